#!/bin/bash
# GPU session: parity tests, then a short bench.  Stops at the first crash/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PYTEST_ARGS=${PYTEST_ARGS:-tests -m gpu -x -q}
timeout -k 10 ${PYTEST_TIMEOUT:-700} python -m pytest $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" | tee -a gpurun_out/pytest_gpu.log
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if grep -qiE "illegal memory|APERTURE_VIOLATION|memory access fault|HSA_STATUS_ERROR|core dumped" gpurun_out/pytest_gpu.log; then
  echo "GPU fault detected: stopping"; exit 3; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py ${BENCH_ARGS:---steps 60 --warmup 30 --no-cpu-baseline} > gpurun_out/bench.log 2>&1
brc=$?
echo "bench rc=$brc"
tail -5 gpurun_out/bench.log
exit $brc
