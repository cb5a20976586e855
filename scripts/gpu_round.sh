#!/bin/bash
# GPU iteration: parity suite (stop on failure / fault), then c2 / c3 / c5 bench lines.
# TESTS=0 skips the suite; CONFIGS overrides the bench configs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_EXTRA} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -5 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && { echo "pytest rc=$rc: stopping"; exit $rc; }
fi
for c in ${CONFIGS:-c3 c5 c2}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline ${BENCH_EXTRA} > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.4g' % d['value'], 'ms/step', d['ms_per_step'], 'kernel ms/launch', d['roofline']['kernel_ms_per_launch'])"
done
