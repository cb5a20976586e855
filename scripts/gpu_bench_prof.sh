#!/bin/bash
# Bench (with CPU baseline) + rocprofv3 kernel-trace stats of the same command.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 300 --warmup 30}
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py $ARGS > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ -z "$NO_PROF" ]; then
  timeout -k 10 ${PROF_TIMEOUT:-400} rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py $ARGS --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \; | head -20
fi
exit $rc
