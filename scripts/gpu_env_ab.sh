#!/bin/bash
# Parity suite once, then the c2 bench + microbench under each environment in $VARIANTS
# (space-separated; each a comma-separated list of VAR=value, "base" = none).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NO_PARITY" ]; then
  SKIP_BENCH=1 PYTEST_ARGS="tests -m gpu -x -q --timeout 300 --timeout-method thread" bash scripts/gpu_check.sh || exit $?
  grep -q " failed" gpurun_out/pytest_gpu.log && { echo "parity failures: stop"; exit 1; }
fi
for v in ${VARIANTS:-base}; do
  envs=""; [ "$v" != "base" ] && envs=$(echo "$v" | tr ',' ' ')
  env $envs timeout -k 10 200 python bench.py --config ${CFG:-c2} --no-cpu-baseline > gpurun_out/bench_ab.log 2>&1 || { tail -5 gpurun_out/bench_ab.log; exit 1; }
  tail -1 gpurun_out/bench_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $v', d['value'], 'ms/step', d['ms_per_step'], 'kern', d['roofline']['kernel_ms_per_launch'])"
  [ -z "$NO_MICRO" ] && { env $envs timeout -k 10 120 python tools/microbench.py --config ${CFG:-c2} || exit 1; }
done
exit 0
