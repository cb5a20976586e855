#!/bin/bash
# Parity suite, then c2 bench + launch microbench with the scalar-bitboard kernels on/off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKIP_BENCH=1 PYTEST_ARGS="tests -m gpu -x -q --timeout 300 --timeout-method thread" bash scripts/gpu_check.sh || exit $?
grep -q " failed" gpurun_out/pytest_gpu.log && { echo "parity failures: stop"; exit 1; }
for sb in 1 0; do
  TMG_SB=$sb timeout -k 10 200 python bench.py --config ${CFG:-c2} --no-cpu-baseline > gpurun_out/bench_sb$sb.log 2>&1 || { tail -5 gpurun_out/bench_sb$sb.log; exit 1; }
  tail -1 gpurun_out/bench_sb$sb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH sb=$sb', d['value'], 'ms/step', d['ms_per_step'], 'kern', d['roofline']['kernel_ms_per_launch'])"
  TMG_SB=$sb timeout -k 10 120 python tools/microbench.py --config ${CFG:-c2} || exit 1
done
for sb in 1 0; do TMG_SB=$sb timeout -k 10 60 python tools/reset_probe.py c2 || exit 1; done
