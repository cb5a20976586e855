#!/bin/bash
# Round-end evidence: GPU parity suite, smoke, default bench (c2 with the CPU
# baseline), the driver's short window, c3 / c5 bench lines.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -20 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 \
  || { echo "smoke failed"; tail -5 gpurun_out/final/smoke.log; exit 1; }
echo "smoke ok: $(tail -1 gpurun_out/final/smoke.log)"
timeout -k 10 400 python bench.py > gpurun_out/final/c2_bench.log 2>&1 || { echo "bench c2 failed"; tail gpurun_out/final/c2_bench.log; exit 1; }
tail -1 gpurun_out/final/c2_bench.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/final/c2_driver_window_bench.log 2>&1 || exit 1
for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/final/${c}_bench.log 2>&1 || { echo "bench $c failed"; exit 1; }
done
for f in c2_bench c2_driver_window_bench c3_bench c5_bench; do
  tail -1 gpurun_out/final/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', '%.4g' % d['value'], 'ms/step', d['ms_per_step'], 'steps', d['steps'])"
done
