#!/bin/bash
# Phase-block bench variants + the regeneration-priority A/B (LIBS) on the latency probe.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k phase --timeout 120 --timeout-method thread > gpurun_out/pytest_phase.log 2>&1 || { tail -20 gpurun_out/pytest_phase.log; exit 1; }
tail -1 gpurun_out/pytest_phase.log
for lib in ${LIBS:-libtmg.so}; do
  export TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/$lib
  if [ -z "$NO_PROBE" ]; then
    timeout -k 10 200 python tools/latency_probe.py --skip-reset > gpurun_out/lat_$lib.log 2>&1 || { tail gpurun_out/lat_$lib.log; exit 1; }
    echo "== $lib"; grep groups gpurun_out/lat_$lib.log
  fi
  for spec in ${SPECS:-3:20:5 3:300:30 1:300:30 0:60:30}; do
    IFS=: read -r p1 p2 p3 p4 <<< "$spec"; set -- $p1 $p2 $p3 $p4
    timeout -k 10 300 python bench.py --phase-blocks $1 --steps $2 --warmup $3 ${4:+--phase-interleave} --no-cpu-baseline > gpurun_out/bench_${lib}_p$1_k$2.log 2>&1 || { tail -3 gpurun_out/bench_${lib}_p$1_k$2.log; exit 1; }
    tail -1 gpurun_out/bench_${lib}_p$1_k$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $lib P=$1 K=$2 I=$4', d['value'], 'ms/step', d['ms_per_step'])"
  done
done
