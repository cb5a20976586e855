#!/bin/bash
# A/B of library builds: RUNS="lib:config lib:config ..." (lib under _lib/), one bench line each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for run in $RUNS; do
  lib=${run%%:*}; cfg=${run##*:}
  TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline ${BENCH_EXTRA} > gpurun_out/ab_${lib}_$cfg.log 2>&1 || { echo "bench $lib $cfg failed"; tail -3 gpurun_out/ab_${lib}_$cfg.log; exit 1; }
  tail -1 gpurun_out/ab_${lib}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('AB $lib $cfg', '%.4g' % d['value'], 'ms/step', d['ms_per_step'])"
done
