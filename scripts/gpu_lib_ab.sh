#!/bin/bash
# Per library build ($LIBS): microbench (normal / storm / quick launch times) + aligned 300-step bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lib in ${LIBS:-libtmg.so}; do
  export TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/$lib
  timeout -k 10 120 python tools/microbench.py --config ${CFG:-c2} > gpurun_out/micro_$lib.log 2>&1 || { tail gpurun_out/micro_$lib.log; exit 1; }
  echo "== $lib $(tail -1 gpurun_out/micro_$lib.log)"
  timeout -k 10 300 python bench.py --config ${CFG:-c2} ${BENCH_ARGS:---phase-blocks 1 --steps 300 --warmup 30} --no-cpu-baseline > gpurun_out/bench_$lib.log 2>&1 || { tail -3 gpurun_out/bench_$lib.log; exit 1; }
  tail -1 gpurun_out/bench_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $lib', d['value'], 'ms/step', d['ms_per_step'])"
done
