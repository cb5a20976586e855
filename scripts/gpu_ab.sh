#!/bin/bash
# A/B: parity + bench for each library given in $LIBS (paths relative to the package _lib dir).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for lib in ${LIBS:-libtmg.so}; do
  export TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/$lib
  echo "== $lib"
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -m pytest ${PYTEST_ARGS:-tests -m gpu -x -q} > gpurun_out/pytest_$lib.log 2>&1
  rc=$?; tail -1 gpurun_out/pytest_$lib.log
  if grep -qiE "illegal memory|APERTURE_VIOLATION|memory access fault|HSA_STATUS_ERROR|core dumped" gpurun_out/pytest_$lib.log; then echo "GPU fault: stop"; exit 3; fi
  [ $rc -ne 0 ] && { echo "parity failed for $lib"; continue; }
  for cfg in ${CONFIGS:-c2}; do
    timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_${lib}_$cfg.log 2>&1 || { tail -3 gpurun_out/bench_${lib}_$cfg.log; exit 1; }
    tail -1 gpurun_out/bench_${lib}_$cfg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', '$lib', '$cfg', d['value'], 'ms/step', d['ms_per_step'])"
  done
done
