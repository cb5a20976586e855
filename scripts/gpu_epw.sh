#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/pytest_epw.log 2>&1; tail -1 gpurun_out/pytest_epw.log
grep -qiE "illegal memory|APERTURE|fault|core dumped" gpurun_out/pytest_epw.log && exit 3
for lib in ${LIBS:-libtmg.so}; do for epw in ${EPWS:-1 4 8 16 64}; do
  TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/$lib TMG_EPW=$epw timeout -k 10 300 python bench.py --no-cpu-baseline ${EXTRA:-} > gpurun_out/b.log 2>&1 || { tail -3 gpurun_out/b.log; exit 1; }
  tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH $lib epw=$epw', d['config']['workload'][:3], d['value'], 'ms/step', d['ms_per_step'])"
done; done
