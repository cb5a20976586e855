#!/bin/bash
# Round-6 bench lines of the phase layouts and the vector-env API (c2), each
# under its own time limit; stops at the first failure.
#   TAG=r06/s7 bash scripts/gpu_r06_lines.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$PWD/gpurun_out/${TAG:-r06/lines}
mkdir -p $OUT
export TMPDIR=/tmp
run() {   # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/$name.log 2>&1 || { echo "bench $name failed"; tail $OUT/$name.log; exit 1; }
  echo "$name $(tail -1 $OUT/$name.log | cut -c80-125)"
}
run raw_p3 --no-cpu-baseline
run raw_p1 --phase-blocks 1 --no-cpu-baseline
run vec_p1 --api vector --phase-blocks 1 --no-cpu-baseline
run vec_p1_i8 --api vector --phase-blocks 1 --obs-dtype int8 --no-cpu-baseline
run vec_p3 --api vector --no-cpu-baseline
run vec_p1_g3 --api vector --phase-blocks 1 --groups 3 --no-cpu-baseline
for i in 1 2 3; do run window_$i --steps 20 --warmup 5 --no-cpu-baseline; done
