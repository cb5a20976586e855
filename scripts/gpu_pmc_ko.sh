#!/bin/bash
# SQ counts per launch kind (tools/microbench.py + tools/pmc_micro.py) for the
# product library and diagnostic knock-out builds (LIBS="ko1 ko2 ..." ->
# _lib/libtmg_ab_<name>.so): attribution of an effective step's instructions.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$PWD/gpurun_out/${TAG:-r06/ko}; mkdir -p $OUT
export TMPDIR=/tmp
LIBDIR=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib
c=${CONFIG:-c2}
nb=$(python3 -c "import bench; print(bench.CONFIGS['$c'][5])")
for ab in product ${LIBS:-}; do
  lib=$LIBDIR/libtmg.so; [ $ab = product ] || lib=$LIBDIR/libtmg_ab_$ab.so
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    TMG_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace -d $OUT/${ab}_${c}_$i -o run --output-format csv -- \
      python3 tools/microbench.py --config $c > $OUT/${ab}_${c}_$i.log 2>&1 || { echo "pmc $ab $i failed"; tail -5 $OUT/${ab}_${c}_$i.log; exit 1; }
  done
  python3 tools/pmc_micro.py $OUT/${ab}_${c}_1 $OUT/${ab}_${c}_2 --boards $nb --eff-frac 0.24 > $OUT/${ab}_${c}.json || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/${ab}_${c}.json'))
for k in ('quick','normal','policy','storm'):
    v=d.get(k,{}); print('$ab', k, 'VALU', round(v.get('SQ_INSTS_VALU',0)), 'SALU', round(v.get('SQ_INSTS_SALU',0)), 'LDS', round(v.get('SQ_INSTS_LDS',0)), 'WC', round(v.get('SQ_WAVE_CYCLES',0)), 'WAIT', round(v.get('SQ_WAIT_INST_ANY',0)))"
done
