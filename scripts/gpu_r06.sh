#!/bin/bash
# Round-6 GPU evidence (same stages as gpu_r06.sh).  Usage (through gpurun, from the repo root):
#   STAGE=tests  bash scripts/gpu_r06.sh   # pytest -m gpu (all but the deep rollouts), smoke, c2 bench
#   STAGE=deep   bash scripts/gpu_r06.sh   # the deep rollouts vs the oracle + the TMG_COVER branch counts
#   STAGE=bench  bash scripts/gpu_r06.sh   # bench lines with the CPU baseline (CONFIGS, POLICY) + driver window
#   STAGE=prof   bash scripts/gpu_r06.sh   # rocprofv3 --kernel-trace --stats of the benches (CONFIGS, POLICY)
#   STAGE=abx    bash scripts/gpu_r06.sh   # A/B: AB="base product <name> ..." (base = the _ab_base/ worktree of
#                                          # the previous commit, <name> = _lib/libtmg_ab_<name>.so), REPS times
#   STAGE=pmcmb  bash scripts/gpu_r06.sh   # SQ counts per launch kind (tools/microbench.py, tools/pmc_micro.py)
#   STAGE=window bash scripts/gpu_r06.sh   # the driver's 20-step window + its kernel timeline
# Each GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r06}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
LIBDIR=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib
# bench arguments of a config name (c4: BASELINE configs[3], one GPU's shard of 1 048 576 / 8 boards)
# (<cfg>-e: the same with the effective-action policy; c2p1: c2 with the episodes aligned, --phase-blocks 1)
bargs() { case $1 in c4) echo "--config c2 --boards 131072";; c2p1) echo "--config c2 --phase-blocks 1";;
                     *-e) echo "--config ${1%-e} --policy effective";; *) echo "--config $1";; esac; }
case "${STAGE:-tests}" in
tests)
  TMG_EVIDENCE_DIR=$OUT/evidence timeout -k 10 900 $PYT tests -m gpu --ignore=tests/test_gpu_deep.py \
    > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
  ;;
deep)
  TMG_COVER_OUT=$OUT/cover.json timeout -k 10 1000 $PYT tests/test_gpu_deep.py > $OUT/pytest_deep.log 2>&1 \
    || { echo "deep failed"; tail -30 $OUT/pytest_deep.log; exit 1; }
  tail -3 $OUT/pytest_deep.log
  ;;
bench)
  for pol in ${POLICY:-uniform}; do
    for c in ${CONFIGS:-c2 c3 c5 c4}; do
      timeout -k 10 400 python bench.py $(bargs $c) --policy $pol ${BENCH_ARGS:-} > $OUT/${c}_${pol}_bench.log 2>&1 \
        || { echo "bench $c $pol failed"; tail $OUT/${c}_${pol}_bench.log; exit 1; }
      echo "$c $pol $(tail -1 $OUT/${c}_${pol}_bench.log | cut -c88-150)"
    done
  done
  if [ -z "${NO_WINDOW:-}" ]; then
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_driver_window_bench.log 2>&1 || exit 1
    echo "window $(tail -1 $OUT/c2_driver_window_bench.log | cut -c88-150)"
  fi
  ;;
prof)
  for pol in ${POLICY:-uniform}; do
    for c in ${CONFIGS:-c2 c3 c5 c4}; do
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_${c}_$pol -o run --output-format csv -- \
        python3 bench.py $(bargs $c) --policy $pol --steps 90 --warmup 30 --no-cpu-baseline > $OUT/${c}_${pol}_prof_bench.log 2>&1 \
        || { echo "prof $c $pol failed"; tail $OUT/${c}_${pol}_prof_bench.log; exit 1; }
      echo "$c $pol $(tail -1 $OUT/${c}_${pol}_prof_bench.log | cut -c88-150)"
    done
  done
  ;;
abx)
  # bench line + per-launch probes per build, REPS times in alternating order (box noise)
  for rep in $(seq 1 ${REPS:-2}); do
    for ab in ${AB:-base product}; do
      dir=$PWD; lib=$LIBDIR/libtmg.so
      case $ab in
        base) dir=$PWD/_ab_base; lib=$dir/tile-match-gym_amd/tile_match_gym_amd/_lib/libtmg.so;;
        product) ;;
        *) lib=$LIBDIR/libtmg_ab_$ab.so;;
      esac
      for c in ${CONFIGS:-c2 c3 c5}; do
        (cd $dir && TMG_LIB=$lib timeout -k 10 300 python bench.py $(bargs $c) ${BENCH_ARGS:-} --no-cpu-baseline) \
          > $OUT/${c}_${ab}_${rep}_bench.log 2>&1 || { echo "bench $ab $c failed"; tail $OUT/${c}_${ab}_${rep}_bench.log; exit 1; }
        if [ -z "${NO_MICRO:-}" ]; then
          (cd $dir && TMG_LIB=$lib timeout -k 10 240 python tools/microbench.py $(bargs $c)) > $OUT/${c}_${ab}_${rep}_micro.log 2>&1 \
            || { echo "micro $ab $c failed"; tail $OUT/${c}_${ab}_${rep}_micro.log; exit 1; }
        fi
        echo "$rep $ab $c $(tail -1 $OUT/${c}_${ab}_${rep}_bench.log | cut -c88-110) $(tail -1 $OUT/${c}_${ab}_${rep}_micro.log 2>/dev/null)"
      done
    done
  done
  ;;
pmcmb)
  # SQ counts per launch kind; TREE=base: the _ab_base/ worktree (previous commit) with its own library
  dir=$PWD; tag=""
  [ "${TREE:-}" = base ] && { dir=$PWD/_ab_base; tag=_base; }
  for c in ${CONFIGS:-c2 c5}; do
    i=0
    for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
               "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
      i=$((i+1))
      (cd $dir && timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace -d $OUT/pmcmb${tag}_${c}_$i -o run --output-format csv -- \
        python3 tools/microbench.py --config $c) > $OUT/pmcmb${tag}_${c}_$i.log 2>&1 || { echo "pmc $c $i failed"; tail -5 $OUT/pmcmb${tag}_${c}_$i.log; exit 1; }
    done
    nb=$(python3 -c "import bench; print(bench.CONFIGS['$c'][5])")
    python3 tools/pmc_micro.py $OUT/pmcmb${tag}_${c}_1 $OUT/pmcmb${tag}_${c}_2 --boards $nb --eff-frac 0.24 > $OUT/pmcmb${tag}_${c}.json \
      && echo "$c$tag" && head -c 300 $OUT/pmcmb${tag}_${c}.json
  done
  ;;
window)
  for k in 20 40 80; do
    timeout -k 10 200 python bench.py --steps $k --warmup 5 --no-cpu-baseline > $OUT/c2_window_$k.log 2>&1 || exit 1
    echo "steps $k: $(tail -1 $OUT/c2_window_$k.log | cut -c88-150)"
  done
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/window_trace -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/window_trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/window_trace.log; exit 1; }
  python3 tools/window_trace.py $OUT/window_trace 20 3 | tee $OUT/window_trace.txt
  ;;
esac
