#!/bin/bash
# Round-4 GPU evidence.  Usage (through gpurun, from the repo root):
#   STAGE=tests bash scripts/gpu_r04.sh   # pytest -m gpu (all but the deep rollouts), smoke, c2 bench
#   STAGE=deep  bash scripts/gpu_r04.sh   # the deep rollouts vs the oracle + the TMG_COVER branch counts
#   STAGE=bench bash scripts/gpu_r04.sh   # c2 / c3 / c5 / c4-shard bench lines with the CPU baseline + driver window
#   STAGE=prof  bash scripts/gpu_r04.sh   # rocprofv3 --kernel-trace --stats of the c2 / c3 / c5 / c4 benches
#   STAGE=abx   bash scripts/gpu_r04.sh   # A/B: product vs _lib/libtmg_ab_<name>.so for AB="name ..." (scripts/build_ab.sh)
#   STAGE=pmcmb bash scripts/gpu_r04.sh   # SQ instruction counts per launch kind (tools/microbench.py, tools/pmc_micro.py)
#   STAGE=window bash scripts/gpu_r04.sh  # the driver's 20-step window vs longer ones + its kernel timeline
#   STAGE=final bash scripts/gpu_r04.sh   # deep, bench, pmcmb (c2 c5), facade probe
#   STAGE=all   bash scripts/gpu_r04.sh   # tests, deep, bench
# Each GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
# LIB=libtmg_<x>.so: every step below runs that build of this tree (TMG_LIB)
[ -n "${LIB:-}" ] && export TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/$LIB
mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
# bench arguments of a config name (c4: BASELINE configs[3], one GPU's shard of 1 048 576 / 8 boards)
bargs() { case $1 in c4) echo "--config c2 --boards 131072";; *) echo "--config $1";; esac; }
case "${STAGE:-tests}" in
tests)
  TMG_EVIDENCE_DIR=$OUT/evidence timeout -k 10 900 $PYT tests -m gpu --ignore=tests/test_gpu_deep.py \
    > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
  timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/c2_bench.log 2>&1 || { echo "bench failed"; tail $OUT/c2_bench.log; exit 1; }
  tail -1 $OUT/c2_bench.log | cut -c1-300
  ;;
deep)
  TMG_COVER_OUT=$OUT/cover.json timeout -k 10 1000 $PYT tests/test_gpu_deep.py > $OUT/pytest_deep.log 2>&1 \
    || { echo "deep failed"; tail -30 $OUT/pytest_deep.log; exit 1; }
  tail -3 $OUT/pytest_deep.log
  ;;
bench)
  for c in ${CONFIGS:-c2 c3 c5 c4}; do
    timeout -k 10 400 python bench.py $(bargs $c) > $OUT/${c}_bench.log 2>&1 || { echo "bench $c failed"; tail $OUT/${c}_bench.log; exit 1; }
    tail -1 $OUT/${c}_bench.log | cut -c1-200
  done
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_driver_window_bench.log 2>&1 || exit 1
  tail -1 $OUT/c2_driver_window_bench.log | cut -c1-200
  ;;
probe)
  # per-launch breakdown: quick-exit floor / normal step / autoreset storm, and a bare reset
  for c in ${CONFIGS:-c2 c3 c5}; do
    timeout -k 10 240 python tools/microbench.py --config $c > $OUT/${c}_microbench.log 2>&1 \
      || { echo "microbench $c failed"; tail $OUT/${c}_microbench.log; exit 1; }
    echo "$c $(tail -1 $OUT/${c}_microbench.log)"
    timeout -k 10 240 python tools/reset_probe.py $c > $OUT/${c}_reset_probe.log 2>&1 \
      || { echo "reset_probe $c failed"; tail $OUT/${c}_reset_probe.log; exit 1; }
    tail -1 $OUT/${c}_reset_probe.log
  done
  ;;
iter)
  # one iteration: GPU parity suite (not the deep rollouts), then c2/c3/c5 bench lines (no CPU baseline) and the
  # per-launch probes; AB="name ..." adds c2/c3 bench lines of _lib/libtmg_ab_<name>.so
  TMG_EVIDENCE_DIR=$OUT/evidence timeout -k 10 900 $PYT tests -m gpu --ignore=tests/test_gpu_deep.py \
    > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  for c in ${CONFIGS:-c2 c3 c5}; do
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/${c}_bench.log 2>&1 || { echo "bench $c failed"; tail $OUT/${c}_bench.log; exit 1; }
    echo "$c $(tail -1 $OUT/${c}_bench.log | cut -c80-140)"
    timeout -k 10 240 python tools/microbench.py --config $c > $OUT/${c}_microbench.log 2>&1 || { echo "microbench $c failed"; exit 1; }
    echo "$c $(tail -1 $OUT/${c}_microbench.log)"
  done
  for ab in ${AB:-}; do
    for c in c2 c3; do
      TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/libtmg_ab_$ab.so timeout -k 10 300 python bench.py --config $c \
        --no-cpu-baseline > $OUT/${c}_ab_${ab}_bench.log 2>&1 || { echo "bench ab $ab $c failed"; tail $OUT/${c}_ab_${ab}_bench.log; exit 1; }
      echo "ab $ab $c $(tail -1 $OUT/${c}_ab_${ab}_bench.log | cut -c80-140)"
    done
  done
  ;;
abx)
  # A/B: bench line + per-launch probes for the product library and each _lib/libtmg_ab_<name>.so in AB, twice
  # each in alternating order (box noise)
  for rep in $(seq 1 ${REPS:-2}); do
    for ab in product ${AB:-}; do
      lib=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/libtmg.so
      [ $ab != product ] && lib=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/libtmg_ab_$ab.so
      for c in ${CONFIGS:-c2 c3}; do
        TMG_LIB=$lib timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $OUT/${c}_${ab}_${rep}_bench.log 2>&1 \
          || { echo "bench $ab $c failed"; tail $OUT/${c}_${ab}_${rep}_bench.log; exit 1; }
        TMG_LIB=$lib timeout -k 10 240 python tools/microbench.py --config $c > $OUT/${c}_${ab}_${rep}_micro.log 2>&1 \
          || { echo "micro $ab $c failed"; exit 1; }
        echo "$rep $ab $c $(tail -1 $OUT/${c}_${ab}_${rep}_bench.log | cut -c88-110) $(tail -1 $OUT/${c}_${ab}_${rep}_micro.log)"
      done
    done
  done
  ;;
pmcmb)
  # SQ instruction counts per launch kind (normal / storm / quick step launches, reset / spill launches) of
  # tools/microbench.py; PMCLIBS="product ab_old": one set per library build
  for lib in ${PMCLIBS:-product}; do
  [ $lib != product ] && export TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/libtmg_$lib.so
  for c in ${CONFIGS:-c2}; do
    i=0
    for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
               "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
      i=$((i+1))
      timeout -s KILL 150 rocprofv3 --pmc $set --kernel-trace -d $OUT/pmcmb_${lib}_${c}_$i -o run --output-format csv -- \
        python3 tools/microbench.py --config $c ${BOARDS:+--boards $BOARDS} > $OUT/pmcmb_${lib}_${c}_$i.log 2>&1 || { echo "pmc $c $i failed"; tail -5 $OUT/pmcmb_${lib}_${c}_$i.log; exit 1; }
    done
    nb=${BOARDS:-$(python3 -c "import bench; print(bench.CONFIGS['$c'][5])")}
    python3 tools/pmc_micro.py $OUT/pmcmb_${lib}_${c}_1 $OUT/pmcmb_${lib}_${c}_2 --boards $nb --eff-frac 0.24 > $OUT/pmcmb_${lib}_${c}.json && echo "$lib $c" && head -c 600 $OUT/pmcmb_${lib}_${c}.json
  done
  done
  ;;
window)
  # the driver's short window (--steps 20 --warmup 5) against longer ones, and its kernel timeline
  for k in 20 40 80; do
    timeout -k 10 200 python bench.py --steps $k --warmup 5 --no-cpu-baseline > $OUT/c2_window_$k.log 2>&1 || exit 1
    echo "steps $k: $(tail -1 $OUT/c2_window_$k.log | cut -c88-140)"
  done
  for v in "--phase-interleave" "--phase-align 0"; do
    for k in 20 300; do
      n=$(echo "$v" | tr -d ' -')_$k
      timeout -k 10 200 python bench.py --steps $k --warmup 5 --no-cpu-baseline $v > $OUT/c2_window_$n.log 2>&1 || exit 1
      echo "$v steps $k: $(tail -1 $OUT/c2_window_$n.log | cut -c88-140)"
    done
  done
  timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/window_trace -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/window_trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/window_trace.log; exit 1; }
  python3 tools/window_trace.py $OUT/window_trace 20 3 | tee $OUT/window_trace.txt
  ;;
final)
  # round-end evidence: deep rollouts + cover counts, bench lines with CPU baselines (c2 c3 c5 and the c4
  # shard) + the driver's window, SQ counts per launch kind (c2, c5), the single-env facade probe
  STAGE=deep bash scripts/gpu_r04.sh && STAGE=bench bash scripts/gpu_r04.sh || exit 1
  STAGE=pmcmb CONFIGS="c2 c5" bash scripts/gpu_r04.sh || exit 1
  timeout -k 10 120 python tools/facade_probe.py > $OUT/facade_probe.log 2>&1 && cat $OUT/facade_probe.log
  ;;
all)
  STAGE=tests bash scripts/gpu_r04.sh && STAGE=deep bash scripts/gpu_r04.sh && STAGE=bench bash scripts/gpu_r04.sh
  ;;
prof)
  for c in ${CONFIGS:-c2 c3 c5 c4}; do
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- \
      python3 bench.py $(bargs $c) --steps 90 --warmup 30 --no-cpu-baseline > $OUT/${c}_prof_bench.log 2>&1 \
      || { echo "prof $c failed"; tail $OUT/${c}_prof_bench.log; exit 1; }
    tail -1 $OUT/${c}_prof_bench.log | cut -c1-200
  done
  ;;
esac
