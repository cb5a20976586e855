#!/bin/bash
# Per profiled run (bench.run_args names: c2 c3 c5, c4 = the c2 shard of 131 072 boards, a "-eff" suffix = the
# effective-action policy): rocprofv3 --kernel-trace --stats of the bench, the SQ instruction-count pass
# (-> gpurun_out/issue.json for roofline.issue) and the FETCH_SIZE / WRITE_SIZE passes (-> gpurun_out/traffic.json
# for roofline.traffic), each pass its own run.  The reducers record each run's build hash and shape from its
# bench line, and bench.py attaches a profile only to a line of the same build and run shape.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/issue gpurun_out/traffic gpurun_out/stats
export TMPDIR=/tmp
S=${STEPS:-60}; W=${WARMUP:-30}
for run in ${RUNS:-c2 c3 c5 c4 c2-eff c3-eff c5-eff}; do
  ARGS="$(python3 -c "import bench; print(' '.join(bench.run_args('$run')))") --steps $S --warmup $W --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats/$run -o run --output-format csv \
    -- python3 bench.py $ARGS > gpurun_out/stats/$run.log 2>&1 || { echo "stats $run failed"; tail -5 gpurun_out/stats/$run.log; exit 1; }
  echo "stats $run ok: $(tail -1 gpurun_out/stats/$run.log | cut -c88-150)"
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-trace -d gpurun_out/issue/$run -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/issue/$run.log 2>&1 \
    || { echo "pmc SQ $run failed"; tail -5 gpurun_out/issue/$run.log; exit 1; }
  echo "pmc SQ $run ok"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/traffic/${run}_$ctr -o run --output-format csv \
      -- python3 bench.py $ARGS > gpurun_out/traffic/${run}_$ctr.log 2>&1 \
      || { echo "pmc $run $ctr failed"; tail -5 gpurun_out/traffic/${run}_$ctr.log; exit 1; }
    echo "pmc $run $ctr ok"
  done
done
python3 tools/issue.py gpurun_out/issue $((S + W)) > gpurun_out/issue.json && head -c 400 gpurun_out/issue.json
python3 tools/traffic.py gpurun_out/traffic $((S + W)) > gpurun_out/traffic.json && head -c 400 gpurun_out/traffic.json
