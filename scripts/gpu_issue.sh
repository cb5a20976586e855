#!/bin/bash
# Per config: rocprofv3 --kernel-trace --stats of the bench, the SQ instruction-count
# pass (-> gpurun_out/issue.json for roofline.issue) and the FETCH_SIZE / WRITE_SIZE
# passes (-> gpurun_out/traffic.json for roofline.traffic), each pass its own run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/issue gpurun_out/traffic gpurun_out/stats
export TMPDIR=/tmp
S=${STEPS:-60}; W=${WARMUP:-30}
# bench arguments of a config name (c4: BASELINE configs[3], one GPU's shard; bench.PROFILE_RUNS)
bargs() { case $1 in c4) echo "--config c2 --boards 131072";; *) echo "--config $1";; esac; }
for cfg in ${CONFIGS:-c2 c3 c5 c4}; do
  ARGS="$(bargs $cfg) --steps $S --warmup $W --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats/$cfg -o run --output-format csv \
    -- python3 bench.py $ARGS > gpurun_out/stats/$cfg.log 2>&1 || { echo "stats $cfg failed"; tail -5 gpurun_out/stats/$cfg.log; exit 1; }
  echo "stats $cfg ok: $(tail -1 gpurun_out/stats/$cfg.log | cut -c1-160)"
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-trace -d gpurun_out/issue/$cfg -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/issue/$cfg.log 2>&1 \
    || { echo "pmc SQ $cfg failed"; tail -5 gpurun_out/issue/$cfg.log; exit 1; }
  echo "pmc SQ $cfg ok"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/traffic/${cfg}_$ctr -o run --output-format csv \
      -- python3 bench.py $ARGS > gpurun_out/traffic/${cfg}_$ctr.log 2>&1 \
      || { echo "pmc $cfg $ctr failed"; tail -5 gpurun_out/traffic/${cfg}_$ctr.log; exit 1; }
    echo "pmc $cfg $ctr ok"
  done
done
python3 tools/issue.py gpurun_out/issue $((S + W)) > gpurun_out/issue.json && cat gpurun_out/issue.json
python3 tools/traffic.py gpurun_out/traffic $((S + W)) > gpurun_out/traffic.json && cat gpurun_out/traffic.json
