#!/bin/bash
# rocprofv3 PMC passes (each its own run, --kernel-trace only) on a short bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 60 --warmup 30 --no-cpu-baseline}
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmc/p$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok"
done
