#!/bin/bash
# HBM traffic per step_kernel launch (roofline.traffic in bench.py), one rocprofv3
# --pmc pass per counter as MI355X_MICROARCH.md "HBM [CDNA4]" prescribes:
# FETCH_SIZE (doubled: gfx950 tallies 128-B requests at 64 B) and WRITE_SIZE in
# separate passes, --kernel-trace only.  Writes gpurun_out/traffic.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/traffic
export TMPDIR=/tmp
for cfg in ${CONFIGS:-c2 c3 c5}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d gpurun_out/traffic/${cfg}_$ctr -o run --output-format csv \
      -- python3 bench.py --config $cfg --steps 60 --warmup 30 --no-cpu-baseline > gpurun_out/traffic/${cfg}_$ctr.log 2>&1 \
      || { echo "pmc $cfg $ctr failed"; tail -5 gpurun_out/traffic/${cfg}_$ctr.log; exit 1; }
    echo "pmc $cfg $ctr ok"
  done
done
python3 tools/traffic.py gpurun_out/traffic > gpurun_out/traffic.json && cat gpurun_out/traffic.json
