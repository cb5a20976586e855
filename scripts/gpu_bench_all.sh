#!/bin/bash
# Default bench (c2, with CPU baseline) + rocprofv3 stats + c3/c5 bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 || { echo "prof failed"; tail gpurun_out/prof_c2.log; exit 1; }
find gpurun_out/prof_c2 -name "*kernel_stats.csv" -exec head -4 {} \;
for c in c3 c5; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
done
