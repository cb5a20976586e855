#!/bin/bash
# One optimisation iteration: GPU parity suite, default bench, SALU/VALU PMC pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
SKIP_BENCH=1 PYTEST_TIMEOUT=${PYTEST_TIMEOUT:-600} bash scripts/gpu_check.sh || exit $?
grep -q "failed" gpurun_out/pytest_gpu.log && { echo "parity failures: not benchmarking"; exit 1; }
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['config']['workload'][:3], d['value'], 'ms/step', d['ms_per_step'])"
if [ -z "$NO_PMC" ]; then
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace -d gpurun_out/pmc_iter -o run --output-format csv -- python3 bench.py --steps 60 --warmup 30 --no-cpu-baseline > gpurun_out/pmc_iter.log 2>&1 || { tail -5 gpurun_out/pmc_iter.log; exit 1; }
  python3 - <<'PY'
import csv, collections, statistics
rows=list(csv.DictReader(open('gpurun_out/pmc_iter/run_counter_collection.csv')))
per=collections.defaultdict(dict)
for r in rows:
    if 'step_kernel' not in r['Kernel_Name']: continue
    d=per[int(r['Dispatch_Id'])]; d[r['Counter_Name']]=d.get(r['Counter_Name'],0)+float(r['Counter_Value'])
names=sorted(next(iter(per.values())).keys())
for n in names:
    v=[per[d][n] for d in per]
    big=sorted(v)[-2:]
    print(f"PMC {n:22s} median {statistics.median(v):14.0f}  max {max(v):14.0f}")
PY
fi
