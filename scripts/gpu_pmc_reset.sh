#!/bin/bash
# PMC passes on the reset kernel (sb on/off): instruction mix and wave states per dispatch.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmcr
export TMPDIR=/tmp
for sb in ${SBS:-1 0}; do
  TMG_SB=$sb timeout -k 10 60 python tools/reset_probe.py c2 || exit 1
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    TMG_SB=$sb timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmcr/sb${sb}_$i -o run --output-format csv -- python3 tools/reset_probe.py c2 > gpurun_out/pmcr/sb${sb}_$i.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmcr/sb${sb}_$i.log; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections, os
for sb in [int(x) for x in os.environ.get('SBS', '1 0').split()]:
    tot = collections.defaultdict(list)
    for f in glob.glob(f'gpurun_out/pmcr/sb{sb}_*/run_counter_collection.csv'):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if 'reset_kernel' not in r['Kernel_Name']: continue
            per[int(r['Dispatch_Id'])][r['Counter_Name']] += float(r['Counter_Value'])
        for d in per.values():
            for k, v in d.items(): tot[k].append(v)
    print('sb', sb, {k: round(sorted(v)[len(v)//2] / 1e6, 2) for k, v in sorted(tot.items())}, '(millions, median dispatch)')
PY
