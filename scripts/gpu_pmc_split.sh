#!/bin/bash
# kernel trace + PMC, split into reset-storm dispatches (top 1/30) and normal ones.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$LIB" ] && export TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/$LIB
ARGS="--steps 90 --warmup 30 --no-cpu-baseline ${EXTRA:-}"
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmcs$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmcs$i.log 2>&1 || { tail -5 gpurun_out/pmcs$i.log; exit 1; }
done
python3 - <<'PY'
import csv, collections, statistics, glob
per=collections.defaultdict(dict); dur={}
for f in glob.glob('gpurun_out/pmcs*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'step_kernel' not in r['Kernel_Name']: continue
        k=(f, int(r['Dispatch_Id']))
        per[k][r['Counter_Name']]=per[k].get(r['Counter_Name'],0)+float(r['Counter_Value'])
        dur[k]=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
byf=collections.defaultdict(list)
for k in per: byf[k[0]].append(k)
for f,ks in sorted(byf.items()):
    ks.sort(key=lambda k: dur[k])
    nres=max(1,len(ks)//30)
    norm, res = ks[:-nres], ks[-nres:]
    names=sorted(per[ks[0]].keys())
    print(f, 'normal us', round(statistics.median([dur[k] for k in norm]),1), 'reset us', round(statistics.median([dur[k] for k in res]),1))
    for n in names:
        print(f"   {n:22s} normal {statistics.median([per[k][n] for k in norm]):14.0f}   reset {statistics.median([per[k][n] for k in res]):14.0f}")
PY
