cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab3
export TMPDIR=/tmp
RUNS="libtmg.so:c3 libtmg_w4.so:c3 libtmg.so:c3 libtmg_w4.so:c3" bash scripts/gpu_libs.sh || exit 1
for lib in libtmg.so libtmg_w4.so; do
  TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/$lib timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/ab3/$lib -o run --output-format csv -- python3 bench.py --config c3 --steps 60 --warmup 30 --no-cpu-baseline > gpurun_out/ab3/$lib.log 2>&1 || exit 1
  python3 - "$lib" <<'PY'
import csv,glob,sys,collections
v=collections.defaultdict(float)
for f in glob.glob(f"gpurun_out/ab3/{sys.argv[1]}/**/*counter_collection.csv",recursive=True):
    for r in csv.DictReader(open(f)):
        if 'step_kernel' in r['Kernel_Name']: v[int(r['Dispatch_Id'])]+=float(r['Counter_Value'])
print(sys.argv[1], 'WRITE_SIZE KiB per step launch', sum(v.values())/max(1,len(v)))
PY
done
