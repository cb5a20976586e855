#!/bin/bash
# Round-6 final evidence on the final build (through gpurun, from the repo root):
#   STAGE=tests  : pytest -m gpu (all, deep rollouts with the TMG_COVER counts included) + smoke
#   STAGE=prof   : scripts/gpu_issue.sh over RUNS (stats, SQ, FETCH_SIZE, WRITE_SIZE per run)
#   STAGE=lines  : bench lines with the CPU baseline (copy gpurun_out/{issue,traffic}.json to profiles/ first,
#                  so the lines carry them) + the driver-like windows
#   STAGE=pmcmb  : SQ counts per launch kind (scripts/gpu_r06.sh STAGE=pmcmb)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$PWD/gpurun_out/r06/${FINAL:-final}; mkdir -p $OUT
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
case "${STAGE:-tests}" in
tests)
  TMG_EVIDENCE_DIR=$OUT/evidence timeout -k 10 600 $PYT tests -m gpu --ignore=tests/test_gpu_deep.py > $OUT/pytest_gpu.log 2>&1 \
    || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  TMG_COVER_OUT=$OUT/cover.json timeout -k 10 1000 $PYT tests/test_gpu_deep.py > $OUT/pytest_deep.log 2>&1 \
    || { echo "deep failed"; tail -30 $OUT/pytest_deep.log; exit 1; }
  tail -1 $OUT/pytest_deep.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
  ;;
prof)
  RUNS="${RUNS:-c2 c2-p1 c2-vec c3 c5 c4 c2-eff c3-eff c5-eff c4-eff}" bash scripts/gpu_issue.sh
  ;;
lines)
  run() {   # name, bench args...
    local name=$1; shift
    timeout -k 10 400 python bench.py "$@" > $OUT/$name.log 2>&1 || { echo "bench $name failed"; tail $OUT/$name.log; exit 1; }
    tail -1 $OUT/$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name', '%.4g' % d['value'], 'ms/step', d['ms_per_step'], 'issue', (r.get('issue') or {}).get('salu_frac'), 'traffic', r.get('traffic_bytes_per_env_step'), 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
  }
  run c2 ; run c2_p1 --phase-blocks 1 ; run c2_vec --api vector ; run c2_eff --policy effective
  run c3 --config c3 ; run c3_eff --config c3 --policy effective ; run c4 --config c2 --boards 131072 ; run c4_eff --config c2 --boards 131072 --policy effective
  run c5 --config c5 ; run c5_eff --config c5 --policy effective ; run g1 --config g1 ; run g2 --config g2
  for i in 1 2 3; do run window20_$i --steps 20 --warmup 5 --no-cpu-baseline; done
  run window40 --steps 40 --warmup 5 --no-cpu-baseline ; run window80 --steps 80 --warmup 5 --no-cpu-baseline
  run gpus2 --gpus 2 --no-cpu-baseline
  ;;
pmcmb)
  STAGE=pmcmb TAG=r06/${FINAL:-final} CONFIGS="${CONFIGS:-c2 c3 c5}" bash scripts/gpu_r06.sh
  ;;
esac
