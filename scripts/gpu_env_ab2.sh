#!/bin/bash
# c3 autoreset-mode A/B through the runtime switches (no rebuild).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in 1 2; do
  for mode in "X=0" "TMG_DEFER=0" "TMG_RESETQ=1"; do
    env $mode timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > gpurun_out/envab_$i.log 2>&1 || { echo "fail $mode"; tail -3 gpurun_out/envab_$i.log; exit 1; }
    tail -1 gpurun_out/envab_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', '%.4g' % d['value'], d['ms_per_step'])"
  done
done
