#!/bin/bash
# Env-group count A/B per config (bench flags only).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/groups
for cfg in ${CONFIGS:-c3 c5}; do
  for g in ${GROUPS_LIST:-2 3}; do
    timeout -k 10 300 python bench.py --config $cfg --groups $g --phase-blocks $g --no-cpu-baseline > gpurun_out/groups/${cfg}_g$g.log 2>&1 || { echo "fail $cfg $g"; exit 1; }
    tail -1 gpurun_out/groups/${cfg}_g$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg groups $g', '%.4g' % d['value'], d['ms_per_step'])"
  done
done
