#!/bin/bash
# Phase-alignment A/B: the driver's short window and the default window.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/align
for i in 1 2; do
  for args in "--steps 20 --warmup 5 --phase-align 0" "--steps 20 --warmup 5 --phase-align 1" "--phase-align 0" "--phase-align 1"; do
    tag=$(echo "$args" | tr -d ' -')
    timeout -k 10 300 python bench.py $args --no-cpu-baseline > gpurun_out/align/c2_$tag.log 2>&1 || { echo "fail $args"; exit 1; }
    tail -1 gpurun_out/align/c2_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 $args', '%.4g' % d['value'], d['ms_per_step'])"
  done
done
for c in c3 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/align/${c}_short.log 2>&1 || exit 1
  tail -1 gpurun_out/align/${c}_short.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c 20/5 aligned', '%.4g' % d['value'], d['ms_per_step'])"
done
