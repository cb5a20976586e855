mkdir -p gpurun_out/grp
for g in 3 4 6 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 --policy effective --groups $g > gpurun_out/grp/c2eff_g$g.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 --policy effective --groups $g --boards 131072 > gpurun_out/grp/c4eff_g$g.log 2>&1 || exit 1
done
