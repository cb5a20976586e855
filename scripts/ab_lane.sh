# A/B of the lane kernel variants (scripts/build_ab.sh names in VARS)
mkdir -p gpurun_out/lane12
for v in ${VARS:-r2 r8}; do
  L=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/libtmg_ab_$v.so
  for rep in 1 2; do
  TMG_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 --policy effective > gpurun_out/lane12/${v}_c2eff_$rep.log 2>&1 || exit 1
  TMG_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 --boards 131072 --policy effective > gpurun_out/lane12/${v}_c4eff_$rep.log 2>&1 || exit 1
  done
done
