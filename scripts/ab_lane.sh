# A/B of the lane kernel variants (scripts/build_ab.sh names in VARS)
mkdir -p gpurun_out/lane5
for v in ${VARS:-old l64 l32}; do
  L=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/libtmg_ab_$v.so
  TMG_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 > gpurun_out/lane5/${v}_c2.log 2>&1 || exit 1
  TMG_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 --policy effective > gpurun_out/lane5/${v}_c2eff.log 2>&1 || exit 1
  TMG_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 --boards 131072 > gpurun_out/lane5/${v}_c4.log 2>&1 || exit 1
  TMG_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 --boards 131072 --policy effective > gpurun_out/lane5/${v}_c4eff.log 2>&1 || exit 1
  TMG_LIB=$L timeout -k 10 120 python tools/microbench.py > gpurun_out/lane5/${v}_mb.log 2>&1 || exit 1
done
