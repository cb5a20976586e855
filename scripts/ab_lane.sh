mkdir -p gpurun_out/lane3
for nb in 131072 262144 524288; do
  for v in old lane; do
    for pol in uniform effective; do
      TMG_LIB=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib/libtmg_ab_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --boards $nb --steps 90 --warmup 30 --policy $pol > gpurun_out/lane3/${v}_${nb}_${pol}.log 2>&1 || exit 1
    done
  done
done
