# parity of the lane + tail hybrid (K=2: the tail path taken most), then c2 / c2-eff / c4 A/B
mkdir -p gpurun_out/tail
L=$PWD/tile-match-gym_amd/tile_match_gym_amd/_lib
for v in old t2; do
  TMG_LIB=$L/libtmg_ab_$v.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_policy.py tests/test_gpu_aux.py > gpurun_out/tail/pytest_$v.log 2>&1 || { tail -30 gpurun_out/tail/pytest_$v.log; exit 1; }
  tail -1 gpurun_out/tail/pytest_$v.log
done
for v in old t2 t3 t4; do
  TMG_LIB=$L/libtmg_ab_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 > gpurun_out/tail/${v}_c2.log 2>&1 || exit 1
  TMG_LIB=$L/libtmg_ab_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 --policy effective > gpurun_out/tail/${v}_c2eff.log 2>&1 || exit 1
  TMG_LIB=$L/libtmg_ab_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --warmup 30 --boards 131072 > gpurun_out/tail/${v}_c4.log 2>&1 || exit 1
  TMG_LIB=$L/libtmg_ab_$v.so timeout -k 10 120 python tools/microbench.py > gpurun_out/tail/${v}_mb.log 2>&1 || exit 1
done
