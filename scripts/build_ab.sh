#!/bin/bash
# Build A/B variants of libtmg.so from this tree (CPU, in-tree):
#   bash scripts/build_ab.sh "name:-DFLAG=1 -DOTHER=2" "name2:-DX=0"
# -> tile_match_gym_amd/_lib/libtmg_<name>.so, variant ab_<name> (same sources, so the loader accepts them via TMG_LIB)
cd "$(dirname "$0")/../tile-match-gym_amd"
rm -f tile_match_gym_amd/_lib/libtmg_ab_*.so
for v in "$@"; do
  n=${v%%:*}; f=${v#*:}
  make -j8 OUT=tile_match_gym_amd/_lib/libtmg_ab_$n.so VARIANT=ab_$n EXTRA="$f" > /tmp/build_ab_$n.log 2>&1 || { echo "build $n failed"; tail /tmp/build_ab_$n.log; exit 1; }
done
ls tile_match_gym_amd/_lib/
