#!/bin/bash
# z tile stride with nt stores on the slab shares (phantom rank) and 512^3
O=gpurun_out/zs5; mkdir -p $O
export TMPDIR=/tmp
for r in 8 4; do
  for zs in 56 0; do
    HEAT3D_TL_ZS=$zs timeout -k 10 200 python3 tools/rank_proxy.py --ranks $r --gbps 64 --steps 120 --warmup 24 --extra=--no-graph > $O/p$r$zs.json 2>&1 || exit 1
    echo "ranks=$r zs=$zs $(grep -o '"ms_per_step[^,]*' $O/p$r$zs.json) $(grep -o '"projected_node_glups[^,}]*' $O/p$r$zs.json)"
  done
done
for n in 512 1280; do
  for zs in 58 56; do
    HEAT3D_TL_ZS=$zs timeout -k 10 200 python3 tools/tune.py --n $n --dtype fp64 --variants tl3 --iters 10 --rounds 2 > $O/t.log 2>&1 || exit 1
    echo "n=$n zs=$zs $(grep -o '"glups_median[^,]*' $O/t.log)"
  done
done
