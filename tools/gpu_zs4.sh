#!/bin/bash
# z tile stride with nt stores: 58 vs 56 columns, fp64 1024^3 and 768^3 kernel level
O=gpurun_out/zs4; mkdir -p $O
export TMPDIR=/tmp
for n in 1024 768; do
  for rep in 1 2; do
    for zs in 58 56; do
      HEAT3D_TL_ZS=$zs timeout -k 10 200 python3 tools/tune.py --n $n --dtype fp64 --variants tl3 --iters 10 --rounds 2 > $O/t.log 2>&1 || exit 1
      echo "n=$n zs=$zs $(grep -o '"glups_median[^,]*' $O/t.log)"
    done
  done
done
