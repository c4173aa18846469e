#!/bin/bash
# fp32 pair kernel: 64-B aligned z stride (112) and nt stores vs the default (120, write-back)
O=gpurun_out/tpzs; mkdir -p $O
P=tl3:2:3:1:16:0:3
for n in 1024 2049; do
for zs in 120 112; do
  HEAT3D_TP_ZS=$zs timeout -k 10 250 python3 tools/tune.py --n $n --dtype fp32 --variants $P $P:2 --iters 8 --rounds 2 > $O/t.log 2>&1 || exit 1
  echo "n=$n zs=$zs $(grep -o '"variant[^,]*, "glups_median[^,]*' $O/t.log | tr '\n' ' ')"
done
done
