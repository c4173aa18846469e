#!/bin/bash
# z-stride robustness: other grid sizes and the 8-slab phantom rank
O=gpurun_out/zs2; mkdir -p $O
run() { env $1 timeout -k 10 200 python3 tools/tune.py --n $2 --dtype fp64 --variants tl3 --iters 8 --rounds 2 > $O/t.log 2>&1 || exit 1; echo "$1 n=$2 $(grep -o '"glups_median[^,]*' $O/t.log)"; }
for n in 512 768 1000 1024 1280; do run HEAT3D_TL_ZS=58 $n; run HEAT3D_TL_ZS=56 $n; done
for zs in 58 56; do
  HEAT3D_TL_ZS=$zs timeout -k 10 200 python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 120 --warmup 24 --extra=--no-graph > $O/p.json 2>/dev/null || exit 1
  echo "proxy8 zs=$zs $(grep -o '"ms_per_step[^,]*' $O/p.json) $(grep -o '"projected_node_glups[^,]*' $O/p.json)"
done
