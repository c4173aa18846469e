#!/bin/bash
# boundary slabs after the interior vs as soon as the halo lands, phantom rank 1 of 8 / 4
O=gpurun_out/bnd; mkdir -p $O
for r in 8 4; do
for g in 64 150 400; do
  for a in 0 1; do
    HEAT3D_BND_AFTER_INT=$a timeout -k 10 200 python3 tools/rank_proxy.py --ranks $r --gbps $g --steps 120 --warmup 24 --extra=--no-graph > $O/p.json 2>&1 || exit 1
    echo "ranks=$r gbps=$g after=$a $(grep -o '"ms_per_step[^,]*' $O/p.json) $(grep -o '"projected_node_glups[^,}]*' $O/p.json)"
  done
done
done
