#!/bin/bash
# z stride on the x-slab shares of the 2/4/8-GPU bench (phantom rank proxy)
O=gpurun_out/zs3; mkdir -p $O
for P in 2 4 8; do for zs in 58 56; do
  HEAT3D_TL_ZS=$zs timeout -k 10 200 python3 tools/rank_proxy.py --ranks $P --gbps 64 --steps 120 --warmup 24 --extra=--no-graph > $O/p.json 2>/dev/null || exit 1
  echo "proxy$P zs=$zs $(grep -o '"ms_per_step[^,]*' $O/p.json) $(grep -o '"projected_node_glups[^,]*' $O/p.json)"
done; done
