#!/bin/bash
O=gpurun_out/proxy2; mkdir -p $O
run() { local name=$1; shift; env "$@" timeout -k 10 200 python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 240 --warmup 24 $PX > $O/$name.json 2>&1 || exit 1; echo "$name $(grep -o '"ms_per_step[^,]*, "kernel[^,]*, "reserved_cus[^,]*, "graph_launches[^,]*, "projected_node_glups[^}]*' $O/$name.json)"; }
PX="--extra=--no-graph" run nograph_res8 HEAT3D_RESERVE_CUS=8
PX="--extra=--no-graph" run nograph_res0 HEAT3D_RESERVE_CUS=0
PX="--extra=--no-graph" run nograph_res8_ch1 HEAT3D_RESERVE_CUS=8 HEAT3D_PHANTOM_CHANNELS=1
PX="" run graph_res8_ch1 HEAT3D_RESERVE_CUS=8 HEAT3D_PHANTOM_CHANNELS=1
PX="--extra=--no-graph" run nograph_res0_ch1_tr3 HEAT3D_RESERVE_CUS=0 HEAT3D_PHANTOM_CHANNELS=1 HEAT3D_KERNEL2=tr3
