#!/bin/bash
# flattened (kernel-node) multi-stream graphs: bitwise tests, proxy speed, trace
O=gpurun_out/graphq2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_graph.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; true
run() { local name=$1; shift; env "$@" timeout -k 10 200 python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 120 --warmup 24 $PX > $O/$name.json 2> $O/$name.err || exit 1; echo "$name $(grep -o '"ms_per_step[^,]*, "kernel[^,]*, "reserved_cus[^,]*, "graph_launches[^,]*, "projected_node_glups[^,]*' $O/$name.json)"; }
PX="--extra=--no-graph" run eager HEAT3D_RESERVE_CUS=8
PX="" run graph_flat HEAT3D_GRAPH_MULTISTREAM=1
PX="" run graph_child HEAT3D_GRAPH_MULTISTREAM=1 HEAT3D_GRAPH_FLATTEN=0
PX="" run graph_flat_res0 HEAT3D_GRAPH_MULTISTREAM=1 HEAT3D_RESERVE_CUS=0
HEAT3D_GRAPH_MULTISTREAM=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 48 --warmup 12 > $O/trace.log 2>&1; echo trace rc=$?
