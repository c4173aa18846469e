#!/bin/bash
# Why does graph replay of the overlapped schedule lose the overlap?  Proxy
# runs under the HIP runtime's graph-execution knobs, plus a kernel trace.
O=gpurun_out/graphq; mkdir -p $O
export TMPDIR=/tmp
run() { local name=$1; shift; env "$@" timeout -k 10 200 python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 120 --warmup 24 $PX > $O/$name.json 2> $O/$name.err || exit 1; echo "$name $(grep -o '"ms_per_step[^,]*, "kernel[^,]*, "reserved_cus[^,]*, "graph_launches[^,]*, "projected_node_glups[^,]*' $O/$name.json)"; }
PX="--extra=--no-graph" run eager HEAT3D_RESERVE_CUS=8
PX="" run graph HEAT3D_GRAPH_MULTISTREAM=1
PX="" run graph_q1 HEAT3D_GRAPH_MULTISTREAM=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1
PX="" run graph_q4 HEAT3D_GRAPH_MULTISTREAM=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
PX="" run graph_nopc HEAT3D_GRAPH_MULTISTREAM=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
PX="" run graph_log HEAT3D_GRAPH_MULTISTREAM=1 AMD_LOG_LEVEL=3 AMD_LOG_MASK=0x7fffffff
grep -E "hipGraph\] Creating|max_streams" $O/graph_log.err | sort | uniq -c | head -20 > $O/graph_log_summary.txt
rm -f $O/graph_log.err
cat $O/graph_log_summary.txt
HEAT3D_GRAPH_MULTISTREAM=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 48 --warmup 12 > $O/trace.log 2>&1; echo trace rc=$?
