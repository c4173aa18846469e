#!/bin/bash
# phantom rank 1 of 8 (1024^3 fp64 slabs): projected node GLUPS and one kernel trace
O=gpurun_out/ptrace; mkdir -p $O
export TMPDIR=/tmp
for g in 64 1000; do
  timeout -k 10 200 python3 tools/rank_proxy.py --ranks 8 --gbps $g --steps 120 --warmup 24 --extra=--no-graph > $O/p$g.json 2>&1 || exit 1
  echo "gbps=$g $(grep -o '"ms_per_step[^,]*' $O/p$g.json) $(grep -o '"projected_node_glups[^,}]*' $O/p$g.json)"
done
timeout -k 10 200 python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 120 --warmup 24 --extra="--no-graph --no-overlap" > $O/pno.json 2>&1 || exit 1
echo "no-overlap $(grep -o '"ms_per_step[^,]*' $O/pno.json) $(grep -o '"projected_node_glups[^,}]*' $O/pno.json)"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 30 --warmup 6 --extra=--no-graph > $O/trace.log 2>&1 || exit 1
echo trace done
