#!/bin/bash
# driver-config gap: 20 timed steps vs 200 (warm-up length, step count modulo K, kernel trace)
O=gpurun_out/steps2; mkdir -p $O
export TMPDIR=/tmp
b() { timeout -k 10 200 python3 bench.py --converge-eps 0 "$@" > $O/b.json 2>>$O/err.log || exit 1; echo "$* $(grep -o '"value[^,]*' $O/b.json) $(grep -o '"ms_per_step[^,]*' $O/b.json) $(grep -o '"graph_launches[^,]*' $O/b.json)"; }
b --steps 20 --warmup 5
b --steps 20 --warmup 5
b --steps 20 --warmup 30
b --steps 21 --warmup 5
b --steps 60 --warmup 5
b --steps 200 --warmup 20
b --steps 20 --warmup 5 --no-graph
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --converge-eps 0 > $O/trace.log 2>&1 || exit 1
echo trace done
