#!/bin/bash
# hipGraph probe: multi-stream schedules as explicitly built graphs, bitwise vs eager
O=gpurun_out/gcap
mkdir -p $O
export HEAT3D_SEGV_TRACE=1
set -o pipefail
run() { local n=$1; shift; echo "== $n"; timeout -k 10 120 "$@" > $O/$n.out 2> $O/$n.err; local rc=$?; tail -3 $O/$n.out; [ $rc -ne 0 ] && tail -5 $O/$n.err; echo "rc=$rc"; return $rc; }
run slab8 python3 tools/graph_multistream_probe.py --n 96 --ranks 8 --decomp 8x1x1 --steps 72 &&
run block8 python3 tools/graph_multistream_probe.py --n 96 --ranks 8 --decomp 2x2x2 --steps 72 &&
run phantom python3 tools/graph_multistream_probe.py --n 256 --decomp 8x1x1 --phantom 1/8 --steps 72 &&
run single python3 tools/graph_multistream_probe.py --n 128 --ranks 1 --decomp 1x1x1 --steps 72 &&
run bench1 python3 bench.py --steps 20 --warmup 5 --converge-eps 0
