#!/bin/bash
# The interior / boundary x plans (HEAT3D_TRACE launch lines) of the BASELINE
# config-4 / config-5 phantom shares and of the 2- / 4- / 8-GPU fp64 slab
# shares: gpurun --timeout 600 -- bash tools/probes/plan_trace.sh
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/plan_trace
mkdir -p "$OUT"
run() {  # tag, rank_proxy args
  local tag=$1; shift
  HEAT3D_TRACE=1 timeout -k 10 300 python3 -u tools/rank_proxy.py --steps 3 --warmup 3 --gbps 64 "$@" \
    > "$OUT/$tag.log" 2>&1
  echo "== $tag"
  grep "heat3d trace\] tl" "$OUT/$tag.log" | sort | uniq -c | sort -rn | head -8
}
run c4 --ranks 8 --decomp 2x2x2 --dtype fp32 --grid 2048 --rank 1
run c5 --ranks 8 --decomp 2x2x2 --dtype fp32 --grid 4096 --rank 7
run s2 --ranks 2
run s4 --ranks 4
run s8 --ranks 8
