#!/bin/bash
# Round-2 GPU probe: 1-GPU bench, RCCL self exchange, self-launched 2-rank bench
# (socket, then real RCCL over loopback), multi-stream hipGraph capture.
# Every step has its own time limit; the chain stops at the first failure.
set -o pipefail
O=gpurun_out/r2probe
mkdir -p $O
export HEAT3D_SEGV_TRACE=1
step() {
  local name=$1 t=$2; shift 2
  echo "== $name" | tee -a $O/steps.log
  timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "rc=$rc" | tee -a $O/steps.log
  tail -3 $O/$name.out
  return $rc
}
step bench1 300 python3 bench.py --steps 20 --warmup 5 &&
step selfx 120 python3 -c "
import heat3d_amd
ext = heat3d_amd.native()
r = ext.rccl_self_exchange(0, [8, 24, 1000, 4093, 1<<20, 3*(1<<20)+5])
print(r)
assert all(r['ok']) and r['touched_outside'] == 0 and r['transport_ranks'] == 1, r
" &&
step bench2_socket 300 python3 bench.py --gpus 2 --comm socket --grid 128 --steps 6 --warmup 3 --converge-eps 0 --timeout 240 &&
step bench2_rccl 300 env NCCL_DEBUG=WARN python3 bench.py --gpus 2 --comm rccl --rccl-host-split --grid 128 --steps 12 --warmup 6 --converge-eps 1e-3 --timeout 240 &&
step graph_ms 180 python3 tools/graph_multistream_probe.py --n 96 --ranks 8 --decomp 8x1x1 --steps 72
echo "done rc=$?" | tee -a $O/steps.log
