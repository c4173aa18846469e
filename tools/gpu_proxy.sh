#!/bin/bash
# phantom-rank proxy of the 8-GPU 1024^3 slab bench: CU reservation on / off,
# projected node GLUPS and a kernel trace of each (check / delay kernel waits)
O=gpurun_out/proxy; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for res in 8 0; do
  HEAT3D_RESERVE_CUS=$res timeout -k 10 200 python3 $R/tools/rank_proxy.py --ranks 8 --gbps 64 --steps 240 --warmup 24 > $R/$O/proxy_res$res.json 2>&1 || exit 1
  grep proxy $R/$O/proxy_res$res.json
done
for res in 8 0; do
  HEAT3D_RESERVE_CUS=$res timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/trace_res$res -o run --output-format csv -- python3 $R/tools/rank_proxy.py --ranks 8 --gbps 64 --steps 60 --warmup 12 > $R/$O/trace_res$res.log 2>&1 || exit 1
  echo traced res=$res
done
