#!/bin/bash
# kernel diagnostics: cache-resident vs HBM-sized grids, K=3 vs K=4 16-wave variants
O=gpurun_out/kdiag; mkdir -p $O
for n in 256 1024; do
  timeout -k 10 200 python3 tools/tune.py --n $n --iters 10 --rounds 3 --variants tr3:1:3:1:16:0:3 tr4:1:3:1:16:0:3 tr3:1:2:1:16:0:4 tr3:1:4:1:16:0:3 tr4:1:6:1:8:0:3 > $O/tune_$n.txt 2>&1 || exit 1
  cat $O/tune_$n.txt | grep -v amdgpu.ids
done
timeout -k 10 200 python3 tools/tune.py --n 1024 --iters 10 --rounds 2 --variants tr3:1:3:1:16:0:3 --probes > $O/probes.txt 2>&1; grep probe $O/probes.txt | grep '"blocks": 8192'
