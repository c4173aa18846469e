#!/bin/bash
O=gpurun_out/tl2; mkdir -p $O
export HEAT3D_ALLOW_SPILL=1
timeout -k 10 300 python3 tools/tune.py --n 1024 --iters 10 --rounds 3 --variants tl3 tl4 tl4:1:3:1:16:0:3 tl4:1:4:1:12:0:3 tl4:1:4:1:12:0:4 tl5:1:3:1:12:0:3 > $O/tune.txt 2>&1; echo tune rc=$?
grep -v amdgpu.ids $O/tune.txt
