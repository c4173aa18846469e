#!/bin/bash
O=gpurun_out/tl3; mkdir -p $O
timeout -k 10 400 python3 tools/tune.py --n 1024 --dtype fp32 --iters 10 --rounds 3 --variants tr3 tl3 tl4:1:3:1:16:0:3 tl4:1:4:1:16:0:3 tl5:1:3:1:16:0:3 tl5:1:4:1:16:0:3 tl6:1:3:1:16:0:3 tl5:1:3:1:16:0:6 tl4:1:4:1:12:0:3 > $O/tune32.txt 2>&1; echo tune rc=$?
grep -v amdgpu.ids $O/tune32.txt
