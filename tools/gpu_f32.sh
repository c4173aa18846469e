#!/bin/bash
# fp32 pair-kernel variants at 1024^3 and the default's counters
O=gpurun_out/f32; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/tune.py --n 1024 --dtype fp32 --variants tl3:2:3:1:16:0:3 tl3:2:3:1:16:0:4 tl3:2:2:1:16:0:3 tl4:2:2:1:16:0:3 tl4:2:2:1:16:0:4 tl4:2:3:1:16:0:3 --iters 10 --rounds 3 > $O/t.log 2>&1 || exit 1
grep -o '"variant[^}]*' $O/t.log
bash tools/pmc_passes.sh $O/pmc tl3 1024 fp32 > $O/pmc.log 2>&1 || exit 1
echo pmc done
