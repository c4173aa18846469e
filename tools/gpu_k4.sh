#!/bin/bash
# 12-wave K = 4 lean tiles with nt stores vs the K = 3 default (fp64 1024^3)
O=gpurun_out/k4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py -k "stencil_k_bitwise" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
HEAT3D_ALLOW_SPILL=1 timeout -k 10 300 python3 tools/tune.py --n 1024 --dtype fp64 --variants tl3 tl4 tl4:1:3:1:12:0:3:2 tl4:1:4:1:12:0:3:2 tl4:1:3:1:12:0:3 tl4:1:4:1:12:0:3 --iters 8 --rounds 3 > $O/t.log 2>&1 || exit 1
grep -o '"variant[^}]*' $O/t.log
