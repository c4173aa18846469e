#!/bin/bash
# lean kernel: correctness (bitwise vs CPU / single steps) then speed
O=gpurun_out/tl; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_temporal.py -k "stencil_k_bitwise or deep_halo_matches" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/tune.py --n 1024 --iters 10 --rounds 3 --variants tl3 tl4 tl4:1:2:1:16:0:6 tl3:1:3:1:16:0:6 tl3:1:2:1:16:0:6 > $O/tune.txt 2>&1; echo tune rc=$?
grep -v amdgpu.ids $O/tune.txt
