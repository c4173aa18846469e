#!/bin/bash
# 8-wave lean tiles (R = 6 rows per wave, <= 256 VGPRs): bitwise checks, then kernel GLUPS vs the default
O=gpurun_out/w8; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py \
  -k "stencil_k_bitwise or deep_halo_matches_cpu" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for dt in fp64 fp32; do
  v="tl3 tl4:1:6:1:8:0:3 tl3:1:6:1:8:0:3 tl4:1:6:1:8:0:4 tl4:1:5:1:8:0:3"
  [ $dt = fp32 ] && v="tl3 tl4:1:6:1:8:0:3 tl4 tl3:1:6:1:8:0:3"
  timeout -k 10 300 python3 tools/tune.py --n 1024 --dtype $dt --variants $v --iters 8 --rounds 2 > $O/tune_$dt.log 2>&1 || exit 1
  grep -o '"variant[^}]*' $O/tune_$dt.log | head -20
done
