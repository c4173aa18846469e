#!/bin/bash
# lean-kernel experiment: numerics of the tl variants, then kernel-level GLUPS
O=gpurun_out/tlx; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_temporal.py -k "tl or lean or ring" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 tools/tune.py --n 1024 --dtype fp64 --variants $V64 --iters 8 --rounds 2 > $O/tune64.log 2>&1; rc=$?; echo "tune64 rc=$rc"; grep -E "variant" $O/tune64.log | cut -c1-150; [ $rc -ne 0 ] && exit $rc
[ -n "$V32" ] && { timeout -k 10 300 python3 tools/tune.py --n 1024 --dtype fp32 --variants $V32 --iters 8 --rounds 2 > $O/tune32.log 2>&1; rc=$?; echo "tune32 rc=$rc"; grep -E "variant" $O/tune32.log | cut -c1-150; }
exit 0
