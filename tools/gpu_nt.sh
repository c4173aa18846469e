#!/bin/bash
# output-store cache policy of the lean kernels (spec field 7): bitwise check, kernel GLUPS
O=gpurun_out/nt; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py \
  -k "stencil_k_bitwise or pair_deep_halo" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
B=tl3:1:3:1:16:0:3
timeout -k 10 250 python3 tools/tune.py --n 1024 --dtype fp64 --variants $B $B:2 $B:3 $B:17 $B:18 $B:19 --iters 10 --rounds 3 > $O/t.log 2>&1 || exit 1
grep -o '"variant[^}]*' $O/t.log
P=tl3:2:3:1:16:0:3
timeout -k 10 250 python3 tools/tune.py --n 1024 --dtype fp32 --variants $P $P:2 $P:3 $P:17 $P:19 --iters 10 --rounds 3 > $O/t32.log 2>&1 || exit 1
grep -o '"variant[^}]*' $O/t32.log
for n in 512 768; do
timeout -k 10 250 python3 tools/tune.py --n $n --dtype fp64 --variants $B $B:2 --iters 10 --rounds 3 > $O/t$n.log 2>&1 || exit 1
grep -o '"variant[^}]*' $O/t$n.log
done
