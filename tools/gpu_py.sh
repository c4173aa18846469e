#!/bin/bash
# tile order probe (HEAT3D_TL_PY = tile rows per band): bitwise check, kernel GLUPS, HBM read bytes
O=gpurun_out/py; mkdir -p $O
export TMPDIR=/tmp
HEAT3D_TL_PY=8 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py \
  -k "stencil_k_bitwise or deep_halo_matches_cpu or ring_kernel_solver" > $O/pytest.log 2>&1
rc=$?; echo "pytest(py=8) rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for py in 0 2 4 8 16 25; do
    HEAT3D_TL_PY=$py timeout -k 10 200 python3 tools/tune.py --n 1024 --dtype fp64 --variants tl3 --iters 10 --rounds 2 > $O/t.log 2>&1 || exit 1
    echo "py=$py $(grep -o '"glups_median[^,]*' $O/t.log)"
  done
done
for py in 0 8 25; do
  HEAT3D_TL_PY=$py timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum -d $O/pmc$py -o run --output-format csv -- \
    python3 tools/tune.py --n 1024 --dtype fp64 --variants tl3 --iters 4 --rounds 1 > $O/pmc$py.log 2>&1 || exit 1
  echo "pmc py=$py rc=$?"
done
