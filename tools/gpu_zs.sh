#!/bin/bash
# z-stride experiment: stored strips aligned to 64 bytes (fp64 lean, fp32 pair)
O=gpurun_out/zs; mkdir -p $O
HEAT3D_TP_ZS=112 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py -k "pair" > $O/pytest.log 2>&1
rc=$?; echo "pytest(tp zs=112) rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
run() { env $1 timeout -k 10 200 python3 tools/tune.py --n 1024 --dtype $2 --variants $3 --iters 8 --rounds 2 > $O/t.log 2>&1 || exit 1; echo "$1 $2 $3 $(grep -o '"glups_median[^,]*' $O/t.log)"; }
run HEAT3D_TL_ZS=58 fp64 tl4
run HEAT3D_TL_ZS=56 fp64 tl4
run HEAT3D_TL_ZS=58 fp64 tl3
run HEAT3D_TL_ZS=56 fp64 tl3
run HEAT3D_TL_ZS=60 fp64 tl2
run HEAT3D_TL_ZS=56 fp64 tl2
run HEAT3D_TP_ZS=120 fp32 tl3
run HEAT3D_TP_ZS=112 fp32 tl3
run HEAT3D_TP_ZS=120 fp32 tl3
run HEAT3D_TP_ZS=112 fp32 tl3
run HEAT3D_TL_ZS=56 fp32 tl4:1:4:1:16:0:3
run HEAT3D_TL_ZS=48 fp32 tl4:1:4:1:16:0:3
