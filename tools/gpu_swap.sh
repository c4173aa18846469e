#!/bin/bash
# y-marching tiles for thin x slabs: bitwise tests, phantom-rank proxies with / without
O=gpurun_out/swap; mkdir -p $O
export TMPDIR=/tmp
HEAT3D_TL_SWAP=1 timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py -k "thin_slab or block_decomposition" > $O/pytest0.log 2>&1
echo "pytest0 rc=$?"; tail -3 $O/pytest0.log; grep "^FAILED" $O/pytest0.log | head
HEAT3D_TL_SWAP=1 timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py tests/test_gpu_solver.py tests/test_gpu_rccl.py tests/test_gpu_multiprocess.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 8 4 2; do
  for sw in 1 0; do
    HEAT3D_TL_SWAP=$sw timeout -k 10 200 python3 tools/rank_proxy.py --ranks $r --gbps 64 --steps 120 --warmup 24 --extra=--no-graph > $O/p$r$sw.json 2>&1 || exit 1
    echo "ranks=$r swap=$sw $(grep -o '"ms_per_step[^,]*' $O/p$r$sw.json) $(grep -o '"projected_node_glups[^,}]*' $O/p$r$sw.json)"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 30 --warmup 6 --extra=--no-graph > $O/trace.log 2>&1 || exit 1
echo trace done
