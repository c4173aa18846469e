#!/bin/bash
# y-marching interior of thin slab shares: bitwise solver tests with the switch, proxies
O=gpurun_out/swapx; mkdir -p $O
export TMPDIR=/tmp
HEAT3D_TL_SWAP_X=400 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py -k "slabs or block_decomposition or ring_kernel_solver" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 8 4; do
  for sx in 400 0; do
    HEAT3D_TL_SWAP_X=$sx timeout -k 10 200 python3 tools/rank_proxy.py --ranks $r --gbps 64 --steps 120 --warmup 24 --extra=--no-graph > $O/p$r$sx.json 2>&1 || exit 1
    echo "ranks=$r swap_x=$sx $(grep -o '"ms_per_step[^,]*' $O/p$r$sx.json) $(grep -o '"projected_node_glups[^,}]*' $O/p$r$sx.json)"
  done
done
for sx in 400 0; do
  HEAT3D_TL_SWAP_X=$sx timeout -k 10 200 python3 tools/rank_proxy.py --ranks 8 --gbps 1000 --steps 120 --warmup 24 --extra=--no-graph > $O/pf$sx.json 2>&1 || exit 1
  echo "ranks=8 gbps=1000 swap_x=$sx $(grep -o '"ms_per_step[^,]*' $O/pf$sx.json) $(grep -o '"projected_node_glups[^,}]*' $O/pf$sx.json)"
done
HEAT3D_TL_SWAP_X=400 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 30 --warmup 6 --extra=--no-graph > $O/trace.log 2>&1 || exit 1
echo trace done
