#!/bin/bash
# paired boundary slabs: bitwise tests, phantom-rank proxies with / without pairing
O=gpurun_out/xpair; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py tests/test_gpu_solver.py tests/test_gpu_rccl.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 8 4 2; do
  for pair in 1 0; do
    HEAT3D_PAIR_SLABS=$pair timeout -k 10 200 python3 tools/rank_proxy.py --ranks $r --gbps 64 --steps 120 --warmup 24 --extra=--no-graph > $O/p$r$pair.json 2>&1 || exit 1
    echo "ranks=$r pair=$pair $(grep -o '"ms_per_step[^,]*' $O/p$r$pair.json) $(grep -o '"projected_node_glups[^,}]*' $O/p$r$pair.json)"
  done
done
HEAT3D_PAIR_SLABS=1 timeout -k 10 200 python3 tools/rank_proxy.py --ranks 8 --gbps 1000 --steps 120 --warmup 24 --extra=--no-graph > $O/p8fast.json 2>&1 || exit 1
echo "ranks=8 gbps=1000 pair=1 $(grep -o '"ms_per_step[^,]*' $O/p8fast.json) $(grep -o '"projected_node_glups[^,}]*' $O/p8fast.json)"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/rank_proxy.py --ranks 8 --gbps 64 --steps 30 --warmup 6 --extra=--no-graph > $O/trace.log 2>&1 || exit 1
echo trace done
