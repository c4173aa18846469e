mkdir -p gpurun_out/t8
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_graph.py > gpurun_out/t8/pytest.log 2>&1
rc=$?; echo pytest rc=$rc; tail -25 gpurun_out/t8/pytest.log
[ $rc -eq 0 ] && HEAT3D_RCCL_GRAPH=1 timeout -k 10 150 python3 bench.py --gpus 2 --comm rccl --rccl-host-split --grid 96 --steps 36 --warmup 6 --converge-eps 1e-3 --timeout 120 > gpurun_out/t8/rcclgraph.out 2> gpurun_out/t8/rcclgraph.err; echo rcclgraph rc=$?; tail -c 1500 gpurun_out/t8/rcclgraph.out; tail -5 gpurun_out/t8/rcclgraph.err
