#!/bin/bash
# quick GPU check: temporal + graph tests, then the driver-config bench
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_temporal.py tests/test_gpu_graph.py tests/test_gpu_solver.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --converge-eps 0 > $O/bench$i.json 2> $O/bench.err; echo bench rc=$?; cut -c1-170 $O/bench$i.json; done
HEAT3D_LONG_SWEEPS=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --converge-eps 0 > $O/bench_nolong.json 2>> $O/bench.err; echo bench_nolong rc=$?; cut -c1-170 $O/bench_nolong.json
