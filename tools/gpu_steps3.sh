#!/bin/bash
# driver-config gap after: nt stores on the K = 2 / 4 sweeps, graph upload, capture during warm-up
O=gpurun_out/steps3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py tests/test_gpu_graph.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
b() { timeout -k 10 200 python3 bench.py --converge-eps 0 "$@" > $O/b.json 2>>$O/err.log || exit 1; echo "$* $(grep -o '"value[^,]*' $O/b.json) $(grep -o '"ms_per_step[^,]*' $O/b.json) $(grep -o '"graph_launches[^,]*' $O/b.json)"; }
b --steps 20 --warmup 5
b --steps 20 --warmup 5
b --steps 20 --warmup 30
b --steps 21 --warmup 5
b --steps 200 --warmup 20
b --steps 20 --warmup 5 --no-graph
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --converge-eps 0 > $O/trace.log 2>&1 || exit 1
echo trace done
