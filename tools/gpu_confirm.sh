#!/bin/bash
# confirmation: temporal/graph GPU tests, benches (driver config x2, default, fp32), rocprofv3 stats, HBM counters
O=gpurun_out/confirm; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_temporal.py tests/test_gpu_graph.py tests/test_gpu_solver.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench.err || exit 1; cut -c1-200 $O/bench_driver.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver2.json 2>> $O/bench.err || exit 1; cut -c1-200 $O/bench_driver2.json
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2>> $O/bench.err || exit 1; cut -c1-200 $O/bench_default.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --dtype fp32 > $O/bench_fp32.json 2>> $O/bench.err || exit 1; cut -c1-200 $O/bench_fp32.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 60 --warmup 6 --converge-eps 0 > $O/stats.log 2>&1 || exit 1
echo stats done
bash tools/pmc_passes.sh $O/pmc tl3 > $O/pmc.log 2>&1 || exit 1
echo pmc done
