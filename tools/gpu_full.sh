#!/bin/bash
# full GPU test suite, smoke, 1-GPU bench (driver config) and fp32 bench
O=gpurun_out/full; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest -x -q --durations 25 --timeout 200 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -32 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo smoke rc=$?; tail -2 $O/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; echo bench rc=$?; cat $O/bench.json | cut -c1-200
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --converge-eps 0 > $O/bench100.json 2>> $O/bench.err; echo bench100 rc=$?; cut -c1-200 $O/bench100.json
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --dtype fp32 --converge-eps 0 > $O/bench32.json 2>> $O/bench.err; echo bench32 rc=$?; cut -c1-200 $O/bench32.json
