#!/bin/bash
# full GPU suite, smoke, driver-config benches, default bench, fp32 driver config
O=gpurun_out/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --durations 5 --timeout 200 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1; tail -1 $O/smoke.log
for i in 1 2; do timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver$i.json 2>> $O/bench.err || exit 1; cut -c1-190 $O/bench_driver$i.json; done
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2>> $O/bench.err || exit 1; cut -c1-190 $O/bench_default.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --dtype fp32 > $O/bench_fp32.json 2>> $O/bench.err || exit 1; cut -c1-190 $O/bench_fp32.json
for r in 2 4 8; do
  timeout -k 10 200 python3 tools/rank_proxy.py --ranks $r --gbps 64 --steps 120 --warmup 24 --extra=--no-graph > $O/proxy$r.json 2>&1 || exit 1
  echo "proxy ranks=$r $(grep -o '"ms_per_step[^,]*' $O/proxy$r.json) $(grep -o '"projected_node_glups[^,}]*' $O/proxy$r.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 60 --warmup 6 --converge-eps 0 > $O/stats.log 2>&1 || exit 1
echo stats done
