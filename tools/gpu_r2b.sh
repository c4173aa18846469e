#!/bin/bash
# round-2 re-entry: full GPU suite, smoke, benches (driver config / default / fp32), phantom-rank
# proxies of the 2/4/8-GPU slab shares with the fp64 nt-store default vs the default store policy
O=gpurun_out/r2b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --durations 10 --timeout 200 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1; tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench.err || exit 1; cut -c1-160 $O/bench_driver.json
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2>> $O/bench.err || exit 1; cut -c1-160 $O/bench_default.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --dtype fp32 > $O/bench_fp32.json 2>> $O/bench.err || exit 1; cut -c1-160 $O/bench_fp32.json
for r in 2 4 8; do
  for pol in "" ":0"; do
    timeout -k 10 200 python3 tools/rank_proxy.py --ranks $r --gbps 64 --steps 120 --warmup 24 \
      --extra="--no-graph --kernel2 tl3:1:3:1:16:0:3$pol" > $O/proxy$r$pol.json 2>&1 || exit 1
    echo "proxy ranks=$r pol=$pol $(grep -o '"ms_per_step[^,]*' $O/proxy$r$pol.json) $(grep -o '"projected_node_glups[^,}]*' $O/proxy$r$pol.json)"
  done
done
