#!/bin/bash
# Round-2 config-5 sizing on one GPU: the corner rank (7 of 8) of a 2x2x2
# decomposition of 4096^3 fp32 (and fp64) as a phantom rank, with
# hipMemGetInfo before / after and the per-rank GLUPS; then the GPU suite.
O=gpurun_out/c5; mkdir -p $O
set -o pipefail
run() { name=$1; shift; timeout -k 10 300 python3 -u tools/rank_proxy.py "$@" > $O/$name.json 2> $O/$name.err; rc=$?; echo "$name rc=$rc"; cut -c1-600 $O/$name.json; return $rc; }
run c5_fp32 --grid 4096 --dtype fp32 --decomp 2x2x2 --rank 7 --steps 24 --warmup 4 --gbps 64 &&
run c5_fp32_k3 --grid 4096 --dtype fp32 --decomp 2x2x2 --rank 7 --steps 24 --warmup 3 --gbps 64 --extra "--temporal 3" &&
run c5_fp64 --grid 4096 --dtype fp64 --decomp 2x2x2 --rank 7 --steps 24 --warmup 3 --gbps 64 || exit $?
timeout -k 10 1200 python3 -u -m pytest -x -q --durations 20 --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 $O/pytest.log; exit $rc
