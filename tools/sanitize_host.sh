#!/bin/bash
# Host AddressSanitizer + UBSan build (HEAT3D_SANITIZE=ON: host C++ only, the
# gfx950 code objects are built as usual) and CPU-backend runs under it: C++
# unit tests, single domain, 8 virtual ranks with K = 3 sweeps + checkpoint,
# restart, 4 socket-connected processes (2x2x1 blocks, deep halos), and the
# round-4 / round-5 schedules: long K+1 sweeps across the halos (slabs and
# blocks, partial remainders, rollback), tile-thick y / z layers, and 3 socket processes timing their sweeps
# and voting (remainder policy, --time-limit cap re-votes).
# CPU only — sanitised GPU runs are not available on this pool.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=${1:-/tmp/build-asan}
cmake -S "$ROOT" -B "$B" -G Ninja -DCMAKE_BUILD_TYPE=RelWithDebInfo -DCMAKE_HIP_ARCHITECTURES=gfx950 \
  -DCMAKE_HIP_COMPILER=/opt/rocm/llvm/bin/clang++ -DHEAT3D_SANITIZE=ON > /dev/null
cmake --build "$B" -j 8 --target heat3d heat3d_unit_tests > /dev/null
export ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
W=$(mktemp -d) && cd "$W"
timeout 600 "$B/heat3d_unit_tests" | tail -1
timeout 300 "$B/heat3d" 27 27 27 100000 1e-4 --backend cpu --threads 2 | grep converged
timeout 300 "$B/heat3d" 33 33 33 100000 1e-4 --backend cpu --threads 2 --virtual-ranks 8 --temporal 3 \
  --checkpoint-every 500 --checkpoint-dir ck --output none | grep converged
timeout 300 "$B/heat3d" 33 33 33 100000 1e-4 --backend cpu --threads 2 --restart ck --output none | grep converged
PORT=$((29000 + RANDOM % 1000))
pids=()
for r in 0 1 2 3; do
  WORLD_SIZE=4 RANK=$r LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT HEAT3D_BOOTSTRAP_PORT=$PORT \
    timeout 300 "$B/heat3d" 27 27 27 100000 1e-4 --backend cpu --threads 1 --decomp 2x2x1 --temporal 3 \
    --output none > mp$r.log 2>&1 &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
grep converged mp0.log
# long sweeps across halos: step counts that are not multiples of K end in
# K+1-step sweeps over K+1-deep ghosts (slabs, blocks), with the rollback of a
# convergence inside a sweep
for c in "3x1x1 --temporal 3" "2x1x1 --temporal 2" "2x2x2 --temporal 3" "1x1x3 --temporal 3"; do
  set -- $c
  n=$(( ${1:0:1} * ${1:2:1} * ${1:4:1} ))
  timeout 300 "$B/heat3d" 33 29 31 100000 1e-4 --backend cpu --threads 2 --virtual-ranks $n --decomp $c \
    --long-sweeps on --check-every 7 --output none > ls_$n.log 2>&1
  grep -q converged ls_$n.log
done
# partial remainder sweeps on 2x2x2 blocks
timeout 300 "$B/heat3d" 33 29 31 100000 1e-4 --backend cpu --threads 2 --virtual-ranks 8 --decomp 2x2x2 \
  --temporal 2 --no-long-sweeps --output none > partial.log 2>&1
grep -q converged partial.log
# tile-thick y / z boundary layers (85 x 117 owned per rank)
timeout 300 "$B/heat3d" 14 172 236 300 0 --backend cpu --threads 2 --virtual-ranks 4 --decomp 1x2x2 \
  --temporal 3 --output none > tile.log 2>&1
grep -q "did not converge" tile.log
# 3 processes over sockets: start-up sweep timing + rank vote of the
# remainder policy, --time-limit cap votes, K+1-deep halos
PORT=$((30000 + RANDOM % 1000))
pids=()
for r in 0 1 2; do
  WORLD_SIZE=3 RANK=$r LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT HEAT3D_BOOTSTRAP_PORT=$PORT \
    timeout 300 "$B/heat3d" 31 31 31 100000 1e-4 --backend cpu --threads 1 --decomp 3x1x1 --temporal 3 \
    --long-sweeps measure --time-limit 60 --check-every 6 --output none > vote$r.log 2>&1 &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
grep converged vote0.log
if grep -lE "runtime error|ERROR: AddressSanitizer" ./*.log 2>/dev/null; then exit 1; fi
echo "sanitizer runs clean"
