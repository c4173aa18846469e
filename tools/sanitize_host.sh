#!/bin/bash
# Host AddressSanitizer + UBSan build (HEAT3D_SANITIZE=ON: host C++ only, the
# gfx950 code objects are built as usual) and CPU-backend runs under it: C++
# unit tests, single domain, 8 virtual ranks with K = 3 sweeps + checkpoint,
# restart, and 4 socket-connected processes (2x2x1 blocks, deep halos).
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
if grep -lE "runtime error|ERROR: AddressSanitizer" ./*.log 2>/dev/null; then exit 1; fi
echo "sanitizer runs clean"
