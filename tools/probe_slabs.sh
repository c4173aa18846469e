# Slab-shaped single-GPU probes: per-GPU work of the strong-scaling bench at N = 2, 4, 8.
B=build/heat3d
run() { echo "## $*"; $B "$@" --output none --quiet 2>&1 | grep -E "heat3d:|device_slots|tbr K"; }
HEAT3D_TRACE=1 $B 130 1024 1024 6 0 --output none --quiet 2>&1 | grep -E "device_slots|tbr K" | head -5
run 1024 1024 1024 600 0 &&
run 514 1024 1024 900 0 &&
run 258 1024 1024 1200 0 &&
run 130 1024 1024 1200 0 &&
for L in 128 64 41 32 20; do run 130 1024 1024 1200 0 --kernel2 tr3:1:3:1:16:$L:3; done &&
for L in 1022 512 256 128 64; do run 1024 1024 1024 300 0 --kernel2 tr3:1:3:1:16:$L:3; done &&
run 1024 1024 1024 300 0 --virtual-ranks 8 --decomp 8x1x1
