# x-segment length sweep of the default ring kernel (kernel2 spec field L).
B=build/heat3d
run() { echo "## $*"; $B "$@" --output none --quiet 2>&1 | grep -oE "kernel=[^ ]+|GLUPS=[0-9.]+" | tr '\n' ' '; echo; }
HEAT3D_TRACE=1 $B 512 512 512 6 0 --output none --quiet 2>&1 | grep "tbr K" | head -1
HEAT3D_TRACE=1 $B 1024 1024 1024 6 0 --output none --quiet 2>&1 | grep "tbr K" | head -1
for L in 0 510 255 170 128 102 85 73 64 51; do run 512 512 512 1200 0 --kernel2 tr3:1:3:1:16:$L:3; done
for L in 0 1022 511 341 256 205 171 146 128 114; do run 1024 1024 1024 300 0 --kernel2 tr3:1:3:1:16:$L:3; done
for L in 0 128 64 43 32; do run 130 1024 1024 1200 0 --kernel2 tr3:1:3:1:16:$L:3; done
