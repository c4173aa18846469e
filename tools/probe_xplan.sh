# x schedule of the ring kernel: split-tail plan (L = 0, default) vs equal
# segments (L = -1, previous policy), interleaved.
B=build/heat3d
run() { echo "## $*"; $B "$@" --output none --quiet 2>&1 | grep -oE "GLUPS=[0-9.]+" ; }
for sh in "1024 1024 1024 300" "512 512 512 1200" "130 1024 1024 1200" "258 1024 1024 900" "514 1024 1024 600"; do
  HEAT3D_TRACE=1 $B $sh 0 --output none --quiet 2>&1 | grep "tbr K" | head -1
  for rep in 1 2; do
    run $sh 0 --kernel2 tr3:1:3:1:16:0:3
    run $sh 0 --kernel2 tr3:1:3:1:16:-1:3
  done
done
HEAT3D_TRACE=1 $B 1024 1024 1024 6 0 --dtype fp32 --output none --quiet 2>&1 | grep "tbr K" | head -1
run 1024 1024 1024 600 0 --dtype fp32
run 1024 1024 1024 600 0 --dtype fp32 --kernel2 tr3:2:4:1:8:-1:3
