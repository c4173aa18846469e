# x schedule of the ring kernel: split-tail plan (L = 0, default) vs equal
# segments (L = -1, previous policy), interleaved on one box.
B=build/heat3d
run() { echo "## $*"; $B "$@" --output none --quiet 2>&1 | grep -oE "GLUPS=[0-9.]+" ; }
ab() {  # $1 = kernel2 prefix, rest = problem
  local k=$1; shift
  HEAT3D_TRACE=1 $B "$@" --output none --quiet 2>&1 | grep "tbr K" | head -1
  HEAT3D_TRACE=1 $B "$@" --kernel2 $k:-1:3 --output none --quiet 2>&1 | grep "tbr K" | head -1
  for rep in 1 2; do run "$@"; run "$@" --kernel2 $k:-1:3; done
}
ab tr3:1:3:1:16 1024 1024 1024 300 0
ab tr3:1:3:1:16 512 512 512 1200 0
ab tr3:1:3:1:16 130 1024 1024 1200 0
ab tr3:1:3:1:16 258 1024 1024 900 0
ab tr3:2:4:1:8 2049 2049 2049 60 0 --dtype fp32
ab tr3:2:4:1:8 1024 1024 1024 600 0 --dtype fp32
