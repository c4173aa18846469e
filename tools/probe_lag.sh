# Lagged convergence check on 8 virtual x slabs (one GPU), with and without an
# emulated all-reduce latency on the reduce stream.
B=build/heat3d
run() { echo "## $*"; env "$@" $B 1024 1024 1024 600 0 --virtual-ranks 8 --decomp 8x1x1 --output none --quiet 2>&1 | grep -E "heat3d:"; }
for us in 0 30; do
  run HEAT3D_LAG=0 HEAT3D_FAKE_ALLREDUCE_US=$us && run HEAT3D_LAG=1 HEAT3D_FAKE_ALLREDUCE_US=$us || exit 1
done
echo "## 2 slabs"
HEAT3D_LAG=0 $B 1024 1024 1024 600 0 --virtual-ranks 2 --output none --quiet 2>&1 | grep heat3d: &&
HEAT3D_LAG=1 $B 1024 1024 1024 600 0 --virtual-ranks 2 --output none --quiet 2>&1 | grep heat3d:
