# Block decompositions on one GPU (virtual ranks): exchange-first vs overlapped
# sweeps, with and without an emulated all-reduce latency.
B=build/heat3d
run() { echo "## $*"; env "$@" --output none --quiet 2>&1 | grep -E "heat3d:"; }
for ov in 0 1; do
  run HEAT3D_BLOCK_OVERLAP=$ov $B 2048 2048 2048 30 0 --dtype fp32 --virtual-ranks 8 --decomp 2x2x2 || exit 1
  run HEAT3D_BLOCK_OVERLAP=$ov $B 1024 1024 1024 300 0 --virtual-ranks 8 --decomp 2x2x2 || exit 1
  run HEAT3D_BLOCK_OVERLAP=$ov HEAT3D_FAKE_ALLREDUCE_US=30 $B 1024 1024 1024 300 0 --virtual-ranks 8 --decomp 2x2x2 || exit 1
done
