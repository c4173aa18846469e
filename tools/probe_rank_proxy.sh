# Per-GPU schedule of the 2/4/8-GPU bench (1024^3 fp64 slabs) on one GPU:
# phantom inner rank, emulated halo bandwidth / all-reduce latency.
run() { timeout -k 10 120 python tools/rank_proxy.py "$@" || exit 1; }
for P in 2 4 8; do
  for g in 1000 64 40; do run --ranks $P --gbps $g --ar-us 20; done
done
run --ranks 8 --gbps 64 --ar-us 20 --extra=--no-overlap
HEAT3D_LAG=0 run --ranks 8 --gbps 64 --ar-us 20
run --ranks 8 --gbps 64 --ar-us 20 --decomp 2x2x2
run --ranks 8 --gbps 64 --ar-us 20 --decomp 4x2x1
