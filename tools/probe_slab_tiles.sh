# Ring-kernel tile shape vs slab thickness: smaller y tiles give more
# workgroups (better round fill on 256 CUs) at more y-halo overlap.
run() { timeout -k 10 120 python tools/rank_proxy.py "$@" || exit 1; }
for v in tr3:1:3:1:16:0:3 tr3:1:2:1:16:0:3 tr3:1:4:1:8:0:3 tr3:1:5:1:8:0:3 tr3:1:2:1:16:0:4; do
  for P in 1 2 4 8; do run --ranks $P --gbps 1000 --ar-us 20 --extra="--kernel2 $v"; done
done
