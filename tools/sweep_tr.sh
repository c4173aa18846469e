# Ring-kernel variant sweep (tools/tune.py, interleaved rounds on one box).
# 8th spec field 1 = non-temporal T^{n+K} stores.
python tools/tune.py --n 1024 --dtype fp64 --rounds 3 --iters 8 --json-out gpurun_out/sweep_fp64.json --variants tr3:1:3:1:16:0:3 tr3:1:6:1:8:0:3 tr4:1:6:1:8:0:3 tr4:1:5:1:8:0:3 tr4:1:4:1:8:0:3 tr5:1:4:1:8:0:3 tr3:1:3:1:16:0:3:1 &&
python tools/tune.py --n 512 --dtype fp64 --rounds 3 --iters 8 --variants tr3:1:3:1:16:0:3 tr4:1:6:1:8:0:3 tr4:1:5:1:8:0:3 tr5:1:4:1:8:0:3
