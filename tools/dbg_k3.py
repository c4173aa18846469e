import sys, numpy as np
sys.path.insert(0, "/root/repo")
import torch, heat3d_amd as h
N = (37, 37, 37)
for vr in (8,):
    for ov in (False,):
        for it in (3, 6, 9, 30):
            g = h.HeatSolver(N, it, 0.0, backend="hip", virtual_ranks=vr, decomp=(vr, 1, 1), overlap=ov,
                             extra_args=["--temporal", "3"])
            c = h.HeatSolver(N, it, 0.0, backend="cpu", extra_args=["--temporal", "1"])
            g.run(); c.run()
            a, b = g.gather(), c.gather()
            d = np.abs(a - b)
            idx = np.argwhere(d > 0)
            print(vr, ov, it, "maxdiff", d.max(), "count", len(idx), "first", idx[:5].tolist() if len(idx) else None,
                  "x-planes", sorted(set(idx[:, 0].tolist()))[:20] if len(idx) else None, flush=True)
