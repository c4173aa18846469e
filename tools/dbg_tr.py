"""Locate mismatches of a multi-step kernel against K reference single steps."""
import sys
import torch
sys.path.insert(0, "/root/repo")
import heat3d_amd as h

ops = h.ops
gpu = torch.device("cuda", 0)
D = (0.06, 0.05, 0.04)
for n in [(9, 13, 130), (17, 21, 259)]:
    g = torch.Generator().manual_seed(5)
    host = ops.PaddedField(n, dtype=torch.float64)
    host.ghosted().copy_(torch.rand(tuple(v + 2 for v in n), generator=g, dtype=torch.float64))
    dev = ops.PaddedField(n, dtype=torch.float64, device=gpu)
    dev.flat.copy_(host.flat)
    for v in sys.argv[1:]:
        K = int(v.split(":")[0][2])
        T = host.ghosted().clone()
        for _ in range(K):
            u, r = ops.ftcs_reference(T, D)
            T = T.clone()
            T[1:-1, 1:-1, 1:-1] = u
        want = T[1:-1, 1:-1, 1:-1]
        for rep in range(3):
            out = ops.PaddedField(n, dtype=torch.float64, device=gpu)
            out.flat.fill_(-3.0)
            st = ops.new_state(gpu)
            ops.ftcs_step2(dev, out, D, kernel=v, state=st, slot=0)
            torch.cuda.synchronize()
            got = out.owned().cpu()
            bad = (got != want).nonzero()
            print(n, v, rep, "bad", len(bad), "planes", sorted(set(bad[:, 0].tolist()))[:10],
                  "rows", sorted(set(bad[:, 1].tolist()))[:10], "cols", sorted(set(bad[:, 2].tolist()))[:12], flush=True)
