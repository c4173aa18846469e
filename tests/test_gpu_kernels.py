"""gfx950 kernel numerics vs a plain-PyTorch reference of the same op.

The kernels evaluate heat3D.cu:128-131 with explicit fused multiply-adds in
nvcc's contraction order (kernels.hpp ftcs_update) and no implicit
contraction, so the HIP result must equal the torch CPU evaluation (exact FMA
emulation, utils/fma.py) bit for bit, fp64 and fp32, for every kernel variant.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

VARIANTS_F64 = ["naive", "tile", "tile:2:4:1:4", "tile:2:4:2:2", "tile:2:8:2:2", "tile:2:8:4:1", "tile:2:6:2:4",
                "tile:2:4:2:4:5:1"]
VARIANTS_F32 = ["naive", "tile", "tile:4:4:2:2", "tile:4:8:1:4", "tile:2:8:2:2:3:1"]


def _random_field(ops, n, dtype, gpu, seed=0):
    g = torch.Generator().manual_seed(seed)
    f = ops.PaddedField(n, dtype=dtype, device="cpu")
    f.ghosted().copy_(torch.rand(tuple(v + 2 for v in n), generator=g, dtype=torch.float64).to(dtype))
    d = ops.PaddedField(n, dtype=dtype, device=gpu)
    d.flat.copy_(f.flat)
    return f, d


@pytest.mark.parametrize("dtype,variants", [(torch.float64, VARIANTS_F64), (torch.float32, VARIANTS_F32)])
@pytest.mark.parametrize("n", [(9, 13, 130), (17, 21, 259), (5, 3, 64), (40, 33, 1022)])
def test_stencil_bitwise(h3d, gpu, dtype, variants, n):
    ops = h3d.ops
    D = (1 / 15, 1 / 15, 1 / 15) if n[0] != 17 else (0.05, 0.07, 0.03)
    host, dev = _random_field(ops, n, dtype, gpu)
    ref, res_ref = ops.ftcs_reference(host.ghosted(), D)
    for v in variants:
        out = ops.PaddedField(n, dtype=dtype, device=gpu)
        state = ops.new_state(gpu)
        ops.ftcs_step(dev, out, D, kernel=v, state=state)
        torch.cuda.synchronize()
        got = out.owned().cpu()
        assert torch.equal(got, ref), f"{v} {dtype} {n}: max diff {(got - ref).abs().max().item()}"
        assert ops.residual_from_state(state) == res_ref, v


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_stencil_subbox(h3d, gpu, dtype):
    """Partial boxes with unaligned z starts (interior/shell split) write only the box."""
    ops = h3d.ops
    n = (12, 14, 200)
    D = (0.06, 0.05, 0.04)
    host, dev = _random_field(ops, n, dtype, gpu, seed=3)
    ref, _ = ops.ftcs_reference(host.ghosted(), D)
    for box in ([1, 11, 1, 13, 1, 199], [0, 1, 0, 14, 0, 200], [3, 7, 2, 9, 5, 133], [0, 12, 0, 14, 0, 1]):
        for v in ("naive", "tile", "tile:2:4:2:4", "tile:2:8:4:1"):
            out = ops.PaddedField(n, dtype=dtype, device=gpu)
            out.flat.fill_(-7.0)
            ops.ftcs_step(dev, out, D, box=box, kernel=v)
            torch.cuda.synchronize()
            got = out.owned().cpu()
            sl = (slice(box[0], box[1]), slice(box[2], box[3]), slice(box[4], box[5]))
            assert torch.equal(got[sl], ref[sl]), (v, box)
            mask = torch.ones(n, dtype=torch.bool)
            mask[sl] = False
            assert bool((got[mask] == -7.0).all()), f"{v} wrote outside box {box}"


def test_done_flag_makes_kernel_noop(h3d, gpu, ext):
    ops = h3d.ops
    n = (8, 8, 128)
    host, dev = _random_field(ops, n, torch.float64, gpu)
    out = ops.PaddedField(n, device=gpu)
    out.flat.fill_(3.0)
    state = ops.new_state(gpu)
    state.view(torch.int32)[h3d.native().STATE_DONE_OFFSET // 4] = 1
    for v in ("naive", "tile"):
        ops.ftcs_step(dev, out, (0.1, 0.1, 0.1), kernel=v, state=state)
    torch.cuda.synchronize()
    assert bool((out.flat == 3.0).all())


def test_init_field_matches_cpu(h3d, gpu):
    ops = h3d.ops
    N = (19, 23, 29)
    n = (7, 10, 27)
    gstart = (5, 1, 1)
    h = tuple(1.0 / (v - 1.0) for v in N)
    for dtype in (torch.float64, torch.float32):
        c = ops.PaddedField(n, dtype=dtype)
        d = ops.PaddedField(n, dtype=dtype, device=gpu)
        ops.init_field(c, gstart, N, h)
        ops.init_field(d, gstart, N, h)
        torch.cuda.synchronize()
        assert torch.equal(c.flat, d.flat.cpu())


@pytest.mark.parametrize("box", [[0, 6, 0, 9, 0, 1], [0, 6, 0, 9, 67, 70], [0, 6, -1, 10, -1, 2],
                                 [1, 5, 2, 7, 10, 27], [0, 6, 0, 9, 0, 70], [0, 1, 0, 9, 0, 70]])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_pack_unpack_box_shapes(h3d, gpu, box, dtype):
    """Pack / unpack of thin z faces (1-3 columns: many rows per workgroup),
    ghost-inclusive and general boxes, against plain tensor slicing."""
    ops = h3d.ops
    n = (6, 9, 70)
    _, dev = _random_field(ops, n, dtype, gpu, seed=7)
    ex, ey, ez = box[1] - box[0], box[3] - box[2], box[5] - box[4]
    buf = torch.empty(ex * ey * ez, dtype=dtype, device=gpu)
    ops.pack_box(dev, box, buf)
    g = dev.ghosted()
    want = g[box[0] + 1:box[1] + 1, box[2] + 1:box[3] + 1, box[4] + 1:box[5] + 1]
    torch.cuda.synchronize()
    assert torch.equal(buf.view(ex, ey, ez).cpu(), want.cpu())
    other = ops.PaddedField(n, dtype=dtype, device=gpu)
    ops.unpack_box(other, box, buf)
    torch.cuda.synchronize()
    got = other.ghosted()[box[0] + 1:box[1] + 1, box[2] + 1:box[3] + 1, box[4] + 1:box[5] + 1]
    assert torch.equal(got.cpu(), want.cpu())


def test_pack_unpack_roundtrip(h3d, gpu):
    ops = h3d.ops
    n = (6, 9, 70)
    _, dev = _random_field(ops, n, torch.float64, gpu, seed=5)
    box = [0, 6, 0, 1, 0, 70]  # a y face (strided)
    buf = torch.empty(6 * 70, dtype=torch.float64, device=gpu)
    ops.pack_box(dev, box, buf)
    other = ops.PaddedField(n, device=gpu)
    ops.unpack_box(other, [0, 6, -1, 0, 0, 70], buf)
    torch.cuda.synchronize()
    assert torch.equal(other.ghosted()[1:-1, 0, 1:-1].cpu(), dev.owned()[:, 0, :].cpu())
