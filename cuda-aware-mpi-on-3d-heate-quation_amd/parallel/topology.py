"""Pure-Python mirrors of the native topology / decomposition (csrc/core/decomp.cpp).

Used for planning (message sizes, memory per GPU) and as an independent check
of the native implementation in tests.  Reference counterparts:
``MPI_Dims_create`` / ``MPI_Cart_create`` / ``MPI_Cart_shift`` /
``MPI_Cart_coords`` (heat3D.cu:224-263) and the chunk rule (heat3D.cu:373-389),
which is replaced by an uneven split of the N-2 interior points with ghost
shells.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

FACES = ("LEFT", "RIGHT", "BOTTOM", "TOP", "BACK", "FRONT")


def dims_create(nprocs: int, fixed: Sequence[int] = (0, 0, 0)) -> Tuple[int, int, int]:
    """Balanced non-increasing 3-factorisation (MPI_Dims_create semantics)."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    fixed = list(fixed)
    fprod = 1
    for f in fixed:
        if f > 0:
            fprod *= f
    if nprocs % fprod:
        raise ValueError(f"fixed dims product {fprod} does not divide {nprocs}")
    rem = nprocs // fprod
    nfree = sum(1 for f in fixed if f <= 0)
    if nfree == 0:
        if rem != 1:
            raise ValueError("fixed dims do not multiply to nprocs")
        return tuple(fixed)  # type: ignore[return-value]
    best = None

    def rec(left, slots, cap, cur):
        nonlocal best
        if slots == 1:
            if left > cap:
                return
            c = cur + [left]
            key = (max(c) - min(c), max(c))
            if best is None or key < best[0]:
                best = (key, c)
            return
        for d in range(min(left, cap), 0, -1):
            if left % d == 0:
                rec(left // d, slots - 1, d, cur + [d])

    rec(rem, nfree, rem, [])
    vals = iter(best[1])
    return tuple(f if f > 0 else next(vals) for f in fixed)  # type: ignore[return-value]


def split_even(n: int, parts: int, p: int) -> Tuple[int, int]:
    base, rem = divmod(n, parts)
    count = base + (1 if p < rem else 0)
    start = p * base + min(p, rem)
    return start, count


@dataclass
class Subdomain:
    rank: int
    coords: Tuple[int, int, int]
    n: Tuple[int, int, int]
    gstart: Tuple[int, int, int]
    neighbors: List[int] = field(default_factory=list)

    def extended(self) -> Tuple[int, int, int, int, int, int]:
        out = []
        for a in range(3):
            lo = self.gstart[a] - (1 if self.neighbors[2 * a] < 0 else 0)
            hi = self.gstart[a] + self.n[a] + (1 if self.neighbors[2 * a + 1] < 0 else 0)
            out += [lo, hi]
        return tuple(out)  # type: ignore[return-value]


def coords_of(rank: int, dims: Sequence[int]) -> Tuple[int, int, int]:
    return (rank // (dims[1] * dims[2]), (rank // dims[2]) % dims[1], rank % dims[2])


def rank_of(c: Sequence[int], dims: Sequence[int]) -> int:
    if any(c[a] < 0 or c[a] >= dims[a] for a in range(3)):
        return -1
    return (c[0] * dims[1] + c[1]) * dims[2] + c[2]


def decompose(N: Sequence[int], dims: Sequence[int]) -> List[Subdomain]:
    subs = []
    P = dims[0] * dims[1] * dims[2]
    for r in range(P):
        c = coords_of(r, dims)
        n, g = [], []
        for a in range(3):
            if N[a] - 2 < dims[a]:
                raise ValueError(f"axis {a}: {N[a] - 2} interior points cannot be split over {dims[a]} ranks")
            st, cnt = split_even(N[a] - 2, dims[a], c[a])
            n.append(cnt)
            g.append(1 + st)
        nb = []
        for a in range(3):
            for side in (-1, 1):
                cc = list(c)
                cc[a] += side
                nb.append(rank_of(cc, dims))
        subs.append(Subdomain(r, c, tuple(n), tuple(g), nb))
    return subs


def reference_legal(N: Sequence[int], dims: Sequence[int]) -> bool:
    """The reference's partition assert (heat3D.cu:375-380)."""
    return all((N[a] - 1) % dims[a] == 0 for a in range(3))


def halo_bytes_per_iteration(N: Sequence[int], dims: Sequence[int], esize: int = 8) -> List[int]:
    """Bytes each rank sends per iteration (faces only; a 7-point stencil
    needs no edge/corner ghosts)."""
    out = []
    for s in decompose(N, dims):
        b = 0
        for f, nb in enumerate(s.neighbors):
            if nb < 0:
                continue
            a = f // 2
            other = [s.n[x] for x in range(3) if x != a]
            b += other[0] * other[1] * esize
        out.append(b)
    return out


def field_bytes_per_rank(N: Sequence[int], dims: Sequence[int], esize: int = 8) -> int:
    """Device bytes of the two ping-pong fields of the largest subdomain."""
    big = max(decompose(N, dims), key=lambda s: s.n[0] * s.n[1] * s.n[2])
    return 2 * (big.n[0] + 2) * (big.n[1] + 2) * (big.n[2] + 2) * esize


def best_dims_for(N: Sequence[int], nprocs: int, prefer: Optional[str] = None) -> Tuple[int, int, int]:
    """Process grid choice: 'slab' -> (P,1,1) (x faces are contiguous: zero-copy
    halos); 'block' -> balanced dims_create; default: slab while each slab is
    at least 16 planes thick, else block."""
    if prefer == "slab":
        return (nprocs, 1, 1)
    if prefer == "block":
        return dims_create(nprocs)
    if (N[0] - 2) // nprocs >= 16:
        return (nprocs, 1, 1)
    return dims_create(nprocs)


# Slab or 2D blocks for a multi-GPU job, from the measured link rate.  The
# reference picks its process grid from the rank count alone
# (MPI_Dims_create, heat3D.cu:243-263).  Phantom-rank proxy of the 1024^3 fp64
# bench at the driver's window (profiles/rank_proxy_r04.md, emulated links):
# 8 ranks as 8x1x1 slabs win from ~55 GB/s per link up (0.2179 vs 0.2377
# ms/step at 96 GB/s), 4x2x1 blocks below (0.2603 vs 0.3256 at 32 GB/s),
# because a slab sends 2 K-deep 1024^2 faces per sweep over one link each
# while 4x2x1 sends 3 smaller ones; 4 ranks keep 4x1x1 at 40-64 GB/s
# (0.4152 vs 0.4239 for 2x2x1) and 2 ranks have nothing else.
SLAB_MIN_LINK_GBPS = {8: 55.0}


def choose_dims(N: Sequence[int], nprocs: int, link_gbps: Optional[float]) -> Tuple[int, int, int]:
    """Round 5's --decomp auto heuristic (kept as a documented rule, no
    longer used by bench.py, which times every candidate grid since round 6:
    decomp_candidates / pick_measured): slabs (best_dims_for) unless the
    job's slowest measured link (Solver.link_probe, GB/s one way) is below
    the phantom-rank proxy's crossover for this rank count — a proxy-derived
    constant, not a measurement of real links — then the 2D block with the x
    extent halved and 2 ranks along y."""
    slab = best_dims_for(N, nprocs)
    cut = SLAB_MIN_LINK_GBPS.get(nprocs)
    if cut is None or link_gbps is None or link_gbps <= 0 or link_gbps >= cut or slab[0] != nprocs:
        return slab
    return (nprocs // 2, 2, 1)


def decomp_candidates(N: Sequence[int], nprocs: int, K: int = 3) -> List[Tuple[int, int, int]]:
    """Process grids the bench's ``--decomp auto`` times at start-up: x slabs,
    the 2D block with two ranks along y, and the balanced 3D block
    (MPI_Dims_create, heat3D.cu:243), in that order, without duplicates and
    only where every split axis keeps an interior between its K-deep boundary
    layers (>= 2K + 1 points: the overlapped sweep)."""
    cands = [(nprocs, 1, 1)]
    if nprocs % 2 == 0 and nprocs >= 4:
        cands.append((nprocs // 2, 2, 1))
    cands.append(dims_create(nprocs))
    out: List[Tuple[int, int, int]] = []
    for d in cands:
        d = tuple(int(v) for v in d)
        if d in out:
            continue
        if all(d[a] == 1 or (N[a] - 2) // d[a] >= 2 * K + 1 for a in range(3)):
            out.append(d)  # type: ignore[arg-type]
    return out


def pick_measured(trials: Sequence[dict], margin: float = 0.02) -> Tuple[int, int, int]:
    """The fastest timed candidate (``{"dims", "ms_per_step"}``, the slowest
    rank's time each); a later candidate must beat the earlier pick by
    ``margin`` (noise of short windows must not flip slabs to blocks)."""
    best = None
    for t in trials:
        if t.get("ms_per_step") is None:
            continue
        if best is None or t["ms_per_step"] < best["ms_per_step"] * (1.0 - margin):
            best = t
    if best is None:
        raise ValueError("no decomposition candidate was timed")
    return tuple(best["dims"])  # type: ignore[return-value]
