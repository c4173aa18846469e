"""Topology (MPI_Dims_create / Cart clone) and decomposition."""
import itertools

import pytest

from heat3d_amd.parallel import topology as T


# MPI_Dims_create(P, 3) results (reference heat3D.cu:243)
MPI_DIMS = {1: (1, 1, 1), 2: (2, 1, 1), 3: (3, 1, 1), 4: (2, 2, 1), 6: (3, 2, 1), 8: (2, 2, 2),
            12: (3, 2, 2), 16: (4, 2, 2), 24: (4, 3, 2), 27: (3, 3, 3), 32: (4, 4, 2), 64: (4, 4, 4)}


@pytest.mark.parametrize("p", sorted(MPI_DIMS))
def test_dims_create_matches_mpi(ext, p):
    assert tuple(ext.dims_create(p)) == MPI_DIMS[p]
    assert T.dims_create(p) == MPI_DIMS[p]


def test_dims_create_fixed(ext):
    assert tuple(ext.dims_create(8, [8, 1, 1])) == (8, 1, 1)
    assert tuple(ext.dims_create(8, [0, 1, 1])) == (8, 1, 1)
    assert tuple(ext.dims_create(8, [0, 0, 1])) == (4, 2, 1)
    with pytest.raises(Exception):
        ext.dims_create(8, [3, 0, 0])


def test_cart_rank_order_z_fastest():
    # rank = (cx * dy + cy) * dz + cz (survey [RUN] from out.dat zone origins)
    dims = (2, 3, 4)
    for r in range(24):
        c = T.coords_of(r, dims)
        assert T.rank_of(c, dims) == r
    assert T.coords_of(1, dims) == (0, 0, 1)
    assert T.coords_of(4, dims) == (0, 1, 0)


@pytest.mark.parametrize("N,dims", [((27, 27, 27), (2, 2, 2)), ((1024, 1024, 1024), (8, 1, 1)),
                                    ((33, 20, 17), (3, 2, 1)), ((2048, 2048, 2048), (2, 2, 2))])
def test_decomposition_native_matches_python(ext, N, dims):
    nat = ext.decomposition(list(N), list(dims))
    py = T.decompose(N, dims)
    for a, b in zip(nat, py):
        assert tuple(a["n"]) == b.n and tuple(a["gstart"]) == b.gstart
        assert list(a["neighbors"]) == b.neighbors
        assert tuple(a["extended"]) == b.extended()


@pytest.mark.parametrize("N,dims", [((27, 19, 33), (2, 2, 2)), ((10, 10, 10), (8, 1, 1)), ((9, 30, 12), (1, 4, 3))])
def test_extended_boxes_tile_grid(N, dims):
    seen = set()
    for s in T.decompose(N, dims):
        e = s.extended()
        for p in itertools.product(range(e[0], e[1]), range(e[2], e[3]), range(e[4], e[5])):
            assert p not in seen
            seen.add(p)
    assert len(seen) == N[0] * N[1] * N[2]


def test_baseline_grids_illegal_in_reference_but_fine_here(ext):
    # 1024^3 / 2048^3 on even process grids violate heat3D.cu:375-380
    assert not T.reference_legal((1024,) * 3, (8, 1, 1))
    assert not T.reference_legal((2048,) * 3, (2, 2, 2))
    assert T.reference_legal((1025,) * 3, (8, 1, 1))
    subs = ext.decomposition([1024] * 3, [8, 1, 1])
    assert sum(s["n"][0] for s in subs) == 1022
    assert max(s["n"][0] for s in subs) - min(s["n"][0] for s in subs) <= 1


def test_split_interior(ext):
    # slab rank with both x neighbours: interior x in [1, n-1), two x shell slabs
    interior, shell = ext.split_interior([16, 10, 12], [3, 5, -1, -1, -1, -1])
    assert tuple(interior) == (1, 15, 0, 10, 0, 12)
    assert sorted(tuple(b) for b in shell) == [(0, 1, 0, 10, 0, 12), (15, 16, 0, 10, 0, 12)]
    interior, shell = ext.split_interior([8, 8, 8], [1, 2, 3, 4, 5, 6])
    assert tuple(interior) == (1, 7, 1, 7, 1, 7)
    vol = sum((b[1] - b[0]) * (b[3] - b[2]) * (b[5] - b[4]) for b in shell)
    assert vol == 8 ** 3 - 6 ** 3


def test_halo_and_memory_planning():
    # 1024^3 fp64 slab over 8 GPUs: ~8 MiB per face, <= 2 faces per rank
    hb = T.halo_bytes_per_iteration((1024,) * 3, (8, 1, 1), 8)
    assert max(hb) == 2 * 1022 * 1022 * 8 and min(hb) == 1022 * 1022 * 8
    # 4096^3 fp32 on 2x2x2: ~69 GB of fields per GPU, fits 288 GB HBM
    fb = T.field_bytes_per_rank((4096,) * 3, (2, 2, 2), 4)
    assert 60e9 < fb < 80e9


def test_layout_alignment(ext):
    for n in ([5, 7, 1022], [1, 1, 1], [3, 4, 127]):
        for es in (8, 4):
            L = ext.layout(n, es)
            assert (L["origin"] * es) % 128 == 0
            assert (L["sy"] * es) % 128 == 0
            assert L["sy"] >= L["zoff"] + n[2] + 1
            assert L["elems"] >= (n[0] + 2) * L["sx"]


def test_choose_dims_from_link_rate():
    """--decomp auto of the bench: slabs at or above the proxy's crossover
    (8 ranks: 55 GB/s), 4x2x1 below it; other rank counts and an unknown
    rate keep the slab (heat3D.cu:243-263 picks by rank count alone)."""
    from heat3d_amd.parallel import SLAB_MIN_LINK_GBPS, choose_dims

    N = (1024, 1024, 1024)
    assert SLAB_MIN_LINK_GBPS[8] == 55.0
    assert choose_dims(N, 8, 64.0) == (8, 1, 1)
    assert choose_dims(N, 8, 55.0) == (8, 1, 1)
    assert choose_dims(N, 8, 40.0) == (4, 2, 1)
    assert choose_dims(N, 8, 3.5) == (4, 2, 1)
    assert choose_dims(N, 8, None) == (8, 1, 1)
    assert choose_dims(N, 4, 10.0) == (4, 1, 1)
    assert choose_dims(N, 2, 1.0) == (2, 1, 1)
    assert choose_dims((40, 1024, 1024), 8, 10.0) == (2, 2, 2)   # slabs too thin: dims_create


def test_decomp_candidates_and_measured_pick():
    """bench.py --decomp auto: the candidate grids it times (slabs, 2D, 3D
    blocks; only where every split axis keeps an interior between its K-deep
    boundary layers) and the pick by the slowest rank's time, with a margin
    that keeps the earlier (slab) candidate on a near tie."""
    from heat3d_amd.parallel import decomp_candidates, pick_measured

    assert decomp_candidates((1024,) * 3, 8) == [(8, 1, 1), (4, 2, 1), (2, 2, 2)]
    assert decomp_candidates((1024,) * 3, 4) == [(4, 1, 1), (2, 2, 1)]
    assert decomp_candidates((1024,) * 3, 2) == [(2, 1, 1)]
    assert decomp_candidates((40, 40, 40), 8) == [(4, 2, 1), (2, 2, 2)]   # 38 / 8 < 7: no slabs
    t = [{"dims": (8, 1, 1), "ms_per_step": 1.00}, {"dims": (4, 2, 1), "ms_per_step": 0.99},
         {"dims": (2, 2, 2), "ms_per_step": 1.20}]
    assert pick_measured(t) == (8, 1, 1)          # within the 2 % margin: slabs stay
    t[1]["ms_per_step"] = 0.95
    assert pick_measured(t) == (4, 2, 1)
    t[2]["ms_per_step"] = 0.90
    assert pick_measured(t) == (2, 2, 2)
    with pytest.raises(ValueError):
        pick_measured([{"dims": (2, 1, 1), "ms_per_step": None}])
