"""--scheme reference: emulation of the reference's own shared-plane domain
decomposition (face update with halos, edge extrapolation, corner averaging,
local norm, any-rank stop; heat3D.cu:373-389, 757-1073, 1093-1106).

SURVEY.md App. B.3b pins its P-dependence at 27^3, eps 1e-5: iteration counts,
what rank 0 prints, and the true global error.  The default scheme of this
framework must instead give the P=1 row for every process grid."""
import numpy as np
import pytest

from conftest import run_cli

B3B = [((1, 1, 1), 2513, 0.0192, 0.0192), ((2, 1, 1), 2511, 0.0189, 0.0194),
       ((2, 2, 1), 2543, 0.0185, 0.0193), ((2, 2, 2), 2615, 0.0180, 0.0193)]


@pytest.mark.parametrize("dims,iters,err_rank0,err_global", B3B)
def test_survey_b3b_table(ext, dims, iters, err_rank0, err_global):
    rs = ext.ReferenceScheme((27, 27, 27), dims)
    assert tuple(rs.chunk) == tuple((27 - 1) // d + 1 for d in dims)
    r = rs.run(10 ** 6, 1e-5)
    assert r["converged"] and r["conv_iter"] == iters
    assert round(r["error_percent_rank0"], 4) == err_rank0
    assert round(r["error_percent_global"], 4) == err_global


def test_single_rank_equals_default_scheme(h3d, ext):
    # P = 1: no shared planes, the two schemes are the same algorithm
    rs = ext.ReferenceScheme((21, 19, 23), (1, 1, 1))
    r = rs.run(300, 0.0)
    s = h3d.HeatSolver((21, 19, 23), 300, 0.0, backend="cpu")
    s.run()
    assert np.array_equal(rs.gather(), s.gather().ravel())


def test_default_scheme_is_p_invariant_where_reference_is_not(h3d, ext):
    base = h3d.HeatSolver((27, 27, 27), 10 ** 6, 1e-5, backend="cpu").run()["conv_iter"]
    for dims in ((2, 1, 1), (2, 2, 2)):
        s = h3d.HeatSolver((27, 27, 27), 10 ** 6, 1e-5, backend="cpu", virtual_ranks=8 if dims == (2, 2, 2) else 2,
                           decomp=dims)
        assert s.run()["conv_iter"] == base == 2513


def test_partition_rule_enforced(ext):
    with pytest.raises(ext.NativeError, match="N-1"):
        ext.ReferenceScheme((28, 27, 27), (2, 1, 1))


def test_cli_reference_scheme(heat3d_bin, tmp_path):
    out = tmp_path / "out.dat"
    p = run_cli(["27", "27", "27", "100000", "1e-5", "--scheme", "reference", "--decomp", "2x2x1",
                             "--output", str(out)], cwd=tmp_path)
    assert p.returncode == 0, p.stderr
    assert "Simulation has converged in 2543 iterations with a convergence threshold of 1.000000e-05" in p.stdout
    assert "L2-norm error: 0.0185 %" in p.stdout
    text = out.read_text().splitlines()
    assert text[1] == 'VARIABLES = "X", "Y", "Z", "T", "rank"'
    zones = [l for l in text if l.startswith("ZONE")]
    assert zones == ['ZONE T = "0", I=14, J=14, K=27, F=POINT'] * 4  # every title "0" 
