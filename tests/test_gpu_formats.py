"""The per-nonzero device formats built on the GPU (formats.hip: block-aligned col / val
streams, x-tile ids and tile indices, value tables / indices / diagonal slots, row ends) are
byte-identical to the host builders (AMG_DEVICE_FORMATS=0) for every operator of a hierarchy:
square A_l on the x-tile path, rectangular P_l / R_l on the tile or gather paths, with and
without value indexing, at one rank and with halo columns (loopback ranks)."""
import pytest

from tests.util import make_ctx

pytestmark = pytest.mark.gpu


def _digests(ra, ctx, kind, dims, coarsen, smoother, monkeypatch, device, boxes=None):
    monkeypatch.setenv("AMG_DEVICE_FORMATS", "1" if device else "0")
    A = ra.par_stencil_grid(ctx, kind, dims)
    ml = ra.ParMultilevel(coarsen=coarsen, smoother=smoother).setup(A)
    out = [A.format_digest()]
    for l in range(ml.num_levels):
        out.append(ml.level_matrix(l, "A").format_digest())
        if l + 1 < ml.num_levels:
            out.append(ml.level_matrix(l, "P").format_digest())
            out.append(ml.level_matrix(l, "R").format_digest())
    return out


@pytest.mark.parametrize("kind,dims,coarsen,smoother", [
    ("7pt", (40, 36, 44), "pmis", "jacobi"),
    ("27pt", (30, 28, 26), "sa", "hybrid_gs"),
    ("5pt", (300, 280), "pmis", "jacobi"),
    ("7pt-lines32", (40, 36, 44), "pmis", "jacobi"),
])
def test_device_formats_equal_host_builders(kind, dims, coarsen, smoother, monkeypatch):
    import raptor_amd as ra

    if kind.endswith("-lines32"):  # 32-byte x-tile lines forced on every tiled operator
        monkeypatch.setenv("AMG_TILE_LINE", "4")
        kind = kind.split("-")[0]
    ctx = make_ctx(0)
    dev = _digests(ra, ctx, kind, dims, coarsen, smoother, monkeypatch, True)
    host = _digests(ra, ctx, kind, dims, coarsen, smoother, monkeypatch, False)
    assert len(dev) >= 4
    assert dev == host
