"""Unstructured inputs on the GPU (SURVEY.md 8f row f2 / BASELINE.json:11 substitute):
generator, reader, writer and RCM through the device C-ABI, and the SA / PMIS V-cycle on
the randomly numbered and the RCM-reordered graph Laplacian, bit-exact against the oracle
(1 rank and 2-3 loopback ranks)."""
import numpy as np
import pytest
import scipy.io

from tests.test_gpu_multirank import level_starts, run_ranks, set_oracle_cuts
from tests.util import loopback_ctx, same_csr, to_dev, to_host

pytestmark = pytest.mark.gpu


def test_graph_laplacian_and_rcm_on_device(ctx, oracle, tmp_path):
    import raptor_amd as ra

    O = oracle
    A = ra.par_graph_laplacian(ctx, 61, 58, seed=4)
    Ao = O.gen_graph_laplacian(61, 58, 4)
    assert same_csr(A.to_scipy_local(), Ao.to_scipy())
    n = A.local_rows
    x = O.vec_uniform(n, 1)
    y = ctx.empty(n)
    A.mult(to_dev(ctx, x), y)
    assert np.array_equal(to_host(ctx, y), Ao.spmv(x))
    B, perm = A.reorder("rcm")
    p = O.rcm(Ao)
    assert np.array_equal(perm, p)
    Bo = O.permute(Ao, p)
    assert same_csr(B.to_scipy_local(), Bo.to_scipy())
    B.mult(to_dev(ctx, x[perm]), y)
    yb = to_host(ctx, y)
    assert np.array_equal(yb, Bo.spmv(x[perm]))
    # the same products, renumbered (row sums now run in the new column order)
    assert np.allclose(yb, Ao.spmv(x)[perm], rtol=1e-13, atol=1e-13 * np.abs(yb).max())
    path = str(tmp_path / "b.bin")
    B.write(path)
    C = ra.read_par_matrix(ctx, path)
    assert same_csr(C.to_scipy_local(), Bo.to_scipy())
    mm = str(tmp_path / "b.mtx")
    scipy.io.mmwrite(mm, Bo.to_scipy(), precision=17)
    D = ra.read_par_matrix(ctx, mm)
    assert same_csr(D.to_scipy_local(), Bo.to_scipy())


@pytest.mark.parametrize("coarsen,smoother,reorder,tol", [("sa", "hybrid_gs", False, 0.0), ("sa", "hybrid_gs", True, 0.0),
                                                          ("sa", "jacobi", True, 0.0), ("pmis", "jacobi", False, 0.0),
                                                          # r6: coarse-operator drop tolerance
                                                          ("sa", "hybrid_gs", True, 0.01)])
def test_vcycle_on_graph_laplacian(ctx, oracle, coarsen, smoother, reorder, tol):
    import raptor_amd as ra

    O = oracle
    A = ra.par_graph_laplacian(ctx, 90, 77, seed=2)
    Ao = O.gen_graph_laplacian(90, 77, 2)
    if reorder:
        A, perm = A.reorder("rcm")
        Ao = O.permute(Ao, perm)
    ml = ra.ParMultilevel(coarsen=coarsen, smoother=smoother, drop_tol=tol).setup(A)
    Ho = O.Hierarchy(Ao, **dict(O.DEFAULTS[coarsen], smoother=O.SMOOTH_JACOBI if smoother == "jacobi"
                                else O.SMOOTH_HYBRID_GS, drop_tol=tol))
    assert ml.num_levels == Ho.num_levels
    for l in range(ml.num_levels):
        assert same_csr(ml.level_matrix(l, "A").to_scipy_local(), Ho.matrix(l, "A"))
    n = Ao.shape[0]
    b = O.vec_uniform(n, 42)
    db = to_dev(ctx, b)
    dx = ctx.zeros(n)
    xo = np.zeros(n)
    for _ in range(3):
        ml.cycle(dx, db)
        xo = Ho.cycle(xo, b)
        assert np.array_equal(to_host(ctx, dx), xo)
    _, hist = ml.pcg(ctx.zeros(n), db, max_iter=10)
    _, hist_o = Ho.pcg(np.zeros(n), b, max_iter=10)
    assert np.all(np.abs(hist - hist_o) <= 1e-9 * hist_o[0])


@pytest.mark.parametrize("nranks,tol", [(2, 0.0), (3, 0.0), (2, 0.01)])
def test_multirank_graph_laplacian(oracle, nranks, tol):
    import raptor_amd as ra

    O = oracle
    Ao = O.gen_graph_laplacian(70, 66, 5)
    p = O.rcm(Ao)
    Bo = O.permute(Ao, p)
    Ho = O.Hierarchy(Bo, **dict(O.DEFAULTS["sa"], drop_tol=tol))
    n = Bo.shape[0]
    b = O.vec_uniform(n, 8)

    def rank(r, nr, world):
        ctx = loopback_ctx(r, nr, world)
        A = ra.par_graph_laplacian(ctx, 70, 66, seed=5)
        B, perm = A.reorder("rcm")
        ml = ra.ParSmoothedAggregationSolver(replicate_below=400, drop_tol=tol).setup(B)
        f, m = B.first_row, B.local_rows
        dx = ctx.zeros(m)
        db = to_dev(ctx, b[f:f + m])
        ml.cycle(dx, db)
        ml.cycle(dx, db)
        return f, m, perm, to_host(ctx, dx), B.info["n_halo"], level_starts(ml)

    res = run_ranks(nranks, rank)
    set_oracle_cuts(Ho, res)
    xo = Ho.cycle(Ho.cycle(np.zeros(n), b), b)
    for f, m, perm, x, halo, _ in res:
        assert np.array_equal(perm, p[f:f + m])
        assert np.array_equal(x, xo[f:f + m])
        assert halo > 0
