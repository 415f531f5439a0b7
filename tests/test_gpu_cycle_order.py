"""Cycle order: on one rank the V-cycle runs the Jacobi levels of a
grid-built hierarchy in a private brick order.  The hierarchy (exported operators, C/F splits)
is unchanged; the cycle's copies are the same operators with rows and columns permuted and each
row's entries in the hierarchy's order.  Bar: every iterate bit-identical to the oracle's cycle
on the hierarchy's own operators, and to the same setup with AMG_CYCLE_ORDER=0."""
import numpy as np
import pytest

from tests.util import oracle_levels, to_dev, to_host

pytestmark = pytest.mark.gpu


def _cycles(ctx, ml, db, n, k):
    dx = ctx.zeros(n)
    out = []
    for _ in range(k):
        ml.cycle(dx, db)
        out.append(to_host(ctx, dx))
    return out


def _is_brick_copy(M, Mc):
    """Mc holds M's rows, permuted, each with M's entries in M's order under a column
    renumbering (square: the same permutation on rows and columns)."""
    a, c = M.to_scipy_local(), Mc.to_scipy_local()
    if a.shape != c.shape or a.nnz != c.nnz:
        return False
    la, lc = np.diff(a.indptr), np.diff(c.indptr)
    # rows of equal multiset of values in the same sequence: match each copy row to a row of M
    key = {}
    for i in range(a.shape[0]):
        key.setdefault(a.data[a.indptr[i]:a.indptr[i + 1]].tobytes(), []).append(i)
    for i in range(c.shape[0]):
        if not key.get(c.data[c.indptr[i]:c.indptr[i + 1]].tobytes()):
            return False
    return sorted(la.tolist()) == sorted(lc.tolist())


@pytest.mark.parametrize("case", ["7pt-pmis", "7pt-sa", "5pt-rs"])
def test_cycle_order_bit_identical(ctx, oracle, monkeypatch, case):
    import raptor_amd as ra

    O = oracle
    kind, coarsen = case.split("-")
    dims = (48, 40, 36) if kind == "7pt" else (160, 144)
    A = ra.par_stencil_grid(ctx, kind, dims)
    n = A.local_rows
    mk = (lambda: ra.ParSmoothedAggregationSolver(smoother="jacobi")) if coarsen == "sa" else \
        (lambda: ra.ParRugeStubenSolver(coarsen=coarsen))
    ml = mk().setup(A)
    # the cycle runs permuted copies on level 1 (>= 4,096 rows)
    A1, A1c = ml.level_matrix(1, "A"), ml.level_matrix(1, "A_cycle")
    assert A1.local_rows >= 4096
    e1, e1c = A1.export(), A1c.export()
    assert not (np.array_equal(e1[1], e1c[1]) and np.array_equal(e1[0], e1c[0])), "no cycle order"
    assert _is_brick_copy(A1, A1c)
    # the hierarchy-order operator's formats wait for a caller (DevMatrix::defer): its first
    # compute call builds them, and it applies in the hierarchy's order
    m1 = A1.local_rows
    x1h, b1h = O.vec_uniform(m1, 5), O.vec_uniform(m1, 6)
    r1 = ctx.empty(m1)
    A1.residual(to_dev(ctx, x1h), to_dev(ctx, b1h), r1)
    A1o = O.Csr.from_arrays(m1, m1, *e1)
    assert np.array_equal(to_host(ctx, r1), A1o.residual(x1h, b1h))
    P0 = ml.level_matrix(0, "P")
    e = ctx.empty(n)
    P0.mult(to_dev(ctx, x1h), e)
    rp, col, val = P0.export()
    assert np.array_equal(to_host(ctx, e), O.Csr.from_arrays(n, m1, rp, col, val).spmv(x1h))
    b = O.vec_uniform(n, 31)
    db = to_dev(ctx, b)
    xs = _cycles(ctx, ml, db, n, 3)
    H = O.Hierarchy(None, levels=oracle_levels(O, ml))
    xo = np.zeros(n)
    for k in range(3):
        xo = H.cycle(xo, b)
        assert np.array_equal(xs[k], xo), ("cycle", k)
    monkeypatch.setenv("AMG_CYCLE_ORDER", "0")
    ml0 = mk().setup(A)
    e0 = ml0.level_matrix(1, "A_cycle").export()
    assert np.array_equal(e0[1], e1[1]) and np.array_equal(e0[2], e1[2])  # the natural operator
    for k, x in enumerate(_cycles(ctx, ml0, db, n, 3)):
        assert np.array_equal(x, xs[k]), ("AMG_CYCLE_ORDER=0", k)
    # PCG preconditioned by the permuted cycle: same history as the natural one
    x1, x0 = ctx.zeros(n), ctx.zeros(n)
    _, h1 = ml.pcg(x1, db, max_iter=8)
    _, h0 = ml0.pcg(x0, db, max_iter=8)
    assert np.array_equal(to_host(ctx, x1), to_host(ctx, x0)) and np.array_equal(h1, h0)


@pytest.mark.parametrize("nranks,boxes", [(2, None), (4, None), (8, (2, 2, 2))], ids=["slabs2", "slabs4", "boxes8"])
def test_cycle_order_multirank(ctx, nranks, boxes):
    """N loopback ranks, each with its own brick order on every permuted level (halo send lists
    in that order): every rank's slice of three V-cycles equals the one-rank iterate."""
    import raptor_amd as ra
    from tests.test_gpu_multirank import run_ranks
    from tests.util import loopback_ctx

    dims = (96, 80, 64)  # level 1 (~151 k rows) above replicate_below = 65,536: distributed
    A = ra.par_stencil_grid(ctx, "7pt", dims, boxes=boxes)
    n = A.local_rows
    ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
    assert ml.level_info(1)["n_global"] > 65536
    b = np.random.default_rng(3).uniform(-1.0, 1.0, n)
    ref = _cycles(ctx, ml, to_dev(ctx, b), n, 3)

    def body(r, nr, world):
        c = loopback_ctx(r, nr, world)
        Ar = ra.par_stencil_grid(c, "7pt", dims, boxes=boxes)
        f, m = Ar.first_row, Ar.local_rows
        mr = ra.ParRugeStubenSolver(coarsen="pmis", replicate_below=65536).setup(Ar)
        permuted = not np.array_equal(mr.level_matrix(1, "A_cycle").export()[1],
                                      mr.level_matrix(1, "A").export()[1])
        xs = _cycles(c, mr, to_dev(c, b[f:f + m]), m, 3)
        return f, m, permuted, xs

    for f, m, permuted, xs in run_ranks(nranks, body):
        assert permuted or m == 0
        for k in range(3):
            assert np.array_equal(xs[k], ref[k][f:f + m]), ("cycle", k, f)
