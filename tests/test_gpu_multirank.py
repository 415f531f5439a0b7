"""Multi-rank device path on ONE GPU: N virtual ranks (threads, loopback transport) run the
same halo plans, pack kernels, interior/boundary overlap, distributed setup and coarse/norm
allgathers as the RCCL path.  Every rank's slice of every kernel output, level operator and
V-cycle iterate must be bit-identical to the serial oracle."""
import threading
import uuid

import numpy as np
import pytest

from tests.util import loopback_ctx, to_dev, to_host

pytestmark = pytest.mark.gpu


def run_ranks(n, fn):
    """fn(rank, nranks, world) in n threads; re-raise the first failure."""
    world = "w-" + uuid.uuid4().hex
    errs = [None] * n
    out = [None] * n

    def body(r):
        try:
            out[r] = fn(r, n, world)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    # a rank that fails leaves its peers timing out at the next loopback barrier: report
    # the root cause first
    bad = [e for e in errs if e is not None]
    bad.sort(key=lambda e: "barrier timed out" in str(e))
    if bad:
        raise bad[0]
    return out


def level_starts(ml):
    """first_row of every level operator on this rank (a replicated level starts at 0)."""
    return [ml.level_matrix(l, "A").first_row for l in range(ml.num_levels)]


def set_oracle_cuts(Ho, res):
    """Hybrid-GS blocks are clipped at rank boundaries: give the oracle each
    level's partition, gathered from the ranks' results (last element = level_starts)."""
    starts = [r[-1] for r in res]
    for l in range(Ho.num_levels):
        Ho.set_cuts(l, sorted({s[l] for s in starts if l < len(s)}))


@pytest.mark.parametrize("tpl", [False, True, "plain"], ids=["csr", "templates", "plain"])
@pytest.mark.parametrize("nranks", [2, 3])
def test_slab_kernels_bit_exact(oracle, monkeypatch, nranks, tpl):
    """templates: interior rows on the row-template kernel, halo rows on the CSR block
    kernel (size floor lowered so the small slabs qualify).  plain: AMG_FORMAT_CSR, the plain
    CSR kernel over local | halo columns after the exchange."""
    import raptor_amd as ra

    if tpl is True:
        monkeypatch.setenv("AMG_TPL_MIN_ROWS", "0")

    O = oracle
    dims = (14, 13, 17)
    Ao = O.gen_7pt(*dims)
    n = Ao.shape[0]
    x = O.vec_uniform(n, 3)
    b = O.vec_uniform(n, 4)
    ref = {"y": Ao.spmv(x), "r": Ao.residual(x, b), "j": Ao.jacobi(x, b, 2.0 / 3.0)}
    rn_ref = O.norm2(Ao.residual(x, b))

    def rank(r, nr, world):
        ctx = loopback_ctx(r, nr, world)
        A = ra.par_stencil_grid(ctx, "7pt", dims)
        if tpl == "plain":
            A.set_format("csr")
        f, m = A.first_row, A.local_rows
        dx, db = to_dev(ctx, x[f:f + m]), to_dev(ctx, b[f:f + m])
        out = ctx.empty(m)
        A.mult(dx, out)
        got = {"y": to_host(ctx, out)}
        A.residual(dx, db, out)
        got["r"] = to_host(ctx, out)
        A.jacobi(dx, db, out)
        got["j"] = to_host(ctx, out)
        got["rn"] = A.residual_norm(dx, db)
        got["halo"] = A.info["n_halo"]
        got["tpl_rows"] = A.info["template_rows"]
        return f, m, got

    res = run_ranks(nranks, rank)
    assert sum(m for _, m, _ in res) == n
    for f, m, got in res:
        for k in ("y", "r", "j"):
            assert np.array_equal(got[k], ref[k][f:f + m]), k
        assert abs(got["rn"] - rn_ref) <= 1e-12 * rn_ref
        assert got["halo"] > 0
        assert (0 < got["tpl_rows"] < m) if tpl is True else got["tpl_rows"] == 0


CASES = [(2, "7pt", (16, 15, 18), "pmis", "jacobi"),
         (3, "7pt", (14, 14, 21), "pmis", "jacobi"),
         (4, "27pt", (10, 11, 16), "sa", "hybrid_gs"),
         (2, "5pt", (40, 34), "pmis", "jacobi"),
         # configs[3]'s partition shape: 8 z-slabs
         (8, "7pt", (48, 48, 96), "pmis", "jacobi"),
         (8, "7pt", (48, 48, 96), "sa", "hybrid_gs")]


@pytest.mark.parametrize("rep", [0, 800, 10 ** 9], ids=["distributed", "rep-deep", "rep-all"])
@pytest.mark.parametrize("nranks,kind,dims,coarsen,smoother", CASES)
def test_multirank_vcycle_bit_exact(oracle, nranks, kind, dims, coarsen, smoother, rep):
    """rep = replicate_below: 0 keeps every level distributed; 800 replicates the coarse
    tail; 1e9 replicates everything below the fine level."""
    _vcycle_vs_oracle(oracle, nranks, kind, dims, coarsen, smoother, rep)


@pytest.mark.parametrize("nranks,kind,dims,boxes,coarsen,smoother",
                         [(8, "7pt", (24, 24, 24), (2, 2, 2), "pmis", "jacobi"),
                          (4, "7pt", (20, 22, 24), (1, 2, 2), "pmis", "jacobi"),
                          (8, "27pt", (12, 12, 12), (2, 2, 2), "sa", "hybrid_gs"),
                          (3, "7pt", (18, 17, 16), (3, 1, 1), "pmis", "jacobi")])
def test_multirank_boxes_vcycle_bit_exact(oracle, nranks, kind, dims, boxes, coarsen, smoother):
    """The box decomposition (bench.py --gpus 8: 2 x 2 x 2 cubes of 256^3): every rank's slice
    of every level operator and V-cycle iterate equals the oracle's hierarchy of P A P^T (the
    box numbering of the same stencil), and the solve history agrees to 1e-10."""
    _vcycle_vs_oracle(oracle, nranks, kind, dims, coarsen, smoother, 0, boxes)


@pytest.mark.parametrize("nranks,kind,dims", [(2, "27pt", (24, 24, 32)), (4, "27pt", (24, 24, 32)),
                                              (8, "7pt", (48, 48, 96))])
def test_multirank_split_gs_bit_exact(oracle, nranks, kind, dims):
    """Split hybrid-GS sweeps on N ranks: every
    distributed Galerkin level of the SA hierarchy runs the CSR-block old-value pass (its halo
    exchanged under the interior blocks) + the chain walk, and the V-cycle iterates stay
    bit-identical to the oracle's rank-cut hybrid GS."""
    split = _vcycle_vs_oracle(oracle, nranks, kind, dims, "sa", "hybrid_gs", 0)
    for per_rank in split:
        assert len(per_rank) >= 2
        assert all(per_rank[1:]), per_rank  # every Galerkin level split, on every rank


def _vcycle_vs_oracle(oracle, nranks, kind, dims, coarsen, smoother, rep, boxes=None):
    import raptor_amd as ra

    O = oracle
    Ao = {"7pt": O.gen_7pt, "5pt": O.gen_5pt, "27pt": O.gen_27pt}[kind](*dims)
    if boxes is not None:
        Ao = O.permute(Ao, ra.box_order(dims, boxes))
    Ho = O.Hierarchy(Ao, **dict(O.DEFAULTS[coarsen], smoother=O.SMOOTH_JACOBI if smoother == "jacobi"
                                else O.SMOOTH_HYBRID_GS))
    n = Ao.shape[0]
    b = Ao.spmv(O.vec_uniform(n, 42))
    levels = [Ho.matrix(l, "A") for l in range(Ho.num_levels)]

    def rank(r, nr, world):
        ctx = loopback_ctx(r, nr, world)
        A = ra.par_stencil_grid(ctx, kind, dims, boxes=boxes)
        ml = ra.ParMultilevel(coarsen=coarsen, smoother=smoother, replicate_below=rep).setup(A)
        f, m = A.first_row, A.local_rows
        bad = []
        if ml.num_levels != Ho.num_levels:
            bad.append(("levels", ml.num_levels, Ho.num_levels))
        for l in range(min(ml.num_levels, Ho.num_levels)):
            M = ml.level_matrix(l, "A")
            loc = M.to_scipy_local()
            G = levels[l][M.first_row:M.first_row + M.local_rows]
            if not (np.array_equal(loc.indptr, G.indptr) and np.array_equal(loc.indices, G.indices)
                    and np.array_equal(loc.data, G.data)):
                bad.append(("A", l))
            # global nonzeros, replicated levels included (held whole by every rank)
            if ml.level_info(l)["nnz_global"] != levels[l].nnz:
                bad.append(("nnz_global", l, ml.level_info(l)["nnz_global"], levels[l].nnz))
        db = to_dev(ctx, b[f:f + m])
        dx = ctx.zeros(m)
        xs = []
        for k in range(3):
            ml.cycle(dx, db)
            xs.append(to_host(ctx, dx))
        dx = ctx.zeros(m)
        _, hist = ml.solve(dx, db, max_iter=6)
        # distributed levels only (a replicated level is whole on every rank)
        split = [bool(ml.level_matrix(l, "A").info["gs_split"]) for l in range(ml.num_levels - 1)
                 if ml.level_matrix(l, "A").local_rows < ml.level_info(l)["n_global"]]
        return bad, hist, f, m, xs, split, level_starts(ml)

    res = run_ranks(nranks, rank)
    set_oracle_cuts(Ho, res)
    xo = np.zeros(n)
    for k in range(3):
        xo = Ho.cycle(xo, b)
        for _, _, f, m, xs, _, _ in res:
            assert np.array_equal(xs[k], xo[f:f + m]), ("cycle", k)
    _, hist_o = Ho.solve(np.zeros(n), b, max_iter=6)
    for bad, hist, *_ in res:
        assert bad == []
        assert np.all(np.abs(hist - hist_o) <= 1e-10 * hist_o)
    assert all(np.array_equal(res[0][1], r[1]) for r in res)  # every rank reports the same
    return [r[5] for r in res]


def test_uneven_partition_from_csr(oracle):
    """ParCSRMatrix.from_csr with a ragged, non-plane-aligned row partition."""
    import raptor_amd as ra

    O = oracle
    Ao = O.gen_27pt(9, 8, 7)
    M = Ao.to_scipy()
    n = M.shape[0]
    cuts = [0, 37, 300, n]
    x = O.vec_uniform(n, 5)
    y_ref = Ao.spmv(x)
    xo = O.Hierarchy(Ao, **O.DEFAULTS["pmis"]).cycle(np.zeros(n), y_ref)

    def rank(r, nr, world):
        ctx = loopback_ctx(r, nr, world)
        lo, hi = cuts[r], cuts[r + 1]
        A = ra.ParCSRMatrix.from_scipy_local(ctx, M[lo:hi], n, lo)
        out = ctx.empty(hi - lo)
        A.mult(to_dev(ctx, x[lo:hi]), out)
        ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
        dx = ctx.zeros(hi - lo)
        ml.cycle(dx, to_dev(ctx, y_ref[lo:hi]))
        return to_host(ctx, out), to_host(ctx, dx)

    res = run_ranks(3, rank)
    for r, (y, xc) in enumerate(res):
        assert np.array_equal(y, y_ref[cuts[r]:cuts[r + 1]])
        assert np.array_equal(xc, xo[cuts[r]:cuts[r + 1]])


def test_multirank_pcg(oracle):
    import raptor_amd as ra

    O = oracle
    dims = (18, 16, 21)
    Ao = O.gen_7pt(*dims)
    n = Ao.shape[0]
    b = O.vec_uniform(n, 5)
    Ho = O.Hierarchy(Ao, **O.DEFAULTS["pmis"])
    _, hist_o = Ho.pcg(np.zeros(n), b, max_iter=10)

    def rank(r, nr, world):
        ctx = loopback_ctx(r, nr, world)
        A = ra.par_stencil_grid(ctx, "7pt", dims)
        ml = ra.ParRugeStubenSolver(coarsen="pmis", replicate_below=500).setup(A)
        f, m = A.first_row, A.local_rows
        _, hist = ml.pcg(ctx.zeros(m), to_dev(ctx, b[f:f + m]), max_iter=10)
        return hist

    for hist in run_ranks(3, rank):
        assert np.all(np.abs(hist - hist_o) <= 1e-9 * hist_o[0])


@pytest.mark.parametrize("values", ["stencil", "random"])
def test_one_row_per_rank(oracle, values):
    """Degenerate partition: one row and one local column per rank with one or two halo
    entries -- the kernel's 8-byte x-tile path (a local or halo vector of one entry);
    value-indexed ("stencil") and value-stream ("random") blocks."""
    import scipy.sparse as sp

    import raptor_amd as ra

    O = oracle
    n = 3
    M = sp.diags([-np.ones(n - 1), 2 * np.ones(n), -np.ones(n - 1)], [-1, 0, 1]).tocsr()
    if values == "random":
        M.data = 1.0 + np.random.default_rng(3).random(M.nnz)
    M.sort_indices()
    Ao = O.Csr.from_scipy(M)
    x, b = O.vec_uniform(n, 7), O.vec_uniform(n, 8)
    ref = {"y": Ao.spmv(x), "r": Ao.residual(x, b), "j": Ao.jacobi(x, b, 2.0 / 3.0)}

    def rank(r, nr, world):
        ctx = loopback_ctx(r, nr, world)
        A = ra.ParCSRMatrix.from_scipy_local(ctx, M[r:r + 1], n, r)
        dx, db, out = to_dev(ctx, x[r:r + 1]), to_dev(ctx, b[r:r + 1]), ctx.empty(1)
        A.mult(dx, out)
        got = {"y": to_host(ctx, out)}
        A.residual(dx, db, out)
        got["r"] = to_host(ctx, out)
        A.jacobi(dx, db, out)
        got["j"] = to_host(ctx, out)
        return got, A.info["n_halo"]

    res = run_ranks(n, rank)
    assert [h for _, h in res] == [1, 2, 1]
    for r, (got, _) in enumerate(res):
        for k in ("y", "r", "j"):
            assert np.array_equal(got[k], ref[k][r:r + 1]), (k, r)


@pytest.mark.parametrize("nranks", [2, 4])
def test_multirank_gs_templates(oracle, monkeypatch, nranks):
    """Hybrid GS per rank with the template kernel on interior blocks (size floor lowered so
    the slabs' stencil rows template), interior ELL slabs before the halo wait, boundary slabs
    after it: forward and backward sweeps bit-identical to the oracle with the rank cuts."""
    import raptor_amd as ra

    monkeypatch.setenv("AMG_TPL_MIN_ROWS", "0")
    O = oracle
    dims = (64, 16, 4 * nranks)  # 4 planes of 1024 rows per rank: first_row % 64 == 0
    Ao = O.gen_27pt(*dims)
    n = Ao.shape[0]
    x, b = O.vec_uniform(n, 3), O.vec_uniform(n, 4)

    def rank(r, nr, world):
        ctx = loopback_ctx(r, nr, world)
        A = ra.par_stencil_grid(ctx, "27pt", dims)
        f, m = A.first_row, A.local_rows
        dx, db, out = to_dev(ctx, x[f:f + m]), to_dev(ctx, b[f:f + m]), ctx.empty(m)
        A.hybrid_gs(dx, db, out, 64)
        fw = to_host(ctx, out)
        A.hybrid_gs(dx, db, out, 64, backward=True)
        return f, m, fw, to_host(ctx, out)

    res = run_ranks(nranks, rank)
    cuts = [f for f, *_ in res]
    fo = Ao.hybrid_gs_cut(x, b, 64, False, cuts)
    bo = Ao.hybrid_gs_cut(x, b, 64, True, cuts)
    for f, m, fw, bw in res:
        assert np.array_equal(fw, fo[f:f + m])
        assert np.array_equal(bw, bo[f:f + m])


@pytest.mark.parametrize("nranks,kind,dims,coarsen", [(2, "7pt", (16, 15, 18), "pmis"), (3, "7pt", (14, 14, 21), "pmis"),
                                                      (8, "7pt", (24, 24, 64), "pmis"), (4, "5pt", (40, 34), "pmis"),
                                                      (3, "27pt", (10, 11, 16), "sa"), (8, "7pt", (24, 24, 64), "sa")])
def test_device_setup_equals_host_multirank(nranks, kind, dims, coarsen):
    """SURVEY 8f row f1 on several ranks: the device PMIS + classical interpolation and MIS(2)
    + smoothed prolongator (rank rows with global column ids, halo states forwarded each round,
    ghost rows of A for the strong F neighbours) build the same hierarchy as the host path,
    level by level and bit for bit -- A, P, R and the C/F split / aggregate ids of every rank."""
    import raptor_amd as ra

    def rank(r, nr, world):
        ctx = loopback_ctx(r, nr, world)
        A = ra.par_stencil_grid(ctx, kind, dims)
        out = []
        for m in (1, 0):
            ml = ra.ParMultilevel(coarsen=coarsen, smoother="jacobi" if coarsen == "pmis" else "hybrid_gs",
                                  setup_device=m, replicate_below=0).setup(A)
            lev = []
            for l in range(ml.num_levels):
                mats = {w: ml.level_matrix(l, w).to_scipy_local() for w in ("APR" if l + 1 < ml.num_levels else "A")}
                split = ml.level_split(l) if l + 1 < ml.num_levels else None
                lev.append((mats, split))
            out.append(lev)
            del ml
        return out

    from tests.util import same_csr

    res = run_ranks(nranks, rank)
    for dev, host in res:
        assert len(dev) == len(host) >= 2
        for (md, sd), (mh, sh) in zip(dev, host):
            assert md.keys() == mh.keys()
            for w in md:
                assert same_csr(md[w], mh[w]), w
            assert (sd is None and sh is None) or np.array_equal(sd, sh)
