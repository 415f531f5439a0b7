"""GPU parity: the HIP level kernels and the V-cycle through the C-ABI against the CPU oracle.

Bar: bit-identical for every kernel and every V-cycle iterate (both sides
round each product and sum as written, same order); residual norms (different reduction
order) within 1e-12 relative; solve histories within 1e-10 relative (BASELINE.json:5).
Parity against Siddarthareddy1/raptor itself is unpinned (no AMG code in the reference)."""
import numpy as np
import pytest
import scipy.sparse as sp

from tests.util import oracle_levels, same_csr, to_dev, to_host

pytestmark = pytest.mark.gpu


def _solve_vs_oracle(ctx, O, ml, b_dev, iters):
    """Solve iterates bit-identical to the oracle's cycle on the product's own operators
    (exported), and the residual history within 1e-10 relative."""
    n = b_dev.numel()
    H = O.Hierarchy(None, levels=oracle_levels(O, ml))
    b = to_host(ctx, b_dev)
    x = ctx.zeros(n)
    _, h = ml.solve(x, b_dev, max_iter=iters)
    xo, ho = H.solve(np.zeros(n), b, max_iter=iters)
    assert np.array_equal(to_host(ctx, x), xo)
    assert h.shape == ho.shape and np.all(np.abs(h - ho) <= 1e-10 * ho)
    return to_host(ctx, x), h


def _problems(O):
    rng = np.random.default_rng(7)
    # ragged random matrix: empty rows, variable row length, a dense-ish row > LDS stage
    n = 3000
    M = sp.random(n, n, density=0.002, random_state=11, format="lil")
    M[5, :] = 0
    M[17, :] = 0
    M[100, :] = rng.standard_normal(n)  # 3000 nnz in one row: long-row path (kCAP = 2048)
    M = (M + sp.eye(n) * 10.0).tocsr()
    M.sort_indices()
    return {
        "7pt_20": O.gen_7pt(20, 20, 20),
        "5pt_37x29": O.gen_5pt(37, 29),
        "27pt_13": O.gen_27pt(13, 13, 13),
        "ragged": O.Csr.from_scipy(M),
    }


@pytest.fixture(scope="module")
def problems(oracle):
    return _problems(oracle)


def _dev_matrix(ra, ctx, Ao):
    rp, col, val = Ao.arrays()
    return ra.ParCSRMatrix.from_csr(ctx, Ao.shape[0], 0, rp, col, val)


@pytest.mark.parametrize("name", ["7pt_20", "5pt_37x29", "27pt_13", "ragged"])
def test_level_kernels_bit_exact(ctx, oracle, problems, name):
    import raptor_amd as ra

    O = oracle
    Ao = problems[name]
    A = _dev_matrix(ra, ctx, Ao)
    n = Ao.shape[0]
    x = O.vec_uniform(n, 3)
    b = O.vec_uniform(n, 4)
    y0 = O.vec_uniform(n, 5)
    dx, db = to_dev(ctx, x), to_dev(ctx, b)
    out = ctx.empty(n)
    A.mult(dx, out)
    assert np.array_equal(to_host(ctx, out), Ao.spmv(x))
    dy = to_dev(ctx, y0)
    A.mult_add(dx, dy)
    assert np.array_equal(to_host(ctx, dy), Ao.spmv_add(x, y0))
    A.residual(dx, db, out)
    assert np.array_equal(to_host(ctx, out), Ao.residual(x, b))
    A.jacobi(dx, db, out, 2.0 / 3.0)
    assert np.array_equal(to_host(ctx, out), Ao.jacobi(x, b, 2.0 / 3.0))
    for blk in (64, 17, 1, 33):
        A.hybrid_gs(dx, db, out, blk)
        assert np.array_equal(to_host(ctx, out), Ao.hybrid_gs(x, b, blk)), blk
        A.hybrid_gs(dx, db, out, blk, backward=True)
        assert np.array_equal(to_host(ctx, out), Ao.hybrid_gs_backward(x, b, blk)), blk
    rn = A.residual_norm(dx, db)
    ro = O.norm2(Ao.residual(x, b))
    assert abs(rn - ro) <= 1e-12 * ro


def _all_modes_equal(ctx, O, A, Ao, seed=3):
    n = Ao.shape[0]
    x, b, y0 = O.vec_uniform(n, seed), O.vec_uniform(n, seed + 1), O.vec_uniform(n, seed + 2)
    dx, db = to_dev(ctx, x), to_dev(ctx, b)
    out = ctx.empty(n)
    A.mult(dx, out)
    assert np.array_equal(to_host(ctx, out), Ao.spmv(x))
    dy = to_dev(ctx, y0)
    A.mult_add(dx, dy)
    assert np.array_equal(to_host(ctx, dy), Ao.spmv_add(x, y0))
    A.residual(dx, db, out)
    assert np.array_equal(to_host(ctx, out), Ao.residual(x, b))
    A.jacobi(dx, db, out, 2.0 / 3.0)
    assert np.array_equal(to_host(ctx, out), Ao.jacobi(x, b, 2.0 / 3.0))
    rn = A.residual_norm(dx, db)
    ro = O.norm2(Ao.residual(x, b))
    assert abs(rn - ro) <= 1e-12 * ro


@pytest.mark.parametrize("var", [74, 66], ids=["persist_vi", "persist"])
@pytest.mark.parametrize("name", ["7pt_20", "5pt_37x29", "27pt_13", "ragged"])
def test_persistent_tile_kernel_bit_exact(ctx, oracle, problems, monkeypatch, name, var):
    """Variant bit 64: the persistent x-tile kernel -- resident grid,
    next block's batch 1 prefetched -- gives the oracle's bits in every mode, with and
    without value-indexed blocks, including the long-row and empty-row blocks of "ragged"."""
    import raptor_amd as ra

    monkeypatch.setenv("AMG_KERNEL_VARIANT", str(var))
    Ao = problems[name]
    A = _dev_matrix(ra, ctx, Ao)
    _all_modes_equal(ctx, oracle, A, Ao)


def test_persistent_tile_kernel_vcycle(ctx, oracle, monkeypatch):
    """A PMIS V-cycle on the persistent x-tile kernel (coarse Galerkin operators: VI and
    fp64-value blocks) and on the default kernels: both solves' iterates bit-identical to the
    oracle's (and so to each other), histories within 1e-10."""
    import raptor_amd as ra

    A = ra.par_stencil_grid(ctx, "7pt", (40, 36, 33))
    n = A.local_rows
    b = ra.vector_uniform(ctx, n, 0, 7)
    res = []
    for var in (None, "106"):
        if var is None:
            monkeypatch.delenv("AMG_KERNEL_VARIANT", raising=False)
        else:
            monkeypatch.setenv("AMG_KERNEL_VARIANT", var)
        ml = ra.ParRugeStubenSolver(coarsen="pmis", use_graph=False).setup(A)
        res.append(_solve_vs_oracle(ctx, oracle, ml, b, 4))
    assert np.array_equal(res[0][0], res[1][0])


@pytest.mark.parametrize("name,ntpl", [("7pt_20", 27), ("5pt_37x29", 9), ("27pt_13", 27)])
def test_row_templates_bit_exact(ctx, oracle, problems, monkeypatch, name, ntpl):
    """Stencil operators are stored as row templates: one template per boundary
    class, every row on the template kernel; all four modes bit-identical to the oracle, and
    to the CSR block kernel (AMG_KERNEL_VARIANT without bit 32)."""
    import raptor_amd as ra

    Ao = problems[name]
    A = _dev_matrix(ra, ctx, Ao)
    assert A.info["n_templates"] == ntpl
    assert A.info["template_rows"] == Ao.shape[0]
    # roofline numerator: 1-byte id + x + y per row, the table counted once
    n = Ao.shape[0]
    assert 17 * n < A.info["spmv_bytes"] <= 17 * n + 12 * (1024 + 255)
    _all_modes_equal(ctx, oracle, A, Ao)
    monkeypatch.setenv("AMG_KERNEL_VARIANT", "10")
    _all_modes_equal(ctx, oracle, A, Ao)


@pytest.mark.parametrize("dims", [(40, 40, 40), (37, 41, 29)])
@pytest.mark.parametrize("kind", ["7pt", "27pt"])
def test_row_templates_march_bit_exact(ctx, oracle, monkeypatch, kind, dims):
    """Variant bit 128: z-marching template kernel -- window slots shared with
    the block one shift back are copied inside LDS -- bit-identical in every mode.  Planes of
    1600 rows (not a multiple of the 512-row block): the shift is the largest multiple of 512
    below, so only part of the window is reused, every chain start reloads it all.  The odd
    row count of 37x41x29 turns the march off (16-byte pairs): the window kernel runs."""
    import raptor_amd as ra

    O = oracle
    Ao = O.gen_7pt(*dims) if kind == "7pt" else O.gen_27pt(*dims)
    monkeypatch.setenv("AMG_KERNEL_VARIANT", "170")
    A = _dev_matrix(ra, ctx, Ao)
    assert A.info["template_rows"] == Ao.shape[0]
    _all_modes_equal(ctx, O, A, Ao)


def test_row_templates_march_vcycle(ctx, oracle, monkeypatch):
    """PMIS V-cycle with the z-marching template kernel on level 0 (7-pt 64^3: plane = 8
    blocks, the whole -plane band and half the centre band reused) and with the default
    kernels: iterates bit-identical to the oracle's, histories within 1e-10."""
    import raptor_amd as ra

    A = ra.par_stencil_grid(ctx, "7pt", (64, 64, 64))
    n = A.local_rows
    b = ra.vector_uniform(ctx, n, 0, 9)
    res = []
    for var in (None, "170"):
        if var is None:
            monkeypatch.delenv("AMG_KERNEL_VARIANT", raising=False)
        else:
            monkeypatch.setenv("AMG_KERNEL_VARIANT", var)
        ml = ra.ParRugeStubenSolver(coarsen="pmis", use_graph=False).setup(A)
        res.append(_solve_vs_oracle(ctx, oracle, ml, b, 3))
    assert np.array_equal(res[0][0], res[1][0])


def test_row_templates_partial_cover(ctx, oracle, monkeypatch):
    """Mixed operator: more distinct row shapes than templates (300 perturbed diagonals), a
    row longer than a template holds (100 entries) and an empty row.  With the size floor
    lowered, the template kernel takes the covered rows and the CSR block kernel the rest,
    in one application; results bit-identical, norm partials from both kernels."""
    import raptor_amd as ra

    O = oracle
    monkeypatch.setenv("AMG_TPL_MIN_ROWS", "0")
    M = O.gen_7pt(24, 23, 22).to_scipy().tolil()
    n = M.shape[0]
    rng = np.random.default_rng(5)
    for k, r in enumerate(rng.choice(n, 300, replace=False)):
        M[r, r] = 6.0 + (k + 1) * 1e-3
    M[77, :100] = rng.standard_normal(100)
    M[4000, :] = 0
    M = M.tocsr()
    M.sort_indices()
    Ao = O.Csr.from_scipy(M)
    A = _dev_matrix(ra, ctx, Ao)
    assert 27 < A.info["n_templates"] <= 255  # capped by kTplEntries (1024 entries)
    assert n // 2 <= A.info["template_rows"] < n
    _all_modes_equal(ctx, O, A, Ao, seed=21)


@pytest.mark.parametrize("name", ["7pt_20", "27pt_13", "ragged"])
def test_spgemm_bit_exact(ctx, oracle, problems, name):
    """Device Galerkin SpGEMM == oracle SpGEMM bit for bit (all LDS table bins; the ragged
    matrix's dense row exceeds the largest bin and takes the host path)."""
    import raptor_amd as ra

    O = oracle
    Ao = problems[name]
    A = _dev_matrix(ra, ctx, Ao)
    C = A.matmat(A)
    Co = (Ao @ Ao).to_scipy()
    assert same_csr(C.to_scipy_local(), Co)


def test_spgemm_large_rows(ctx, oracle):
    """Rows whose upper bound exceeds the largest LDS table: a dense row's product (12000
    distinct columns) overflows it and takes the host path; rows with a large bound but few
    distinct columns (long rows of a narrow band) stay on the GPU's largest table.  Both
    bit-identical to the oracle's canonical order."""
    import raptor_amd as ra

    O = oracle
    n = 12000
    M = sp.random(n, n, density=0.0008, random_state=3, format="lil")
    M.setdiag(4.0)
    M[3, :] = np.linspace(-1.0, 1.0, n)                 # dense row: > 8192 distinct outputs
    band = sp.diags([np.full(n - abs(d), 1.0 + 0.01 * d) for d in range(-60, 61)],
                    list(range(-60, 61)), format="lil")
    M[100:300, :] = band[100:300, :]                    # 121 x 121 entries: bound > 8192, ~250 distinct
    M = M.tocsr()
    M.sort_indices()
    Ao = O.Csr.from_scipy(M)
    A = _dev_matrix(ra, ctx, Ao)
    C = A.matmat(A)
    assert same_csr(C.to_scipy_local(), (Ao @ Ao).to_scipy())


@pytest.mark.parametrize("interp", ["default", "wave", "thread"])
@pytest.mark.parametrize("kind,dims,coarsen", [("7pt", (22, 21, 20), "pmis"), ("27pt", (30, 28, 26), "sa"),
                                               ("5pt", (70, 61), "pmis"), ("7pt", (19, 18, 17), "sa")])
def test_device_setup_equals_host(ctx, oracle, monkeypatch, kind, dims, coarsen, interp):
    """setup_device = 1 (strength, PMIS / MIS(2), P and R = P^T on the GPU, SURVEY 8f row
    f1), 2 (Galerkin SpGEMM only) and 0 (host): identical hierarchies -- every level's A,
    P, R and integer split bit for bit -- and R A P via matmat reproduces A_1.  Classical
    interpolation with a wave per row on every level (wave), a thread per row everywhere
    (thread), or the default rule (a wave per row from 12 entries per row on average)."""
    import raptor_amd as ra

    if interp != "default" and coarsen != "pmis":
        pytest.skip("classical interpolation only")
    if interp != "default":
        monkeypatch.setenv("AMG_INTERP_WAVE_NPR", "0" if interp == "wave" else "1000000")

    A = ra.par_stencil_grid(ctx, kind, dims)
    ms = [ra.ParMultilevel(coarsen=coarsen, setup_device=m).setup(A) for m in (1, 2, 0)]
    nl = ms[0].num_levels
    assert all(m.num_levels == nl for m in ms) and nl >= 2
    for l in range(nl):
        for w in ("APR" if l + 1 < nl else "A"):
            ref = ms[2].level_matrix(l, w).to_scipy_local()
            for m in ms[:2]:
                assert same_csr(m.level_matrix(l, w).to_scipy_local(), ref), (l, w)
        if l + 1 < nl:
            for m in ms[:2]:
                assert np.array_equal(m.level_split(l), ms[2].level_split(l)), l
    R, P = ms[0].level_matrix(0, "R"), ms[0].level_matrix(0, "P")
    Ac = R.matmat(A.matmat(P))
    assert same_csr(Ac.to_scipy_local(), ms[0].level_matrix(1, "A").to_scipy_local())


def test_empty_and_tiny(ctx, oracle):
    import raptor_amd as ra

    O = oracle
    # 1x1 and a matrix whose rows are all empty except the diagonal
    for n in (1, 2, 65):
        M = sp.eye(n, format="csr") * 3.0
        Ao = O.Csr.from_scipy(M)
        A = _dev_matrix(ra, ctx, Ao)
        x = O.vec_uniform(n, 9)
        out = ctx.empty(n)
        A.mult(to_dev(ctx, x), out)
        assert np.array_equal(to_host(ctx, out), Ao.spmv(x))


def test_bad_arguments_fail_loudly(ctx):
    import raptor_amd as ra

    with pytest.raises(ra.AmgError):
        ra.ParCSRMatrix.from_csr(ctx, 3, 0, [0, 1, 2, 3], [0, 1, 5], [1.0, 1.0, 1.0])
    with pytest.raises(ra.AmgError):
        ra.ParCSRMatrix.from_csr(ctx, 3, 0, [0, 2, 2, 3], [1, 1, 2], [1.0, 1.0, 1.0])
    A = ra.par_stencil_grid(ctx, "5pt", (4, 4))
    x = ctx.zeros(16)
    with pytest.raises(ra.AmgError):
        A.hybrid_gs(x, x, x, 64)  # in-place GS refused
    with pytest.raises(ra.AmgError):
        A.hybrid_gs(x, x, ctx.zeros(16), 1000)  # block > 256


def test_setup_failure_with_overlapped_gs_builds_is_an_error(ctx):
    """a setup that throws while the format workers still hold jobs that
    push GS builds (hybrid GS, overlapped setup) comes back as AmgError -- the workers drain
    before the GS worker is freed -- and the context stays usable."""
    import raptor_amd as ra

    # 44^3 PMIS: the first coarse level has ~27 k rows > the dense-solve limit (20000), so
    # max_levels=2 throws after level 0 was handed to the workers
    A = ra.par_stencil_grid(ctx, "7pt", (44, 44, 44))
    for _ in range(2):
        with pytest.raises(ra.AmgError, match="coarsest level too large"):
            ra.ParMultilevel(coarsen="pmis", smoother="hybrid_gs", max_levels=2).setup(A)
    ml = ra.ParMultilevel(coarsen="pmis", smoother="hybrid_gs").setup(A)
    n = A.local_rows
    _, hist = ml.solve(ctx.zeros(n), to_dev(ctx, np.ones(n)), max_iter=3)
    assert hist[-1] < hist[0]


@pytest.mark.parametrize("kind,dims", [("7pt", (40, 36, 33)), ("27pt", (20, 18, 22))])
def test_vcycle_ext_i_bit_exact(ctx, oracle, kind, dims):
    """Extended+i interpolation (r6 option, P_max 4): the product's hierarchy equals the
    oracle's on every level, and the GPU V-cycle (cycle-order copies included) is bit-identical
    to the oracle's; an 8-cycle history within 1e-10."""
    import raptor_amd as ra

    O = oracle
    Ao = {"7pt": O.gen_7pt, "27pt": O.gen_27pt}[kind](*dims)
    A = ra.par_stencil_grid(ctx, kind, dims)
    ml = ra.ParRugeStubenSolver(coarsen="pmis", interp="ext+i", p_max=4).setup(A)
    Ho = O.Hierarchy(Ao, interp=O.INTERP_EXT_I, p_max=4)
    assert ml.num_levels == Ho.num_levels >= 3
    for l in range(ml.num_levels):
        assert same_csr(ml.level_matrix(l, "A").to_scipy_local(), Ho.matrix(l, "A")), l
        if l + 1 < ml.num_levels:
            assert same_csr(ml.level_matrix(l, "P").to_scipy_local(), Ho.matrix(l, "P")), l
    n = Ao.shape[0]
    b = Ao.spmv(O.vec_uniform(n, 42))
    db, dx, xo = to_dev(ctx, b), ctx.zeros(n), np.zeros(n)
    for _ in range(3):
        ml.cycle(dx, db)
        xo = Ho.cycle(xo, b)
        assert np.array_equal(to_host(ctx, dx), xo)
    _, hist = ml.solve(ctx.zeros(n), db, max_iter=8)
    _, hist_o = Ho.solve(np.zeros(n), b, max_iter=8)
    assert np.all(np.abs(hist - hist_o) <= 1e-10 * hist_o)


@pytest.mark.parametrize("kind,dims,coarsen,smoother,tol", [("27pt", (30, 28, 26), "sa", "hybrid_gs", 0.02),
                                                           ("7pt", (40, 36, 33), "pmis", "jacobi", 0.05)])
def test_vcycle_drop_tol_bit_exact(ctx, oracle, kind, dims, coarsen, smoother, tol):
    """Coarse-operator drop tolerance (r6 option): the device setup (Galerkin product on the GPU,
    then the drop) equals the oracle on every level; the V-cycle is bit-identical."""
    import raptor_amd as ra

    O = oracle
    Ao = {"7pt": O.gen_7pt, "27pt": O.gen_27pt}[kind](*dims)
    A = ra.par_stencil_grid(ctx, kind, dims)
    ml = ra.ParMultilevel(coarsen=coarsen, smoother=smoother, drop_tol=tol).setup(A)
    Ho = O.Hierarchy(Ao, **dict(O.DEFAULTS[coarsen], smoother=O.SMOOTH_JACOBI if smoother == "jacobi"
                                else O.SMOOTH_HYBRID_GS, drop_tol=tol))
    assert ml.num_levels == Ho.num_levels >= 3
    for l in range(ml.num_levels):
        assert same_csr(ml.level_matrix(l, "A").to_scipy_local(), Ho.matrix(l, "A")), l
        if l + 1 < ml.num_levels:
            assert same_csr(ml.level_matrix(l, "P").to_scipy_local(), Ho.matrix(l, "P")), l
    n = Ao.shape[0]
    b = Ao.spmv(O.vec_uniform(n, 42))
    db, dx, xo = to_dev(ctx, b), ctx.zeros(n), np.zeros(n)
    for _ in range(3):
        ml.cycle(dx, db)
        xo = Ho.cycle(xo, b)
        assert np.array_equal(to_host(ctx, dx), xo)


@pytest.mark.parametrize("coarsen,smoother", [("pmis", "jacobi"), ("sa", "hybrid_gs")])
def test_cycle_timeline(ctx, oracle, coarsen, smoother):
    """amg_solver_cycle_timeline (the bench's in-graph durations): one labelled, positive time
    per operation of the cycle, replayed from a captured graph, and the reps cycles it ran
    leave x exactly where as many ordinary cycles do."""
    import raptor_amd as ra

    O = oracle
    dims = (28, 26, 24)
    A = ra.par_stencil_grid(ctx, "7pt", dims)
    ml = ra.ParMultilevel(coarsen=coarsen, smoother=smoother).setup(A)
    n = A.local_rows
    b = to_dev(ctx, O.vec_uniform(n, 42))
    x = ctx.zeros(n)
    ops, mode = ml.cycle_timeline(x, b, reps=5)
    assert mode >= 1  # replayed from captured graphs
    labels = [lab for lab, _ in ops]
    L = ml.num_levels
    for l in range(L - 1):
        for op in ("residual", "interp", "post-smooth"):
            assert f"L{l} {op}" in labels, (l, op, labels)
    assert "L0 pre-smooth" in labels and f"L{L - 1} coarse solve" in labels
    assert all(us > 0.0 for lab, us in ops if lab != "event-node gap")
    if mode == 2:  # the calibration entry: what one event-record node adds
        assert labels[-1] == "event-node gap" and 0.0 <= ops[-1][1] < 50.0
    x2 = ctx.zeros(n)
    for _ in range(5):
        ml.cycle(x2, b)
    assert np.array_equal(to_host(ctx, x), to_host(ctx, x2))


CASES = [
    ("7pt", (24, 24, 24), "pmis", "jacobi"),
    ("5pt", (48, 40), "rs", "jacobi"),
    ("27pt", (14, 14, 14), "sa", "hybrid_gs"),
    ("7pt", (20, 18, 22), "sa", "hybrid_gs"),
    ("5pt", (64, 64), "pmis", "hybrid_gs"),
]


@pytest.mark.parametrize("kind,dims,coarsen,smoother", CASES)
def test_vcycle_bit_exact(ctx, oracle, kind, dims, coarsen, smoother):
    """Product hierarchy == oracle hierarchy (bit-exact, integer + fp64) and GPU V-cycle
    iterates == oracle iterates (bit-exact); residual history within 1e-10."""
    import raptor_amd as ra

    O = oracle
    gen = {"7pt": O.gen_7pt, "5pt": O.gen_5pt, "27pt": O.gen_27pt}[kind]
    Ao = gen(*dims)
    A = ra.par_stencil_grid(ctx, kind, dims)
    assert same_csr(A.to_scipy_local(), Ao.to_scipy())  # generators agree bit for bit
    ml = ra.ParMultilevel(coarsen=coarsen, smoother=smoother).setup(A)
    Ho = O.Hierarchy(Ao, coarsen={"rs": O.COARSEN_RS, "pmis": O.COARSEN_PMIS, "sa": O.COARSEN_SA}[coarsen],
                     smoother={"jacobi": O.SMOOTH_JACOBI, "hybrid_gs": O.SMOOTH_HYBRID_GS}[smoother],
                     strong_threshold=0.08 if coarsen == "sa" else 0.25)
    assert ml.num_levels == Ho.num_levels >= 2
    for l in range(ml.num_levels):
        assert same_csr(ml.level_matrix(l, "A").to_scipy_local(), Ho.matrix(l, "A"))
        if l + 1 < ml.num_levels:
            assert same_csr(ml.level_matrix(l, "P").to_scipy_local(), Ho.matrix(l, "P"))
            assert same_csr(ml.level_matrix(l, "R").to_scipy_local(), Ho.matrix(l, "R"))
            assert np.array_equal(ml.level_split(l), Ho.split(l))
            # P and R run the x-tile kernel (variant bit 4 clear: blocks that reuse x lines)
            # or the gather kernel with 16-bit column codes (bit 256): every block's columns
            # fit in <= 4 bands of 16384 at these sizes
            for w in ("P_cycle", "R_cycle"):  # the operators the cycle runs
                v = ml.level_matrix(l, w).info["kernel_variant"]
                assert (v & 256) or not (v & 4), (l, w, v)
    n = Ao.shape[0]
    b = Ao.spmv(O.vec_uniform(n, 42))
    db = to_dev(ctx, b)
    dx = ctx.zeros(n)
    xo = np.zeros(n)
    for _ in range(3):
        ml.cycle(dx, db)
        xo = Ho.cycle(xo, b)
        assert np.array_equal(to_host(ctx, dx), xo)
    dx = ctx.zeros(n)
    _, hist = ml.solve(dx, db, max_iter=8)
    _, hist_o = Ho.solve(np.zeros(n), b, max_iter=8)
    assert hist.shape == hist_o.shape
    assert np.all(np.abs(hist - hist_o) <= 1e-10 * hist_o)
    assert hist[-1] < hist[0]


def test_configs0_5pt_256_rs_jacobi(ctx, oracle):
    """BASELINE.json:7 (configs[0]) at its stated size: 2D 5-pt Poisson 256 x 256 (65,536 rows),
    Ruge-Stueben coarsening + Jacobi.  The product's hierarchy equals the oracle's own serial
    setup (O.Hierarchy(gen_5pt(256, 256), COARSEN_RS)) on every level -- A, P, R bit for bit and
    the C/F split -- and the GPU V-cycle iterates are bit-identical; an 8-cycle solve history
    within 1e-10 relative (BASELINE.json:5)."""
    import raptor_amd as ra

    O = oracle
    Ao = O.gen_5pt(256, 256)
    A = ra.par_stencil_grid(ctx, "5pt", (256, 256))
    assert A.local_rows == 65536
    assert same_csr(A.to_scipy_local(), Ao.to_scipy())
    ml = ra.ParRugeStubenSolver(coarsen="rs").setup(A)
    Ho = O.Hierarchy(Ao, **O.DEFAULTS["rs"])
    assert ml.num_levels == Ho.num_levels >= 3
    for l in range(ml.num_levels):
        assert same_csr(ml.level_matrix(l, "A").to_scipy_local(), Ho.matrix(l, "A")), ("A", l)
        if l + 1 < ml.num_levels:
            assert same_csr(ml.level_matrix(l, "P").to_scipy_local(), Ho.matrix(l, "P")), ("P", l)
            assert same_csr(ml.level_matrix(l, "R").to_scipy_local(), Ho.matrix(l, "R")), ("R", l)
            assert np.array_equal(ml.level_split(l), Ho.split(l)), ("C/F", l)
    n = Ao.shape[0]
    b = Ao.spmv(O.vec_uniform(n, 42))
    db = to_dev(ctx, b)
    dx = ctx.zeros(n)
    xo = np.zeros(n)
    for _ in range(3):
        ml.cycle(dx, db)
        xo = Ho.cycle(xo, b)
        assert np.array_equal(to_host(ctx, dx), xo)
    dx = ctx.zeros(n)
    _, hist = ml.solve(dx, db, max_iter=8)
    xso, hist_o = Ho.solve(np.zeros(n), b, max_iter=8)
    assert np.array_equal(to_host(ctx, dx), xso)
    assert hist.shape == hist_o.shape == (9,)
    assert np.all(np.abs(hist - hist_o) <= 1e-10 * hist_o)
    assert hist[-1] < 1e-3 * hist[0]  # RS + Jacobi on the 2D Poisson problem converges


def test_graph_and_eager_agree(ctx, oracle):
    """hipGraph replay and eager launches: both solves bit-identical to the oracle's iterates
    (and to each other, history included)."""
    import raptor_amd as ra

    A = ra.par_stencil_grid(ctx, "7pt", (30, 30, 30))
    n = A.local_rows
    b = ra.vector_uniform(ctx, n, 0, 1)
    res = []
    for g in (True, False):
        ml = ra.ParRugeStubenSolver(use_graph=g).setup(A)
        res.append(_solve_vs_oracle(ctx, oracle, ml, b, 5))
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1])


def test_solve_tolerance_stops(ctx):
    import raptor_amd as ra

    A = ra.par_stencil_grid(ctx, "5pt", (64, 64))
    ml = ra.ParRugeStubenSolver(coarsen="rs").setup(A)
    n = A.local_rows
    b = ra.vector_uniform(ctx, n, 0, 2)
    x = ctx.zeros(n)
    _, h = ml.solve(x, b, max_iter=100, tol=1e-8)
    assert h[-1] / h[0] < 1e-8 and len(h) < 101
    assert np.all(h[1:-1] / h[0] >= 1e-8)


@pytest.mark.slow
def test_full_size_spmv_and_cycle_256(ctx, oracle, say):
    """BASELINE.json configs[1] size: 7-pt 256^3 (117M nnz).  GPU SpMV bit-exact vs the
    oracle at full size; A*1 equals the exact integer row sums; one full V-cycle iterate
    bit-exact vs the oracle on the same hierarchy."""
    import raptor_amd as ra

    O = oracle
    N = 256
    A = ra.par_stencil_grid(ctx, "7pt", (N, N, N))
    n = A.local_rows
    ones = to_dev(ctx, np.ones(n))
    y = ctx.empty(n)
    A.mult(ones, y)
    yh = to_host(ctx, y)
    g = np.arange(n)
    i, j, k = g % N, (g // N) % N, g // (N * N)
    expect = sum((c == 0).astype(float) + (c == N - 1).astype(float) for c in (i, j, k))
    assert np.array_equal(yh, expect)
    x = O.vec_uniform(n, 77)
    dx = to_dev(ctx, x)
    A.mult(dx, y)
    Ao = O.gen_7pt(N, N, N)
    assert np.array_equal(to_host(ctx, y), Ao.spmv(x))
    del Ao
    say("SpMV bit-exact; setup")
    ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
    say("setup done; exporting the hierarchy to the oracle")
    H = O.Hierarchy(None, levels=oracle_levels(O, ml))
    say("oracle cycle")
    b = to_host(ctx, y)
    dx = ctx.zeros(n)
    ml.cycle(dx, y)
    xo = H.cycle(np.zeros(n), b)
    assert np.array_equal(to_host(ctx, dx), xo)


@pytest.mark.slow
def test_full_size_hierarchy_independent_oracle_256(ctx, oracle, say):
    """configs[1] at full size with an INDEPENDENT oracle hierarchy (the 256^3
    cycle test built the oracle from the product's exported levels).  The oracle's serial
    setup of 7-pt 256^3 (strength, PMIS, classical interpolation, transpose, Galerkin) against
    the product's GPU setup: every P_l, R_l and A_{l+1} bit-identical, then two V-cycle iterates
    and a 4-cycle solve history on the oracle's own hierarchy."""
    import raptor_amd as ra

    O = oracle
    N = 256
    A = ra.par_stencil_grid(ctx, "7pt", (N, N, N))
    ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
    say("GPU setup done; oracle setup (serial)")
    Ao = O.gen_7pt(N, N, N)
    Ho = O.Hierarchy(Ao, **O.DEFAULTS["pmis"])
    assert ml.num_levels == Ho.num_levels
    say("oracle setup done; comparing levels")
    for l in range(ml.num_levels):
        say(f"level {l}")
        if l > 0:
            assert same_csr(ml.level_matrix(l, "A").to_scipy_local(), Ho.matrix(l, "A")), ("A", l)
        if l + 1 < ml.num_levels:
            assert same_csr(ml.level_matrix(l, "P").to_scipy_local(), Ho.matrix(l, "P")), ("P", l)
            assert same_csr(ml.level_matrix(l, "R").to_scipy_local(), Ho.matrix(l, "R")), ("R", l)
    n = N ** 3
    b = Ao.spmv(O.vec_uniform(n, 42))
    db = to_dev(ctx, b)
    dx = ctx.zeros(n)
    xo = np.zeros(n)
    for _ in range(2):
        ml.cycle(dx, db)
        xo = Ho.cycle(xo, b)
        assert np.array_equal(to_host(ctx, dx), xo)
    _, h = ml.solve(ctx.zeros(n), db, max_iter=4)
    _, ho = Ho.solve(np.zeros(n), b, max_iter=4)
    assert np.all(np.abs(h - ho) <= 1e-10 * ho)


@pytest.mark.parametrize("coarsen,smoother", [("pmis", "jacobi"), ("sa", "hybrid_gs")])
def test_pcg_matches_oracle(ctx, oracle, coarsen, smoother):
    """AMG-preconditioned CG: same hierarchy, same V-cycle bits; dot products differ only in
    reduction order, so histories agree to 1e-9 relative over 12 iterations."""
    import raptor_amd as ra

    O = oracle
    A = ra.par_stencil_grid(ctx, "7pt", (26, 25, 24))
    ml = ra.ParMultilevel(coarsen=coarsen, smoother=smoother).setup(A)
    H = O.Hierarchy(None, levels=oracle_levels(O, ml),
                    smoother=O.SMOOTH_JACOBI if smoother == "jacobi" else O.SMOOTH_HYBRID_GS)
    n = A.local_rows
    b = O.vec_uniform(n, 11)
    x, hist = ml.pcg(ctx.zeros(n), to_dev(ctx, b), max_iter=12)
    xo, hist_o = H.pcg(np.zeros(n), b, max_iter=12)
    assert hist.shape == hist_o.shape
    assert np.all(np.abs(hist - hist_o) <= 1e-9 * hist_o[0])
    assert np.max(np.abs(to_host(ctx, x) - xo)) <= 1e-9 * np.max(np.abs(xo))
    _, hv = ml.solve(ctx.zeros(n), to_dev(ctx, b), max_iter=12)
    assert hist[-1] < hv[-1]  # CG accelerates the plain V-cycle iteration
    _, ht = ml.pcg(ctx.zeros(n), to_dev(ctx, b), max_iter=100, tol=1e-10)
    assert ht[-1] / ht[0] < 1e-10 and len(ht) < 101
