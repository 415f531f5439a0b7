"""Product host setup (libraptor_amd.so, amg_host_hierarchy_*; the code amg_solver_setup runs
before upload) against the oracle: bit-identical level operators (integer pattern AND fp64
values), splittings and coarse inverse.  CPU only, no GPU needed."""
import numpy as np
import pytest

from tests.util import same_csr

CASES = [
    ("5pt", (48, 40), "rs"),
    ("5pt", (33, 31), "pmis"),
    ("5pt", (40, 40), "sa"),
    ("7pt", (18, 17, 16), "rs"),
    ("7pt", (20, 20, 20), "pmis"),
    ("7pt", (16, 18, 20), "sa"),
    ("27pt", (12, 12, 12), "pmis"),
    ("27pt", (13, 12, 11), "sa"),
]


def gen(O, kind, dims):
    return {"5pt": O.gen_5pt, "7pt": O.gen_7pt, "27pt": O.gen_27pt}[kind](*dims)


@pytest.mark.parametrize("kind,dims,coarsen", CASES)
def test_host_hierarchy_bit_exact(oracle, kind, dims, coarsen):
    from raptor_amd import host

    O = oracle
    A = gen(O, kind, dims)
    rp, col, val = A.arrays()
    n = A.shape[0]
    Hp = host.HostHierarchy(n, 0, rp, col, val, host.options(coarsen=coarsen, max_coarse=64))
    Ho = O.Hierarchy(A, **dict(O.DEFAULTS[coarsen], max_coarse=64))
    assert Hp.num_levels == Ho.num_levels >= 3
    for l in range(Ho.num_levels):
        assert same_csr(Hp.to_scipy(l, "A"), Ho.matrix(l, "A")), l
        if l + 1 < Ho.num_levels:
            assert same_csr(Hp.to_scipy(l, "P"), Ho.matrix(l, "P")), l
            assert same_csr(Hp.to_scipy(l, "R"), Ho.matrix(l, "R")), l
            assert np.array_equal(Hp.split(l), Ho.split(l)), l
    Ac = O.Csr.from_scipy(Ho.matrix(Ho.num_levels - 1, "A"))
    assert np.array_equal(Hp.coarse_inverse(), O.dense_inverse(Ac))


@pytest.mark.parametrize("kind,dims,p_max", [("7pt", (18, 17, 16), 4), ("27pt", (12, 11, 13), 4),
                                             ("5pt", (40, 36), 0)])
def test_host_hierarchy_ext_i_bit_exact(oracle, kind, dims, p_max):
    """Extended+i interpolation (r6 option) on the PMIS split: the product's host
    setup equals the oracle's level for level, P_max truncation included."""
    from raptor_amd import host

    O = oracle
    A = gen(O, kind, dims)
    rp, col, val = A.arrays()
    Hp = host.HostHierarchy(A.shape[0], 0, rp, col, val,
                            host.options(coarsen="pmis", max_coarse=64, interp="ext+i", p_max=p_max))
    Ho = O.Hierarchy(A, **dict(O.DEFAULTS["pmis"], max_coarse=64, interp=O.INTERP_EXT_I, p_max=p_max))
    assert Hp.num_levels == Ho.num_levels >= 3
    for l in range(Ho.num_levels):
        assert same_csr(Hp.to_scipy(l, "A"), Ho.matrix(l, "A")), l
        if l + 1 < Ho.num_levels:
            assert same_csr(Hp.to_scipy(l, "P"), Ho.matrix(l, "P")), l
            assert np.array_equal(Hp.split(l), Ho.split(l)), l
    if p_max:
        for l in range(Ho.num_levels - 1):
            assert np.diff(Ho.matrix(l, "P").indptr).max() <= p_max


@pytest.mark.parametrize("kind,dims,coarsen,tol", [("27pt", (13, 12, 11), "sa", 0.02), ("7pt", (20, 20, 20), "pmis", 0.05),
                                                  ("graph", (60, 50), "sa", 0.01), ("7pt", (18, 17, 16), "pmis+ext+i", 0.02)])
def test_host_hierarchy_drop_tol_bit_exact(oracle, kind, dims, coarsen, tol):
    """Coarse-operator drop tolerance (r6 option): the product's host setup equals
    the oracle's level for level; every coarse operator keeps its Galerkin row sums (up to
    rounding) and loses entries."""
    from raptor_amd import host

    O = oracle
    if kind == "graph":
        G = O.gen_graph_laplacian(*dims, 1)
        A = O.permute(G, O.rcm(G))
    else:
        A = gen(O, kind, dims)
    rp, col, val = A.arrays()
    ext = coarsen.endswith("+ext+i")  # with extended+i interpolation (P_max 4)
    coarsen = coarsen.split("+")[0]
    Hp = host.HostHierarchy(A.shape[0], 0, rp, col, val,
                            host.options(coarsen=coarsen, max_coarse=64, drop_tol=tol,
                                         interp="ext+i" if ext else "classical"))
    ikw = dict(interp=O.INTERP_EXT_I, p_max=4) if ext else {}
    Ho = O.Hierarchy(A, **dict(O.DEFAULTS[coarsen], max_coarse=64, drop_tol=tol, **ikw))
    Hg = O.Hierarchy(A, **dict(O.DEFAULTS[coarsen], max_coarse=64, **ikw))
    assert Hp.num_levels == Ho.num_levels >= 3
    for l in range(Ho.num_levels):
        assert same_csr(Hp.to_scipy(l, "A"), Ho.matrix(l, "A")), l
        if l + 1 < Ho.num_levels:
            assert same_csr(Hp.to_scipy(l, "P"), Ho.matrix(l, "P")), l
            assert np.array_equal(Hp.split(l), Ho.split(l)), l
    assert np.array_equal(Hp.coarse_inverse(), O.dense_inverse(O.Csr.from_scipy(Ho.matrix(Ho.num_levels - 1, "A"))))
    # level 1 from the same P: the Galerkin product less the dropped entries, row sums kept
    A1, G1 = Ho.matrix(1, "A"), Hg.matrix(1, "A")
    assert A1.nnz < G1.nnz
    assert np.allclose(np.asarray(A1.sum(axis=1)).ravel(), np.asarray(G1.sum(axis=1)).ravel(),
                       rtol=0, atol=1e-12 * abs(G1).max())
    assert np.array_equal(O.sparsify(O.Csr.from_scipy(G1), tol).to_scipy().toarray(), A1.toarray())


def test_drop_tol_edge_cases(oracle):
    """sparsify: a row without a stored diagonal keeps every entry (d_i = 0 drops
    nothing, and no column can be lumped onto it); a huge tolerance leaves a diagonal operator,
    after which coarsening stops -- host setup and oracle agree level for level.  (Setup only:
    the lumped diagonal is the Galerkin row sum, ~0 for a Laplacian's interior rows, so that
    coarse operator is near-singular and no cycle is run on it.)"""
    import scipy.sparse as sp

    from raptor_amd import host

    O = oracle
    M = sp.csr_matrix(np.array([[4.0, -0.001, -1.0, 0.0],
                                [-0.001, 0.0, -0.5, 0.2],   # no stored diagonal
                                [-1.0, -0.5, 3.0, -0.002],
                                [0.0, 0.2, -0.002, 2.0]]))
    M.eliminate_zeros()
    B = O.sparsify(O.Csr.from_scipy(M), 0.01).to_scipy().toarray()
    # row 1 (no diagonal): unchanged; rows 0, 2, 3: the entries below 0.01 sqrt(|a_ii a_jj|)
    # against a stored neighbour diagonal are lumped (a_jj = 0 for j = 1 keeps them)
    assert np.array_equal(B[1], M.toarray()[1])
    assert B[0, 1] == -0.001 and B[2, 1] == -0.5
    assert B[2, 3] == 0.0 and B[2, 2] == 3.0 + -0.002 and B[3, 2] == 0.0 and B[3, 3] == 2.0 + -0.002
    for kind, dims, coarsen in [("7pt", (16, 15, 14), "pmis"), ("27pt", (12, 11, 10), "sa")]:
        A = gen(O, kind, dims)
        rp, col, val = A.arrays()
        Hp = host.HostHierarchy(A.shape[0], 0, rp, col, val,
                                host.options(coarsen=coarsen, max_coarse=16, drop_tol=10.0))
        Ho = O.Hierarchy(A, **dict(O.DEFAULTS[coarsen], max_coarse=16, drop_tol=10.0))
        assert Hp.num_levels == Ho.num_levels == 2, (kind, Ho.num_levels)
        A1 = Ho.matrix(1, "A")
        assert same_csr(Hp.to_scipy(1, "A"), A1)
        assert (sp.csr_matrix(A1) - sp.diags(A1.diagonal())).count_nonzero() == 0  # diagonal only


def test_drop_tol_must_be_finite_and_nonnegative(oracle):
    from raptor_amd import host
    from raptor_amd._lib import AmgError

    A = oracle.gen_5pt(12, 12)
    rp, col, val = A.arrays()
    for bad in (-0.01, float("nan"), float("inf")):
        with pytest.raises(AmgError, match="drop_tol"):
            host.HostHierarchy(A.shape[0], 0, rp, col, val, host.options(coarsen="pmis", drop_tol=bad))


def test_unsorted_input_rows_are_sorted(oracle):
    from raptor_amd import host

    O = oracle
    A = O.gen_5pt(20, 20)
    rp, col, val = A.arrays()
    rng = np.random.default_rng(0)
    col2, val2 = col.copy(), val.copy()
    for i in range(rp.size - 1):
        p = rng.permutation(np.arange(rp[i], rp[i + 1]))
        col2[rp[i]:rp[i + 1]], val2[rp[i]:rp[i + 1]] = col[p], val[p]
    Hp = host.HostHierarchy(A.shape[0], 0, rp, col2, val2, host.options(coarsen="pmis"))
    assert same_csr(Hp.to_scipy(0, "A"), A.to_scipy())


def test_invalid_input_is_an_error(oracle):
    from raptor_amd import AmgError, host

    with pytest.raises(AmgError):
        host.HostHierarchy(3, 0, [0, 1, 2, 3], [0, 1, 3], [1.0, 1.0, 1.0], host.options())
    with pytest.raises(AmgError):  # duplicate column
        host.HostHierarchy(2, 0, [0, 2, 3], [0, 0, 1], [1.0, 1.0, 1.0], host.options())
    with pytest.raises(AmgError):  # RS is serial only -> fine here; bad first_row is not
        host.HostHierarchy(3, 1, [0, 1, 2, 3], [0, 1, 2], [1.0, 1.0, 1.0], host.options())
