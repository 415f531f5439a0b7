"""Unstructured inputs on the CPU: the G3_circuit-substitute generator,
Matrix Market / binary CSR readers, the binary writer and RCM reordering.

Parity: the generator and RCM are checked bit for bit against the oracle's independent C
restatement (oracle/io_oracle.c; both specs in DESIGN.md 8 -- parity unpinned against the
reference, which has no such code).  The Matrix Market reader is pinned by scipy.io.mmwrite
/ scipy.sparse (an independent implementation of the format); RCM quality by
scipy.sparse.csgraph.reverse_cuthill_mckee (its tie-breaking differs, so only the bandwidth
is compared)."""
import os

import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp
from scipy.sparse.csgraph import connected_components, reverse_cuthill_mckee


def _host():
    from raptor_amd import host

    return host


def _bw(M):
    C = M.tocoo()
    return int(np.abs(C.row - C.col).max()) if C.nnz else 0


def _same(A, B):
    A, B = A.tocsr().sorted_indices(), B.tocsr().sorted_indices()
    return (A.shape == B.shape and np.array_equal(A.indptr, B.indptr)
            and np.array_equal(A.indices, B.indices) and np.array_equal(A.data, B.data))


@pytest.mark.parametrize("nx,ny,seed", [(40, 37, 1), (64, 64, 7), (33, 95, 123)])
def test_graph_laplacian_properties(oracle, nx, ny, seed):
    M = oracle.gen_graph_laplacian(nx, ny, seed).to_scipy()
    n = nx * ny
    assert M.shape == (n, n)
    assert (abs(M - M.T)).max() == 0.0  # exactly symmetric
    off = M - sp.diags(M.diagonal())
    assert off.max() <= 0.0 and -off.min() <= 10.0 and -off.data.max() >= 0.1
    # strictly diagonally dominant by the grounding term (>= 1e-6)
    assert np.all(M.diagonal() - np.asarray(abs(off).sum(axis=1)).ravel() >= 1e-6 * 0.999)
    assert 5.0 < M.nnz / n < 6.0  # G3_circuit: 4.8 nnz/row
    # randomly numbered: the natural bandwidth is ~n
    assert _bw(M) > n // 2
    deg = np.diff(M.indptr) - 1
    assert deg.max() <= 7 and len(np.unique(deg)) >= 5  # irregular degrees


def test_graph_laplacian_seeded(oracle):
    A = oracle.gen_graph_laplacian(30, 30, 5).to_scipy()
    B = oracle.gen_graph_laplacian(30, 30, 5).to_scipy()
    C = oracle.gen_graph_laplacian(30, 30, 6).to_scipy()
    assert _same(A, B) and not _same(A, C)


@pytest.mark.parametrize("nranks", [1, 3])
def test_host_generator_matches_oracle(oracle, nranks):
    host = _host()
    nx, ny = 70, 45
    G = oracle.gen_graph_laplacian(nx, ny, 3).to_scipy()
    n = nx * ny
    for r in range(nranks):
        H = host.HostCSR.graph_laplacian(nx, ny, 3, rank=r, nranks=nranks)
        s = H.sizes()
        lo, hi = n * r // nranks, n * (r + 1) // nranks
        assert s["first_row"] == lo and s["n_local_rows"] == hi - lo
        assert _same(H.to_scipy_local(), G[lo:hi])


def _rcm_cases(O):
    rng = np.random.default_rng(3)
    M7 = O.gen_7pt(9, 8, 7).to_scipy()
    p = rng.permutation(M7.shape[0])
    shuffled7 = M7[p][:, p].tocsr()
    # disconnected: two blocks + isolated diagonal-only rows
    blk = sp.block_diag([O.gen_5pt(7, 6).to_scipy(), sp.eye(5) * 2.0, O.gen_5pt(4, 9).to_scipy()]).tocsr()
    # unsymmetric pattern: RCM works on pattern(A + A^T)
    U = sp.random(300, 300, density=0.01, random_state=5, format="csr") + sp.eye(300)
    U = U.tocsr()
    U.sort_indices()
    return {"shuffled7": shuffled7, "disconnected": blk, "unsym": U,
            "graph": O.gen_graph_laplacian(50, 41, 2).to_scipy()}


@pytest.mark.parametrize("name", ["shuffled7", "disconnected", "unsym", "graph"])
def test_rcm_matches_oracle_and_scipy_quality(oracle, name):
    host = _host()
    O = oracle
    M = _rcm_cases(O)[name]
    n = M.shape[0]
    A = O.Csr.from_scipy(M)
    p = O.rcm(A)
    assert np.array_equal(np.sort(p), np.arange(n))
    B = O.permute(A, p).to_scipy()
    assert _same(B, M[p][:, p])
    q = reverse_cuthill_mckee(M.tocsr(), symmetric_mode=False)
    assert _bw(B) <= 1.25 * _bw(M[q][:, q]) + 2
    # product host reorder == oracle, serial and every slice of a 3-way partition
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "m.mtx")
        scipy.io.mmwrite(path, M, symmetry="general")
        H = host.HostCSR.read(path)
        Hb, perm = H.reorder("rcm")
        assert np.array_equal(perm, p)
        assert _same(Hb.to_scipy_local(), B)
    ncomp, _ = connected_components(M, directed=False)
    assert ncomp >= 1


def test_rcm_reduces_graph_bandwidth(oracle):
    M = oracle.gen_graph_laplacian(200, 180, 1).to_scipy()
    p = oracle.rcm(oracle.Csr.from_scipy(M))
    assert _bw(M[p][:, p]) < _bw(M) // 10


@pytest.mark.parametrize("symmetry", ["general", "symmetric"])
@pytest.mark.parametrize("field", ["real", "integer", "pattern"])
def test_matrix_market_read_matches_scipy(tmp_path, symmetry, field):
    host = _host()
    rng = np.random.default_rng(11)
    M = sp.random(157, 157, density=0.03, random_state=7, format="csr")
    if symmetry == "symmetric":
        M = (M + M.T).tocsr()
    if field == "integer":
        M.data = rng.integers(-50, 50, M.nnz).astype(float)
        M.eliminate_zeros()
    if field == "pattern":
        M.data[:] = 1.0
    M = M + sp.eye(157)  # every row nonempty
    M = M.tocsr()
    M.sort_indices()
    path = tmp_path / "a.mtx"
    scipy.io.mmwrite(str(path), M, field=field, symmetry=symmetry, precision=17)
    ref = scipy.io.mmread(str(path)).tocsr()
    ref.sum_duplicates()
    ref.sort_indices()
    for nranks in (1, 2, 5):
        n = 157
        for r in range(nranks):
            H = host.HostCSR.read(path, rank=r, nranks=nranks)
            lo, hi = n * r // nranks, n * (r + 1) // nranks
            assert _same(H.to_scipy_local(), ref[lo:hi]), (nranks, r)


def test_matrix_market_details(tmp_path):
    """Duplicates summed in file order, skew-symmetric mirroring, comments and blank lines,
    rectangular general matrices, upper-triangle symmetric entries."""
    host = _host()
    text = """%%MatrixMarket matrix coordinate real general
% a comment

%another
3 4 6
1 1 1.5
1 1 2.25
3 4 -1e-3
2 2 4
1 1 0.125
2 3 7
"""
    p = tmp_path / "d.mtx"
    p.write_text(text)
    M = host.HostCSR.read(p).to_scipy_local().toarray()
    E = np.zeros((3, 4))
    E[0, 0] = (1.5 + 2.25) + 0.125
    E[2, 3], E[1, 1], E[1, 2] = -1e-3, 4, 7
    assert np.array_equal(M, E)
    p.write_text("%%MatrixMarket matrix coordinate real skew-symmetric\n3 3 2\n2 1 5\n3 1 -2\n")
    S = host.HostCSR.read(p).to_scipy_local().toarray()
    assert np.array_equal(S, np.array([[0, -5, 2], [5, 0, 0], [-2, 0, 0]], float))
    p.write_text("%%MatrixMarket matrix coordinate real symmetric\n2 2 2\n1 2 3\n2 2 1\n")
    S = host.HostCSR.read(p).to_scipy_local().toarray()
    assert np.array_equal(S, np.array([[0, 3], [3, 1]], float))


@pytest.mark.parametrize("text", [
    "%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n",
    "%%MatrixMarket matrix coordinate complex general\n1 1 1\n1 1 1 0\n",
    "%%MatrixMarket matrix coordinate real general\n2 2 2\n1 1 1\n3 1 1\n",
    "%%MatrixMarket matrix coordinate real general\n2 2 3\n1 1 1\n2 2 1\n",
    "%%MatrixMarket matrix coordinate real symmetric\n2 3 1\n1 1 1\n",
    "hello world, not a matrix\n",
])
def test_bad_files_fail_loudly(tmp_path, text):
    import raptor_amd as ra

    host = _host()
    p = tmp_path / "bad.mtx"
    p.write_text(text)
    with pytest.raises(ra.AmgError):
        host.HostCSR.read(p)
    with pytest.raises(ra.AmgError):
        host.HostCSR.read(tmp_path / "missing.mtx")


def test_binary_round_trip(oracle, tmp_path):
    host = _host()
    H = host.HostCSR.graph_laplacian(31, 29, 4)
    path = tmp_path / "g.bin"
    H.write(path)
    assert path.stat().st_size == 32 + 8 * (31 * 29 + 1) + 16 * H.sizes()["nnz_local"]
    G = H.to_scipy_local()
    n = G.shape[0]
    for nranks in (1, 4):
        for r in range(nranks):
            R = host.HostCSR.read(path, rank=r, nranks=nranks)
            lo, hi = n * r // nranks, n * (r + 1) // nranks
            assert _same(R.to_scipy_local(), G[lo:hi])
    raw = bytearray(path.read_bytes())
    raw[0] = ord("X")
    (tmp_path / "bad.bin").write_bytes(bytes(raw))
    import raptor_amd as ra

    with pytest.raises(ra.AmgError):
        host.HostCSR.read(tmp_path / "bad.bin")
