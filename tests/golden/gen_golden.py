"""Generate tests/golden/*.npz: independent fixtures that pin the oracle.

The reference (Siddarthareddy1/raptor) holds no AMG code or vectors, so the
oracle is pinned here by implementations that share no code with it:
  * scipy.sparse 1.15.3 -- model-problem matrices built from Kronecker products, SpMV,
    residual, Jacobi, transposes and Galerkin products R (A P);
  * numpy uint64 arithmetic -- the splitmix64 vector generator and hashes;
  * small pure-Python loop restatements -- RS first pass, PMIS, MIS(2) aggregation, hybrid GS
    (small sizes only), written from DESIGN.md section 3, not from the C code;
  * (r5) the floating-point setup and the cycle, restated the same way:
    classical (modified) interpolation weights, SA's tentative prolongator T, rho and smoothed
    P = T - (4/3 rho) (D^-1 A_F T) (r6: signed strength, filtered A_F, max-norm power rho),
    the Gauss-Jordan coarse inverse (numpy row operations), the
    64-way interleaved butterfly coarse solve, and whole hierarchies + V-cycles built from
    these restatements, scipy's Galerkin products and the loop smoothers only
    (setup_<case>.npz).
Run: python tests/golden/gen_golden.py   (writes the .npz files next to this script)
"""
from __future__ import annotations

import heapq
import math
import os

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
M64 = (1 << 64) - 1


# --------------------------------------------------------------------------------------
# model problems by Kronecker products (independent of the C generators)
# --------------------------------------------------------------------------------------
def lap1d(n):
    return sp.diags([-np.ones(n - 1), 2 * np.ones(n), -np.ones(n - 1)], [-1, 0, 1], format="csr")


def eye(n):
    return sp.identity(n, format="csr")


def poisson5(nx, ny):
    # row id = i + nx*j: x fastest => kron(Iy, Tx) + kron(Ty, Ix)
    return (sp.kron(eye(ny), lap1d(nx)) + sp.kron(lap1d(ny), eye(nx))).tocsr()


def poisson7(nx, ny, nz):
    return (sp.kron(eye(nz), sp.kron(eye(ny), lap1d(nx)))
            + sp.kron(eye(nz), sp.kron(lap1d(ny), eye(nx)))
            + sp.kron(lap1d(nz), sp.kron(eye(ny), eye(nx)))).tocsr()


def fe27(nx, ny, nz, ex=1.0, ey=1.0, ez=1e-3):
    """36 x Q1 stiffness of -div(diag(ex,ey,ez) grad u): K1 = tridiag(-1,2,-1),
    m1 = tridiag(1,4,1); A = ex Kx.my.mz + ey mx.Ky.mz + ez mx.my.Kz (x fastest)."""
    def m1(n):
        return sp.diags([np.ones(n - 1), 4 * np.ones(n), np.ones(n - 1)], [-1, 0, 1], format="csr")

    t1 = ex * sp.kron(m1(nz), sp.kron(m1(ny), lap1d(nx)))
    t2 = ey * sp.kron(m1(nz), sp.kron(lap1d(ny), m1(nx)))
    t3 = ez * sp.kron(lap1d(nz), sp.kron(m1(ny), m1(nx)))
    return ((t1 + t2) + t3).tocsr()


def mixed_graph(n, deg, seed):
    """Unstructured SPD test matrix (r6): a symmetric random graph (deg random partners per
    node, numpy Generator(PCG64(seed))), couplings -U(0.5, 1.5) with one in eight positive
    +U(0.05, 0.6), diagonal sum |a_ij| + 0.01 -- positive couplings and weak entries
    exercise SA's signed strength and the filtered operator."""
    rng = np.random.Generator(np.random.PCG64(seed))
    i = np.repeat(np.arange(n), deg)
    j = rng.integers(0, n, size=n * deg)
    keep = i != j
    i, j = i[keep], j[keep]
    w = -rng.uniform(0.5, 1.5, size=i.size)
    pos = rng.integers(0, 8, size=i.size) == 0
    w[pos] = rng.uniform(0.05, 0.6, size=int(pos.sum()))
    W = sp.coo_matrix((w, (i, j)), shape=(n, n)).tocsr()
    W = ((W + W.T) * 0.5).tocsr()
    W.sum_duplicates()
    d = np.asarray(abs(W).sum(axis=1)).ravel() + 0.01
    return (W + sp.diags(d)).tocsr()


# --------------------------------------------------------------------------------------
# splitmix64 in numpy uint64
# --------------------------------------------------------------------------------------
def mix64(z):
    z = np.asarray(z, np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniform(n, seed, first=0):
    with np.errstate(over="ignore"):
        base = np.uint64((seed * 0xD1B54A32D192ED03) & M64)
        u = mix64(base + np.arange(first, first + n, dtype=np.uint64))
    return (u >> np.uint64(11)).astype(np.float64) * 2.0 ** -52 - 1.0


def hash32(ids, seed):
    with np.errstate(over="ignore"):
        s = np.uint64((seed * 0x9E3779B97F4A7C15) & M64)
        return (mix64(np.asarray(ids, np.uint64) ^ s) >> np.uint64(32)).astype(np.uint64)


# --------------------------------------------------------------------------------------
# pure-Python restatements
# --------------------------------------------------------------------------------------
def rows(M):
    M = M.tocsr()
    M.sort_indices()
    return [(M.indices[M.indptr[i]:M.indptr[i + 1]].tolist(),
             M.data[M.indptr[i]:M.indptr[i + 1]].tolist()) for i in range(M.shape[0])]


def strength_classical(A, theta):
    R = rows(A)
    out = []
    for i, (cols, vals) in enumerate(R):
        off = [-v for c, v in zip(cols, vals) if c != i]
        keep = []
        if off and max(off) > 0.0:
            thr = theta * max(off)
            keep = [c for c, v in zip(cols, vals) if c != i and -v >= thr]
        out.append(keep)
    return out


def sa_strong(v, di, dc, theta):
    """SA strength, signed (r6): -a_ij >= theta sqrt(|a_ii a_jj|); positive couplings never."""
    return -v >= theta * np.sqrt(abs(di * dc))


def strength_symmetric(A, theta):
    R = rows(A)
    d = A.diagonal()
    return [[(c, v) for c, v in zip(cols, vals)
             if c != i and sa_strong(v, d[i], d[c], theta)] for i, (cols, vals) in enumerate(R)]


def transpose_lists(S, n):
    T = [[] for _ in range(n)]
    for i, cols in enumerate(S):
        for c in cols:
            T[c].append(i)
    return T


def rs_split(S):
    n = len(S)
    ST = transpose_lists(S, n)
    U, F, Cc = -1, 0, 1
    cf = [F if (not S[i] and not ST[i]) else U for i in range(n)]
    lam = [len(ST[i]) for i in range(n)]
    heap = [(-lam[i], i) for i in range(n) if cf[i] == U]
    heapq.heapify(heap)
    while heap:
        nl, i = heapq.heappop(heap)
        if cf[i] != U or -nl != lam[i]:
            continue
        cf[i] = Cc
        for j in ST[i]:
            if cf[j] == U:
                cf[j] = F
                for k in S[j]:
                    if cf[k] == U:
                        lam[k] += 1
                        heapq.heappush(heap, (-lam[k], k))
        for j in S[i]:
            if cf[j] == U:
                lam[j] -= 1
                heapq.heappush(heap, (-lam[j], j))
    return np.array(cf, np.int32)


def pmis_split(S, seed):
    n = len(S)
    ST = transpose_lists(S, n)
    h = hash32(np.arange(n), seed)
    key = [(len(ST[i]) << 32) | int(h[i]) for i in range(n)]
    U, F, Cc = -1, 0, 1
    cf = [F if not ST[i] else U for i in range(n)]
    while any(c == U for c in cf):
        newc = []
        for i in range(n):
            if cf[i] != U:
                continue
            if all(not (cf[j] == U and (key[j], j) > (key[i], i)) for j in S[i] + ST[i]):
                newc.append(i)
        for i in newc:
            cf[i] = Cc
        for i in range(n):
            if cf[i] == U and any(cf[j] == Cc for j in S[i]):
                cf[i] = F
    return np.array(cf, np.int32)


def mis2_aggregate(Sv, seed):
    n = len(Sv)
    S = [[c for c, _ in r] for r in Sv]
    h = [int(v) for v in hash32(np.arange(n), seed)]
    OUT, UND, IN = 0, 1, 2
    st = [UND] * n
    while UND in st:
        t = [(st[i], h[i], i) for i in range(n)]
        for _ in range(2):
            t = [max([t[i]] + [t[j] for j in S[i]]) for i in range(n)]
        for i in range(n):
            if st[i] == UND:
                if t[i][2] == i:
                    st[i] = IN
                elif t[i][0] == IN:
                    st[i] = OUT
    roots = [i for i in range(n) if st[i] == IN]
    agg = [-1] * n
    for a, r in enumerate(roots):
        agg[r] = a
    a1 = list(agg)
    for i in range(n):
        if a1[i] < 0:
            for j in S[i]:
                if st[j] == IN:
                    a1[i] = agg[j]
                    break
    out = list(a1)
    for i in range(n):
        if a1[i] < 0:
            best, ba = -1.0, -1
            for j, v in Sv[i]:
                if a1[j] < 0:
                    continue
                w = abs(v)
                if w > best or (w == best and a1[j] < ba):
                    best, ba = w, a1[j]
            out[i] = ba
    return np.array(out, np.int32), len(roots)


def _l1_gs_block(R, d, x, b, out, s, e, backward):
    """l1 hybrid GS on block [s, e): acc = b_i - sum of old-value couplings
    (incl. the diagonal, CSR order) - sum of new-value in-block couplings (sweep order);
    x_i' = x_i + acc / (a_ii + sum_{j outside [s, e)} |a_ij|)."""
    order = range(e - 1, s - 1, -1) if backward else range(s, e)
    for i in order:
        cols, vals = R[i]
        lo, hi = (i + 1, e) if backward else (s, i)
        l1 = 0.0
        for c, v in zip(cols, vals):
            if c < s or c >= e:
                l1 += abs(v)
        acc = b[i]
        for c, v in zip(cols, vals):
            if lo <= c < hi:
                continue
            acc -= v * x[c]
        new = [(c, v) for c, v in zip(cols, vals) if lo <= c < hi]
        for c, v in (reversed(new) if backward else new):
            acc -= v * out[c]
        out[i] = x[i] + acc * (1.0 / (d[i] + l1))


def hybrid_gs(A, x, b, block):
    R = rows(A)
    n = len(R)
    out = np.zeros(n)
    d = A.diagonal()
    for s in range(0, n, block):
        _l1_gs_block(R, d, x, b, out, s, min(n, s + block), False)
    return out


def hybrid_gs_backward(A, x, b, block):
    """Backward sweep: rows of each block in descending order, new values for in-block j > i."""
    R = rows(A)
    n = len(R)
    out = np.zeros(n)
    d = A.diagonal()
    for s in range(0, n, block):
        _l1_gs_block(R, d, x, b, out, s, min(n, s + block), True)
    return out


# --------------------------------------------------------------------------------------
# floating-point setup and the V-cycle, restated from DESIGN.md section 3 (r5)
# --------------------------------------------------------------------------------------
def interp_classical(A, S, cf):
    """Classical (modified) interpolation, distance 1.  C row: 1 at its coarse index.  F row
    i: C_i = strong C neighbours; d = a_ii + the weak a_ij (row order); num_j = a_ij for
    j in C_i; then for each strong F neighbour k (row order): s_k = sum of a_km over m in C_i
    with sign(a_km) = -sign(a_kk) (row k order); s_k = 0 adds a_ik to d, else num_m +=
    (a_ik a_km) / s_k over those m.  w_ij = -num_j / d (columns ascending)."""
    R = rows(A)
    n = len(R)
    cidx = np.cumsum(cf == 1) - 1
    diag = {i: dict(zip(*R[i])).get(i, 0.0) for i in range(n)}
    indptr, indices, data = [0], [], []
    for i in range(n):
        if cf[i] == 1:
            indices.append(int(cidx[i]))
            data.append(1.0)
            indptr.append(len(indices))
            continue
        Si = set(S[i])
        cols, vals = R[i]
        d = diag[i]
        num = {}
        for c, v in zip(cols, vals):
            if c == i:
                continue
            if c in Si and cf[c] == 1:
                num[c] = v
            elif c not in Si:
                d = d + v
        if num:
            for k, aik in zip(cols, vals):
                if k == i or k not in Si or cf[k] == 1:
                    continue
                kc, kv = R[k]
                pos = diag[k] > 0.0
                sel = [(m, v) for m, v in zip(kc, kv) if m in num and ((v < 0.0) if pos else (v > 0.0))]
                sk = 0.0
                for _, v in sel:
                    sk = sk + v
                if sk == 0.0:
                    d = d + aik
                else:
                    for m, v in sel:
                        num[m] = num[m] + (aik * v) / sk
        for c in sorted(num):
            indices.append(int(cidx[c]))
            data.append(-num[c] / d)
        indptr.append(len(indices))
    return sp.csr_matrix((np.array(data), np.array(indices, np.int64), np.array(indptr, np.int64)),
                         shape=(n, int((cf == 1).sum())))


def interp_ext_i(A, S, cf, p_max):
    """Extended+i (distance two, r6 option).  F row i: Chat_i = strong C
    neighbours, then the strong C neighbours of each strong F neighbour; num_j from 0.0;
    d = a_ii; row i in order: a_ij to num_j (j in Chat_i) or to d (weak j); each strong F
    neighbour k (row i order): abar = a_kl of sign opposite to a_kk, s_k = sum of abar over
    Chat_i u {i} (row k order) -- 0 adds a_ik to d, else num_l += (a_ik abar_kl) / s_k (l in
    Chat_i), d += (a_ik abar_ki) / s_k; w = -num / d by ascending column; more than p_max
    entries: keep the p_max largest |w| (ties: smaller column), scale them by
    (sum of all w) / (sum of kept w), sums in column order."""
    R = rows(A)
    n = len(R)
    cidx = np.cumsum(cf == 1) - 1
    diag = {i: dict(zip(*R[i])).get(i, 0.0) for i in range(n)}
    indptr, indices, data = [0], [], []
    for i in range(n):
        if cf[i] == 1:
            indices.append(int(cidx[i]))
            data.append(1.0)
            indptr.append(len(indices))
            continue
        Si = S[i]
        sset = set(Si)
        ch = []
        for j in Si:
            if cf[j] == 1 and j not in ch:
                ch.append(j)
        for k in Si:
            if cf[k] != 1:
                for j in S[k]:
                    if cf[j] == 1 and j not in ch:
                        ch.append(j)
        chs = set(ch)
        num = {j: 0.0 for j in ch}
        d = diag[i]
        cols, vals = R[i]
        for c, v in zip(cols, vals):
            if c == i:
                continue
            if c in chs:
                num[c] = num[c] + v
            elif c not in sset:
                d = d + v
        for k, aik in zip(cols, vals):
            if k == i or k not in sset or cf[k] == 1:
                continue
            kc, kv = R[k]
            pos = diag[k] > 0.0
            ab = [(c, v) for c, v in zip(kc, kv) if ((v < 0.0) if pos else (v > 0.0))]
            sk = 0.0
            for c, v in ab:
                if c in chs or c == i:
                    sk = sk + v
            if sk == 0.0:
                d = d + aik
                continue
            for c, v in ab:
                if c in chs:
                    num[c] = num[c] + (aik * v) / sk
                elif c == i:
                    d = d + (aik * v) / sk
        order = sorted(ch)
        w = [-num[j] / d for j in order]
        keep = [True] * len(w)
        if p_max > 0 and len(w) > p_max:
            tot = 0.0
            for v in w:
                tot = tot + v
            ranked = sorted(range(len(w)), key=lambda t: (-abs(w[t]), t))
            keep = [False] * len(w)
            for t in ranked[:p_max]:
                keep[t] = True
            kept = 0.0
            for t, v in enumerate(w):
                if keep[t]:
                    kept = kept + v
            if kept != 0.0:
                f = tot / kept
                w = [v * f if keep[t] else v for t, v in enumerate(w)]
        for t, j in enumerate(order):
            if keep[t]:
                indices.append(int(cidx[j]))
                data.append(w[t])
        indptr.append(len(indices))
    return sp.csr_matrix((np.array(data), np.array(indices, np.int64), np.array(indptr, np.int64)),
                         shape=(n, int((cf == 1).sum())))


def sa_filter(A, theta):
    """Filtered operator (r6): the diagonal and the strong off-diagonals in row order; the
    diagonal value f_i = a_ii + the weak off-diagonal a_ij (row order).  Explicit zeros kept."""
    R = rows(A)
    d = A.diagonal()
    n = len(R)
    indptr, indices, data = [0], [], []
    for i, (cols, vals) in enumerate(R):
        f = d[i]
        for c, v in zip(cols, vals):
            if c != i and not sa_strong(v, d[i], d[c], theta):
                f = f + v
        for c, v in zip(cols, vals):
            if c == i:
                indices.append(c)
                data.append(f)
            elif sa_strong(v, d[i], d[c], theta):
                indices.append(c)
                data.append(v)
        indptr.append(len(indices))
    return sp.csr_matrix((np.array(data, np.float64), np.array(indices, np.int64), np.array(indptr, np.int64)),
                         shape=A.shape)


def sa_rho(F, d, seed, iters=10):
    """rho(D^-1 A_F) by power steps in the max norm: x = u / max|u| (u = uniform(seed));
    y = (A_F x) / a_ii, lam = max|y|, stop at lam = 0, x = y / lam."""
    x = uniform(F.shape[0], seed)
    m = float(np.max(np.abs(x))) if x.size else 0.0
    if m > 0.0:
        x = x / m
    lam = 0.0
    for _ in range(iters):
        y = (F @ x) / d
        lam = float(np.max(np.abs(y))) if y.size else 0.0
        if lam == 0.0:
            break
        x = y / lam
    return lam


def sa_prolongator(A, agg, na, theta, seed):
    """T_{i,agg(i)} = 1 / sqrt(|agg(i)|); A_F = sa_filter(A, theta); rho = sa_rho(A_F, diag A,
    seed); P = T - ((4/3) / rho) (1 / a_ii) (A_F T) on the union pattern (r6)."""
    n = A.shape[0]
    size = np.bincount(agg, minlength=na)
    T = sp.csr_matrix((1.0 / np.sqrt(size[agg].astype(np.float64)), agg.astype(np.int64), np.arange(n + 1)),
                      shape=(n, na))
    d = A.diagonal()
    F = sa_filter(A, theta)
    rho = sa_rho(F, d, seed)
    omega = (4.0 / 3.0) / rho if rho > 0.0 else 0.0
    c = omega * (1.0 / d)
    FT = (F @ T).tocsr()
    return (T - sp.diags(c) @ FT).tocsr()


def gauss_jordan_inverse(M):
    """Dense inverse: for each column c, pivot = first row r >= c of max |M_rc|, swap, scale
    the pivot row by 1 / M_cc, subtract f = M_rc times it from every other row with f != 0."""
    M = np.array(M, np.float64, copy=True)
    n = M.shape[0]
    inv = np.eye(n)
    for c in range(n):
        p = c + int(np.argmax(np.abs(M[c:, c])))
        if p != c:
            M[[c, p]] = M[[p, c]]
            inv[[c, p]] = inv[[p, c]]
        ip = 1.0 / M[c, c]
        M[c] = M[c] * ip
        inv[c] = inv[c] * ip
        f = M[:, c].copy()
        f[c] = 0.0
        rs = np.nonzero(f)[0]
        M[rs] = M[rs] - f[rs, None] * M[c][None, :]
        inv[rs] = inv[rs] - f[rs, None] * inv[c][None, :]
    return inv


def coarse_solve(inv, b):
    """x_i = sum_j inv_ij b_j as 64 partial sums p_l over j = l mod 64 (ascending j, from 0.0)
    combined by the butterfly p_l <- p_l + p_{l xor m}, m = 32 ... 1; x_i = p_0."""
    n = b.size
    x = np.empty(n)
    lanes = np.arange(64)
    for i in range(n):
        p = np.zeros(64)
        for j in range(n):
            p[j % 64] = p[j % 64] + inv[i, j] * b[j]
        m = 32
        while m >= 1:
            p = p + p[lanes ^ m]
            m >>= 1
        x[i] = p[0]
    return x


def norm2(v):
    s = 0.0
    for t in v.tolist():
        s = s + t * t
    return float(np.sqrt(s))


def sparsify(A, tau):
    """Coarse-operator drop tolerance (r6 option): off-diagonal a_ij with |a_ij| <
    tau sqrt(|a_ii a_jj|) move onto the diagonal, summed in row order from a_ii; rows without a
    stored diagonal stay as they are.  Loops over the CSR arrays, written from the definition
    in DESIGN.md 3 (not from the C)."""
    A = sp.csr_matrix(A)
    n = A.shape[0]
    d = np.zeros(n)
    has = np.zeros(n, bool)
    for i in range(n):
        for k in range(A.indptr[i], A.indptr[i + 1]):
            if A.indices[k] == i:
                d[i], has[i] = A.data[k], True
                break
    rp, ci, va = [0], [], []
    for i in range(n):
        cols = A.indices[A.indptr[i]:A.indptr[i + 1]]
        vals = A.data[A.indptr[i]:A.indptr[i + 1]]
        if not has[i]:
            ci.extend(cols)
            va.extend(vals)
            rp.append(len(ci))
            continue
        drop = [j != i and abs(v) < tau * math.sqrt(abs(d[i] * d[j])) for j, v in zip(cols, vals)]
        f = d[i]
        for v, dr in zip(vals, drop):
            if dr:
                f += v
        for j, v, dr in zip(cols, vals, drop):
            if j == i:
                ci.append(j)
                va.append(f)
            elif not dr:
                ci.append(j)
                va.append(v)
        rp.append(len(ci))
    return sp.csr_matrix((np.array(va, float), np.array(ci, np.int64), np.array(rp, np.int64)), shape=A.shape)


def canon(M):
    M = sp.csr_matrix(M)
    M.eliminate_zeros()
    M.sort_indices()
    return M


class PyHierarchy:
    """The setup and V-cycle of DESIGN.md 3 from the restatements above: strength (theta; SA:
    signed, theta_l = theta (3/4)^l rounded per level), RS / PMIS (seed + l) + classical interpolation or MIS(2) (seed + l)
    + smoothed P; R = P^T; A_c = R (A P) (scipy); stop at n <= max_coarse, n_c = 0, n_c >= n
    or (n <= 8192 and 5 n_c > 4 n); Gauss-Jordan inverse on the coarsest level.  Cycle: one
    pre-smooth (Jacobi 2/3 or forward l1 hybrid GS(64)), r = b - A x, b_c = R r, x_c = 0,
    recurse, x += P x_c, one post-smooth (Jacobi or backward GS)."""

    def __init__(self, A, coarsen, smoother, theta, max_coarse=256, seed=0x5EED, max_levels=25,
                 interp="classical", p_max=4, drop_tol=0.0):
        self.smoother = smoother
        self.A, self.P, self.R, self.split = [canon(A)], [], [], []
        th = theta
        while len(self.A) < max_levels and self.A[-1].shape[0] > max_coarse:
            l = len(self.A) - 1
            Al = self.A[-1]
            n = Al.shape[0]
            if coarsen == "sa":
                Sv = strength_symmetric(Al, th)
                agg, na = mis2_aggregate(Sv, seed + l)
                P = sa_prolongator(Al, agg, na, th, seed + l)
                split = agg
            else:
                S = strength_classical(Al, theta)
                cf = rs_split(S) if coarsen == "rs" else pmis_split(S, seed + l)
                P = interp_ext_i(Al, S, cf, p_max) if interp == "ext+i" else interp_classical(Al, S, cf)
                split = cf
            nc = P.shape[1]
            if nc == 0 or nc >= n or (n <= 8192 and 5 * nc > 4 * n):
                break
            P = canon(P)
            R = canon(P.T.tocsr())
            self.P.append(P)
            self.R.append(R)
            self.split.append(np.asarray(split, np.int32))
            Ac = canon(R @ (Al @ P))
            self.A.append(canon(sparsify(Ac, drop_tol)) if drop_tol > 0 else Ac)
            th = th * 0.75  # SA: theta_{l+1} = theta_l * 3/4 (r6)
        self.inv = gauss_jordan_inverse(self.A[-1].toarray())

    def smooth(self, l, x, b, post):
        A = self.A[l]
        if self.smoother == "hybrid_gs":
            return (hybrid_gs_backward if post else hybrid_gs)(A, x, b, 64)
        return x + (2.0 / 3.0) * ((1.0 / A.diagonal()) * (b - A @ x))

    def cycle(self, x, b, l=0):
        if l == len(self.A) - 1:
            return coarse_solve(self.inv, b)
        x = self.smooth(l, x, b, False)
        r = b - self.A[l] @ x
        xc = self.cycle(np.zeros(self.A[l + 1].shape[0]), self.R[l] @ r, l + 1)
        x = x + self.P[l] @ xc
        return self.smooth(l, x, b, True)

    def solve(self, b, iters):
        x = np.zeros(b.size)
        hist = [norm2(b - self.A[0] @ x)]
        for _ in range(iters):
            x = self.cycle(x, b)
            hist.append(norm2(b - self.A[0] @ x))
        return x, np.array(hist)


# (name, generator, coarsen, smoother, theta, max_coarse)
SETUP_CASES = [
    ("p5_32x32_rs_jacobi", lambda: poisson5(32, 32), "rs", "jacobi", 0.25, 256),
    ("p5_32x32_rs_jacobi_mc16", lambda: poisson5(32, 32), "rs", "jacobi", 0.25, 16),
    ("p7_10x9x8_pmis_jacobi_mc16", lambda: poisson7(10, 9, 8), "pmis", "jacobi", 0.25, 16),
    ("fe27_8x7x6_sa_gs_mc16", lambda: fe27(8, 7, 6), "sa", "hybrid_gs", 0.08, 16),
    ("p7_10x9x8_sa_gs_mc16", lambda: poisson7(10, 9, 8), "sa", "hybrid_gs", 0.08, 16),
    ("mixed_600_sa_gs_mc16", lambda: mixed_graph(600, 2, 11), "sa", "hybrid_gs", 0.08, 16),
    # r6: extended+i interpolation (P_max 4) on the PMIS split; the mixed-sign graph exercises
    # the sign rule and empty s_k
    ("p7_10x9x8_pmis_exti4_jacobi_mc16", lambda: poisson7(10, 9, 8), "pmis+ext+i", "jacobi", 0.25, 16),
    ("mixed_600_pmis_exti4_jacobi_mc16", lambda: mixed_graph(600, 2, 11), "pmis+ext+i", "jacobi", 0.25, 16),
    # r6: coarse-operator drop tolerance 0.01 (non-Galerkin lumping) on SA
    ("mixed_600_sa_gs_drop01_mc16", lambda: mixed_graph(600, 2, 11), "sa", "hybrid_gs", 0.08, 16, 0.01),
    ("fe27_8x7x6_sa_gs_drop01_mc16", lambda: fe27(8, 7, 6), "sa", "hybrid_gs", 0.08, 16, 0.01),
]


def gen_setup_case(name, gen, coarsen, smoother, theta, max_coarse, drop_tol=0.0):
    A = gen()
    interp = "ext+i" if coarsen.endswith("+ext+i") else "classical"
    H = PyHierarchy(A, coarsen.split("+")[0], smoother, theta, max_coarse, interp=interp, drop_tol=drop_tol)
    n = A.shape[0]
    b = A @ uniform(n, 42)
    out = {"nlev": np.array(len(H.A), np.int64), "inv": H.inv, "b": b}
    out.update(csr_arrays("Ain", canon(A)))  # the input (the unstructured case has no C generator)
    if coarsen == "sa":  # level 0's filtered operator and rho, for the oracle's pieces
        F = sa_filter(canon(A), theta)
        out.update(csr_arrays("F0", F))
        out["rho0"] = np.array(sa_rho(F, canon(A).diagonal(), seed=0x5EED))
    for l in range(len(H.A)):
        out.update(csr_arrays(f"A{l}", H.A[l]))
        if l + 1 < len(H.A):
            out.update(csr_arrays(f"P{l}", H.P[l]))
            out[f"split{l}"] = H.split[l]
    x = np.zeros(n)
    for k in range(3):
        x = H.cycle(x, b)
        out[f"x{k}"] = x
    xs, hist = H.solve(b, 8)
    out["xsolve"] = xs
    out["hist"] = hist
    save(f"setup_{name}.npz", **out)
    print(name, "levels", [M.shape[0] for M in H.A], "hist", hist[0], "->", hist[-1])


def save(name, **arrays):
    np.savez_compressed(os.path.join(HERE, name), **arrays)


def csr_arrays(prefix, M):
    M = M.tocsr()
    M.sort_indices()
    return {f"{prefix}_indptr": M.indptr.astype(np.int64), f"{prefix}_indices": M.indices.astype(np.int64),
            f"{prefix}_data": M.data, f"{prefix}_shape": np.array(M.shape, np.int64)}


def main():
    problems = {
        "p5_16x12": poisson5(16, 12),
        "p5_32x32": poisson5(32, 32),
        "p7_10x9x8": poisson7(10, 9, 8),
        "fe27_8x7x6": fe27(8, 7, 6),
    }
    for name, A in problems.items():
        n = A.shape[0]
        x = uniform(n, 3)
        b = uniform(n, 4)
        d = A.diagonal()
        out = dict(csr_arrays("A", A))
        out["x"] = x
        out["b"] = b
        out["y"] = A @ x
        out["r"] = b - A @ x
        out["jac"] = x + (2.0 / 3.0) * ((1.0 / d) * (b - A @ x))
        out["gs64"] = hybrid_gs(A, x, b, 64)
        out["gs7"] = hybrid_gs(A, x, b, 7)
        out["gsb64"] = hybrid_gs_backward(A, x, b, 64)
        out["gsb7"] = hybrid_gs_backward(A, x, b, 7)
        S = strength_classical(A, 0.25)
        out["S_classical_nnz"] = np.array([len(s) for s in S], np.int64)
        out["cf_rs"] = rs_split(S)
        out["cf_pmis"] = pmis_split(S, 0x5EED)
        Ss = strength_symmetric(A, 0.08)
        agg, na = mis2_aggregate(Ss, 0x5EED)
        out["agg_mis2"] = agg
        out["n_agg"] = np.array(na, np.int64)
        out["hash32_seed5eed"] = hash32(np.arange(n), 0x5EED).astype(np.int64)
        save(f"{name}.npz", **out)
        print(name, n, A.nnz, "C(rs)", int(out["cf_rs"].sum()), "C(pmis)", int(out["cf_pmis"].sum()),
              "aggs", na)
    for case in SETUP_CASES:
        gen_setup_case(*case)
    # vector generator at an offset (partition independence of the generator)
    save("uniform.npz", u0=uniform(1000, 42), u_off=uniform(1000, 42, first=123456789),
         u_seed7=uniform(17, 7))


if __name__ == "__main__":
    main()
