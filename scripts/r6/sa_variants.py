"""SA setup variants for configs[2] (27-pt Q1 anisotropic, eps = (1, 1, 1e-3)): convergence study.

VERDICT r5 "next" 2: the SA hierarchy (|a_ij| strength, Gershgorin rho, P smoothed with A) stalls
(asymptotic factor >= 0.98).  This prototype builds hierarchies from scipy with the oracle's own
MIS(2) aggregation and V-cycle (hybrid GS 1+1) and measures, per variant, the factor over many
cycles, PCG iterations to 1e-8 and the operator complexity.  Prototype only (scipy Galerkin
products, not the oracle's bit-exact order): it picks the definition; the oracle, the golden
restatement and the product then implement the chosen one together.

usage: python scripts/r6/sa_variants.py N [cycles]
"""
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402


def strength(A, theta, signed):
    A = A.tocsr()
    d = A.diagonal()
    coo = A.tocoo()
    off = coo.row != coo.col
    r, c, v = coo.row[off], coo.col[off], coo.data[off]
    thr = theta * np.sqrt(np.abs(d[r] * d[c]))
    keep = (-v >= thr) if signed else (np.abs(v) >= thr)
    return sp.csr_matrix((v[keep], (r[keep], c[keep])), shape=A.shape)


def filtered(A, S):
    """A_F: strong off-diagonals kept, the rest of each row lumped onto the diagonal."""
    A = A.tocsr()
    n = A.shape[0]
    d = A.diagonal()
    off_sum = np.asarray(A.sum(axis=1)).ravel() - d
    Sd = S.copy()
    Sd.data = np.ones_like(Sd.data)
    AF_off = A.multiply(Sd).tocsr()
    AF_off.eliminate_zeros()
    kept = np.asarray(AF_off.sum(axis=1)).ravel()
    dF = d + (off_sum - kept)
    return (AF_off + sp.diags(dF)).tocsr()


def rho_power(A, iters=15):
    Dinv = sp.diags(1.0 / A.diagonal())
    M = Dinv @ A
    x = np.ones(A.shape[0]) + np.arange(A.shape[0]) % 7 * 0.1
    lam = 0.0
    for _ in range(iters):
        y = M @ x
        lam = np.linalg.norm(y) / np.linalg.norm(x)
        x = y / np.linalg.norm(y)
    return lam


def rho_inf(A, d=None, iters=10, seed=7):
    """Power iteration on D^-1 A normalised in the max norm (order-independent: bit-exact on
    any partition); start x0 = vec_uniform(seed)."""
    dinv = 1.0 / (A.diagonal() if d is None else d)
    x = O.vec_uniform(A.shape[0], seed)
    x = x / np.max(np.abs(x))
    lam = 0.0
    for _ in range(iters):
        y = dinv * (A @ x)
        lam = np.max(np.abs(y))
        x = y / lam
    return lam


def rho_gersh(A):
    return np.max(np.asarray(abs(A).sum(axis=1)).ravel() / np.abs(A.diagonal()))


def build(A0, v, max_coarse=256, theta0=0.08, seed=0x5EED, verbose=False):
    levels = []
    A = A0.tocsr()
    l = 0
    while A.shape[0] > max_coarse and l < 24:
        theta = theta0 * v.get("q", 0.5 if v.get("halve", True) else 1.0) ** l
        S = strength(A, theta, v["signed"])
        agg, na = O.mis2_aggregate(O.Csr.from_scipy(S), seed + l)
        n = A.shape[0]
        if na == 0 or na >= n or (n <= 8192 and 5 * na > 4 * n):
            break
        sizes = np.bincount(agg, minlength=na)
        T = sp.csr_matrix((1.0 / np.sqrt(sizes[agg]), (np.arange(n), agg)), shape=(n, na))
        As = filtered(A, S) if v["filter"] else A
        dsc = A.diagonal() if v.get("dA", False) else As.diagonal()
        if verbose and v["filter"]:
            r = As.diagonal() / A.diagonal()
            print(f"    d_F/a_ii min={r.min():.3g} p1={np.percentile(r, 1):.3g} neg={np.sum(r <= 0)}")
        rho = {"power": rho_power, "gersh": rho_gersh, "inf": rho_inf}[v["rho"]](As, dsc) if v["rho"] == "inf" else {"power": rho_power, "gersh": rho_gersh}[v["rho"]](As)
        om = 4.0 / 3.0 / rho
        P = (T - sp.diags(om / dsc) @ (As @ T)).tocsr()
        if v.get("drop", 0) > 0:
            P = drop_small(P, v["drop"])
        R = P.T.tocsr()
        Ac = (R @ (A @ P)).tocsr()
        if verbose:
            print(f"  L{l}: n={n} nnz={A.nnz} na={na} rho={rho:.3f} P nnz/row={P.nnz/n:.1f}")
        levels.append((A, P, R))
        A = Ac
        l += 1
    levels.append((A, None, None))
    return levels


def drop_small(P, tol):
    P = P.tocsr().copy()
    for i in range(P.shape[0]):
        s, e = P.indptr[i], P.indptr[i + 1]
        row = P.data[s:e]
        if row.size:
            m = np.max(np.abs(row))
            row[np.abs(row) < tol * m] = 0.0
    P.eliminate_zeros()
    return P


def evaluate(A0, v, cycles, name):
    t0 = time.time()
    levels = build(A0, v, verbose=True)
    ts = time.time() - t0
    cx = sum(L[0].nnz for L in levels) / levels[0][0].nnz
    lv = [tuple(O.Csr.from_scipy(M) if M is not None else None for M in L) for L in levels]
    H = O.Hierarchy(lv[0][0], coarsen=O.COARSEN_SA, smoother=O.SMOOTH_HYBRID_GS, levels=lv)
    n = A0.shape[0]
    b = lv[0][0].spmv(O.vec_uniform(n, 42))
    x, hist = H.solve(np.zeros(n), b, max_iter=cycles)
    rel = hist / hist[0]
    k = min(cycles, 50)
    asym = (rel[-1] / rel[-1 - k]) ** (1.0 / k)
    reach = np.nonzero(rel <= 1e-8)[0]
    _, hp = H.pcg(np.zeros(n), b, max_iter=300, tol=1e-8)
    print(f"{name}: levels={len(levels)} cx={cx:.2f} setup={ts:.1f}s factor(last {k})={asym:.4f} "
          f"cycles_to_1e-8={reach[0] if reach.size else None} final={rel[-1]:.2e} pcg_iters={hp.size - 1}",
          flush=True)


if __name__ == "__main__":
    N = int(sys.argv[1])
    cycles = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    which = sys.argv[3].split("|") if len(sys.argv) > 3 else None
    A0 = O.gen_27pt(N, N, N).to_scipy().tocsr()
    variants = {
        "current(abs,gersh,A)": dict(signed=False, rho="gersh", filter=False),
        "signed,gersh,A": dict(signed=True, rho="gersh", filter=False),
        "signed,power,A": dict(signed=True, rho="power", filter=False),
        "signed,gersh,AF": dict(signed=True, rho="gersh", filter=True),
        "signed,power,AF": dict(signed=True, rho="power", filter=True),
        "abs,power,AF": dict(signed=False, rho="power", filter=True),
    }
    for name, v in variants.items():
        if which and name not in which:
            continue
        evaluate(A0, v, cycles, name)
