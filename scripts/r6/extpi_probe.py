"""Extended+i (distance-two) interpolation vs the product's distance-one classical interpolation
on the 7-pt PMIS hierarchy (VERDICT r5 "next" 7): a prototype that decides whether the option
is worth defining in the oracle, the restatement and the device setup.

Extended+i (De Sterck, Falgout, Nolting, Yang 2008): for an F point i with strong C set C_i,
strong F set F_i and interpolatory set Chat_i = C_i u (union of C_k over k in F_i),
  abar_kl = a_kl if sign(a_kl) != sign(a_kk) else 0,
  s_k = sum_{l in Chat_i u {i}} abar_kl           (k in F_i),
  d_i = a_ii + sum_{weak n not in Chat_i} a_in + sum_{k in F_i} a_ik abar_ki / s_k,
  w_ij = -(a_ij + sum_{k in F_i} a_ik abar_kj / s_k) / d_i      (j in Chat_i).
Same strength (classical, theta 0.25), same PMIS split and seeds as the product; Galerkin
products by scipy; the oracle's V-cycle (Jacobi 1+1) on the resulting levels.

usage: python scripts/r6/extpi_probe.py N
"""
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402


def ext_i(A, S, cf):
    A = A.tocsr()
    S = S.tocsr()
    n = A.shape[0]
    cidx = np.cumsum(cf == 1) - 1
    diag = A.diagonal()
    rows, cols, vals = [], [], []
    Aind, Aptr, Adat = A.indices, A.indptr, A.data
    Sind, Sptr = S.indices, S.indptr
    for i in range(n):
        if cf[i] == 1:
            rows.append(i); cols.append(cidx[i]); vals.append(1.0)
            continue
        si = set(Sind[Sptr[i]:Sptr[i + 1]].tolist())
        Ci = {j for j in si if cf[j] == 1}
        Fi = [k for k in si if cf[k] != 1]
        Ch = set(Ci)
        for k in Fi:
            Ch.update(j for j in Sind[Sptr[k]:Sptr[k + 1]] if cf[j] == 1)
        num = {j: 0.0 for j in Ch}
        d = diag[i]
        for t in range(Aptr[i], Aptr[i + 1]):
            j = Aind[t]
            if j == i:
                continue
            if j in Ch:
                num[j] += Adat[t]
            elif j not in si:
                d += Adat[t]
        for t in range(Aptr[i], Aptr[i + 1]):
            k = Aind[t]
            if k == i or k not in si or cf[k] == 1:
                continue
            aik = Adat[t]
            kc = Aind[Aptr[k]:Aptr[k + 1]]
            kv = Adat[Aptr[k]:Aptr[k + 1]]
            sgn = diag[k] > 0
            ab = np.where((kv < 0) if sgn else (kv > 0), kv, 0.0)
            sel = np.array([(c in Ch) or c == i for c in kc])
            sk = ab[sel].sum()
            if sk == 0.0:
                d += aik
                continue
            for c, v in zip(kc, ab):
                if v == 0.0:
                    continue
                if c in Ch:
                    num[c] += aik * v / sk
                elif c == i:
                    d += aik * v / sk
        for j, v in num.items():
            rows.append(i); cols.append(cidx[j]); vals.append(-v / d)
    return sp.csr_matrix((vals, (rows, cols)), shape=(n, int((cf == 1).sum())))


def truncate(P, kmax):
    """hypre-style P_max truncation: keep the kmax largest |w| of each row, rescale to the row sum."""
    P = P.tocsr().copy()
    for i in range(P.shape[0]):
        s0, e0 = P.indptr[i], P.indptr[i + 1]
        if e0 - s0 <= kmax:
            continue
        v = P.data[s0:e0]
        keep = np.zeros(v.size, bool)
        keep[np.argsort(-np.abs(v), kind="stable")[:kmax]] = True
        tot, kept = v.sum(), v[keep].sum()
        v[~keep] = 0.0
        if kept != 0.0:
            v[keep] *= tot / kept
    P.eliminate_zeros()
    return P


def hierarchy(A0, interp, max_coarse=256):
    levels = []
    A = A0
    l = 0
    while A.shape[0] > max_coarse and l < 24:
        S = O.strength_classical(A, 0.25)
        cf = O.pmis_split(S, 0x5EED + l)
        if interp == "classical":
            P = O.interp_classical(A, S, cf).to_scipy()
        else:
            P = ext_i(A.to_scipy(), S.to_scipy(), cf)
            if interp.startswith("ext+i/"):
                P = truncate(P, int(interp.split("/")[1]))
        nc = P.shape[1]
        if nc == 0 or nc >= A.shape[0]:
            break
        R = P.T.tocsr()
        Ac = (R @ (A.to_scipy() @ P)).tocsr()
        levels.append((A, O.Csr.from_scipy(P), O.Csr.from_scipy(R)))
        A = O.Csr.from_scipy(Ac)
        l += 1
    levels.append((A, None, None))
    return levels


if __name__ == "__main__":
    N = int(sys.argv[1])
    A0 = O.gen_7pt(N, N, N)
    n = A0.shape[0]
    b = A0.spmv(O.vec_uniform(n, 42))
    for interp in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("classical", "ext+i", "ext+i/4")):
        t = time.time()
        lv = hierarchy(A0, interp)
        ts = time.time() - t
        nnz = [L[0].nnz for L in lv]
        pnnz = sum(L[1].nnz for L in lv if L[1] is not None) + sum(L[2].nnz for L in lv if L[2] is not None)
        H = O.Hierarchy(A0, levels=lv)
        _, h = H.solve(np.zeros(n), b, max_iter=200, tol=1e-8)
        _, hp = H.pcg(np.zeros(n), b, max_iter=200, tol=1e-8)
        # cycle cost model: stored bytes ~ 3 sweeps of every A_l (2 Jacobi + residual) + P + R
        work = 3 * sum(nnz) + pnnz
        print(f"{interp}: setup {ts:.0f}s levels {[L[0].shape[0] for L in lv]} op. complexity "
              f"{sum(nnz) / nnz[0]:.3f} nnz/row {[round(L[0].nnz / L[0].shape[0], 1) for L in lv]} "
              f"cycles to 1e-8 {h.size - 1} PCG {hp.size - 1} cycle work (nnz units) {work / 1e6:.1f}M "
              f"solve work {(h.size - 1) * work / 1e6:.0f}M PCG work {(hp.size - 1) * work / 1e6:.0f}M", flush=True)
