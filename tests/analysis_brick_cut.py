"""Block-cut simulation: x-tile bytes per operator of the 7-pt PMIS hierarchy
with the coarse levels in the hierarchy's order vs a private 8x8x8-brick order (rows and
columns permuted, as a cycle-order copy would be).  Usage: python tests/analysis_brick_cut.py 64
(analysis, not a test: it lives under tests/ because it runs the oracle)"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle as O
N = int(sys.argv[1])
t = time.time()
Ao = O.gen_7pt(N, N, N)
H = O.Hierarchy(Ao, **O.DEFAULTS["pmis"])
print("setup", time.time() - t, "levels", H.num_levels, flush=True)

def cut(M, order, colmap, LW, cap_l, cap_e=2048, cap_r=256):
    M = M.tocsr() if hasattr(M, "tocsr") else M
    ip, ix = M.indptr, colmap[M.indices]
    nb = lt = 0; cur = set(); ce = cr = 0
    for r in order:
        ls = set((ix[ip[r]:ip[r+1]] // LW).tolist()); ne = ip[r+1] - ip[r]
        u = cur | ls
        if ce and (ce + ne > cap_e or len(u) > cap_l or cr + 1 > cap_r):
            nb += 1; lt += len(cur); cur = set(ls); ce = ne; cr = 1
        else:
            cur = u; ce += ne; cr += 1
    return nb + 1, lt + len(cur)


# coordinates of each level's points (fine-grid coordinates of the C points)
pts = {0: np.arange(N ** 3)}
for l in range(1, H.num_levels):
    s = np.asarray(H.split(l - 1))
    pts[l] = pts[l - 1][np.nonzero(s == 1)[0]]
def brick_perm(p, b=8):
    i, j, k = p % N, (p // N) % N, p // (N * N)
    nb = (N + b - 1) // b
    key = (((k // b) * nb + (j // b)) * nb + (i // b)) * b ** 3 + ((k % b) * b + (j % b)) * b + (i % b)
    return np.argsort(key, kind="stable")  # new position -> old index
L = min(3, H.num_levels - 1)
perm = {0: np.arange(N ** 3)}
for l in range(1, L + 1):
    perm[l] = brick_perm(pts[l])
inv = {l: np.argsort(perm[l]) for l in perm}  # old index -> new position
ident = {l: np.arange(len(perm[l])) for l in perm}
for l in range(0, L):
    for w, rl, cl in (("A", l, l), ("R", l + 1, l), ("P", l, l + 1)):
        if l == 0 and w == "A":
            continue
        M = H.matrix(l, w)
        for LW, capl in ((8, 256), (4, 512)):
            nb0, lt0 = cut(M, ident[rl], ident[cl], LW, capl)
            nb1, lt1 = cut(M, perm[rl], inv[cl], LW, capl)
            print(f"L{l} {w} {M.shape} nnz {M.nnz} LW{LW}: natural blocks {nb0} tile MB {lt0*LW*8/1e6:.2f} | brick blocks {nb1} tile MB {lt1*LW*8/1e6:.2f}", flush=True)
