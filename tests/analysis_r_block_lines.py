"""Block-cut simulation for SA restrictions: x-tile lines per block for the
product's row order vs rows sorted by their first / median column, on the oracle's sa27
hierarchy.  Usage: python tests/analysis_r_block_lines.py 64 (analysis, not a test:
it lives under tests/ because it runs the oracle)"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import oracle as O
N = int(sys.argv[1])
t = time.time()
Ao = O.gen_27pt(N, N, N)
H = O.Hierarchy(Ao, **O.DEFAULTS["sa"])
print("setup", time.time() - t, "levels", H.num_levels, flush=True)

def cut(R, order, LW=4, cap_e=2048, cap_l=512):
    ip, ix = R.indptr, R.indices
    nb = 0; lines_tot = 0; ent = 0
    cur = set(); ce = 0
    for r in order:
        ls = set((ix[ip[r]:ip[r+1]] // LW).tolist())
        ne = ip[r+1] - ip[r]
        u = cur | ls
        if ce and (ce + ne > cap_e or len(u) > cap_l):
            nb += 1; lines_tot += len(cur); cur = set(ls); ce = ne
        else:
            cur = u; ce += ne
    nb += 1; lines_tot += len(cur)
    return nb, lines_tot

for lvl in (0, 1):
    R = H.matrix(lvl, "R")
    n = R.shape[0]
    print(f"level {lvl} R: {R.shape} nnz {R.nnz} per row {R.nnz/n:.1f}")
    ident = np.arange(n)
    mins = np.array([R.indices[R.indptr[r]:R.indptr[r+1]].min() if R.indptr[r+1] > R.indptr[r] else 0 for r in range(n)])
    meds = np.array([np.median(R.indices[R.indptr[r]:R.indptr[r+1]]) if R.indptr[r+1] > R.indptr[r] else 0 for r in range(n)])
    for name, order in (("identity", ident), ("by min col", np.argsort(mins, kind="stable")), ("by median col", np.argsort(meds, kind="stable"))):
        for LW in (4, 8):
            nb, lt = cut(R, order, LW=LW, cap_l=512 if LW == 4 else 256)
            print(f"  {name:14s} LW{LW}: blocks {nb} lines {lt} bytes {lt*LW*8/1e6:.1f} MB entries/line {R.nnz/lt:.2f}", flush=True)
