"""Probe (not product): how fast would the 7-pt level-1 / level-2 block kernels run if the coarse
points were numbered in 3D bricks instead of fine-grid (lexicographic) order?  DESIGN.md 4.1 r5.

Builds the 7-pt N^3 PMIS hierarchy, takes A_1 (and A_2 through the level-1 split) to the host,
renumbers the coarse points by brick of the fine grid (coordinates from the C/F split), rebuilds
the operator as a device matrix and times residual / Jacobi with HIP events against the natural
numbering.  Timing only: the permuted rows sum in sorted-column order, not the hierarchy's."""
import json
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
import raptor_amd as ra  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    ctx = ra.Context.native(0)
    A = ra.par_stencil_grid(ctx, "7pt", (N, N, N))
    ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
    e0, e1 = ra.Event(ctx), ra.Event(ctx)

    def t_us(fn, reps=30):
        fn()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        ctx.synchronize()
        return e0.elapsed_ms(e1) / reps * 1e3

    # coordinates of level-1 points (fine-grid coordinates of the C points of level 0)
    s0 = ml.level_split(0)
    c1 = np.nonzero(s0 == 1)[0]
    coords = {1: (c1 % N, (c1 // N) % N, c1 // (N * N))}
    s1 = ml.level_split(1)
    c2 = c1[np.nonzero(s1 == 1)[0]]
    coords[2] = (c2 % N, (c2 // N) % N, c2 // (N * N))
    out = {"grid": N, "levels": []}
    for l in (1, 2):
        M = ml.level_matrix(l, "A").to_scipy_local().tocsr()
        n = M.shape[0]
        i, j, k = coords[l]
        assert len(i) == n
        rows = []
        for name, spec in [("natural", None), ("brick8", (8, 8, 8)), ("brick16", (16, 16, 16)),
                           ("brick16x16x8", (16, 16, 8))]:
            if spec is None:
                Mp = M
            else:
                bx, by, bz = spec
                nbx, nby = (N + bx - 1) // bx, (N + by - 1) // by
                key = (((k // bz) * nby + (j // by)) * nbx + (i // bx)) * (bx * by * bz) + \
                      ((k % bz) * by + (j % by)) * bx + (i % bx)
                p = np.argsort(key, kind="stable")
                Mp = M[p][:, p].tocsr()
                Mp.sort_indices()
            D = ra.ParCSRMatrix.from_scipy_local(ctx, Mp, n, 0)
            x, b, t = ra.vector_uniform(ctx, n, 0, 5), ra.vector_uniform(ctx, n, 0, 6), ctx.empty(n)
            r = {"order": name, "resid_us": round(t_us(lambda: D.residual(x, b, t)), 1),
                 "jacobi_us": round(t_us(lambda: D.jacobi(x, b, t)), 1), "info": {k2: D.info[k2] for k2 in
                 ("n_blocks", "tile_line_bytes", "spmv_fmt_bytes") if k2 in D.info}}
            rows.append(r)
            print(l, r, file=sys.stderr, flush=True)
            del D
        out["levels"].append({"level": l, "n": n, "nnz": int(M.nnz), "orders": rows})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
