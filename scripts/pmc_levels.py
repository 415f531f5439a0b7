"""Driver for rocprofv3 --pmc passes: runs each level operator of the 7-pt 256^3 PMIS
hierarchy 3 times (SpMV; Jacobi for A_l) so per-dispatch counters can be read per kernel
and grid size, then the level-0 SpMV on the plain CSR format (csr_plain_kernel<0>, the bench's
roofline kernel).  See profiles/README.md for the counter recipe."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import raptor_amd as ra  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ctx = ra.Context.native(0)  # torch-free, like bench.py
A = ra.par_stencil_grid(ctx, "7pt", (N, N, N))
ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
mats = [("A0", A)] + [(f"A{l}", ml.level_matrix(l, "A")) for l in (1, 2)] + \
       [("P0", ml.level_matrix(0, "P")), ("R0", ml.level_matrix(0, "R"))]
for name, M in mats:
    x = ra.vector_uniform(ctx, M.local_cols, 0, 1)
    b = ra.vector_uniform(ctx, M.local_rows, 0, 2)
    y = ctx.empty(M.local_rows)
    for _ in range(3):
        M.mult(x, y)
    if name.startswith("A"):
        for _ in range(3):
            M.jacobi(x, b, y)
    ctx.synchronize()
    print(name, "rows", M.local_rows, "nnz", M.nnz, "blocks", M.info["n_blocks"], flush=True)
A.set_format("csr")
x = ra.vector_uniform(ctx, A.local_cols, 0, 1)
y = ctx.empty(A.local_rows)
for _ in range(3):
    A.mult(x, y)
ctx.synchronize()
print("A0 plain CSR", A.info["csr_bytes"], flush=True)
