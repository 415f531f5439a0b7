"""Driver for counter / trace passes over the level-0 template kernels: 27-pt and 7-pt 256^3
operators, 3 launches each of mult, residual, Jacobi (7-pt) and a forward hybrid GS sweep
(27-pt).  RAPTOR_AMD_LIB selects an alternative build for same-box A/B."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import raptor_amd as ra  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ctx = ra.Context(0)
for st in ("27pt", "7pt"):
    A = ra.par_stencil_grid(ctx, st, (N, N, N))
    x = ra.vector_uniform(ctx, A.local_cols, 0, 1)
    b = ra.vector_uniform(ctx, A.local_rows, 0, 2)
    y = ctx.empty(A.local_rows)
    for _ in range(3):
        A.mult(x, y)
    for _ in range(3):
        A.residual(x, b, y)
    for _ in range(3):
        A.residual_norm(x, b)
    if st == "7pt":
        for _ in range(3):
            A.jacobi(x, b, y)
    else:
        for _ in range(3):
            A.hybrid_gs(x, b, y)
    ctx.synchronize()
    print(st, "rows", A.local_rows, "nnz", A.nnz, "variant", A.info["kernel_variant"], flush=True)
    del A
