"""Driver for counter passes over the plain-CSR roofline kernel (csr_plain_kernel<SPMV>):
7-pt 256^3, AMG_FORMAT_CSR, 5 launches of mult, plus 5 of the read-ceiling kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import raptor_amd as ra  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ctx = ra.Context(0)
A = ra.par_stencil_grid(ctx, "7pt", (N, N, N)).set_format("csr")
x = ra.vector_uniform(ctx, A.local_cols, 0, 1)
y = ctx.empty(A.local_rows)
for _ in range(5):
    A.mult(x, y)
ctx.synchronize()
print("rows", A.local_rows, "nnz", A.nnz, "variant", A.info["kernel_variant"], flush=True)
