"""Driver for rocprofv3 --pmc passes over the 27-pt 256^3 level-0 hybrid-GS sweep (sa27's
level 0: tpl_gs_acc_kernel + tpl_gs_chain_kernel at B = 64), forward and backward, 3 each.
Algorithmic bytes per row: acc kernel 1 B id + 8 b + 8 x + 8 acc out; chain kernel 8 acc +
8 x + 1 id in, 8 y out."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import raptor_amd as ra  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ctx = ra.Context.native(0)
A = ra.par_stencil_grid(ctx, "27pt", (N, N, N))
n = A.local_rows
x = ra.vector_uniform(ctx, n, 0, 1)
b = ra.vector_uniform(ctx, n, 0, 2)
y = ctx.empty(n)
for back in (False, True):
    for _ in range(3):
        A.hybrid_gs(x, b, y, 64, backward=back)
ctx.synchronize()
print("27pt", n, "rows; hybrid GS B=64 fwd/bwd x3", flush=True)
