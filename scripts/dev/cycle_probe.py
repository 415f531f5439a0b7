"""V-cycles only (7-pt 256^3 PMIS hierarchy, b = A x*), for kernel traces of the solve:
cycle_probe.py [n] [cycles]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import raptor_amd as ra  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ctx = ra.Context(0)
A = ra.par_stencil_grid(ctx, "7pt", (n, n, n))
ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
b = ra.vector_uniform(ctx, A.local_rows, 0, 42)
for k in (3, K):
    x = ctx.zeros(A.local_rows)
    ml.solve(x, b, max_iter=k, tol=0.0)
ctx.synchronize()
print("done", flush=True)
