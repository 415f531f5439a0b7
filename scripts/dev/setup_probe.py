"""Setup only (hierarchy + device formats) of a bench config, for kernel traces of the setup
phase: setup_probe.py 7pt|sa27 [n]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import raptor_amd as ra  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "7pt"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
ctx = ra.Context(0)
A = ra.par_stencil_grid(ctx, "27pt" if cfg == "sa27" else "7pt", (n, n, n))
t = time.perf_counter()
if cfg == "sa27":
    ml = ra.ParSmoothedAggregationSolver().setup(A)
else:
    ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
ctx.synchronize()
print(cfg, "setup", round(time.perf_counter() - t, 2), "s levels", ml.num_levels, flush=True)
