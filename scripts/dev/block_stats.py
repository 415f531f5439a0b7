import sys, os
sys.path.insert(0, os.getcwd())
import torch
import raptor_amd as ra
torch.cuda.set_device(0)
ctx = ra.Context(0)
cfg = sys.argv[1]
if cfg == "7pt":
    A = ra.par_stencil_grid(ctx, "7pt", (256, 256, 256)); ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
elif cfg == "sa27":
    A = ra.par_stencil_grid(ctx, "27pt", (256, 256, 256)); ml = ra.ParSmoothedAggregationSolver().setup(A)
else:
    A = ra.par_graph_laplacian(ctx, 1225, 1225, seed=1); A, _ = A.reorder("rcm"); ml = ra.ParSmoothedAggregationSolver().setup(A)
print("done", cfg, flush=True)
