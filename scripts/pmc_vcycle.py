"""Driver for the per-cycle-kernel PMC passes: the exact operations of
bench.py's `vcycle_kernels` table (7-pt 256^3 PMIS hierarchy, levels with >= 1e5 rows: Jacobi,
residual, R r, x += P e), each launched 3 times, with a marker kernel between operations
(uniform_kernel on 1000 + 2 op workgroups before an operation's 3 launches, 1000 + 2 op + 1
after them) so scripts/pmc_vcycle_traffic.py can cut the per-dispatch counter stream into
operations; the warm-up launch of each operation stays outside its segment.  Run under one rocprofv3 --pmc pass per counter
(FETCH_SIZE, WRITE_SIZE); see scripts/gpu_pmc_vcycle.sh."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import raptor_amd as ra  # noqa: E402

# torch-free, like bench.py: the library on the ROCm runtime it was built for
N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
CFG = sys.argv[2] if len(sys.argv) > 2 else "7pt"  # "sa27": configs[2]'s operations (bench.py --config sa27)
ctx = ra.Context.native(0)
if CFG == "sa27":
    A = ra.par_stencil_grid(ctx, "27pt", (N, N, N))
    ml = ra.ParSmoothedAggregationSolver().setup(A)
elif CFG == "g3sub":  # configs[4]'s substitute, as bench.py --config g3sub builds it (N unused)
    A, _ = ra.par_graph_laplacian(ctx, 1225, 1225, seed=1).reorder("rcm")
    ml = ra.ParSmoothedAggregationSolver(drop_tol=0.005).setup(A)
else:
    A = ra.par_stencil_grid(ctx, "7pt", (N, N, N))
    ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
ops = []


def marker(idx):
    ra.vector_uniform(ctx, (1000 + idx) * 256, 0, 1)


for l in range(ml.num_levels - 1):
    if ml.level_info(l)["n_global"] < 100000:
        break
    # the operators as the cycle runs them (cycle-order copies on Jacobi levels)
    Al = A if l == 0 else ml.level_matrix(l, "A_cycle")
    P, R = ml.level_matrix(l, "P_cycle"), ml.level_matrix(l, "R_cycle")
    nl, nc = Al.local_rows, P.local_cols
    xl, bl, tl = ra.vector_uniform(ctx, nl, 0, 5), ra.vector_uniform(ctx, nl, 0, 6), ctx.empty(nl)
    xc, bc = ra.vector_uniform(ctx, nc, 0, 7), ctx.empty(R.local_rows)
    if CFG in ("sa27", "g3sub"):  # hybrid GS(64) sweeps; gs_bytes after the first sweep builds the formats
        Al.hybrid_gs(xl, bl, tl, 64)
        table = [("pre GS (forward)", lambda: Al.hybrid_gs(xl, bl, tl, 64), Al._info()["gs_bytes"]),
                 ("residual", lambda: Al.residual(xl, bl, tl), Al.info["residual_bytes"]),
                 ("restrict R r", lambda: R.mult(tl, bc), R.info["spmv_bytes"]),
                 ("interp x += P e", lambda: P.mult_add(xc, xl), P.info["mult_add_bytes"]),
                 ("post GS (backward)", lambda: Al.hybrid_gs(xl, bl, tl, 64, backward=True), Al._info()["gs_bytes"])]
    else:
        table = [("Jacobi", lambda: Al.jacobi(xl, bl, tl), Al.info["jacobi_bytes"]),
                 ("residual", lambda: Al.residual(xl, bl, tl), Al.info["residual_bytes"]),
                 ("restrict R r", lambda: R.mult(tl, bc), R.info["spmv_bytes"]),
                 ("interp x += P e", lambda: P.mult_add(xc, xl), P.info["mult_add_bytes"])]
    for name, fn, nbytes in table:
        fn()  # warm (first-use builds, caches): outside the segment
        ctx.synchronize()
        marker(2 * len(ops))  # segment start
        for _ in range(3):
            fn()
        marker(2 * len(ops) + 1)  # segment end
        ctx.synchronize()
        ops.append({"level": l, "op": name, "stored_bytes": int(nbytes)})
    del xl, bl, tl, xc, bc
ctx.synchronize()
out = os.environ.get("AMG_PMC_OPS", os.path.join(ROOT, "gpurun_out", "pmc_vcycle_ops.json"))
json.dump({"grid": [N, N, N], "launches_per_op": 3, "ops": ops}, open(out, "w"), indent=1)
print(json.dumps(ops))
# no explicit teardown: raptor_amd's atexit hook releases the library's objects in order
# while the runtime and the profiler's tool are still up
