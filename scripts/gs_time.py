"""Time the hybrid GS sweeps (forward / backward, block 64) on the 27-pt 256^3 operator:
interleaved rounds, HIP events on the context stream.  RAPTOR_AMD_LIB selects the build."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import raptor_amd as ra  # noqa: E402


def timeit(ctx, fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(ctx.stream):
        e0.record(ctx.stream)
        for _ in range(reps):
            fn()
        e1.record(ctx.stream)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    kind = sys.argv[2] if len(sys.argv) > 2 else "27pt"
    ctx = ra.Context(0)
    A = ra.par_stencil_grid(ctx, kind, (N, N, N))
    n = A.local_rows
    x = ra.vector_uniform(ctx, n, 0, 1)
    b = ra.vector_uniform(ctx, n, 0, 2)
    y = ctx.empty(n)
    ops = {"gs_fwd": lambda: A.hybrid_gs(x, b, y, 64), "gs_bwd": lambda: A.hybrid_gs(x, b, y, 64, backward=True),
           "resid": lambda: A.residual(x, b, y)}
    res = {k: [] for k in ops}
    for fn in ops.values():
        fn()
    for _ in range(5):
        for k, fn in ops.items():
            res[k].append(timeit(ctx, fn, 5))
    print(kind, N, "nnz", A.nnz, "  ".join(f"{k}: {statistics.median(v) * 1e3:8.1f}us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
