"""GS kernel probe: 27-pt N^3 level-0 hybrid GS on the template kernel vs sliced ELL (A/B in
one process), HIP-event timed; run under rocprofv3 --kernel-trace --stats for kernel names."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import raptor_amd as ra  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
kind = sys.argv[2] if len(sys.argv) > 2 else "27pt"
ctx = ra.Context(0)


def timed(fn, reps=10):
    with torch.cuda.stream(ctx.stream):
        for _ in range(2):
            fn()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(ctx.stream)
        for _ in range(reps):
            fn()
        e1.record(ctx.stream)
        e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for tpl in (sys.argv[3].split(",") if len(sys.argv) > 3 else ("1", "0")):
    os.environ["AMG_GS_TEMPLATES"] = tpl
    A = ra.par_stencil_grid(ctx, kind, (N, N, N))
    n = A.local_rows
    x, b, y = ra.vector_uniform(ctx, n, 0, 1), ra.vector_uniform(ctx, n, 0, 2), ctx.empty(n)
    A.hybrid_gs(x, b, y, 64)
    inf = A._info()
    tf = timed(lambda: A.hybrid_gs(x, b, y, 64))
    tb = timed(lambda: A.hybrid_gs(x, b, y, 64, backward=True))
    tr = timed(lambda: A.residual(x, b, y))
    print(f"GS templates={tpl}: fwd {tf:.1f} us, bwd {tb:.1f} us, resid {tr:.1f} us, gs_bytes "
          f"{inf['gs_bytes']}, lanes {inf['tpl_lanes']}, tpl rows {inf['template_rows']}", flush=True)
    del A, x, b, y
