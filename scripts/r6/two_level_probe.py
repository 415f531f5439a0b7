"""Two-level V-cycles on one GPU against the oracle (diagnostic): the drop tolerance 10 case
(diagonal, near-singular coarse operator) and max_levels = 2 without it -- NaN / inf counts and
the largest difference of the finite entries after each of 3 cycles."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import raptor_amd as ra  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.util import to_dev, to_host  # noqa: E402

ctx = ra.Context(0)
dims = (20, 18, 16)
Ao = O.gen_7pt(*dims)
A = ra.par_stencil_grid(ctx, "7pt", dims)
n = Ao.shape[0]
b = Ao.spmv(O.vec_uniform(n, 42))
for name, kw in [("drop10", dict(drop_tol=10.0)), ("maxlev2", dict(max_levels=2, max_coarse=16))]:
    ml = ra.ParRugeStubenSolver(coarsen="pmis", **kw).setup(A)
    Ho = O.Hierarchy(Ao, **dict(O.DEFAULTS["pmis"], **kw))
    dx, xo = ctx.zeros(n), np.zeros(n)
    db = to_dev(ctx, b)
    for k in range(3):
        ml.cycle(dx, db)
        xo = Ho.cycle(xo, b)
        xg = to_host(ctx, dx)
        fin = np.isfinite(xg) & np.isfinite(xo)
        print(name, "levels", ml.num_levels, Ho.num_levels, "cycle", k, "nonfinite gpu/oracle",
              int((~np.isfinite(xg)).sum()), int((~np.isfinite(xo)).sum()),
              "max|diff| finite", float(np.max(np.abs(xg[fin] - xo[fin]))) if fin.any() else None,
              "equal (nan-aware)", bool(np.array_equal(xg, xo, equal_nan=True)), flush=True)
