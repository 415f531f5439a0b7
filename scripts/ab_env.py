"""In-process A/B of run-time knobs that select bit-identical kernel paths.

    python scripts/ab_env.py CONFIG "NAME=VAL[,NAME=VAL...]" ["..."] ...

CONFIG: 7pt | sa27 | g3sub (bench.py's workloads, 1 GPU).  Each argument after CONFIG is one
setting (empty string: the defaults).  The hierarchy is built once; for every setting in turn
(alternating, ROUNDS times) the captured graphs are dropped and recaptured, then the solve
(K fused cycles, graph replay) and each level operation of the cycle's large levels are timed
with HIP events.  Knobs must be read per launch (e.g. AMG_TPL_MARCH_CHUNKS).  Prints one JSON line
with the per-setting medians and the solve histories' agreement (bit-identical expected)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import raptor_amd as ra  # noqa: E402

K, ROUNDS, REPS = 20, 5, 10


def parse(spec):
    out = {}
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=", 1)
        out[k] = v
    return out


def main():
    cfg = sys.argv[1]
    settings = [parse(s) for s in sys.argv[2:]] or [{}]
    ctx = ra.Context.native(0)
    if cfg == "g3sub":
        A, _ = ra.par_graph_laplacian(ctx, 1225, 1225, seed=1).reorder("rcm")
        ml = ra.ParSmoothedAggregationSolver().setup(A)
    elif cfg == "sa27":
        A = ra.par_stencil_grid(ctx, "27pt", (256, 256, 256))
        ml = ra.ParSmoothedAggregationSolver().setup(A)
    else:
        A = ra.par_stencil_grid(ctx, "7pt", (256, 256, 256))
        ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
    gs = cfg != "7pt"
    n = A.local_rows
    xs = ra.vector_uniform(ctx, n, 0, 42)
    b = ctx.empty(n)
    A.mult(xs, b)
    x = ctx.zeros(n)
    e0, e1 = ra.Event(ctx), ra.Event(ctx)

    def ev_time(fn, reps):
        fn()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        ctx.synchronize()
        return e0.elapsed_ms(e1) / reps

    ops = []
    for l in range(ml.num_levels - 1):
        if ml.level_info(l)["n_global"] < 100000:
            break
        Al = A if l == 0 else ml.level_matrix(l, "A_cycle")
        P, R = ml.level_matrix(l, "P_cycle"), ml.level_matrix(l, "R_cycle")
        nl, nc = Al.local_rows, P.local_cols
        v = [ra.vector_uniform(ctx, nl, 0, 5), ra.vector_uniform(ctx, nl, 0, 6), ctx.empty(nl),
             ra.vector_uniform(ctx, nc, 0, 7), ctx.empty(R.local_rows)]

        def mk(Al=Al, P=P, R=R, v=v):
            xl, bl, tl, xc, bc = v
            if gs:
                return [("fwd GS", lambda: Al.hybrid_gs(xl, bl, tl, 64)),
                        ("residual", lambda: Al.residual(xl, bl, tl)),
                        ("R r", lambda: R.mult(tl, bc)), ("x += P e", lambda: P.mult_add(xc, xl)),
                        ("bwd GS", lambda: Al.hybrid_gs(xl, bl, tl, 64, backward=True))]
            return [("Jacobi", lambda: Al.jacobi(xl, bl, tl)), ("residual", lambda: Al.residual(xl, bl, tl)),
                    ("R r", lambda: R.mult(tl, bc)), ("x += P e", lambda: P.mult_add(xc, xl))]
        ops += [(l, name, fn) for name, fn in mk()]

    res = [{"setting": s, "solve_ms": [], "ops": {f"L{l} {nm}": [] for l, nm, _ in ops}, "hist": None}
           for s in settings]
    base_env = dict(os.environ)
    for _ in range(ROUNDS):
        for r, s in zip(res, settings):
            os.environ.clear()
            os.environ.update(base_env)
            os.environ.update(s)
            ml.set_graph(False)
            ml.set_graph(True)  # recapture with this setting
            ml.solve(x, b, max_iter=3)
            x.zero_()
            ctx.synchronize()
            e0.record()
            _, h = ml.solve(x, b, max_iter=K)
            e1.record()
            ctx.synchronize()
            r["solve_ms"].append(e0.elapsed_ms(e1) / K)
            x.zero_()
            r["hist"] = [float(v) for v in h] if r["hist"] is None else r["hist"]
            for l, nm, fn in ops:
                r["ops"][f"L{l} {nm}"].append(ev_time(fn, REPS) * 1e3)
    os.environ.clear()
    os.environ.update(base_env)
    out = {"config": cfg, "cycles": K, "rounds": ROUNDS, "results": []}
    for r in res:
        out["results"].append({
            "setting": r["setting"],
            "ms_per_cycle_median": round(statistics.median(r["solve_ms"]), 4),
            "ms_per_cycle_all": [round(v, 4) for v in r["solve_ms"]],
            "ops_us_median": {k: round(statistics.median(v), 1) for k, v in r["ops"].items()},
            "history_equal_first": r["hist"] == res[0]["hist"],
        })
    print(json.dumps(out))
    for r in out["results"]:
        print(r["setting"], r["ms_per_cycle_median"], r["history_equal_first"], file=sys.stderr)


if __name__ == "__main__":
    main()
