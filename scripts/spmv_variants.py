"""A/B the CSR-stream kernel variants (env AMG_KERNEL_VARIANT) on the 7-pt 256^3 level-0
operator and on the coarse levels of the PMIS hierarchy: interleaved rounds in one process
(cdna_hip_programming.md 5.4 rule 24), HIP events on the context stream."""
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
    variants = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2,3").split(",")]
    ctx = ra.Context(0)
    A = ra.par_stencil_grid(ctx, "7pt", (N, N, N))
    ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
    mats = [("A0", A)] + [(f"A{l}", ml.level_matrix(l, "A")) for l in (1, 2)] + \
           [("P0", ml.level_matrix(0, "P")), ("R0", ml.level_matrix(0, "R"))]
    res = {}
    for name, M in mats:
        n, nc = M.local_rows, M.local_cols
        x = ra.vector_uniform(ctx, nc, 0, 1)
        b = ra.vector_uniform(ctx, n, 0, 2)
        y = ctx.empty(n)
        byt = {"spmv": 12 * M.nnz + 4 * (n + 1) + 8 * nc + 8 * n}
        ops = {"spmv": lambda: M.mult(x, y)}
        if name.startswith("A"):
            ops["jacobi"] = lambda: M.jacobi(x, b, y)
            byt["jacobi"] = 12 * M.nnz + 4 * (n + 1) + 32 * n
        for op, fn in ops.items():
            for v in variants:
                res[(name, op, v)] = []
        for rnd in range(7):
            for op, fn in ops.items():
                for v in variants:
                    os.environ["AMG_KERNEL_VARIANT"] = str(v)
                    fn()
                    res[(name, op, v)].append(timeit(ctx, fn, 10))
        for op in ops:
            line = [f"{name:3s} {op:7s} n={n:9d} nnz={M.nnz:10d}"]
            for v in variants:
                t = statistics.median(res[(name, op, v)])
                line.append(f"v{v}: {t*1e3:8.1f}us {byt[op]/t/1e6:7.0f}GB/s")
            print("  ".join(line), flush=True)
    # correctness: every variant gives the same bits
    x = ra.vector_uniform(ctx, A.local_rows, 0, 3)
    outs = []
    for v in variants:
        os.environ["AMG_KERNEL_VARIANT"] = str(v)
        y = ctx.empty(A.local_rows)
        A.mult(x, y)
        ctx.synchronize()
        outs.append(y.cpu())
    print("variants bit-identical:", all(torch.equal(outs[0], o) for o in outs[1:]))


if __name__ == "__main__":
    main()
