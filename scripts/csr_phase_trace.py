"""Where the x-tile block kernel's time goes, block by block (diagnostic).

    RAPTOR_AMD_LIB=raptor_amd/libraptor_amd_phase.so python scripts/csr_phase_trace.py [N]

Needs the phase-trace build (make -C raptor_amd/csrc EXTRA=-DAMG_CSR_PHASES=1
BUILD=build_phase OUT=../libraptor_amd_phase.so): thread 0 of every block stamps s_memtime when
its own loads of each phase have landed (kernels.hip, AMG_PHASE) and s_memrealtime (100 MHz) at
entry and exit.  Runs the 7-pt N^3 PMIS hierarchy's level-1 and level-2 residual and Jacobi
(the cycle's dominant launches) three times each and prints, per operation: the median /
mean of each phase in ns, the block lifetime, the kernel span, the mean number of live blocks
(sum of lifetimes / span) and the spread of block start times.  Output: one JSON line."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import raptor_amd as ra  # noqa: E402

PHASES = ["batch1", "batch2", "tile_to_lds", "products", "row_sums"]


def read_launches(path):
    raw = open(path, "rb").read()
    out, o = [], 0
    while o < len(raw):
        mode, nb, n, nnz = np.frombuffer(raw, np.int64, 4, o)
        o += 32
        st = np.frombuffer(raw, np.uint64, int(nb) * 8, o).reshape(int(nb), 8).astype(np.float64)
        o += int(nb) * 8 * 8
        out.append((int(mode), int(nb), int(n), int(nnz), st))
    return out


def summarize(st):
    ok = st[:, 7] > 0
    st = st[ok]
    rt0, rt1 = st[:, 6], st[:, 7]
    life_ns = (rt1 - rt0) * 10.0
    cyc = st[:, 5] - st[:, 0]
    ghz = float(np.median(cyc / np.maximum(life_ns, 1.0)))  # shader clock from the two counters
    res = {"blocks_traced": int(ok.sum()), "shader_GHz": round(ghz, 3)}
    for k, name in enumerate(PHASES):
        d = (st[:, k + 1] - st[:, k]) / ghz
        res[name + "_ns"] = {"median": round(float(np.median(d)), 1), "mean": round(float(d.mean()), 1),
                             "p90": round(float(np.percentile(d, 90)), 1)}
    span_ns = (rt1.max() - rt0.min()) * 10.0
    res["life_ns"] = {"median": round(float(np.median(life_ns)), 1), "mean": round(float(life_ns.mean()), 1)}
    res["span_us"] = round(span_ns / 1e3, 2)
    res["mean_live_blocks"] = round(float(life_ns.sum() / span_ns), 1)
    # start times: how evenly the dispatcher fills the grid (first / last block start)
    starts = np.sort(rt0 - rt0.min()) * 10.0
    res["start_spread_us"] = {"p10": round(float(np.percentile(starts, 10)) / 1e3, 2),
                              "p50": round(float(np.percentile(starts, 50)) / 1e3, 2),
                              "p90": round(float(np.percentile(starts, 90)) / 1e3, 2)}
    # exit-to-next-entry on the chip: blocks retired per us in the steady middle
    return res


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    path = os.path.join(ROOT, "gpurun_out", "csr_phases.bin")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    if os.path.exists(path):
        os.remove(path)
    ctx = ra.Context.native(0)
    A = ra.par_stencil_grid(ctx, "7pt", (N, N, N))
    ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
    report = {"grid": N, "ops": []}
    for l in (1, 2):
        Al = ml.level_matrix(l, "A_cycle")
        n = Al.local_rows
        x, b, t = ra.vector_uniform(ctx, n, 0, 5), ra.vector_uniform(ctx, n, 0, 6), ctx.empty(n)
        for name, fn in (("residual", lambda: Al.residual(x, b, t)), ("Jacobi", lambda: Al.jacobi(x, b, t))):
            fn()  # warm
            ctx.synchronize()
            os.environ["AMG_CSR_PHASES_FILE"] = path
            for _ in range(3):
                fn()
            ctx.synchronize()
            del os.environ["AMG_CSR_PHASES_FILE"]
            launches = read_launches(path)
            os.remove(path)
            for i, (mode, nb, nr, nnz, st) in enumerate(launches):
                s = summarize(st)
                s.update({"level": l, "op": name, "launch": i, "blocks": nb, "rows": nr, "nnz": nnz,
                          "tile_line_bytes": Al.info["tile_line_bytes"]})
                report["ops"].append(s)
                print(json.dumps(s), file=sys.stderr, flush=True)
    print(json.dumps(report))


if __name__ == "__main__":
    main()
