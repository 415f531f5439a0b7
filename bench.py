#!/usr/bin/env python
"""bench.py -- V-cycle iterations/s and SpMV HBM GB/s, 3D 7-pt Poisson (BASELINE.json:2).

Workload (BASELINE.json configs[1], weak-scaled for --gpus N):
  N=1: 256^3   N=2: 256x256x512   N=4: 256x512x512   N=8: 512^3   (16.8M rows per GPU)
  partitioned into one 256^3 box per rank (N=8: 2 x 2 x 2 cubes, the grid numbered box by box;
  --partition slabs: z-slabs of the natural numbering)
  PMIS coarsening + classical interpolation, 1 pre / 1 post Jacobi sweep (omega 2/3),
  dense solve at <= 256 rows; b = A x*, x* ~ U(-1,1) (splitmix64, seed 42), x0 = 0.
One "step" = one ParMultilevel::solve iteration (V-cycle + residual norm) of the global
problem.  Timed: K steps of amg_solver_solve (no host sync inside; cycles and the last norm
replay captured hipGraphs on every rank count), barrier + device sync on both sides, max over
ranks.

No torch in this process: the library binds the ROCm HIP runtime and RCCL it was built
against (a torch-first process binds torch's bundled HIP 7.0 / RCCL 2.26, where multi-rank
graph capture is refused).  Device buffers and events go through the C-ABI
(raptor_amd.Context.native); ranks find each other over a Unix-socket mesh keyed by the
launcher's MASTER_PORT (raptor_amd.SocketComm: RCCL id, setup exchange, barriers, max over
ranks).  value = V-cycles/s x (global rows / 256^3): 256^3-equivalent
V-cycles per second, the whole-job aggregate (equals plain iterations/s at N=1).

roofline: the level-0 ParCSRMatrix::mult on the plain CSR format (csr_plain_kernel: int32 row_ptr
/ col, fp64 val) timed live with HIP events on the context stream, scored on SURVEY.md 8(d)'s
algorithmic bytes 12 nnz + 4 (n+1) + 16 n.  roofline_stored: the same mult in the product's
default format (row templates / CSR-VI blocks) on the bytes that format streams.
vcycle_kernels: every V-cycle operation of the large levels (eager, events), stored bytes and
fraction of the 8 TB/s peak; the hipGraph'd durations are in profiles/ (rocprofv3).
cpu_baseline (rank 0, N=1): the oracle's V-cycle (C, OpenMP) on the same hierarchy and
inputs, timed for --cpu-seconds at the host's CPU quota (cgroup cpu.max) and at 1 thread;
"port" = this repo's CPU restatement (the reference has no AMG code).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GRIDS = {1: (256, 256, 256), 2: (256, 256, 512), 4: (256, 512, 512), 8: (512, 512, 512)}
# box decomposition per rank count: every rank holds one 256^3 cube; the
# z-slab alternative (--partition slabs) gives 512 x 512 x 64 slabs at N = 8
BOXES = {1: (1, 1, 1), 2: (1, 1, 2), 4: (1, 2, 2), 8: (2, 2, 2)}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MALL_BYTES = 256 << 20  # Infinity Cache (MALL) capacity


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--grid", type=str, default=None, help="override nx,ny,nz")
    ap.add_argument("--spmv-reps", type=int, default=50)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--quick", action="store_true",
                    help="the timed solve only (no mode comparison, time to tolerance, kernel "
                         "table or CPU baseline): rehearsals and attribution runs")
    ap.add_argument("--interp", choices=["classical", "ext+i"], default="classical",
                    help="7pt: interpolation of the PMIS hierarchy (ext+i: distance two, P_max 4, one "
                         "rank; DESIGN.md 3) -- the default stays classical (time to 1e-8, DESIGN.md 6)")
    ap.add_argument("--config", choices=["7pt", "sa27", "g3sub"], default="7pt",
                    help="7pt: the metric workload (default); sa27: BASELINE.json configs[2], "
                         "27-pt anisotropic Q1 diffusion, smoothed aggregation + hybrid GS; "
                         "g3sub: BASELINE.json configs[4] with the offline substitute for "
                         "G3_circuit (seeded unstructured graph Laplacian, RCM-reordered), SA")
    ap.add_argument("--lattice", type=int, default=1225,
                    help="g3sub: lattice side (1225^2 = 1.5M rows, G3_circuit size)")
    ap.add_argument("--no-reorder", action="store_true", help="g3sub: keep the random numbering")
    ap.add_argument("--drop-tol", type=float, default=None,
                    help="coarse-operator drop tolerance (non-Galerkin lumping, DESIGN.md 3); default "
                         "0.005 for g3sub (VERDICT r5 item 8: complexity), 0 (Galerkin) otherwise")
    ap.add_argument("--partition", choices=["boxes", "slabs"], default="boxes",
                    help="7pt/sa27 over N ranks: boxes (default; 2 x 2 x 2 cubes of 256^3 at N = 8, "
                         "the grid numbered box by box) or z-slabs of the natural numbering")
    ap.add_argument("--traffic-json", type=str,
                    default=os.path.join(ROOT, "profiles", "pmc_level0_spmv.json"),
                    help="PMC-measured per-launch HBM traffic of the level-0 SpMV "
                         "(scripts/gpu_profile.sh); reported as roofline.traffic")
    args = ap.parse_args()

    # the bench line is the only thing on stdout: native libraries (RCCL's version banner at
    # communicator init) write to fd 1 directly, so fd 1 is pointed at stderr for the run and
    # the JSON line goes to a duplicate of the original stdout
    out_stream = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import raptor_amd as ra

    assert "torch" not in sys.modules, "bench.py runs torch-free (DESIGN.md 5)"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    comm = None
    if world > 1:
        device = local_rank
        if os.environ.get("AMG_BENCH_SHARED_GPU") == "1":
            # rehearsal of the N-GPU path on a 1-GPU box: every rank on device 0, each its own
            # RCCL "host" (RCCL refuses two ranks of one host on one device; it then connects
            # them over its socket transport, as tests/test_gpu_rccl.py does).  Timings of such
            # a run are not a scaling measurement.
            device = 0
            os.environ["NCCL_HOSTID"] = f"amg-bench-rank{rank}"
        comm = ra.SocketComm(rank, world)
        ctx = ra.Context.native(device, comm=comm)
    else:
        ctx = ra.Context.native(0)

    g3 = args.config == "g3sub"
    if g3:
        grid = (args.lattice, args.lattice, 1)
    elif args.grid:
        grid = tuple(int(v) for v in args.grid.split(","))
    else:
        grid = GRIDS.get(world, (256, 256, 256 * world))
    n_global = grid[0] * grid[1] * grid[2]
    # 7pt/sa27 are weak-scaled and reported in 256^3-equivalent cycles; g3sub is one fixed
    # matrix (strong scaling), reported in plain cycles/s
    scale = 1.0 if g3 else n_global / float(256 ** 3)

    def barrier():
        if world > 1:
            comm.barrier()

    t0 = time.perf_counter()
    sa27 = args.config == "sa27"
    reorder_s = None
    if g3:
        A = ra.par_graph_laplacian(ctx, grid[0], grid[1], seed=1)
        if not args.no_reorder:
            tr = time.perf_counter()
            A, _ = A.reorder("rcm")
            reorder_s = time.perf_counter() - tr
    boxes = None
    if not g3:
        if args.partition == "boxes" and world > 1:
            boxes = BOXES.get(world) if not args.grid else None
            if boxes is None:  # other rank counts / grids: boxes along z (= slabs)
                boxes = (1, 1, world)
        A = ra.par_stencil_grid(ctx, "27pt" if sa27 else "7pt", grid, boxes=boxes)
    part_label = ("one rank" if world == 1 else "even row partition" if g3 else
                  "boxes " + "x".join(str(v) for v in boxes) + " (grid numbered box by box)"
                  if boxes and tuple(boxes) != (1, 1, world) else "z-slab row partition")
    log(rank, f"matrix {grid} built in {time.perf_counter() - t0:.1f}s; local rows {A.local_rows}")
    t1 = time.perf_counter()
    graph = False if args.no_graph else None
    drop_tol = args.drop_tol if args.drop_tol is not None else (0.005 if g3 else 0.0)
    if sa27 or g3:  # BASELINE.json configs[2]/[4]: smoothed aggregation + hybrid Gauss-Seidel
        ml = ra.ParSmoothedAggregationSolver(use_graph=graph, drop_tol=drop_tol).setup(A)
    else:     # BASELINE.json configs[1]/[3]: PMIS + classical interpolation, Jacobi
        ml = ra.ParRugeStubenSolver(coarsen="pmis", use_graph=graph, interp=args.interp,
                                    drop_tol=drop_tol).setup(A)
    setup_s = time.perf_counter() - t1
    nlev = ml.num_levels
    infos = [ml.level_info(l) for l in range(nlev)]
    log(rank, f"setup {setup_s:.1f}s, levels {nlev}: " +
        " ".join(f"{i['n_global']}/{i['nnz_global']}" for i in infos))

    # hybrid-GS sweep form per level on every rank (1 = split: CSR-block old-value pass + chain
    # walk; multi-rank since r5)
    gs_split = None
    if sa27 or g3:
        mine = [int(ml.level_matrix(l, "A").info["gs_split"]) for l in range(nlev - 1)]
        if world > 1:
            flat = comm.allgather_bytes(bytes(mine))
            gs_split = [list(v) for v in flat]
        else:
            gs_split = [mine]

    n = A.local_rows
    xs = ra.vector_uniform(ctx, n, A.first_row, 42)
    b = ctx.empty(n)
    A.mult(xs, b)
    x = ctx.zeros(n)
    y = ctx.empty(n)
    ctx.synchronize()

    # ---- measurement legs first: level kernels, roofline legs, copy / read ceilings ----------
    # (timed live with HIP events on the context stream).  They run before the warmup and the
    # timed solve so the timed cycles see a GPU in its steady working state: the first solve
    # after an idle setup ran ~3 % slower than the same solve repeated later in the process
    # (profiles/r5/r5d_bench_7pt.json: 1.254 vs 1.212-1.213 ms per cycle).
    if not args.quick:
        # ---- level kernels, timed live with HIP events on the context stream -----------------
        n = A.local_rows

        e0, e1 = ra.Event(ctx), ra.Event(ctx)

        def timed(fn, reps, flush=None):
            """avg ms per launch of fn() over reps (HIP events recorded on the context stream, the
            stream the kernels run on).  flush: run before each launch and excluded (cache-cold
            timing: a 1 GiB copy evicts the 256 MiB Infinity Cache and the L2s)."""
            for _ in range(3):
                fn()
            if flush is None:
                e0.record()
                for _ in range(reps):
                    fn()
                e1.record()
                return e0.elapsed_ms(e1) / reps
            tot = 0.0
            for _ in range(reps):
                flush()
                e0.record()
                fn()
                e1.record()
                tot += e0.elapsed_ms(e1)
            return tot / reps

        fl_src = ra.vector_uniform(ctx, 1 << 27, 0, 9)
        fl_dst = ctx.empty(1 << 27)

        def flush():
            ra.vector_copy(ctx, fl_src, fl_dst)

        barrier()
        # roofline: level-0 ParCSRMatrix::mult on the plain CSR format -- int32
        # row_ptr, int32 col, fp64 val, exactly the arrays 8(d) prices -- scored on 8(d)'s
        # algorithmic bytes 12 nnz + 4 (n+1) + 8 (cols + halo) + 8 n
        A.set_format("csr")
        csr_bytes = int(A.info["csr_bytes"])
        csr_warm_ms = timed(lambda: A.mult(x, y), args.spmv_reps)
        csr_cold_ms = timed(lambda: A.mult(x, y), 10, flush)
        A.set_format("auto")
        # an operator whose plain-CSR stream fits the 256 MiB Infinity Cache (the G3 substitute)
        # is scored on cache-cold launches (a 1 GiB copy between them), so the HBM roofline is
        # not credited with MALL hits; larger ones on back-to-back launches
        mall = csr_bytes < MALL_BYTES
        csr_ms = csr_cold_ms if mall else csr_warm_ms
        # the product's default format on the same operator (row templates / CSR-VI blocks),
        # scored on the bytes that format streams
        spmv_bytes = int(A.info["spmv_bytes"])
        spmv_ms = timed(lambda: A.mult(x, y), args.spmv_reps)
        spmv_cold_ms = timed(lambda: A.mult(x, y), 10, flush)
        # measured STREAM-copy ceiling: the 16-byte nontemporal copy kernel, 1 GiB
        copy_ms = timed(flush, 10)
        copy_gbs = 2 * fl_src.numel() * 8 / (copy_ms * 1e-3) / 1e9
        # read ceiling: the same 16-byte loads without the stores (the level kernels read 5-20x
        # what they write, so this, not the copy rate, is the rate they can approach)
        rd_part = ctx.empty(4 * ((fl_src.numel() // 2 + 1023) // 1024))
        read_ms = timed(lambda: ra.vector_read(ctx, fl_src, rd_part), 10)
        read_gbs = fl_src.numel() * 8 / (read_ms * 1e-3) / 1e9
        barrier()

        # per-level V-cycle kernels (rank 0's share; eager launches of the ops the cycle runs, on
        # levels whose kernels outlast the launch overhead).  The in-graph durations are in the
        # rocprofv3 summary committed under profiles/.
        table = []
        gs = sa27 or g3
        for l in range(nlev - 1):
            if infos[l]["n_global"] // world < 100000:  # same decision on every rank
                break
            Al = A if l == 0 else ml.level_matrix(l, "A_cycle")
            nl = Al.local_rows
            P, R = ml.level_matrix(l, "P_cycle"), ml.level_matrix(l, "R_cycle")
            nc = P.local_cols
            xl, bl, tl = ra.vector_uniform(ctx, nl, 0, 5), ra.vector_uniform(ctx, nl, 0, 6), ctx.empty(nl)
            xc, bc = ra.vector_uniform(ctx, nc, 0, 7), ctx.empty(R.local_rows)
            ai, pi, ri = Al.info, P.info, R.info
            # per_cycle: launches of the op in one V-cycle (Jacobi: pre + post on level 0; on
            # coarser levels the pre-sweep from x = 0 is fused into the restriction above)
            if gs:
                Al.hybrid_gs(xl, bl, tl, 64)  # builds the sliced-ELL copy if the cycle has not
                ai = Al._info()
                ops = [("pre GS (forward)", lambda: Al.hybrid_gs(xl, bl, tl, 64), ai["gs_bytes"], 1),
                       ("residual", lambda: Al.residual(xl, bl, tl), ai["residual_bytes"], 1),
                       ("restrict R r", lambda: R.mult(tl, bc), ri["spmv_bytes"], 1),
                       ("interp x += P e", lambda: P.mult_add(xc, xl), pi["mult_add_bytes"], 1),
                       ("post GS (backward)", lambda: Al.hybrid_gs(xl, bl, tl, 64, backward=True), ai["gs_bytes"], 1)]
            else:
                ops = [("Jacobi", lambda: Al.jacobi(xl, bl, tl), ai["jacobi_bytes"], 2 if l == 0 else 1),
                       ("residual", lambda: Al.residual(xl, bl, tl), ai["residual_bytes"], 1),
                       ("restrict R r", lambda: R.mult(tl, bc), ri["spmv_bytes"], 1),
                       ("interp x += P e", lambda: P.mult_add(xc, xl), pi["mult_add_bytes"], 1)]
            for name, fn, nbytes, per in ops:
                ms = timed(fn, 10)
                M = P if name.startswith("interp") else R if name.startswith("restrict") else Al
                table.append({"level": l, "op": name, "kernel": kernel_name(M.info, name),
                              "us": round(ms * 1e3, 1), "per_cycle": per,
                              "stored_bytes": int(nbytes),
                              "mall_resident": int(nbytes) < MALL_BYTES,
                              "GBps": round(nbytes / (ms * 1e-3) / 1e9, 1),
                              "frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)})
            del xl, bl, tl, xc, bc
        # PMC-measured traffic of the same operations (scripts/gpu_pmc_vcycle.sh, 7-pt 256^3):
        # 2 x FETCH_SIZE + WRITE_SIZE per launch beside the stored-format byte model; a ratio
        # above 1.1 is wasted traffic (re-reads), below 1 means cache hits served part of the model
        pmc_path = os.path.join(ROOT, "profiles", "pmc_vcycle_kernels.json" if args.config == "7pt"
                                else f"pmc_vcycle_kernels_{args.config}.json")
        if ((args.config in ("7pt", "sa27") and grid == (256, 256, 256)) or (g3 and args.lattice == 1225 and
                                                                           not args.no_reorder)) \
                and world == 1 and os.path.exists(pmc_path):
            try:
                pm = {(o["level"], o["op"]): o for o in json.load(open(pmc_path))["ops"]}
                for row in table:
                    o = pm.get((row["level"], row["op"]))
                    if o and o["stored_bytes"] == row["stored_bytes"]:
                        row["traffic"] = int(o["traffic_bytes"])
                        row["traffic_over_stored"] = o["traffic_over_stored"]
                        row["traffic_GBps"] = round(o["traffic_bytes"] / (row["us"] * 1e-6) / 1e9, 1)
                    else:
                        # no counters for this library's format of the operation (the file was
                        # taken on another build): said so, not silently dropped
                        row["traffic"] = None
                        row["traffic_stale"] = o is not None
            except (OSError, KeyError, ValueError):
                pass
        # in-graph durations: one rank captures the cycle with a timing
        # event after every operation and replays it (amg_solver_cycle_timeline); each table
        # row gets its operation's in-graph time where the cycle runs it on the same bytes
        # (level 0's pre-smoothing carries the norm in the timed solve, coarse levels' first
        # sweep rides with the restriction above: those rows keep their eager time only)
        timeline = None
        if world == 1 and ml.graph_enabled:
            ops, tl_mode = ml.cycle_timeline(x, b, reps=max(5, args.steps))
            in_graph = tl_mode > 0
            timeline = {"in_graph": in_graph, "mode": {2: "event-record nodes inside one captured cycle",
                                                       1: "one captured graph per operation",
                                                       0: "eager"}[tl_mode],
                        "reps": max(5, args.steps),
                        "ops": [{"op": lab, "us": round(us, 1)} for lab, us in ops],
                        "sum_us": round(sum(us for lab, us in ops if lab != "event-node gap"), 1),
                        "what": "median event-to-event time of each operation of one V-cycle, "
                                "timing events after every operation (mode above); the table's "
                                "in_graph_us subtract event_node_gap_us"}
            # the calibration pseudo-operation: what one event-record node adds to the operation
            # before it; subtracted from every in-graph time (raw times stay in "ops")
            gap = next((us for lab, us in ops if lab == "event-node gap"), 0.0)
            timeline["event_node_gap_us"] = round(gap, 2)
            tl = {lab: max(0.0, us - gap) for lab, us in ops} if in_graph else {}
            for row in table:
                lab = {"residual": "residual", "interp x += P e": "interp", "restrict R r": "restrict",
                       "Jacobi": "post-smooth", "post GS (backward)": "post-smooth",
                       "pre GS (forward)": "pre-smooth"}.get(row["op"])
                us = tl.get(f"L{row['level']} {lab}") if lab else None
                if us is not None:
                    row["in_graph_us"] = round(us, 1)
                    row["in_graph_frac"] = round(row["stored_bytes"] / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        # the dominant kernel: the cycle's longest single launch (the roofline below; in-graph
        # where the timeline has it); the largest share of a cycle (us x launches per cycle) is
        # named beside it
        def launch_us(t):
            return t.get("in_graph_us", t["us"])

        dominant = max(table, key=launch_us) if table else None
        top_share = max(table, key=lambda t: launch_us(t) * t["per_cycle"]) if table else None
        del fl_src, fl_dst, rd_part
        barrier()

    # warmup (captures the cycle and norm hipGraphs, on every rank)
    if args.warmup > 0:
        ml.solve(x, b, max_iter=args.warmup)
    x.zero_()
    ctx.synchronize()
    graph_avail = ml.graph_enabled
    # N > 1: graph replay or eager cycles, decided on this machine before the timed region
    # (the one-GPU socket rehearsal favoured eager, xGMI is expected to
    # favour replay): --steps cycles per mode, twice, alternating, max over ranks -- every rank
    # sees the same times and takes the same mode; the faster is timed below, both are reported
    mode_probe = None
    if world > 1 and graph_avail and not args.no_graph:
        pr = {"eager": [], "graph": []}
        for _ in range(2):
            for mode in ("eager", "graph"):
                ml.set_graph(mode == "graph")
                ml.solve(x, b, max_iter=max(1, args.warmup))  # (re)capture outside the timing
                x.zero_()
                ctx.synchronize()
                barrier()
                t = time.perf_counter()
                ml.solve(x, b, max_iter=args.steps)
                ctx.synchronize()
                barrier()
                pr[mode].append(round(comm.allreduce_max(time.perf_counter() - t) * 1e3 / args.steps, 4))
        use_graph = min(pr["graph"]) <= min(pr["eager"])
        ml.set_graph(use_graph)
        ml.solve(x, b, max_iter=max(1, args.warmup))
        x.zero_()
        ctx.synchronize()
        mode_probe = {"ms_per_step": pr, "chosen": "graph" if use_graph else "eager",
                      "what": "before the timed region: --steps cycles per mode, twice, alternating; "
                              "the mode with the smaller minimum is timed"}
        log(rank, f"mode probe {pr}: timing {mode_probe['chosen']}")

    barrier()
    ctx.synchronize()
    ts = time.perf_counter()
    _, hist = ml.solve(x, b, max_iter=args.steps)
    ctx.synchronize()
    barrier()
    dt = time.perf_counter() - ts
    graph_used = ml.graph_enabled
    if world > 1:
        dt = comm.allreduce_max(dt)
        graph_all = [bool(v) for v in comm.allgather_f64(1.0 if graph_used else 0.0)]
    else:
        graph_all = [graph_used]
    iters_per_s = args.steps / dt
    value = iters_per_s * scale
    conv = float((hist[-1] / hist[0]) ** (1.0 / max(1, len(hist) - 1))) if hist[0] > 0 else None
    # the geometric mean over all steps depends on the step count (the first cycles reduce
    # the residual faster): the factor over the last 5 cycles is the asymptotic one
    conv_last5 = (float((hist[-1] / hist[-6]) ** 0.2) if len(hist) >= 6 and hist[-6] > 0 else None)
    log(rank, f"{args.steps} V-cycles in {dt * 1e3:.2f} ms -> {iters_per_s:.1f} it/s, conv {conv}")

    def timed_solve(fn):
        """max over ranks of the wall time of fn() (a collective solve), barrier + device sync
        on both sides, like the timed region"""
        x.zero_()
        ctx.synchronize()
        barrier()
        ctx.synchronize()
        t = time.perf_counter()
        res = fn()
        ctx.synchronize()
        barrier()
        t = time.perf_counter() - t
        return (comm.allreduce_max(t) if world > 1 else t), res

    if args.quick:
        if rank == 0:
            print(json.dumps({"metric": "V-cycle iters/sec (quick rehearsal line)", "value": round(value, 3),
                              "n_gpus": world, "steps": args.steps, "ms_per_step": round(dt * 1e3 / args.steps, 4),
                              "grid": list(grid), "hipgraph_all_ranks": graph_all, "graph_available": graph_avail,
                              "mode_probe": mode_probe, "partition": part_label,
                              "setup_s": round(setup_s, 2)}), file=out_stream, flush=True)
        del ml, A
        if world > 1:
            comm.close()
        return

    # the other cycle mode, same solve, same process (at N > 1 graph replay
    # is the default on an expectation about xGMI; both are measured so a SCALE run decides)
    modes = None
    if not args.no_graph:
        # alternating repetitions (the first timed region above is not reused: order effects)
        reps = {"graph": [], "eager": []}
        for _ in range(3):
            for mode in ("eager", "graph"):
                ml.set_graph(mode == "graph" and graph_avail)
                ml.solve(x, b, max_iter=max(1, args.warmup))  # (re)capture outside the timing
                t_m, _ = timed_solve(lambda: ml.solve(x, b, max_iter=args.steps))
                reps[mode].append(round(t_m * 1e3 / args.steps, 4))
        ml.set_graph(graph_used)
        ml.solve(x, b, max_iter=max(1, args.warmup))
        med = {k: sorted(v)[1] for k, v in reps.items()}
        modes = {"graph_ms_per_step": med["graph"] if graph_avail else None,
                 "eager_ms_per_step": med["eager"],
                 "repetitions_ms_per_step": reps,
                 "timed_mode": "graph" if graph_used else "eager",
                 "mode_probe": mode_probe,
                 "what": "median of 3 alternating timed solves of --steps cycles per mode, same process"}
        log(rank, f"cycle modes (median of 3): graph {med['graph']} eager {med['eager']} ms/step")

    # time to solution: stationary solve and AMG-PCG to 1e-8 relative
    # residual, setup excluded (reported beside it).  tol > 0 reads the norm back every
    # iteration (one host wait each); the same iteration count without the check is the
    # asynchronous figure.
    tol = 1e-8
    # each form runs once untimed first: its hipGraphs are captured there, not in the timing
    # (tol = 1 stops after one cycle, but sizes the device history for 1000 first: a larger
    # history later would drop the captured graphs)
    timed_solve(lambda: ml.solve(x, b, max_iter=1000, tol=1.0))
    timed_solve(lambda: ml.solve(x, b, max_iter=2))
    t_s, (_, h_s) = timed_solve(lambda: ml.solve(x, b, max_iter=1000, tol=tol))
    n_s = len(h_s) - 1
    t_sa, _ = timed_solve(lambda: ml.solve(x, b, max_iter=n_s))
    timed_solve(lambda: ml.pcg(x, b, max_iter=3))
    t_p, (_, h_p) = timed_solve(lambda: ml.pcg(x, b, max_iter=1000, tol=tol))
    n_p = len(h_p) - 1
    t_pa, _ = timed_solve(lambda: ml.pcg(x, b, max_iter=n_p))
    time_to_tol = {
        "tol_rel": tol,
        "setup_s": round(setup_s, 3),
        "solve": {"cycles": n_s, "reached": bool(h_s[-1] <= tol * h_s[0]), "seconds": round(t_s, 5),
                  "seconds_no_check": round(t_sa, 5)},
        "pcg": {"iterations": n_p, "reached": bool(h_p[-1] <= tol * h_p[0]), "seconds": round(t_p, 5),
                "seconds_no_check": round(t_pa, 5)},
        # a drop-in level solver's time to solution: setup (hierarchy + device formats) + solve
        "setup_plus_solve_s": round(setup_s + t_s, 4),
        "setup_plus_pcg_s": round(setup_s + t_p, 4),
        "what": "rel. residual <= tol from x0 = 0; 'seconds' with the per-iteration norm check "
                "(host wait), 'seconds_no_check' the same iteration count without it; setup "
                "(hierarchy + device formats) not included there, added in setup_plus_*",
    }
    log(rank, f"time to {tol:g}: solve {n_s} cycles {t_s * 1e3:.1f} ms, pcg {n_p} its {t_p * 1e3:.1f} ms")

    # bytes of one V-cycle on all ranks: plain-CSR and stored-format (what
    # the kernels stream).  The per-iteration residual norm is fused into the next cycle's
    # first sweep, so a solve iteration moves one cycle's bytes.
    def allsum(v):
        return float(v) if world == 1 else comm.allreduce_sum(float(v))

    cyc_bytes = allsum(ml.bytes_per_cycle())
    cyc_stored = allsum(sum(i["stored_bytes_per_cycle_local"] for i in infos))


    traffic = None
    traffic_src = None
    if (args.config == "7pt" and grid == (256, 256, 256) and args.traffic_json
            and os.path.exists(args.traffic_json)):
        try:
            tj = json.load(open(args.traffic_json))
            traffic = float(tj["traffic_bytes"])
            traffic_src = (f"{os.path.relpath(args.traffic_json, ROOT)}: {tj.get('kernel', 'level-0 SpMV')}, "
                           "2xFETCH_SIZE+WRITE_SIZE per launch (MI355X_MICROARCH.md correction)")
        except (OSError, KeyError, ValueError):
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(ml, b, args.cpu_seconds, scale, hybrid_gs=sa27 or g3)

    if rank == 0:
        out = {
            "metric": "V-cycle iters/sec + SpMV HBM GB/s, 3D 7-pt Poisson 256^3, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": ("V-cycles/s (fixed 1.5M-row graph)" if g3 else
                     "V-cycles/s (256^3-equivalent: rows*cycles/s / 256^3)"),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if g3 else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (b = A x*, x* splitmix64 U(-1,1) seed 42, x0 = 0)" +
                     ("; matrix: seeded graph-Laplacian SUBSTITUTE for SuiteSparse G3_circuit "
                      "(not available offline)" if g3 else "")),
            "config": {
                "workload": (f"G3_circuit substitute: graph Laplacian on a {grid[0]}x{grid[1]} lattice "
                             f"({n_global} rows, {infos[0]['nnz_global']} nnz, seed 1), "
                             f"{'random numbering' if args.no_reorder else 'RCM-reordered'}, smoothed "
                             f"aggregation (MIS(2)), hybrid GS(64) 1+1 V-cycle, {part_label}" +
                             (f", coarse drop tolerance {drop_tol:g}" if drop_tol else ""))
                if g3 else
                (f"3D 27-pt Q1 anisotropic diffusion (1,1,1e-3) {grid[0]}x{grid[1]}x{grid[2]}, "
                             f"smoothed aggregation (MIS(2)), hybrid GS(64) 1+1 V-cycle, {part_label}" +
                             (f", coarse drop tolerance {drop_tol:g}" if drop_tol else ""))
                if sa27 else
                (f"3D 7-pt Poisson {grid[0]}x{grid[1]}x{grid[2]}, PMIS + "
                 f"{'classical' if args.interp == 'classical' else 'extended+i (P_max 4)'} interp, "
                 f"Jacobi(2/3) 1+1 V-cycle, {part_label}" +
                 (f", coarse drop tolerance {drop_tol:g} (non-Galerkin)" if drop_tol else "")),
                "grid": list(grid),
                "global_rows": n_global,
                "levels": nlev,
                "level_rows": [i["n_global"] for i in infos],
                "level_nnz": [i["nnz_global"] for i in infos],
                "operator_complexity": round(sum(i["nnz_global"] for i in infos) / infos[0]["nnz_global"], 3),
                # the densest coarse level's mean nonzeros per row
                "coarse_nnz_per_row_max": max((round(i["nnz_global"] / max(1, i["n_global"]), 1)
                                               for i in infos[1:]), default=None),
                "drop_tol": drop_tol,
                "parallelism": f"row-partition x{world}, RCCL halo",
                "partition": part_label,
                "setup_s": round(setup_s, 2),
                "reorder_s": None if reorder_s is None else round(reorder_s, 2),
                "hipgraph": graph_used,
                "hipgraph_all_ranks": graph_all,  # the timed mode (the probe's choice at N > 1)
                "graph_available": graph_avail,
                "gs_split_per_rank_level": gs_split,
            },
            "iters_per_s": round(iters_per_s, 3),
            "convergence_factor": conv,
            "convergence_factor_last5": conv_last5,
            # bytes one cycle streams in the stored formats (<= peak x time) and the plain-CSR
            # count of SURVEY.md 8(d) (what a CSR implementation of the same cycle would move)
            "vcycle_stored_bytes": cyc_stored,
            "vcycle_stored_GBps": round(cyc_stored * iters_per_s / 1e9, 1),
            "vcycle_csr_equiv_bytes": cyc_bytes,
            # roofline: the timed cycle's dominant kernel (its longest single launch), timed
            # live with HIP events on the context stream (eager launches of the same operation,
            # rank 0), scored on the bytes its stored format must move;
            # traffic: PMC 2 x FETCH_SIZE + WRITE_SIZE per launch of the same operation
            # (profiles/pmc_vcycle_kernels*.json) when taken on this build's format
            "roofline": None if dominant is None else {
                "bound": "hbm",
                "kernel": f"{dominant['kernel']} -- level-{dominant['level']} {dominant['op']}, rank 0",
                "achieved": round(dominant["stored_bytes"] / (launch_us(dominant) * 1e-6) / 1e9, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(dominant["stored_bytes"] / (launch_us(dominant) * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                "timing": (f"in-graph: median over replays, {timeline['mode']} "
                           "(amg_solver_cycle_timeline)" if "in_graph_us" in dominant
                           else "eager back-to-back launches, HIP events"),
                "eager": {"avg_launch_ms": round(dominant["us"] * 1e-3, 5), "achieved": dominant["GBps"],
                          "frac": dominant["frac"]},
                "traffic": dominant.get("traffic"),
                "traffic_unit": "bytes per launch",
                "bytes_per_launch": dominant["stored_bytes"],
                "bytes_definition": "stored-format HBM bytes per launch (DESIGN.md 4, 8(d) per-unit "
                                    "figures in the operator's stored format)",
                "avg_launch_ms": round(launch_us(dominant) * 1e-3, 5),
                "stream_copy_GBps": round(copy_gbs, 1),
                "stream_read_GBps": round(read_gbs, 1),
                "largest_cycle_share": None if top_share is None else
                    {k: top_share.get(k) for k in ("level", "op", "kernel", "us", "in_graph_us", "per_cycle", "frac")},
            },
            # SURVEY.md 8(d)'s SpMV leg (north_star: >= 60 % of the HBM roofline on the 256^3
            # 7-pt SpMV): the level-0 mult on the plain CSR arrays 8(d) prices
            "spmv_roofline_csr": {
                "bound": "hbm",
                "kernel": "csr_plain_kernel<SPMV> -- level-0 ParCSRMatrix::mult, plain CSR "
                          "(AMG_FORMAT_CSR: int32 row_ptr/col, fp64 val), rank 0",
                "achieved": round(csr_bytes / (csr_ms * 1e-3) / 1e9, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(csr_bytes / (csr_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else round(traffic / 1e9, 4),
                "traffic_unit": "GB per launch",
                "traffic_source": traffic_src,
                "bytes_per_launch": csr_bytes,
                "bytes_definition": "SURVEY.md 8(d): 12 nnz + 4 (n+1) + 8 (local + halo cols) + 8 n",
                "avg_launch_ms": round(csr_ms, 5),
                "timing": ("cache-cold launches (operator fits the 256 MiB Infinity Cache)" if mall
                           else "back-to-back launches"),
                "warm_avg_launch_ms": round(csr_warm_ms, 5),
                "cold_avg_launch_ms": round(csr_cold_ms, 5),
                "cold_GBps": round(csr_bytes / (csr_cold_ms * 1e-3) / 1e9, 1),
                "stream_copy_GBps": round(copy_gbs, 1),
                "stream_read_GBps": round(read_gbs, 1),
                "frac_of_stream_copy": round(csr_bytes / (csr_ms * 1e-3) / 1e9 / copy_gbs, 4),
            },
            "roofline_stored": {
                "kernel": (("tpl_march_kernel" if A.info["tpl_march_shift"] > 0 else "tpl_kernel") +
                           "<SPMV> (row templates" +
                           (")" if A.info["template_rows"] == A.local_rows else " + csr_block_kernel)")
                           if A.info["template_rows"] > 0 else "csr_block_kernel<SPMV> (CSR-VI blocks)") +
                          " -- level-0 mult, default format, rank 0",
                "achieved": round(spmv_bytes / (spmv_ms * 1e-3) / 1e9, 1),
                "frac": round(spmv_bytes / (spmv_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "bytes_per_launch": spmv_bytes,
                "bytes_definition": "stored-format HBM bytes per launch (DESIGN.md 4)",
                "avg_launch_ms": round(spmv_ms, 5),
                "cold_avg_launch_ms": round(spmv_cold_ms, 5),
                "csr_speedup": round(csr_ms / spmv_ms, 3),
                "row_templates": A.info["n_templates"],
                "template_rows_frac": round(A.info["template_rows"] / max(1, A.local_rows), 4),
                "vi_blocks_frac": round(A.info["n_vi_blocks"] / max(1, A.info["n_blocks"]), 4),
            },
            # the runtimes the library actually bound in this process (torch, imported
            # first, brings its own HIP / RCCL)
            "runtime": ra.runtime_versions(),
            "vcycle_kernels": table,
            "vcycle_dominant_kernel": dominant,
            "cycle_timeline": timeline,
            "cycle_modes": modes,
            "time_to_tol": time_to_tol,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), file=out_stream, flush=True)
    del ml, A
    if world > 1:
        comm.close()


def kernel_name(info, op):
    """The kernel family an operation of a matrix runs, from its format info."""
    if op.startswith(("pre GS", "post GS")):
        if info["template_rows"] > 0:
            return "tpl_gs_acc_kernel + tpl_gs_chain_kernel"
        return "csr_block_kernel<GSACC> + gs_chain_kernel" if info["gs_split"] else "hybrid_gs_kernel"
    mode = {"Jacobi": "JACOBI", "residual": "RESID", "restrict R r": "SPMV",
            "interp x += P e": "SPMV_ADD"}[op]
    if info["template_rows"] > 0:
        fam = "tpl_march_kernel" if info["tpl_march_shift"] > 0 else "tpl_kernel"
        if info["template_rows"] < info["n_local_rows"]:
            fam += " + csr_block_kernel"
        return f"{fam}<{mode}>"
    vi = info["n_vi_blocks"] / max(1, info["n_blocks"])
    return (f"csr_block_kernel<{mode}> ({info['tile_line_bytes']}-byte x-tile lines, "
            f"{vi:.0%} value-indexed blocks, {info['n_blocks']} blocks)")


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_quota():
    """CPUs this process may keep busy: the cgroup v2 quota (cpu.max "quota period"), capped by
    the affinity mask; None when there is no quota ("max") or it cannot be read."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q == "max":
            return None
        cpus = max(1, int(float(q) / float(per) + 0.5))
    except (OSError, ValueError):
        return None
    try:
        cpus = min(cpus, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    return cpus


def cpu_baseline(ml, b, seconds, scale, hybrid_gs=False):
    """Oracle V-cycle (C, OpenMP) on the product's own level operators, rank 0, N=1.

    Timed at the host's CPU share -- the cgroup quota (cpu.max; 16 CPUs on the GPU box), else
    OMP_NUM_THREADS / the affinity mask -- and at one thread, for half of `seconds` each.  More
    threads than the quota only time the scheduler's throttling (a 256-thread team on a
    16-CPU quota ran 31x slower than 16 threads, BENCH_r03.json), so no run exceeds it.
    `value` / `cores` are the faster run; both are listed under `runs`."""
    import numpy as np

    from oracle import oracle as O

    levels = []
    for l in range(ml.num_levels):
        mats = []
        for w in "APR":
            if w != "A" and l == ml.num_levels - 1:
                mats.append(None)
                continue
            rp, col, val = ml.level_matrix(l, w).export()
            ncols = ml.level_matrix(l, w).info["n_global_cols"]
            mats.append(O.Csr.from_arrays(rp.size - 1, ncols, rp, col, val))
            del rp, col, val
        levels.append(tuple(mats))
    H = O.Hierarchy(levels[0][0], levels=levels,
                    smoother=O.SMOOTH_HYBRID_GS if hybrid_gs else O.SMOOTH_JACOBI)
    bh = b.numpy()
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    L = O.lib()
    default_threads = int(L.orc_num_threads())
    quota = cpu_quota()
    share = quota or min(default_threads, affinity or default_threads)
    runs = []
    for threads in dict.fromkeys([share, 1]):
        L.orc_set_num_threads(threads)
        x = np.zeros(bh.size)
        x = H.cycle(x, bh)  # untimed first touch / thread start-up
        t0 = time.perf_counter()
        k = 0
        while True:
            x = H.cycle(x, bh)
            k += 1
            el = time.perf_counter() - t0
            if el >= seconds / 2:
                break
        runs.append({"threads": threads, "cycles": k, "seconds": round(el, 2),
                     "value": round(k / el * scale, 4),
                     "what": "host CPU share (cgroup quota)" if threads == quota and quota else
                             "OMP_NUM_THREADS / affinity" if threads == share else "one thread"})
    L.orc_set_num_threads(default_threads)
    best = max(runs, key=lambda r: r["value"])
    return {
        "value": best["value"],
        "unit": "V-cycles/s" if scale == 1.0 else "V-cycles/s (256^3-equivalent)",
        "cores": best["threads"],
        "kind": "port",
        "runs": runs,
        "cpu_model": _cpu_model(),
        "nproc": os.cpu_count(),
        "affinity_cpus": affinity,
        "cgroup_cpu_quota": quota,
        "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
        "sample": f"oracle V-cycles (C/OpenMP, same hierarchy and b): " +
                  ", ".join(f"{r['cycles']} in {r['seconds']}s at {r['threads']} threads" for r in runs) +
                  "; build CPU restatement, not RAPtor (the reference has no AMG CPU path, SURVEY.md 0)",
    }


if __name__ == "__main__":
    main()
