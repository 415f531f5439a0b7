"""One rank of tests/test_gpu_rccl.py: the product's RCCL transport, one process per rank.

Launched by the test as a child process (never imported by it) with RANK / WORLD_SIZE /
MASTER_* set.  spec["native"]: torch-free (raptor_amd.Context.native over a SocketComm, the
bench's own form, on ROCm's HIP / RCCL); otherwise torch's gloo group and torch's bundled
runtime.  Every rank joins the host exchange (setup) and an RCCL communicator
(solve-time halo exchange, norm and coarse allgathers), runs the level kernels and a few
V-cycles on its z-slab, and writes its slices to ``<out>.<rank>.npz``.  The parent compares
them with the serial oracle: this is the path the bench takes for --gpus N > 1.

The development boxes have one GPU and RCCL refuses two ranks on one device of one host, so
the test gives each rank its own NCCL_HOSTID: RCCL then treats the ranks as separate hosts and
moves the data over its socket transport on the loopback interface.  Every call the product
makes (ncclSend/ncclRecv groups on the comm stream, ncclAllGather, graph capture of both) is
the same call it makes over xGMI on an 8-GPU node; only the wire differs.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    spec = json.loads(sys.argv[1])
    out = sys.argv[2]
    sys.path.insert(0, ROOT)
    import numpy as np

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    native = bool(spec.get("native"))
    if native:
        # torch-free: the library binds ROCm's HIP runtime and RCCL; the ranks
        # meet over raptor_amd.SocketComm, vectors are C-ABI device buffers
        import raptor_amd as ra

        comm = ra.SocketComm(rank, world)
        ctx = ra.Context.native(0, comm=comm)

        def host(t):
            ctx.synchronize()
            return t.numpy()

        def barrier():
            comm.barrier()

        def barrier_and_close():
            comm.barrier()
            comm.close()

        def zero(t):
            t.zero_()
    else:
        import torch
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        import raptor_amd as ra

        ctx = ra.Context.distributed(0)

        def host(t):
            ctx.synchronize()
            return t.detach().cpu().numpy().copy()

        def barrier():
            dist.barrier()

        def barrier_and_close():
            dist.barrier()
            dist.destroy_process_group()

        def zero(t):
            with torch.cuda.stream(ctx.stream):
                t.zero_()

    A = ra.par_stencil_grid(ctx, spec["kind"], spec["dims"], boxes=spec.get("boxes"))
    f, m = A.first_row, A.local_rows
    res = {"f": f, "m": m, "n_halo": A.info["n_halo"]}
    if spec.get("big"):
        # full-size case (tests/test_gpu_zfull_512.py): setup, one V-cycle from x = 0 on
        # b = A x* and a few timed cycles; only this rank's first iterate is written
        import time

        t = time.perf_counter()
        ml = ra.ParMultilevel(coarsen=spec["coarsen"], smoother=spec["smoother"],
                              replicate_below=spec["rep"], use_graph=spec["graph"],
                              drop_tol=spec.get("drop", 0.0)).setup(A)
        barrier()
        res["setup_s"] = time.perf_counter() - t
        res["levels"] = np.array([[ml.level_info(l)["n_global"], ml.level_info(l)["nnz_global"]]
                                  for l in range(ml.num_levels)])
        xs = ra.vector_uniform(ctx, m, f, 42)
        bb = ctx.empty(m)
        A.mult(xs, bb)
        dx = ctx.zeros(m)
        ml.cycle(dx, bb)
        res["x1"] = host(dx)
        zero(dx)
        ml.solve(dx, bb, max_iter=2)
        ctx.synchronize()
        barrier()
        t = time.perf_counter()
        _, hist = ml.solve(dx, bb, max_iter=5)
        ctx.synchronize()
        res["cycle_ms"] = (time.perf_counter() - t) / 5 * 1e3
        res["graph_used"] = ml.graph_enabled
        np.savez(f"{out}.{rank}.npz", **res)
        del ml, A
        barrier_and_close()
        return

    x = ra.vector_uniform(ctx, m, f, 3)
    b = ra.vector_uniform(ctx, m, f, 4)
    y = ctx.empty(m)
    A.mult(x, y)
    res["y"] = host(y)
    A.residual(x, b, y)
    res["r"] = host(y)
    A.jacobi(x, b, y)
    res["j"] = host(y)
    res["rn"] = A.residual_norm(x, b)

    res.update(ra.runtime_versions())
    try:
        ml = ra.ParMultilevel(coarsen=spec["coarsen"], smoother=spec["smoother"],
                              replicate_below=spec["rep"], use_graph=spec["graph"],
                              drop_tol=spec.get("drop", 0.0)).setup(A)
    except ra.AmgError as e:
        # graph=True on a runtime whole-cycle capture is not validated on: the gate's error
        # is the result (tests/test_gpu_rccl.py checks it)
        if spec["graph"] is not True:
            raise
        res["gate_error"] = str(e)
        np.savez(f"{out}.{rank}.npz", **res)
        barrier_and_close()
        return
    res["levels"] = ml.num_levels
    res["starts"] = np.array([ml.level_matrix(l, "A").first_row for l in range(ml.num_levels)])
    xs = ra.vector_uniform(ctx, m, f, 42)
    bb = ctx.empty(m)
    A.mult(xs, bb)
    dx = ctx.zeros(m)
    for k in range(3):
        ml.cycle(dx, bb)
        res[f"x{k}"] = host(dx)
    dx = ctx.zeros(m)
    _, hist = ml.solve(dx, bb, max_iter=6)
    res["hist"] = hist
    res["xsolve"] = host(dx)
    # a second solve: rank 0 alone moves its x to a new buffer (the others reuse theirs), so
    # only rank 0's captured graphs are stale -- the ranks must decide to recapture together
    if rank == 0:
        dx = ctx.zeros(m)
    else:
        zero(dx)
    _, hist2 = ml.solve(dx, bb, max_iter=6)
    res["hist2"] = hist2
    dx = ctx.zeros(m)
    _, hp = ml.pcg(dx, bb, max_iter=5)
    res["pcg"] = hp
    if spec.get("trace_pcg"):
        # a second PCG on the same buffers: its iteration graphs are fresh, so under
        # AMG_TRACE_RCCL nothing between the markers may capture or wait in the eager fence
        zero(dx)
        os.write(2, b"@@pcg2-begin\n")
        _, hp2 = ml.pcg(dx, bb, max_iter=5)
        os.write(2, b"@@pcg2-end\n")
        res["pcg2"] = hp2
    res["graph_used"] = ml.graph_enabled
    np.savez(f"{out}.{rank}.npz", **res)
    del ml, A
    barrier_and_close()


if __name__ == "__main__":
    main()
