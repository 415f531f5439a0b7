"""(Named to run after the other -m gpu files: a failure here cannot stop them under -x.)

configs[3] at its real size (BASELINE.json:10): 7-pt Poisson 512^3 = 134,217,728 rows and
937,951,232 nonzeros, near the int32 index ranges of the device formats, the device setup and
the SpGEMM.  On one MI355X, with no scaling claim:
  * 1 rank, GPU setup (strength, PMIS, interpolation, transpose, Galerkin SpGEMM on the device);
  * 8 loopback ranks (z-slabs of 64 planes), GPU setup on every rank (halo states of each
    round through the host exchange), the host's distributed transpose;
and the two must agree: identical per-level global sizes and nonzero counts, and every rank's
slice of the first V-cycle iterate bit-identical to the 1-rank iterate.  Twice: z-slabs of the
natural numbering, and the partition bench.py --gpus 8 runs -- 2 x 2 x 2 boxes of 256^3, the
grid numbered box by box (the 1-rank reference is the same box-numbered operator on one rank).  The plain-CSR A*1
equals the integer row sums (the number of missing neighbours of each grid point), exactly.
At this size no oracle runs (it would take the CPU minutes per cycle); the properties above are
size-independent, and the same code is bit-exact against the oracle at the smaller sizes of
test_gpu_parity.py / test_gpu_multirank.py.

Progress goes to the terminal (capture disabled) so a long phase never looks hung."""
import json
import os
import threading
import time
import uuid

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

DIMS = (512, 512, 512)
NRANKS = 8


def boundary_faces(torch, n, dims, device):
    """(A 1)_i for the Dirichlet 7-pt operator: 6 - (#neighbours) = missing faces of point i."""
    nx, ny, nz = dims
    idx = torch.arange(n, device=device, dtype=torch.int64)
    i, j, k = idx % nx, (idx // nx) % ny, idx // (nx * ny)
    faces = ((i == 0).to(torch.int8) + (i == nx - 1).to(torch.int8) + (j == 0).to(torch.int8) +
             (j == ny - 1).to(torch.int8) + (k == 0).to(torch.int8) + (k == nz - 1).to(torch.int8))
    del idx, i, j, k
    return faces.to(torch.float64)


# the z-slab form is opt-in since r6 (AMG_TEST_512_SLABS=1; ~50 s): the -m gpu step keeps its
# time for the full-size configs[2] / configs[4] checks (test_gpu_zfull_configs.py); boxes are
# the partition bench.py --gpus 8 runs
@pytest.mark.parametrize("partition", [
    pytest.param("slabs", marks=pytest.mark.skipif(os.environ.get("AMG_TEST_512_SLABS") != "1",
                                                   reason="opt-in: AMG_TEST_512_SLABS=1")),
    "boxes"])
def test_512cubed_one_rank_vs_eight_loopback_ranks(capfd, monkeypatch, partition):
    import torch

    import raptor_amd as ra

    t_start = time.perf_counter()
    report = {"partition": partition}
    boxes = (2, 2, 2) if partition == "boxes" else None

    def say(msg):
        with capfd.disabled():
            print(f"[512^3 {partition} {time.perf_counter() - t_start:7.1f}s] {msg}", flush=True)

    monkeypatch.setenv("AMG_LOOPBACK_TIMEOUT", "900")
    n = DIMS[0] * DIMS[1] * DIMS[2]

    # ---- 1 rank, device setup -------------------------------------------------------------
    ctx = ra.Context(0)
    t = time.perf_counter()
    A = ra.par_stencil_grid(ctx, "7pt", DIMS, boxes=boxes)
    report["matrix_s"] = time.perf_counter() - t
    assert A.local_rows == n == 134217728
    assert A.nnz == 937951232
    say(f"1 rank: A built ({A.nnz} nnz) in {report['matrix_s']:.1f}s")
    if boxes is None:  # (the face count below is written in the natural numbering)
        with torch.cuda.stream(ctx.stream):
            ones = ctx.empty(n).fill_(1.0)
            y = ctx.empty(n)
        A.set_format("csr")  # plain int32 row_ptr / col: 938M entries
        A.mult(ones, y)
        ctx.synchronize()
        faces = boundary_faces(torch, n, DIMS, ctx.torch_device)
        assert torch.equal(y, faces), "plain-CSR A*1 differs from the integer row sums"
        A.set_format("auto")  # row templates
        A.mult(ones, y)
        ctx.synchronize()
        assert torch.equal(y, faces), "template-format A*1 differs from the integer row sums"
        del faces, ones, y
        say("A*1 = integer row sums (plain CSR and row templates)")

    t = time.perf_counter()
    ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
    report["setup_1rank_s"] = time.perf_counter() - t
    sizes1 = [(ml.level_info(l)["n_global"], ml.level_info(l)["nnz_global"]) for l in range(ml.num_levels)]
    report["levels"] = sizes1
    say(f"1 rank: device setup {report['setup_1rank_s']:.1f}s, levels {sizes1}")
    assert all(nz < 2 ** 31 for _, nz in sizes1)
    with torch.cuda.stream(ctx.stream):
        xs = ra.vector_uniform(ctx, n, 0, 42)
        b = ctx.empty(n)
    A.mult(xs, b)
    x = ctx.zeros(n)
    ml.cycle(x, b)
    ctx.synchronize()
    x1 = x.cpu().numpy()
    assert np.all(np.isfinite(x1))
    # one more cycle must reduce the residual (the 1-rank solve is the reference below)
    rn0 = A.residual_norm(ctx.zeros(n), b)
    rn1 = A.residual_norm(x, b)
    assert rn1 < 0.5 * rn0
    report["rn0"], report["rn1"] = rn0, rn1
    say(f"1 rank: first V-cycle done, ||r1||/||r0|| = {rn1 / rn0:.4f}")
    del ml, A, xs, b, x
    ctx.synchronize()
    torch.cuda.empty_cache()

    # ---- 8 loopback ranks ------------------------------------------------------------------
    world = f"w512{partition}-" + uuid.uuid4().hex
    out = [None] * NRANKS
    errs = [None] * NRANKS

    def rank(r):
        try:
            c = ra.Context.loopback(r, NRANKS, world)
            Ar = ra.par_stencil_grid(c, "7pt", DIMS, boxes=boxes)
            f, m = Ar.first_row, Ar.local_rows
            tr = time.perf_counter()
            mr = ra.ParRugeStubenSolver(coarsen="pmis").setup(Ar)
            st = time.perf_counter() - tr
            if r == 0:
                say(f"{NRANKS} ranks: setup {st:.1f}s")
            sizes = [(mr.level_info(l)["n_global"], mr.level_info(l)["nnz_global"]) for l in range(mr.num_levels)]
            with torch.cuda.stream(c.stream):
                xr = ra.vector_uniform(c, m, f, 42)
                br = c.empty(m)
            Ar.mult(xr, br)
            xc = c.zeros(m)
            mr.cycle(xc, br)
            c.synchronize()
            same = bool(np.array_equal(xc.cpu().numpy(), x1[f:f + m]))
            out[r] = (f, m, sizes, same, st)
            del mr, Ar
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    th = [threading.Thread(target=rank, args=(r,)) for r in range(NRANKS)]
    for t_ in th:
        t_.start()
    for t_ in th:
        t_.join(timeout=1200)
    bad = [e for e in errs if e is not None]
    bad.sort(key=lambda e: "barrier timed out" in str(e))
    if bad:
        raise bad[0]
    report["setup_8rank_s"] = max(o[4] for o in out)
    say(f"{NRANKS} ranks: first V-cycle done")
    assert sum(o[1] for o in out) == n
    # 64-plane z-slabs / one 256^3 box per rank: equal row counts either way
    assert [o[0] for o in out] == [r * n // NRANKS for r in range(NRANKS)]
    for f, m, sizes, same, _ in out:
        assert sizes == sizes1, "level sizes / nnz differ between 1 and 8 ranks"
        assert same, f"rank slice [{f}, {f + m}) of the first V-cycle differs from the 1-rank iterate"
    rep_dir = os.environ.get("AMG_TEST_REPORT_DIR")
    if rep_dir:
        with open(os.path.join(rep_dir, f"test_512_{partition}_report.json"), "w") as fh:
            json.dump(report, fh)
    say(f"done: {report}")


@pytest.mark.skipif(os.environ.get("AMG_TEST_RCCL_512") != "1",
                    reason="opt-in (AMG_TEST_RCCL_512=1): eight RCCL processes of 512^3 on one GPU")
def test_512cubed_rccl_eight_processes_vs_one_rank(tmp_path, capfd):
    """configs[3] at its size over the product's RCCL transport: eight
    torch-free processes, 2 x 2 x 2 boxes of 256^3 (the bench's --gpus 8 partition), device
    setup, RCCL halo exchange and captured cycles -- on one GPU, each process its own RCCL
    "host" (tests/test_gpu_rccl.py) -- against one rank of the same box-numbered problem: every
    rank's slice of the first V-cycle iterate bit-identical, and the same hierarchy."""
    import raptor_amd as ra

    from tests.test_gpu_rccl import run_rccl

    t_start = time.perf_counter()

    def say(msg):
        with capfd.disabled():
            print(f"[512^3 rccl {time.perf_counter() - t_start:7.1f}s] {msg}", flush=True)

    n = DIMS[0] * DIMS[1] * DIMS[2]
    report = {}
    ctx = ra.Context.native(0)
    A = ra.par_stencil_grid(ctx, "7pt", DIMS, boxes=(2, 2, 2))
    t = time.perf_counter()
    ml = ra.ParMultilevel(coarsen="pmis", smoother="jacobi", replicate_below=262144, use_graph=True).setup(A)
    report["setup_1rank_s"] = time.perf_counter() - t
    sizes1 = [[ml.level_info(l)["n_global"], ml.level_info(l)["nnz_global"]] for l in range(ml.num_levels)]
    xs = ra.vector_uniform(ctx, n, 0, 42)
    b = ctx.empty(n)
    A.mult(xs, b)
    x = ctx.zeros(n)
    ml.cycle(x, b)
    ctx.synchronize()
    x1 = x.numpy()
    assert np.all(np.isfinite(x1))
    say(f"1 rank: setup {report['setup_1rank_s']:.1f}s, levels {sizes1}")
    del ml, A, xs, b, x
    ctx.synchronize()
    del ctx

    spec = dict(kind="7pt", dims=list(DIMS), boxes=[2, 2, 2], coarsen="pmis", smoother="jacobi", rep=262144,
                native=True, graph=True, big=True)
    res = run_rccl(NRANKS, spec, tmp_path, timeout=900)
    say(f"{NRANKS} RCCL processes: setup {max(float(r['setup_s']) for r in res):.1f}s, "
        f"cycle {max(float(r['cycle_ms']) for r in res):.1f} ms (one shared GPU, socket transport)")
    assert [int(r["f"]) for r in res] == [q * n // NRANKS for q in range(NRANKS)]
    for r in res:
        assert r["levels"].tolist() == sizes1, "hierarchy differs between 1 rank and 8 RCCL ranks"
        f, m = int(r["f"]), int(r["m"])
        assert np.array_equal(r["x1"], x1[f:f + m]), f"rank slice [{f}, {f + m}) of the first V-cycle differs"
        assert bool(r["graph_used"])
    report.update(setup_8proc_s=max(float(r["setup_s"]) for r in res),
                  cycle_8proc_ms=max(float(r["cycle_ms"]) for r in res), levels=sizes1)
    rep_dir = os.environ.get("AMG_TEST_REPORT_DIR")
    if rep_dir:
        with open(os.path.join(rep_dir, "test_512_rccl_report.json"), "w") as fh:
            json.dump(report, fh)
    say(f"done: {report}")
