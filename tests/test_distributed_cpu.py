"""Multi-rank setup over gloo on the CPU (world_size 2 and 3): every rank's slice of every
level operator, splitting and the coarse inverse must be bit-identical to the serial
oracle -- the partition-independence that lets 1, 2, 4, 8 GPUs build one hierarchy
(SURVEY.md 7 "Bit-exact integer coarsening", 8e)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from oracle import oracle as O
        from raptor_amd import host

        fails = []
        cases = [("7pt", O.gen_7pt(14, 13, 12), "pmis", 0.0), ("5pt", O.gen_5pt(40, 37), "pmis", 0.0),
                 ("27pt", O.gen_27pt(11, 10, 12), "sa", 0.0), ("7pt", O.gen_7pt(16, 12, 14), "sa", 0.0),
                 # r6: coarse-operator drop tolerance (off-rank diagonals through the halo)
                 ("27pt drop", O.gen_27pt(11, 10, 12), "sa", 0.02), ("7pt drop", O.gen_7pt(14, 13, 12), "pmis", 0.05)]
        for name, A, coarsen, tol in cases:
            M = A.to_scipy()
            n = M.shape[0]
            # uneven contiguous partition (not plane aligned)
            cuts = [0] + [n * (r + 1) // ws - (5 * (ws - 1 - r)) for r in range(ws)]
            cuts[-1] = n
            lo, hi = cuts[rank], cuts[rank + 1]
            Ml = M[lo:hi]
            Hp = host.HostHierarchy(n, lo, Ml.indptr, Ml.indices, Ml.data,
                                    host.options(coarsen=coarsen, max_coarse=32, drop_tol=tol),
                                    rank=rank, nranks=ws, group=dist.group.WORLD)
            Ho = O.Hierarchy(A, **dict(O.DEFAULTS[coarsen], max_coarse=32, drop_tol=tol))
            if Hp.num_levels != Ho.num_levels:
                fails.append((name, "levels", Hp.num_levels, Ho.num_levels))
                continue
            for l in range(Ho.num_levels):
                for w in "APR":
                    if w != "A" and l == Ho.num_levels - 1:
                        continue
                    P = Hp.to_scipy(l, w)
                    f = Hp.sizes(l, w)["first_row"]
                    G = Ho.matrix(l, w)[f:f + P.shape[0]]
                    if not (np.array_equal(P.indptr, G.indptr) and np.array_equal(P.indices, G.indices)
                            and np.array_equal(P.data, G.data)):
                        fails.append((name, coarsen, l, w))
                if l + 1 < Ho.num_levels:
                    f = Hp.sizes(l, "A")["first_row"]
                    s = Hp.split(l)
                    if not np.array_equal(s, Ho.split(l)[f:f + s.size]):
                        fails.append((name, coarsen, l, "split"))
            inv = O.dense_inverse(O.Csr.from_scipy(Ho.matrix(Ho.num_levels - 1, "A")))
            if not np.array_equal(Hp.coarse_inverse(), inv):
                fails.append((name, coarsen, "inverse"))
        q.put((rank, fails))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, [repr(e)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_distributed_setup_matches_serial_oracle(oracle, ws):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
    for rank, fails in res:
        assert fails == [], (rank, fails)


def _io_worker(rank, ws, port, path, q):
    """Reorder (gathers the graph over gloo) and the collective binary writer, ws ranks."""
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from oracle import oracle as O
        from raptor_amd import host

        fails = []
        nx, ny = 53, 47
        A = O.gen_graph_laplacian(nx, ny, 9)
        p = O.rcm(A)
        B = O.permute(A, p).to_scipy()
        n = nx * ny
        lo, hi = n * rank // ws, n * (rank + 1) // ws
        H = host.HostCSR.graph_laplacian(nx, ny, 9, rank=rank, nranks=ws, group=dist.group.WORLD)
        Hb, perm = H.reorder("rcm")
        if not np.array_equal(perm, p[lo:hi]):
            fails.append("perm")
        L = Hb.to_scipy_local()
        G = B[lo:hi]
        if not (np.array_equal(L.indptr, G.indptr) and np.array_equal(L.indices, G.indices)
                and np.array_equal(L.data, G.data)):
            fails.append("reordered rows")
        Hb.write(path)
        dist.barrier()
        R = host.HostCSR.read(path).to_scipy_local()  # every rank reads the whole file
        if not (np.array_equal(R.indptr, B.indptr) and np.array_equal(R.indices, B.indices)
                and np.array_equal(R.data, B.data)):
            fails.append("written file")
        q.put((rank, fails))
    except Exception as e:
        q.put((rank, [repr(e)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 3])
def test_distributed_reorder_and_write(oracle, tmp_path, ws):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    path = str(tmp_path / "rcm.bin")
    procs = [ctx.Process(target=_io_worker, args=(r, ws, port, path, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
    for rank, fails in res:
        assert fails == [], (rank, fails)
