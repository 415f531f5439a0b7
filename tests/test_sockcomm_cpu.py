"""The torch-free host exchange (raptor_amd.SocketComm) on the CPU: the Unix-socket
mesh the bench's ranks use for the RCCL id, the setup all-to-all-v and barriers.  Its
collectives are checked directly, and the multi-rank host setup run over it must give every
rank the serial oracle's slices bit for bit (as test_distributed_cpu.py does over gloo)."""
import multiprocessing as mp
import os
import sys
import uuid

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _prims(rank, ws, key, q):
    sys.path.insert(0, ROOT)
    try:
        from raptor_amd._sockcomm import SocketComm

        c = SocketComm(rank, ws, key=key, timeout=60)
        fails = []
        rng = np.random.default_rng(7)
        # sizes[a][b]: bytes rank a sends to rank b (some empty, some large)
        sizes = rng.integers(0, 3 << 20, size=(ws, ws))
        sizes[0, ws - 1] = 0
        send = [bytes(np.full(sizes[rank][b], (rank * 16 + b) & 255, np.uint8)) for b in range(ws)]
        got = c.alltoallv(send, [int(sizes[a][rank]) for a in range(ws)])
        for a in range(ws):
            if bytes(got[a]) != bytes(np.full(sizes[a][rank], (a * 16 + rank) & 255, np.uint8)):
                fails.append(("alltoallv", a))
        if c.allgather_f64(rank + 0.5) != [r + 0.5 for r in range(ws)]:
            fails.append("allgather")
        if c.allreduce_max(float(rank)) != ws - 1 or c.allreduce_sum(1.0) != ws:
            fails.append("allreduce")
        if c.bcast_bytes(b"id-from-root" if rank == 0 else None) != b"id-from-root":
            fails.append("bcast")
        c.barrier()
        c.close()
        q.put((rank, fails))
    except Exception as e:
        q.put((rank, [repr(e)]))


def _setup(rank, ws, key, q):
    sys.path.insert(0, ROOT)
    try:
        from oracle import oracle as O
        from raptor_amd import host
        from raptor_amd._sockcomm import SocketComm

        assert "torch" not in sys.modules
        c = SocketComm(rank, ws, key=key, timeout=60)
        fails = []
        for name, A, coarsen in [("7pt", O.gen_7pt(14, 13, 12), "pmis"), ("27pt", O.gen_27pt(11, 10, 12), "sa")]:
            M = A.to_scipy()
            n = M.shape[0]
            lo, hi = n * rank // ws, n * (rank + 1) // ws
            Ml = M[lo:hi]
            Hp = host.HostHierarchy(n, lo, Ml.indptr, Ml.indices, Ml.data,
                                    host.options(coarsen=coarsen, max_coarse=32),
                                    rank=rank, nranks=ws, group=c)
            Ho = O.Hierarchy(A, **dict(O.DEFAULTS[coarsen], max_coarse=32))
            if Hp.num_levels != Ho.num_levels:
                fails.append((name, "levels"))
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
                        fails.append((name, l, w))
        c.close()
        q.put((rank, fails))
    except Exception as e:
        q.put((rank, [repr(e)]))


def _run(target, ws):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    key = "test-" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=target, args=(r, ws, key, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
    for rank, fails in res:
        assert fails == [], (rank, fails)


@pytest.mark.parametrize("ws", [2, 3, 5])
def test_socketcomm_collectives(ws):
    _run(_prims, ws)


@pytest.mark.parametrize("ws", [2, 3])
def test_socketcomm_host_setup_matches_oracle(oracle, ws):
    _run(_setup, ws)


def test_socketcomm_single_rank_is_trivial():
    sys.path.insert(0, ROOT)
    from raptor_amd._sockcomm import SocketComm

    c = SocketComm(0, 1, key="solo")
    assert c.allreduce_max(3.0) == 3.0 and c.bcast_bytes(b"x") == b"x"
    c.barrier()
