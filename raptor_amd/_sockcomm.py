"""Host exchange for torch-free multi-rank runs: a full mesh of Unix stream sockets.

One process per GPU (the bench's ranks under ``torch.distributed.run``, the RCCL test workers)
needs three host-side things besides RCCL: the RCCL unique id from rank 0, the setup-time
all-to-all-v of the C-ABI (``amg_alltoallv_fn``: halo plans, ghost rows, coarse numbering) and
barriers / small reductions around timed regions.  ``SocketComm`` provides them without
importing torch, so the process binds the HIP runtime and RCCL libraptor_amd.so was built
against (a torch-first process binds torch's bundled copies).

The mesh uses Linux abstract-namespace Unix sockets named after ``key``, so it is confined to
one node -- as the bench is (one node, 1-8 GPUs).  Rank r listens on ``raptor-amd/<key>/<r>``,
connects to every lower rank and accepts every higher one; each connection starts with the
connecting rank's id.  The default key is per job: ``RAPTOR_AMD_MESH_KEY`` if set, else the
launcher's MASTER_PORT joined with torchrun's TORCHELASTIC_RUN_ID or, without one, the parent
(launcher) process id -- two jobs on a node never share a name.  Abstract sockets
carry no file permissions, so both ends check the peer's credentials (SO_PEERCRED): only a
process of the same user joins the mesh."""
from __future__ import annotations

import ctypes as C
import os
import socket
import struct
import threading
import time

import numpy as np

from ._lib import ALLTOALLV_FN


def _name(key: str, rank: int) -> str:
    return f"\0raptor-amd/{key}/{rank}"


def default_key() -> str:
    """The per-job mesh name (module docstring)."""
    k = os.environ.get("RAPTOR_AMD_MESH_KEY")
    if k:
        return k
    run = os.environ.get("TORCHELASTIC_RUN_ID", "")
    if not run or run == "none":
        run = f"ppid{os.getppid()}"
    return f"{os.environ.get('MASTER_PORT', '0')}.{run}"


def _check_peer(sock):
    """The peer runs as this user (SO_PEERCRED: pid, uid, gid)."""
    cred = sock.getsockopt(socket.SOL_SOCKET, socket.SO_PEERCRED, struct.calcsize("3i"))
    _, uid, _ = struct.unpack("3i", cred)
    if uid != os.getuid():
        raise ConnectionError(f"mesh peer runs as uid {uid}, not {os.getuid()}")


def _recv_into(sock, view):
    got = 0
    n = len(view)
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed the socket")
        got += k


class SocketComm:
    """rank / nranks with a socket to every other rank (see the module docstring)."""

    def __init__(self, rank: int, nranks: int, key: str | None = None, timeout: float = 600.0):
        self.rank, self.nranks = int(rank), int(nranks)
        if not 0 <= self.rank < self.nranks:
            raise ValueError("bad rank / nranks")
        key = str(key if key is not None else default_key())
        self.peers: dict[int, socket.socket] = {}
        if self.nranks == 1:
            return
        lst = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        lst.bind(_name(key, self.rank))
        lst.listen(self.nranks)
        deadline = time.monotonic() + timeout
        try:
            for q in range(self.rank):  # connect to the lower ranks (they may not listen yet)
                while True:
                    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                    try:
                        s.connect(_name(key, q))
                        break
                    except (ConnectionRefusedError, FileNotFoundError):
                        s.close()
                        if time.monotonic() > deadline:
                            raise TimeoutError(f"rank {self.rank}: rank {q} never listened")
                        time.sleep(0.05)
                _check_peer(s)
                s.sendall(struct.pack("<q", self.rank))
                self.peers[q] = s
            lst.settimeout(max(1.0, deadline - time.monotonic()))
            for _ in range(self.rank + 1, self.nranks):  # accept the higher ranks
                s, _ = lst.accept()
                _check_peer(s)
                s.settimeout(None)
                hdr = bytearray(8)
                _recv_into(s, memoryview(hdr))
                q = struct.unpack("<q", hdr)[0]
                if not self.rank < q < self.nranks or q in self.peers:
                    raise ConnectionError(f"unexpected peer id {q}")
                self.peers[q] = s
        finally:
            lst.close()
        for s in self.peers.values():
            s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 1 << 22)
            s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 22)

    # ---- collectives -----------------------------------------------------------------
    def alltoallv(self, send: list[bytes | memoryview], recv_sizes: list[int]) -> list[bytearray]:
        """send[q] goes to rank q; returns what each rank sent here (sizes known in advance).
        A sender thread writes while this thread reads, so no pair blocks on full buffers."""
        out = [bytearray(int(n)) for n in recv_sizes]
        out[self.rank][:] = send[self.rank]
        err = []

        def tx():
            try:
                for q in range(self.nranks):
                    if q != self.rank and len(send[q]):
                        self.peers[q].sendall(send[q])
            except Exception as e:  # reported after the receives
                err.append(e)

        th = threading.Thread(target=tx, daemon=True)
        th.start()
        for q in range(self.nranks):
            if q != self.rank and recv_sizes[q]:
                _recv_into(self.peers[q], memoryview(out[q]))
        th.join()
        if err:
            raise err[0]
        return out

    def allgather_bytes(self, data: bytes) -> list[bytes]:
        n = np.array([len(data)], np.int64).tobytes()
        sizes = [struct.unpack("<q", b)[0] for b in self.alltoallv([n] * self.nranks, [8] * self.nranks)]
        return [bytes(b) for b in self.alltoallv([data] * self.nranks, sizes)]

    def allgather_f64(self, v: float) -> list[float]:
        return [struct.unpack("<d", b)[0] for b in self.allgather_bytes(struct.pack("<d", float(v)))]

    def allreduce_max(self, v: float) -> float:
        return max(self.allgather_f64(v))

    def allreduce_sum(self, v: float) -> float:
        return sum(self.allgather_f64(v))  # rank order: the same sum on every rank

    def barrier(self):
        if self.nranks > 1:
            self.allgather_bytes(b"\1")

    def bcast_bytes(self, data: bytes | None, root: int = 0) -> bytes:
        return self.allgather_bytes(data if self.rank == root else b"")[root]

    # ---- the C-ABI's setup exchange ---------------------------------------------------
    def exchange_fn(self):
        """An ``amg_alltoallv_fn`` over this mesh (keep the returned object alive)."""
        nr = self.nranks

        def _cb(user, send, sbytes, recv, rbytes):
            try:
                sb = [int(sbytes[q]) for q in range(nr)]
                rb = [int(rbytes[q]) for q in range(nr)]
                base = C.cast(send, C.c_void_p).value or 0
                offs = np.concatenate([[0], np.cumsum(sb)]).astype(np.int64)
                parts = [C.string_at(base + int(offs[q]), sb[q]) if sb[q] else b"" for q in range(nr)]
                got = self.alltoallv(parts, rb)
                dst = C.cast(recv, C.c_void_p).value or 0
                o = 0
                for q in range(nr):
                    if rb[q]:
                        C.memmove(dst + o, bytes(got[q]), rb[q])
                    o += rb[q]
                return 0
            except Exception as e:  # never let an exception unwind through C
                import sys

                print(f"raptor_amd socket exchange failed on rank {self.rank}: {e!r}", file=sys.stderr)
                return 1

        return ALLTOALLV_FN(_cb)

    def close(self):
        for s in self.peers.values():
            try:
                s.close()
            except OSError:
                pass
        self.peers = {}

    def __del__(self):
        self.close()
