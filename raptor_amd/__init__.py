"""raptor_amd -- MI355X-native AMG V-cycle hot path behind a ParCSRMatrix / ParMultilevel API.

The compute path is ``libraptor_amd.so`` (hand-written gfx950 HIP kernels + C++ host setup +
RCCL halo exchange) reached through the C-ABI in ``include/raptor_amd.h``.  This module is
the Python host mirror of that API (BASELINE.json:5: "keeps the ParMultilevel/ParCSRMatrix
API surface"); it holds no numerics of its own and never falls back to a CPU path: if the
shared library or a GPU is missing, it raises.

    import raptor_amd as ra
    ctx = ra.Context()                               # one per GPU / rank
    A = ra.par_stencil_grid(ctx, "7pt", (256, 256, 256))
    ml = ra.ParRugeStubenSolver(coarsen="pmis")       # PMIS + classical interp, Jacobi
    ml.setup(A)
    x, hist = ml.solve(x, b, max_iter=20)

Vectors are rank-local float64 device vectors: torch tensors on the context's device, or --
for a torch-free process (``Context.native``; the bench, so the library binds the ROCm HIP
runtime and RCCL it was built against instead of torch's bundled copies) -- ``DeviceVector``s
allocated through the C-ABI.
"""
from __future__ import annotations

import atexit
import ctypes as C
import os
import weakref

import numpy as np

from ._sockcomm import SocketComm  # noqa: F401
from ._lib import (  # noqa: F401  (re-exported constants)
    AMG_FORMAT_AUTO,
    AMG_FORMAT_BLOCKS,
    AMG_FORMAT_CSR,
    AMG_COARSEN_PMIS,
    AMG_REORDER_RCM,
    AMG_COARSEN_RS,
    AMG_COARSEN_SA,
    AMG_INTERP_CLASSICAL,
    AMG_INTERP_EXT_I,
    AMG_SMOOTH_HYBRID_GS,
    AMG_SMOOTH_JACOBI,
    AMG_STENCIL_5PT,
    AMG_STENCIL_7PT,
    AMG_STENCIL_27PT,
    AmgError,
    LevelInfo,
    MatrixInfo,
    Options,
    check,
    lib,
    lib_path,
)

__all__ = [
    "Context",
    "DeviceVector",
    "Event",
    "SocketComm",
    "ParCSRMatrix",
    "ParMultilevel",
    "ParRugeStubenSolver",
    "ParSmoothedAggregationSolver",
    "par_stencil_grid",
    "par_graph_laplacian",
    "read_par_matrix",
    "vector_uniform",
    "AmgError",
]


def _torch():
    import torch

    return torch


# ---- teardown --------------------------------------------------------------------------
# Objects left alive at interpreter exit used to be freed by their __del__s during module
# teardown, after the HIP runtime's (and a profiler tool's) own finalisation had begun: a
# late hipFree faulted under rocprofv3.  Every live handle is registered
# here and destroyed by an atexit hook -- Python's atexit runs before the C runtime's exit
# handlers -- in dependency order: solvers, then matrices, then vectors and events, then
# contexts.  After it ran, every __del__ is a no-op.
_live = {k: weakref.WeakSet() for k in ("solver", "matrix", "buffer", "context")}
_finalized = False


def _track(kind: str, obj):
    _live[kind].add(obj)


@atexit.register
def _teardown():
    global _finalized
    if _finalized:
        return
    for kind in ("solver", "matrix", "buffer", "context"):
        for obj in list(_live[kind]):
            try:
                obj._release()
            except Exception:
                pass
    _finalized = True


class DeviceVector:
    """float64 device vector of a native (torch-free) context, allocated through the C-ABI
    (amg_device_malloc); freed when collected.  ``numpy()`` copies it to the host."""

    def __init__(self, ctx: "Context", n: int):
        self.ctx = ctx
        self.n = int(n)
        self.ptr = C.c_void_p()
        check(lib().amg_device_malloc(ctx.h, 8 * self.n, C.byref(self.ptr)))
        _track("buffer", self)

    def numel(self) -> int:
        return self.n

    def __len__(self):
        return self.n

    def numpy(self) -> np.ndarray:
        out = np.empty(self.n, np.float64)
        if self.n:
            check(lib().amg_memcpy(self.ctx.h, out.ctypes.data_as(C.c_void_p), self.ptr, 8 * self.n))
        return out

    def cpu(self):  # torch-tensor-like spelling for code that takes either kind
        return self

    def copy_from(self, arr):
        a = np.ascontiguousarray(arr, np.float64)
        if a.size != self.n:
            raise ValueError("copy_from: sizes differ")
        if self.n:
            check(lib().amg_memcpy(self.ctx.h, self.ptr, a.ctypes.data_as(C.c_void_p), 8 * self.n))
        return self

    def zero_(self):
        if self.n:
            check(lib().amg_memset_async(self.ctx.h, self.ptr, 0, 8 * self.n))
        return self

    def _release(self):
        p = getattr(self, "ptr", None)
        self.ptr = None
        if p and p.value and self.ctx.h:
            lib().amg_device_free(self.ctx.h, p)

    def __del__(self):
        if not _finalized:
            try:
                self._release()
            except Exception:
                pass


class Event:
    """Timing event on a context's stream (amg_event_*): works for native and torch contexts."""

    def __init__(self, ctx: "Context"):
        self.ctx = ctx
        self.h = C.c_void_p()
        check(lib().amg_event_create(ctx.h, C.byref(self.h)))
        _track("buffer", self)

    def record(self):
        check(lib().amg_event_record(self.h))
        return self

    def elapsed_ms(self, end: "Event") -> float:
        ms = C.c_float()
        check(lib().amg_event_elapsed_ms(self.h, end.h, C.byref(ms)))
        return ms.value

    def _release(self):
        h = getattr(self, "h", None)
        self.h = None
        if h:
            lib().amg_event_destroy(h)

    def __del__(self):
        if not _finalized:
            try:
                self._release()
            except Exception:
                pass


def _ptr(t):
    """Device pointer of a DeviceVector or a float64 torch tensor (checked)."""
    if t is None:
        return None
    if isinstance(t, DeviceVector):
        return t.ptr
    torch = _torch()
    if not isinstance(t, torch.Tensor) or t.dtype != torch.float64 or not t.is_cuda:
        raise TypeError("vectors must be float64 CUDA(HIP) torch tensors")
    if not t.is_contiguous():
        raise ValueError("vectors must be contiguous")
    return C.c_void_p(t.data_ptr())


class Context:
    """One GPU / rank.  ``Context(device, stream)``; multi-rank via ``Context.distributed``.

    The context's HIP stream is a torch stream, so torch events and the C-ABI kernels share
    one queue (``ctx.stream``).  ``Context.native(device)`` makes a torch-free context: its
    own stream, ``DeviceVector``s for ``empty`` / ``zeros``, multi-rank over a ``SocketComm``
    (``Context.native(device, comm=...)``)."""

    is_native = False  # torch-free context (Context.native)

    def __init__(self, device: int | None = None, stream=None):
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError("raptor_amd needs an AMD GPU (torch.cuda.is_available() is False)")
        if device is None:
            device = torch.cuda.current_device()
        self.device = int(device)
        self.torch_device = torch.device("cuda", self.device)
        self.stream = stream if stream is not None else torch.cuda.Stream(device=self.torch_device)
        self.h = C.c_void_p()
        check(lib().amg_context_create(self.device, C.c_void_p(self.stream.cuda_stream),
                                       C.byref(self.h)))
        _track("context", self)
        self.rank, self.nranks = 0, 1
        self._keep = []

    @classmethod
    def distributed(cls, device: int | None = None, group=None, stream=None):
        """Collective: every rank of ``torch.distributed`` calls this.  Setup-time metadata
        moves over a gloo group; the solve-time halo exchange is RCCL (created here)."""
        import torch.distributed as dist

        from ._comm import make_exchange

        ctx = cls(device, stream)
        rank, nranks = dist.get_rank(group), dist.get_world_size(group)
        gloo = dist.new_group(backend="gloo") if group is None else group
        uid = (C.c_char * 128)()
        if rank == 0:
            check(lib().amg_rccl_unique_id(uid))
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0, group=gloo)
        uid = (C.c_char * 128).from_buffer_copy(obj[0])
        cb = make_exchange(gloo, nranks)
        ctx._keep.append(cb)
        check(lib().amg_context_set_comm(ctx.h, rank, nranks, uid, cb, None))
        ctx.rank, ctx.nranks, ctx.group = rank, nranks, gloo
        return ctx

    @classmethod
    def native(cls, device: int = 0, comm=None):
        """A torch-free context (no torch import): the library's own stream and device
        buffers.  comm: a ``SocketComm`` for multi-rank runs (collective: every rank calls
        this; rank 0's RCCL id travels over the mesh, the setup exchange too)."""
        ctx = cls.__new__(cls)
        ctx.is_native = True
        ctx.device = int(device)
        ctx.torch_device = None
        ctx.stream = None
        ctx.h = C.c_void_p()
        check(lib().amg_context_create(ctx.device, None, C.byref(ctx.h)))
        _track("context", ctx)
        ctx.rank, ctx.nranks = 0, 1
        ctx._keep = []
        if comm is not None and comm.nranks > 1:
            uid = (C.c_char * 128)()
            if comm.rank == 0:
                check(lib().amg_rccl_unique_id(uid))
            raw = comm.bcast_bytes(bytes(uid) if comm.rank == 0 else None)
            uid = (C.c_char * 128).from_buffer_copy(raw)
            cb = comm.exchange_fn()
            ctx._keep.append(cb)
            check(lib().amg_context_set_comm(ctx.h, comm.rank, comm.nranks, uid, cb, None))
            ctx.rank, ctx.nranks, ctx.comm = comm.rank, comm.nranks, comm
        return ctx

    @classmethod
    def loopback(cls, rank: int, nranks: int, world: str, device: int = 0, stream=None,
                 native: bool = False):
        """In-process virtual rank ``rank`` of ``nranks`` (one thread per rank, shared GPU):
        the multi-rank path with device-to-device copies in place of RCCL.  native: a
        torch-free rank (``Context.native``; its own stream, ``DeviceVector``s)."""
        ctx = cls.native(device) if native else cls(device, stream)
        check(lib().amg_context_set_loopback(ctx.h, int(rank), int(nranks), world.encode()))
        ctx.rank, ctx.nranks = int(rank), int(nranks)
        return ctx

    def synchronize(self):
        check(lib().amg_context_synchronize(self.h))

    def empty(self, n: int):
        """Allocate on the context's stream (torch's caching allocator is stream-aware)."""
        if self.is_native:
            return DeviceVector(self, n)
        torch = _torch()
        with torch.cuda.stream(self.stream):
            return torch.empty(int(n), dtype=torch.float64, device=self.torch_device)

    def zeros(self, n: int):
        if self.is_native:
            return DeviceVector(self, n).zero_()
        torch = _torch()
        with torch.cuda.stream(self.stream):
            return torch.zeros(int(n), dtype=torch.float64, device=self.torch_device)

    def _release(self):
        h = getattr(self, "h", None)
        self.h = None
        if h:
            lib().amg_context_destroy(h)

    def __del__(self):
        if not _finalized:
            try:
                self._release()
            except Exception:
                pass


class ParCSRMatrix:
    """Row-partitioned CSR on the GPU (RAPtor ParCSRMatrix analogue).

    Rank-local rows ``[first_row, first_row + local_rows)``; ``mult`` performs the RCCL halo
    exchange it needs, overlapped with the interior rows."""

    def __init__(self, ctx: Context, handle, owner=None):
        self.ctx = ctx
        self.h = handle
        self._owner = owner  # solver that owns a borrowed level matrix
        if owner is None:
            _track("matrix", self)

    @property
    def info(self) -> dict:
        """amg_par_csr_info, read on every access (formats change with set_format and with the
        first compute call).  A borrowed level operator the V-cycle runs as a cycle-order copy
        reports deferred = 1 and zero format fields until a compute call builds it (info never
        builds it: ADVICE r5)."""
        return self._info()

    # ---- construction -------------------------------------------------------------
    @classmethod
    def from_csr(cls, ctx: Context, n_global: int, first_row: int, row_ptr, col, val):
        rp = np.ascontiguousarray(row_ptr, np.int64)
        cg = np.ascontiguousarray(col, np.int64)
        v = np.ascontiguousarray(val, np.float64)
        if rp.ndim != 1 or rp.size < 1 or cg.size != rp[-1] or v.size != rp[-1]:
            raise ValueError("row_ptr / col / val sizes are inconsistent")
        h = C.c_void_p()
        i64 = C.POINTER(C.c_int64)
        check(lib().amg_par_csr_create(ctx.h, int(n_global), int(first_row), rp.size - 1,
                                       rp.ctypes.data_as(i64), cg.ctypes.data_as(i64),
                                       v.ctypes.data_as(C.POINTER(C.c_double)), C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_scipy_local(cls, ctx: Context, M, n_global: int, first_row: int):
        M = M.tocsr()
        return cls.from_csr(ctx, n_global, first_row, M.indptr, M.indices, M.data)

    def _info(self):
        inf = MatrixInfo()
        check(lib().amg_par_csr_info(self.h, C.byref(inf)))
        return {k: getattr(inf, k) for k, _ in MatrixInfo._fields_}

    @property
    def global_rows(self):
        return self.info["n_global_rows"]

    @property
    def local_rows(self):
        return self.info["n_local_rows"]

    @property
    def first_row(self):
        return self.info["first_row"]

    @property
    def local_cols(self):
        return self.info["n_local_cols"]

    @property
    def nnz(self):
        return self.info["nnz_local"]

    def export(self):
        """Host copy of the local rows: (row_ptr, global cols, vals) as numpy arrays."""
        n, nnz = self.local_rows, self.nnz
        rp = np.empty(n + 1, np.int64)
        col = np.empty(nnz, np.int64)
        val = np.empty(nnz, np.float64)
        i64 = C.POINTER(C.c_int64)
        check(lib().amg_par_csr_export(self.h, rp.ctypes.data_as(i64), col.ctypes.data_as(i64),
                                       val.ctypes.data_as(C.POINTER(C.c_double))))
        return rp, col, val

    def to_scipy_local(self):
        import scipy.sparse as sp

        rp, col, val = self.export()
        return sp.csr_matrix((val, col, rp), shape=(self.local_rows, self.info["n_global_cols"]))

    # ---- files and orderings (row f2) ------------------------------------------------
    def write(self, path):
        """Binary CSR file ("RAMGCSR1", read back by read_par_matrix).  Collective."""
        check(lib().amg_par_csr_write(self.h, os.fsencode(path)))

    def reorder(self, method="rcm"):
        """(P A P^T, new_to_old_local): reverse Cuthill-McKee renumbering, even row
        partition; x_new = x_old[new_to_old_local] (gathered).  Collective."""
        if method != "rcm":
            raise ValueError("only 'rcm' is supported")
        n = self.global_rows
        r, p = self.ctx.rank, self.ctx.nranks
        perm = np.empty(n * (r + 1) // p - n * r // p, np.int64)
        h = C.c_void_p()
        check(lib().amg_par_csr_reorder(self.h, AMG_REORDER_RCM, C.byref(h),
                                        perm.ctypes.data_as(C.POINTER(C.c_int64))))
        return ParCSRMatrix(self.ctx, h), perm

    # ---- level kernels (ParCSRMatrix::mult & friends) -------------------------------
    _FORMATS = {"auto": AMG_FORMAT_AUTO, "csr": AMG_FORMAT_CSR, "blocks": AMG_FORMAT_BLOCKS}

    def set_format(self, fmt: str):
        """Storage format of the level kernels: "auto" (row templates + CSR blocks, default),
        "blocks" (CSR blocks with x tiles / value indexing on every row) or "csr" (plain
        row_ptr / col / val, the SURVEY.md 8(d) format).  Results are identical."""
        check(lib().amg_par_csr_set_format(self.h, self._FORMATS[fmt]))
        return self

    def format_digest(self) -> int:
        """FNV-1a digest of this matrix's device format arrays (diagnostic: two builds of
        one operator compare byte for byte)."""
        d = C.c_uint64()
        check(lib().amg_par_csr_format_digest(self.h, C.byref(d)))
        return d.value

    def mult(self, x, y):
        check(lib().amg_par_csr_mult(self.h, _ptr(x), _ptr(y)))
        return y

    def mult_add(self, x, y):
        check(lib().amg_par_csr_mult_add(self.h, _ptr(x), _ptr(y)))
        return y

    def residual(self, x, b, r):
        check(lib().amg_par_csr_residual(self.h, _ptr(x), _ptr(b), _ptr(r)))
        return r

    def jacobi(self, x, b, x_out, omega=2.0 / 3.0):
        check(lib().amg_par_csr_jacobi(self.h, _ptr(x), _ptr(b), _ptr(x_out), float(omega)))
        return x_out

    def hybrid_gs(self, x, b, x_out, block=64, backward=False):
        """One hybrid GS sweep (GS inside blocks of `block` rows, Jacobi across blocks and
        ranks); backward=True walks each block's rows in descending order."""
        fn = lib().amg_par_csr_hybrid_gs_backward if backward else lib().amg_par_csr_hybrid_gs
        check(fn(self.h, _ptr(x), _ptr(b), _ptr(x_out), int(block)))
        return x_out

    def matmat(self, B: "ParCSRMatrix") -> "ParCSRMatrix":
        """C = self * B on the GPU (Galerkin SpGEMM kernel; collective)."""
        h = C.c_void_p()
        check(lib().amg_par_csr_matmat(self.h, B.h, C.byref(h)))
        return ParCSRMatrix(self.ctx, h)

    def residual_norm(self, x, b) -> float:
        out = C.c_double()
        check(lib().amg_par_csr_residual_norm(self.h, _ptr(x), _ptr(b), C.byref(out)))
        return out.value

    def _release(self):
        h = getattr(self, "h", None)
        self.h = None
        if h and self._owner is None:
            lib().amg_par_csr_destroy(h)

    def __del__(self):
        if not _finalized:
            try:
                self._release()
            except Exception:
                pass


_STENCILS = {"5pt": AMG_STENCIL_5PT, "7pt": AMG_STENCIL_7PT, "27pt": AMG_STENCIL_27PT}


def _grid3(kind, dims):
    dims = tuple(int(d) for d in dims)
    if kind == "5pt":
        if len(dims) != 2:
            raise ValueError("5pt takes (nx, ny)")
        return dims[0], dims[1], 1
    if len(dims) != 3:
        raise ValueError(f"{kind} takes (nx, ny, nz)")
    return dims


def par_stencil_grid(ctx: Context, kind: str, dims, eps=(1.0, 1.0, 1e-3), boxes=None) -> ParCSRMatrix:
    """Model problem of SURVEY.md 8d.  Default: this rank's z-slab (2D: y-slab) of the
    natural ordering.  boxes=(bx, by, bz): the grid numbered box by box, ranks holding
    contiguous box ranges (e.g. (2, 2, 2) cubes for 8 ranks).  Collective."""
    nx, ny, nz = _grid3(kind, dims)
    e = (C.c_double * 3)(*eps)
    h = C.c_void_p()
    if boxes is None:
        check(lib().amg_par_stencil_create(ctx.h, _STENCILS[kind], nx, ny, nz, e, C.byref(h)))
    else:
        bx, by, bz = (int(v) for v in boxes)
        check(lib().amg_par_stencil_create_boxes(ctx.h, _STENCILS[kind], nx, ny, nz, bx, by, bz, e, C.byref(h)))
    return ParCSRMatrix(ctx, h)


def box_order(dims, boxes):
    """new_to_old of the box numbering of par_stencil_grid(boxes=...) relative to the natural
    lexicographic order (numpy; for oracle comparisons: B = P A P^T = permute(A, new_to_old))."""
    dims = tuple(int(d) for d in dims) + (1,) * (3 - len(dims))
    boxes = tuple(int(b) for b in boxes) + (1,) * (3 - len(boxes))
    nx, ny, nz = dims
    out = []
    for iz in range(boxes[2]):
        for iy in range(boxes[1]):
            for ix in range(boxes[0]):
                x0, x1 = nx * ix // boxes[0], nx * (ix + 1) // boxes[0]
                y0, y1 = ny * iy // boxes[1], ny * (iy + 1) // boxes[1]
                z0, z1 = nz * iz // boxes[2], nz * (iz + 1) // boxes[2]
                k, j, i = np.meshgrid(np.arange(z0, z1), np.arange(y0, y1), np.arange(x0, x1), indexing="ij")
                out.append((i + nx * (j + ny * k)).ravel())
    return np.concatenate(out).astype(np.int64)


def par_graph_laplacian(ctx: Context, nx: int, ny: int, seed: int = 1) -> ParCSRMatrix:
    """Seeded, randomly numbered unstructured graph Laplacian on an nx x ny lattice (the
    offline G3_circuit substitute).  Even row partition.  Collective."""
    h = C.c_void_p()
    check(lib().amg_par_graph_laplacian_create(ctx.h, int(nx), int(ny), C.c_uint64(seed), C.byref(h)))
    return ParCSRMatrix(ctx, h)


def read_par_matrix(ctx: Context, path) -> ParCSRMatrix:
    """readParMatrix analogue: Matrix Market or binary CSR, even row partition.  Collective."""
    h = C.c_void_p()
    check(lib().amg_par_csr_read(ctx.h, os.fsencode(path), C.byref(h)))
    return ParCSRMatrix(ctx, h)


def runtime_versions() -> dict:
    """The HIP runtime and RCCL versions this process actually bound (hipRuntimeGetVersion,
    ncclGetVersion): a process that imported torch first runs the library on torch's bundled
    copies, which need not be the ROCm release the library was built against."""
    hv, nv = C.c_int32(), C.c_int32()
    check(lib().amg_runtime_versions(C.byref(hv), C.byref(nv)))
    return {"hip_runtime": hv.value, "rccl": nv.value}


def vector_copy(ctx: Context, src, dst):
    """dst = src with the 16-byte nontemporal copy kernel (the bench's copy ceiling)."""
    if src.numel() != dst.numel():
        raise ValueError("vector_copy: sizes differ")
    check(lib().amg_vector_copy(ctx.h, int(src.numel()), _ptr(src), _ptr(dst)))
    return dst


def vector_read(ctx: Context, src, partials):
    """One read pass over src (16-byte loads) leaving per-wave partial sums in `partials`
    (>= 4 * ceil(n / 2048) entries): the bench's read-bandwidth ceiling."""
    check(lib().amg_vector_read(ctx.h, int(src.numel()), _ptr(src), _ptr(partials), int(partials.numel())))
    return partials


def vector_uniform(ctx: Context, n: int, first_gid: int = 0, seed: int = 42):
    """Device vector u_i = uniform(-1, 1) of splitmix64(seed, first_gid + i)."""
    out = ctx.empty(n)
    check(lib().amg_vector_uniform(ctx.h, int(n), int(first_gid), C.c_uint64(seed), _ptr(out)))
    return out


class ParMultilevel:
    """AMG hierarchy + V-cycle (RAPtor ParMultilevel analogue).

    ``coarsen``: "rs" (serial Ruge-Stueben), "pmis", or "sa" (smoothed aggregation over MIS(2)
    aggregates).  ``smoother``: "jacobi" or "hybrid_gs".  ``interp`` (RS / PMIS): "classical"
    (distance one) or "ext+i" (distance two, ``p_max`` entries kept per row; one rank).
    ``drop_tol`` > 0: coarse operators lose their off-diagonals below drop_tol sqrt(|a_ii a_jj|),
    lumped onto the diagonal (non-Galerkin)."""

    _COARSEN = {"rs": AMG_COARSEN_RS, "pmis": AMG_COARSEN_PMIS, "sa": AMG_COARSEN_SA}
    _INTERP = {"classical": AMG_INTERP_CLASSICAL, "ext+i": AMG_INTERP_EXT_I}
    _SMOOTH = {"jacobi": AMG_SMOOTH_JACOBI, "hybrid_gs": AMG_SMOOTH_HYBRID_GS}

    def __init__(self, coarsen="pmis", smoother="jacobi", strong_threshold=None,
                 jacobi_omega=2.0 / 3.0, pre_sweeps=1, post_sweeps=1, max_levels=25,
                 max_coarse=256, gs_block=64, seed=0x5EED, use_graph=None, setup_device=True,
                 replicate_below=262144, interp="classical", p_max=4, drop_tol=0.0):
        if strong_threshold is None:
            strong_threshold = 0.08 if coarsen == "sa" else 0.25
        self.options = Options(self._COARSEN[coarsen], self._SMOOTH[smoother],
                               float(strong_threshold), float(jacobi_omega), int(pre_sweeps),
                               int(post_sweeps), int(max_levels), int(max_coarse), int(gs_block),
                               int(seed), int(setup_device), int(replicate_below),
                               self._INTERP[interp], int(p_max), float(drop_tol))
        self.use_graph = use_graph
        self.h = None
        self.A = None

    def setup(self, A: ParCSRMatrix):
        if self.h:
            lib().amg_solver_destroy(self.h)
        self.A = A
        self.h = C.c_void_p()
        check(lib().amg_solver_setup(A.h, C.byref(self.options), C.byref(self.h)))
        _track("solver", self)
        if self.use_graph is not None:
            check(lib().amg_solver_set_graph(self.h, 1 if self.use_graph else 0))
        return self

    @property
    def num_levels(self) -> int:
        n = C.c_int32()
        check(lib().amg_solver_num_levels(self.h, C.byref(n)))
        return n.value

    def level_info(self, level: int) -> dict:
        inf = LevelInfo()
        check(lib().amg_solver_level_info(self.h, int(level), C.byref(inf)))
        return {k: getattr(inf, k) for k, _ in LevelInfo._fields_}

    def level_matrix(self, level: int, which: str = "A") -> ParCSRMatrix:
        h = C.c_void_p()
        # "A" / "P" / "R": the hierarchy's operators; "A_cycle" / "P_cycle" / "R_cycle": the same
        # operators as the V-cycle runs them (a private brick order on Jacobi levels)
        check(lib().amg_solver_level_matrix(self.h, int(level), {"A": 0, "P": 1, "R": 2, "A_cycle": 3,
                                                                 "P_cycle": 4, "R_cycle": 5}[which],
                                            C.byref(h)))
        return ParCSRMatrix(self.A.ctx, h, owner=self)

    def level_split(self, level: int):
        n = self.level_info(level)["n_local"]
        out = np.empty(n, np.int32)
        check(lib().amg_solver_level_split(self.h, int(level),
                                           out.ctypes.data_as(C.POINTER(C.c_int32))))
        return out

    def set_graph(self, enable: bool):
        """Replay captured hipGraphs (True) or launch cycles eagerly (False).  Collective."""
        check(lib().amg_solver_set_graph(self.h, 1 if enable else 0))
        return self

    @property
    def graph_enabled(self) -> bool:
        """True while cycles replay a captured hipGraph."""
        v = C.c_int32()
        check(lib().amg_solver_get_graph(self.h, C.byref(v)))
        return bool(v.value)

    def cycle_timeline(self, x, b, reps=20):
        """In-graph time of each operation of one V-cycle (one rank): ([(label, us), ...],
        mode) -- mode 2: event nodes inside one captured cycle, 1: one graph per operation,
        0: eager.  Runs `reps` cycles on x (amg_solver_cycle_timeline)."""
        nmax, lb = 256, 64
        us = np.zeros(nmax)
        buf = C.create_string_buffer(nmax * lb)
        n, g = C.c_int32(), C.c_int32()
        check(lib().amg_solver_cycle_timeline(self.h, _ptr(x), _ptr(b), int(reps), nmax,
                                              us.ctypes.data_as(C.POINTER(C.c_double)), buf, lb,
                                              C.byref(n), C.byref(g)))
        raw = buf.raw
        ops = [(raw[k * lb:(k + 1) * lb].split(b"\0", 1)[0].decode(), float(us[k]))
               for k in range(min(n.value, nmax))]
        return ops, int(g.value)

    def bytes_per_cycle(self) -> int:
        """Algorithmic HBM bytes of one V-cycle on this rank."""
        return sum(self.level_info(l)["bytes_per_cycle_local"] for l in range(self.num_levels))

    def cycle(self, x, b):
        check(lib().amg_solver_cycle(self.h, _ptr(x), _ptr(b)))
        return x

    def solve(self, x, b, max_iter=20, tol=0.0):
        hist = np.zeros(int(max_iter) + 1)
        it = C.c_int32()
        check(lib().amg_solver_solve(self.h, _ptr(x), _ptr(b), int(max_iter), float(tol),
                                     hist.ctypes.data_as(C.POINTER(C.c_double)), C.byref(it)))
        return x, hist[: it.value + 1]

    def pcg(self, x, b, max_iter=20, tol=0.0):
        """Conjugate gradients with one V-cycle as the preconditioner."""
        hist = np.zeros(int(max_iter) + 1)
        it = C.c_int32()
        check(lib().amg_solver_pcg(self.h, _ptr(x), _ptr(b), int(max_iter), float(tol),
                                   hist.ctypes.data_as(C.POINTER(C.c_double)), C.byref(it)))
        return x, hist[: it.value + 1]

    def _release(self):
        h = getattr(self, "h", None)
        self.h = None
        if h:
            lib().amg_solver_destroy(h)

    def __del__(self):
        if not _finalized:
            try:
                self._release()
            except Exception:
                pass


class ParRugeStubenSolver(ParMultilevel):
    """Classical AMG: strength theta = 0.25, RS (serial) or PMIS coarsening, classical
    interpolation, Jacobi smoothing."""

    def __init__(self, coarsen="pmis", **kw):
        if coarsen not in ("rs", "pmis"):
            raise ValueError("ParRugeStubenSolver coarsen must be 'rs' or 'pmis'")
        super().__init__(coarsen=coarsen, **kw)


class ParSmoothedAggregationSolver(ParMultilevel):
    """Smoothed aggregation: signed strength 0.08 (x 0.75 per level), MIS(2) aggregates,
    prolongator smoothed with the filtered operator (omega = 4 / (3 rho)), hybrid Gauss-Seidel
    smoothing."""

    def __init__(self, smoother="hybrid_gs", **kw):
        super().__init__(coarsen="sa", smoother=smoother, **kw)
