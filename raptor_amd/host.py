"""Host-only (CPU) view of the product's AMG setup: ``amg_host_hierarchy_*`` of the C-ABI.

This is the exact setup code ``ParMultilevel.setup`` runs before uploading the hierarchy to
the GPU, callable without a GPU so the CPU test suite can check
it -- serial and multi-rank over gloo or a ``SocketComm`` -- bit for bit against the oracle."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from ._lib import ALLTOALLV_FN, AMG_REORDER_RCM, Options, check, lib

_WHICH = {"A": 0, "P": 1, "R": 2}
_NULL_FN = ALLTOALLV_FN()


def _exchange(group, nranks):
    """The setup exchange over `group`: a SocketComm (torch-free) or a torch.distributed group."""
    from ._sockcomm import SocketComm

    if isinstance(group, SocketComm):
        return group.exchange_fn()
    from ._comm import make_exchange

    return make_exchange(group, nranks)


class HostHierarchy:
    def __init__(self, n_global, first_row, row_ptr, col, val, options: Options, rank=0,
                 nranks=1, group=None):
        rp = np.ascontiguousarray(row_ptr, np.int64)
        cg = np.ascontiguousarray(col, np.int64)
        v = np.ascontiguousarray(val, np.float64)
        fn = _NULL_FN
        if nranks > 1:
            fn = _exchange(group, nranks)
        self._fn = fn
        self.rank = rank
        self.h = C.c_void_p()
        i64 = C.POINTER(C.c_int64)
        check(lib().amg_host_hierarchy_build(rank, nranks, fn, None, int(n_global), int(first_row),
                                             rp.size - 1, rp.ctypes.data_as(i64),
                                             cg.ctypes.data_as(i64),
                                             v.ctypes.data_as(C.POINTER(C.c_double)),
                                             C.byref(options), C.byref(self.h)))

    @property
    def num_levels(self):
        n = C.c_int32()
        check(lib().amg_host_hierarchy_num_levels(self.h, C.byref(n)))
        return n.value

    def sizes(self, level, which="A"):
        s = np.zeros(5, np.int64)
        check(lib().amg_host_hierarchy_level_size(self.h, level, _WHICH[which],
                                                  s.ctypes.data_as(C.POINTER(C.c_int64))))
        return dict(zip(("n_global_rows", "n_global_cols", "first_row", "n_local_rows",
                         "nnz_local"), s.tolist()))

    def export(self, level, which="A"):
        sz = self.sizes(level, which)
        rp = np.empty(sz["n_local_rows"] + 1, np.int64)
        col = np.empty(sz["nnz_local"], np.int64)
        val = np.empty(sz["nnz_local"], np.float64)
        i64 = C.POINTER(C.c_int64)
        check(lib().amg_host_hierarchy_level_export(self.h, level, _WHICH[which],
                                                    rp.ctypes.data_as(i64), col.ctypes.data_as(i64),
                                                    val.ctypes.data_as(C.POINTER(C.c_double))))
        return rp, col, val, sz

    def to_scipy(self, level, which="A"):
        import scipy.sparse as sp

        rp, col, val, sz = self.export(level, which)
        return sp.csr_matrix((val, col, rp), shape=(sz["n_local_rows"], sz["n_global_cols"]))

    def split(self, level):
        n = self.sizes(level, "A")["n_local_rows"]
        out = np.empty(n, np.int32)
        check(lib().amg_host_hierarchy_level_split(self.h, level,
                                                   out.ctypes.data_as(C.POINTER(C.c_int32))))
        return out

    def coarse_inverse(self):
        n = self.sizes(self.num_levels - 1, "A")["n_global_rows"]
        out = np.empty((n, n))
        check(lib().amg_host_hierarchy_coarse_inverse(self.h,
                                                      out.ctypes.data_as(C.POINTER(C.c_double))))
        return out

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            try:
                lib().amg_host_hierarchy_destroy(h)
            except Exception:
                pass
            self.h = None


class HostCSR:
    """This rank's rows (even row partition) of a host-side matrix: ``amg_host_csr_*``.
    The unstructured-input code run without a GPU."""

    def __init__(self, handle, rank=0, nranks=1, group=None):
        self.h = handle
        self.rank, self.nranks, self.group = rank, nranks, group

    def _fn(self):
        if self.nranks == 1:
            return _NULL_FN
        self._keep = _exchange(self.group, self.nranks)
        return self._keep

    @classmethod
    def graph_laplacian(cls, nx, ny, seed=1, rank=0, nranks=1, group=None):
        h = C.c_void_p()
        check(lib().amg_host_csr_graph_laplacian(rank, nranks, int(nx), int(ny), C.c_uint64(seed),
                                                 C.byref(h)))
        return cls(h, rank, nranks, group)

    @classmethod
    def stencil(cls, kind, dims, boxes=(1, 1, 1), eps=(1.0, 1.0, 1e-3), rank=0, nranks=1, group=None):
        """The box-ordered model problem of par_stencil_grid(boxes=...), host only."""
        kinds = {"5pt": 0, "7pt": 1, "27pt": 2}
        dims = tuple(int(d) for d in dims) + (1,) * (3 - len(dims))
        b = tuple(int(v) for v in boxes) + (1,) * (3 - len(boxes))
        e = (C.c_double * 3)(*eps)
        h = C.c_void_p()
        check(lib().amg_host_csr_stencil(rank, nranks, kinds[kind], dims[0], dims[1], dims[2], b[0], b[1], b[2],
                                         e, C.byref(h)))
        return cls(h, rank, nranks, group)

    @classmethod
    def read(cls, path, rank=0, nranks=1, group=None):
        h = C.c_void_p()
        check(lib().amg_host_csr_read(rank, nranks, os.fsencode(path), C.byref(h)))
        return cls(h, rank, nranks, group)

    def write(self, path):
        check(lib().amg_host_csr_write(self.rank, self.nranks, self._fn(), None, self.h,
                                       os.fsencode(path)))

    def reorder(self, method="rcm"):
        """(P A P^T, new_to_old_local) for the RCM permutation (collective)."""
        if method != "rcm":
            raise ValueError("only 'rcm' is supported")
        n = self.sizes()
        lo = n["n_global_rows"] * self.rank // self.nranks
        hi = n["n_global_rows"] * (self.rank + 1) // self.nranks
        perm = np.empty(hi - lo, np.int64)
        h = C.c_void_p()
        check(lib().amg_host_csr_reorder(self.rank, self.nranks, self._fn(), None, self.h,
                                         AMG_REORDER_RCM, C.byref(h),
                                         perm.ctypes.data_as(C.POINTER(C.c_int64))))
        return HostCSR(h, self.rank, self.nranks, self.group), perm

    def sizes(self):
        s = np.empty(5, np.int64)
        check(lib().amg_host_csr_size(self.h, s.ctypes.data_as(C.POINTER(C.c_int64))))
        return dict(zip(("n_global_rows", "n_global_cols", "first_row", "n_local_rows", "nnz_local"),
                        (int(v) for v in s)))

    def export(self):
        s = self.sizes()
        rp = np.empty(s["n_local_rows"] + 1, np.int64)
        col = np.empty(s["nnz_local"], np.int64)
        val = np.empty(s["nnz_local"])
        i64 = C.POINTER(C.c_int64)
        check(lib().amg_host_csr_export(self.h, rp.ctypes.data_as(i64), col.ctypes.data_as(i64),
                                        val.ctypes.data_as(C.POINTER(C.c_double))))
        return rp, col, val

    def to_scipy_local(self):
        import scipy.sparse as sp

        s = self.sizes()
        rp, col, val = self.export()
        return sp.csr_matrix((val, col, rp), shape=(s["n_local_rows"], s["n_global_cols"]))

    def __del__(self):
        h = getattr(self, "h", None)
        if h:
            try:
                lib().amg_host_csr_destroy(h)
            except Exception:
                pass
            self.h = None


def options(coarsen="pmis", smoother="jacobi", strong_threshold=None, jacobi_omega=2.0 / 3.0,
            pre_sweeps=1, post_sweeps=1, max_levels=25, max_coarse=256, gs_block=64, seed=0x5EED,
            interp="classical", p_max=4, drop_tol=0.0):
    from . import ParMultilevel

    return ParMultilevel(coarsen, smoother, strong_threshold, jacobi_omega, pre_sweeps,
                         post_sweeps, max_levels, max_coarse, gs_block, seed, interp=interp,
                         p_max=p_max, drop_tol=drop_tol).options
