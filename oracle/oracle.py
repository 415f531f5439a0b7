"""ctypes binding for the CPU oracle (liboracle_amg.so).  TEST INFRASTRUCTURE ONLY.

Imported only by tests/, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py``, as the checker.  The product (``raptor_amd``) never imports this module.
Parity is UNPINNED against Siddarthareddy1/raptor (the reference has no AMG code; see
SURVEY.md section 0); the oracle is pinned to scipy fixtures in ``tests/golden``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_amg.so")

COARSEN_RS, COARSEN_PMIS, COARSEN_SA = 0, 1, 2
SMOOTH_JACOBI, SMOOTH_HYBRID_GS = 0, 1
INTERP_CLASSICAL, INTERP_EXT_I = 0, 1

_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_f64p = C.POINTER(C.c_double)


class _Opt(C.Structure):
    _fields_ = [
        ("coarsen", C.c_int32),
        ("smoother", C.c_int32),
        ("strong_threshold", C.c_double),
        ("jacobi_omega", C.c_double),
        ("pre_sweeps", C.c_int32),
        ("post_sweeps", C.c_int32),
        ("max_levels", C.c_int32),
        ("max_coarse", C.c_int64),
        ("gs_block", C.c_int64),
        ("seed", C.c_uint64),
        ("interp", C.c_int32),
        ("p_max", C.c_int64),
        ("drop_tol", C.c_double),
    ]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        vp = C.c_void_p
        sig = {
            "orc_csr_new": (vp, [C.c_int64, C.c_int64, _i64p, _i64p, _f64p]),
            "orc_csr_free": (None, [vp]),
            "orc_csr_nnz": (C.c_int64, [vp]),
            "orc_csr_rows": (C.c_int64, [vp]),
            "orc_csr_cols": (C.c_int64, [vp]),
            "orc_csr_export": (None, [vp, _i64p, _i64p, _f64p]),
            "orc_gen_5pt": (vp, [C.c_int64, C.c_int64]),
            "orc_gen_7pt": (vp, [C.c_int64, C.c_int64, C.c_int64]),
            "orc_gen_27pt": (vp, [C.c_int64] * 3 + [C.c_double] * 3),
            "orc_gen_graph_laplacian": (vp, [C.c_int64, C.c_int64, C.c_uint64]),
            "orc_rcm": (None, [vp, _i64p]),
            "orc_hier_set_cuts": (None, [vp, C.c_int32, C.c_int32, _i64p]),
            "orc_permute": (vp, [vp, _i64p]),
            "orc_vec_uniform": (None, [C.c_int64, C.c_int64, C.c_uint64, _f64p]),
            "orc_spmv": (None, [vp, _f64p, _f64p]),
            "orc_spmv_add": (None, [vp, _f64p, _f64p]),
            "orc_residual": (None, [vp, _f64p, _f64p, _f64p]),
            "orc_jacobi": (None, [vp, _f64p, _f64p, _f64p, C.c_double]),
            "orc_hybrid_gs": (None, [vp, _f64p, _f64p, _f64p, C.c_int64]),
            "orc_hybrid_gs_backward": (None, [vp, _f64p, _f64p, _f64p, C.c_int64]),
            "orc_hybrid_gs_cut": (None, [vp, _f64p, _f64p, _f64p, C.c_int64, C.c_int32, C.c_int32,
                                         _i64p]),
            "orc_norm2": (C.c_double, [C.c_int64, _f64p]),
            "orc_transpose": (vp, [vp]),
            "orc_spgemm": (vp, [vp, vp]),
            "orc_strength_classical": (vp, [vp, C.c_double]),
            "orc_strength_symmetric": (vp, [vp, C.c_double]),
            "orc_rs_split": (None, [vp, _i32p]),
            "orc_pmis_split": (None, [vp, C.c_uint64, _i32p]),
            "orc_interp_classical": (vp, [vp, vp, _i32p]),
            "orc_interp_ext_i": (vp, [vp, vp, _i32p, C.c_int64]),
            "orc_mis2_aggregate": (C.c_int64, [vp, C.c_uint64, _i32p]),
            "orc_sa_prolongator": (vp, [vp, _i32p, C.c_int64, C.c_double, C.c_uint64]),
            "orc_sa_filter": (vp, [vp, C.c_double]),
            "orc_sa_rho": (C.c_double, [vp, _f64p, C.c_uint64]),
            "orc_sa_theta_next": (C.c_double, [C.c_double]),
            "orc_sparsify": (vp, [vp, C.c_double]),
            "orc_dense_inverse": (None, [C.c_int64, vp, _f64p]),
            "orc_hier_setup": (vp, [vp, C.POINTER(_Opt)]),
            "orc_hier_free": (None, [vp]),
            "orc_hier_from_levels": (vp, [C.c_int32, C.POINTER(vp), C.POINTER(vp),
                                          C.POINTER(vp), C.POINTER(_Opt)]),
            "orc_hier_levels": (C.c_int32, [vp]),
            "orc_num_threads": (C.c_int32, []),
            "orc_set_num_threads": (None, [C.c_int32]),
            "orc_hier_pcg": (C.c_int32, [vp, _f64p, _f64p, C.c_int32, C.c_double, _f64p]),
            "orc_hier_matrix": (vp, [vp, C.c_int32, C.c_int32]),
            "orc_hier_split": (None, [vp, C.c_int32, _i32p]),
            "orc_hier_cycle": (None, [vp, _f64p, _f64p]),
            "orc_hier_solve": (C.c_int32, [vp, _f64p, _f64p, C.c_int32, C.c_double, _f64p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


class Csr:
    """Owned oracle CSR handle (int64 indices, fp64 values)."""

    def __init__(self, handle):
        if not handle:
            raise RuntimeError("oracle returned a null matrix")
        self.h = handle

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_csr_free(self.h)
            self.h = None

    @classmethod
    def from_arrays(cls, n_rows, n_cols, rp, col, val):
        rp = np.ascontiguousarray(rp, np.int64)
        col = np.ascontiguousarray(col, np.int64)
        val = np.ascontiguousarray(val, np.float64)
        return cls(lib().orc_csr_new(n_rows, n_cols, _p(rp, _i64p), _p(col, _i64p), _p(val, _f64p)))

    @classmethod
    def from_scipy(cls, M):
        M = M.tocsr()
        M.sort_indices()
        return cls.from_arrays(M.shape[0], M.shape[1], M.indptr, M.indices, M.data)

    @property
    def shape(self):
        return (lib().orc_csr_rows(self.h), lib().orc_csr_cols(self.h))

    @property
    def nnz(self):
        return lib().orc_csr_nnz(self.h)

    def arrays(self):
        n, _ = self.shape
        rp = np.empty(n + 1, np.int64)
        col = np.empty(self.nnz, np.int64)
        val = np.empty(self.nnz, np.float64)
        lib().orc_csr_export(self.h, _p(rp, _i64p), _p(col, _i64p), _p(val, _f64p))
        return rp, col, val

    def to_scipy(self):
        import scipy.sparse as sp

        rp, col, val = self.arrays()
        return sp.csr_matrix((val, col, rp), shape=self.shape)

    # level kernels ---------------------------------------------------------------
    def spmv(self, x):
        x = np.ascontiguousarray(x, np.float64)
        y = np.empty(self.shape[0])
        lib().orc_spmv(self.h, _p(x, _f64p), _p(y, _f64p))
        return y

    def spmv_add(self, x, y):
        x = np.ascontiguousarray(x, np.float64)
        y = np.array(y, np.float64, copy=True)
        lib().orc_spmv_add(self.h, _p(x, _f64p), _p(y, _f64p))
        return y

    def residual(self, x, b):
        x = np.ascontiguousarray(x, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        r = np.empty(self.shape[0])
        lib().orc_residual(self.h, _p(x, _f64p), _p(b, _f64p), _p(r, _f64p))
        return r

    def jacobi(self, x, b, omega):
        x = np.ascontiguousarray(x, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        out = np.empty(self.shape[0])
        lib().orc_jacobi(self.h, _p(x, _f64p), _p(b, _f64p), _p(out, _f64p), omega)
        return out

    def hybrid_gs(self, x, b, block):
        x = np.ascontiguousarray(x, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        out = np.empty(self.shape[0])
        lib().orc_hybrid_gs(self.h, _p(x, _f64p), _p(b, _f64p), _p(out, _f64p), block)
        return out

    def hybrid_gs_backward(self, x, b, block):
        x = np.ascontiguousarray(x, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        out = np.empty(self.shape[0])
        lib().orc_hybrid_gs_backward(self.h, _p(x, _f64p), _p(b, _f64p), _p(out, _f64p), block)
        return out

    def hybrid_gs_cut(self, x, b, block, backward, cuts):
        """Hybrid GS with GS blocks clipped at the rank starts `cuts` (amg_oracle.c:255)."""
        x = np.ascontiguousarray(x, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        c = np.ascontiguousarray(cuts, np.int64)
        out = np.empty(self.shape[0])
        lib().orc_hybrid_gs_cut(self.h, _p(x, _f64p), _p(b, _f64p), _p(out, _f64p), block,
                                1 if backward else 0, int(c.size), _p(c, _i64p))
        return out

    def transpose(self):
        return Csr(lib().orc_transpose(self.h))

    def __matmul__(self, other):
        return Csr(lib().orc_spgemm(self.h, other.h))


def gen_5pt(nx, ny):
    return Csr(lib().orc_gen_5pt(nx, ny))


def gen_7pt(nx, ny, nz):
    return Csr(lib().orc_gen_7pt(nx, ny, nz))


def gen_27pt(nx, ny, nz, ex=1.0, ey=1.0, ez=1e-3):
    return Csr(lib().orc_gen_27pt(nx, ny, nz, ex, ey, ez))


def gen_graph_laplacian(nx, ny, seed=1):
    """G3_circuit substitute (io_oracle.c; spec DESIGN.md 8)."""
    return Csr(lib().orc_gen_graph_laplacian(nx, ny, seed))


def rcm(A):
    """Reverse Cuthill-McKee order: new_to_old (io_oracle.c orc_rcm)."""
    out = np.empty(A.shape[0], np.int64)
    lib().orc_rcm(A.h, _p(out, _i64p))
    return out


def permute(A, new_to_old):
    """P A P^T with B[k, :] = A[new_to_old[k], :] renumbered."""
    p = np.ascontiguousarray(new_to_old, np.int64)
    return Csr(lib().orc_permute(A.h, _p(p, _i64p)))


def vec_uniform(n, seed, first_gid=0):
    out = np.empty(n)
    lib().orc_vec_uniform(n, first_gid, seed, _p(out, _f64p))
    return out


def norm2(v):
    v = np.ascontiguousarray(v, np.float64)
    return lib().orc_norm2(v.size, _p(v, _f64p))


def strength_classical(A, theta):
    return Csr(lib().orc_strength_classical(A.h, theta))


def strength_symmetric(A, theta):
    return Csr(lib().orc_strength_symmetric(A.h, theta))


def rs_split(S):
    cf = np.empty(S.shape[0], np.int32)
    lib().orc_rs_split(S.h, _p(cf, _i32p))
    return cf


def pmis_split(S, seed):
    cf = np.empty(S.shape[0], np.int32)
    lib().orc_pmis_split(S.h, seed, _p(cf, _i32p))
    return cf


def interp_classical(A, S, cf):
    cf = np.ascontiguousarray(cf, np.int32)
    return Csr(lib().orc_interp_classical(A.h, S.h, _p(cf, _i32p)))


def interp_ext_i(A, S, cf, p_max=4):
    """Extended+i interpolation with P_max truncation."""
    cf = np.ascontiguousarray(cf, np.int32)
    return Csr(lib().orc_interp_ext_i(A.h, S.h, _p(cf, _i32p), p_max))


def mis2_aggregate(S, seed):
    agg = np.empty(S.shape[0], np.int32)
    na = lib().orc_mis2_aggregate(S.h, seed, _p(agg, _i32p))
    return agg, na


def sa_prolongator(A, agg, n_agg, theta, seed):
    agg = np.ascontiguousarray(agg, np.int32)
    return Csr(lib().orc_sa_prolongator(A.h, _p(agg, _i32p), n_agg, theta, seed))


def sa_filter(A, theta):
    """SA smoothing's filtered operator."""
    return Csr(lib().orc_sa_filter(A.h, theta))


def sa_rho(F, d, seed):
    d = np.ascontiguousarray(d, np.float64)
    return lib().orc_sa_rho(F.h, _p(d, _f64p), seed)


def sparsify(A, tau):
    """Coarse-operator drop tolerance."""
    return Csr(lib().orc_sparsify(A.h, tau))


def sa_theta_next(theta):
    return lib().orc_sa_theta_next(theta)


def dense_inverse(A):
    n = A.shape[0]
    inv = np.empty((n, n))
    lib().orc_dense_inverse(n, A.h, _p(inv, _f64p))
    return inv


DEFAULTS = {
    "pmis": dict(coarsen=COARSEN_PMIS, smoother=SMOOTH_JACOBI, strong_threshold=0.25),
    "rs": dict(coarsen=COARSEN_RS, smoother=SMOOTH_JACOBI, strong_threshold=0.25),
    "sa": dict(coarsen=COARSEN_SA, smoother=SMOOTH_HYBRID_GS, strong_threshold=0.08),
}


class Hierarchy:
    """Serial oracle ParMultilevel: setup / cycle / solve."""

    def __init__(self, A, coarsen=COARSEN_PMIS, smoother=SMOOTH_JACOBI, strong_threshold=0.25,
                 jacobi_omega=2.0 / 3.0, pre_sweeps=1, post_sweeps=1, max_levels=25,
                 max_coarse=256, gs_block=64, seed=0x5EED, levels=None, interp=INTERP_CLASSICAL,
                 p_max=4, drop_tol=0.0):
        """Serial setup of A; or, with ``levels=[(A_l, P_l, R_l), ...]`` (Csr objects, P/R
        None on the coarsest level), a hierarchy made of those operators.  ``interp``
        (RS / PMIS): INTERP_CLASSICAL or INTERP_EXT_I (``p_max`` entries kept per row)."""
        o = _Opt(coarsen, smoother, strong_threshold, jacobi_omega, pre_sweeps, post_sweeps,
                 max_levels, max_coarse, gs_block, seed, interp, p_max, drop_tol)
        self.A = A
        if levels is None:
            self.h = lib().orc_hier_setup(A.h, C.byref(o))
        else:
            n = len(levels)
            arr = lambda i: (C.c_void_p * n)(*[lv[i].h if lv[i] is not None else None
                                               for lv in levels])
            self._levels = levels
            self.h = lib().orc_hier_from_levels(n, arr(0), arr(1), arr(2), C.byref(o))
        if not self.h:
            raise RuntimeError("oracle setup failed")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_hier_free(self.h)
            self.h = None

    @property
    def num_levels(self):
        return lib().orc_hier_levels(self.h)

    def matrix(self, level, which):
        """which: 'A', 'P' or 'R'.  Returns a scipy CSR copy."""
        w = {"A": 0, "P": 1, "R": 2}[which]
        ptr = lib().orc_hier_matrix(self.h, level, w)
        if not ptr:
            return None
        tmp = Csr.__new__(Csr)
        tmp.h = ptr
        out = tmp.to_scipy()
        tmp.h = None  # borrowed
        return out

    def split(self, level):
        n = self.matrix(level, "A").shape[0]
        out = np.empty(n, np.int32)
        lib().orc_hier_split(self.h, level, _p(out, _i32p))
        return out

    def cycle(self, x, b):
        x = np.array(x, np.float64, copy=True)
        b = np.ascontiguousarray(b, np.float64)
        lib().orc_hier_cycle(self.h, _p(x, _f64p), _p(b, _f64p))
        return x

    def solve(self, x, b, max_iter=10, tol=0.0):
        x = np.array(x, np.float64, copy=True)
        b = np.ascontiguousarray(b, np.float64)
        hist = np.zeros(max_iter + 1)
        it = lib().orc_hier_solve(self.h, _p(x, _f64p), _p(b, _f64p), max_iter, tol,
                                  _p(hist, _f64p))
        return x, hist[: it + 1]

    def set_cuts(self, level, cuts):
        """Rank partition (start rows, cuts[0] = 0) of level ``level``: hybrid-GS blocks are
        clipped to it, as on the product's ranks."""
        c = np.ascontiguousarray(cuts, np.int64)
        lib().orc_hier_set_cuts(self.h, int(level), int(c.size), _p(c, _i64p))

    def pcg(self, x, b, max_iter=10, tol=0.0):
        x = np.array(x, np.float64, copy=True)
        b = np.ascontiguousarray(b, np.float64)
        hist = np.zeros(max_iter + 1)
        it = lib().orc_hier_pcg(self.h, _p(x, _f64p), _p(b, _f64p), max_iter, tol,
                                _p(hist, _f64p))
        return x, hist[: it + 1]
