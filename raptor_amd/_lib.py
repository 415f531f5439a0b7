"""ctypes declarations of the C-ABI in include/raptor_amd.h (libraptor_amd.so).

The library is built in-tree (``__graft_entry__.build()`` / ``make -C raptor_amd/csrc``).
Loading fails loudly when it is missing: there is no fallback path."""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
lib_path = os.environ.get("RAPTOR_AMD_LIB") or os.path.join(_HERE, "libraptor_amd.so")  # override: A/B builds

AMG_OK = 0
AMG_STENCIL_5PT, AMG_STENCIL_7PT, AMG_STENCIL_27PT = 0, 1, 2
AMG_COARSEN_RS, AMG_COARSEN_PMIS, AMG_COARSEN_SA = 0, 1, 2
AMG_SMOOTH_JACOBI, AMG_SMOOTH_HYBRID_GS = 0, 1
AMG_INTERP_CLASSICAL, AMG_INTERP_EXT_I = 0, 1
AMG_PRESET_PMIS_JACOBI, AMG_PRESET_RS_JACOBI, AMG_PRESET_SA_HYBRID_GS = 0, 1, 2
AMG_REORDER_RCM = 1
AMG_FORMAT_AUTO, AMG_FORMAT_CSR, AMG_FORMAT_BLOCKS = 0, 1, 2

ERROR_NAMES = {1: "INVALID", 2: "HIP", 3: "RCCL", 4: "COMM", 5: "INTERNAL", 6: "NOMEM"}


class AmgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"raptor_amd error {ERROR_NAMES.get(code, code)}: {msg}")
        self.code = code


class Options(C.Structure):
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
        ("setup_device", C.c_int32),
        ("replicate_below", C.c_int64),
        ("interp", C.c_int32),
        ("p_max", C.c_int32),
        ("drop_tol", C.c_double),
    ]


class MatrixInfo(C.Structure):
    _fields_ = [
        ("n_global_rows", C.c_int64),
        ("n_global_cols", C.c_int64),
        ("first_row", C.c_int64),
        ("n_local_rows", C.c_int64),
        ("first_col", C.c_int64),
        ("n_local_cols", C.c_int64),
        ("nnz_local", C.c_int64),
        ("n_halo", C.c_int64),
        ("n_send", C.c_int64),
        ("n_neighbors", C.c_int32),
        ("n_blocks", C.c_int32),
        ("n_vi_blocks", C.c_int32),
        ("spmv_bytes", C.c_int64),
        ("n_templates", C.c_int32),
        ("template_rows", C.c_int64),
        ("format", C.c_int32),
        ("kernel_variant", C.c_int32),
        ("csr_bytes", C.c_int64),
        ("tpl_window", C.c_int32),
        ("tpl_lanes", C.c_int32),
        ("tpl_march_shift", C.c_int32),
        ("mult_add_bytes", C.c_int64),
        ("residual_bytes", C.c_int64),
        ("jacobi_bytes", C.c_int64),
        ("gs_bytes", C.c_int64),
        ("tpl_master", C.c_int32),
        ("tile_line_bytes", C.c_int32),
        ("gs_split", C.c_int32),
        ("gs_chain_maxw", C.c_int32),
        ("deferred", C.c_int32),
    ]


class LevelInfo(C.Structure):
    _fields_ = [
        ("n_global", C.c_int64),
        ("nnz_global", C.c_int64),
        ("n_local", C.c_int64),
        ("nnz_local", C.c_int64),
        ("p_nnz_local", C.c_int64),
        ("r_nnz_local", C.c_int64),
        ("bytes_per_cycle_local", C.c_int64),
        ("stored_bytes_per_cycle_local", C.c_int64),
    ]


ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64), C.c_void_p,
                           C.POINTER(C.c_int64))

_vp = C.c_void_p
_i32, _i64, _f64 = C.c_int32, C.c_int64, C.c_double
_pi64 = C.POINTER(C.c_int64)
_pf64 = C.POINTER(C.c_double)

# name -> (restype, argtypes); every symbol declared in include/raptor_amd.h
SIGNATURES = {
    "amg_last_error": (C.c_char_p, []),
    "amg_version": (C.c_int, []),
    "amg_runtime_versions": (C.c_int, [C.POINTER(_i32), C.POINTER(_i32)]),
    "amg_context_create": (C.c_int, [C.c_int, _vp, C.POINTER(_vp)]),
    "amg_context_set_comm": (C.c_int, [_vp, C.c_int, C.c_int, _vp, ALLTOALLV_FN, _vp]),
    "amg_rccl_unique_id": (C.c_int, [_vp]),
    "amg_context_set_loopback": (C.c_int, [_vp, C.c_int, C.c_int, C.c_char_p]),
    "amg_context_stream": (C.c_int, [_vp, C.POINTER(_vp)]),
    "amg_context_synchronize": (C.c_int, [_vp]),
    "amg_context_destroy": (C.c_int, [_vp]),
    "amg_par_csr_create": (C.c_int, [_vp, _i64, _i64, _i64, _pi64, _pi64, _pf64, C.POINTER(_vp)]),
    "amg_par_stencil_create": (C.c_int, [_vp, C.c_int, _i64, _i64, _i64, _pf64, C.POINTER(_vp)]),
    "amg_par_stencil_create_boxes": (C.c_int, [_vp, C.c_int, _i64, _i64, _i64, _i64, _i64, _i64, _pf64,
                                               C.POINTER(_vp)]),
    "amg_host_csr_stencil": (C.c_int, [C.c_int, C.c_int, C.c_int, _i64, _i64, _i64, _i64, _i64, _i64, _pf64,
                                       C.POINTER(_vp)]),
    "amg_par_csr_info": (C.c_int, [_vp, C.POINTER(MatrixInfo)]),
    "amg_par_csr_export": (C.c_int, [_vp, _pi64, _pi64, _pf64]),
    "amg_par_csr_set_format": (C.c_int, [_vp, _i32]),
    "amg_par_csr_format_digest": (C.c_int, [_vp, C.POINTER(C.c_uint64)]),
    "amg_par_graph_laplacian_create": (C.c_int, [_vp, _i64, _i64, C.c_uint64, C.POINTER(_vp)]),
    "amg_par_csr_read": (C.c_int, [_vp, C.c_char_p, C.POINTER(_vp)]),
    "amg_par_csr_write": (C.c_int, [_vp, C.c_char_p]),
    "amg_par_csr_reorder": (C.c_int, [_vp, C.c_int, C.POINTER(_vp), _pi64]),
    "amg_par_csr_mult": (C.c_int, [_vp, _vp, _vp]),
    "amg_par_csr_mult_add": (C.c_int, [_vp, _vp, _vp]),
    "amg_par_csr_residual": (C.c_int, [_vp, _vp, _vp, _vp]),
    "amg_par_csr_jacobi": (C.c_int, [_vp, _vp, _vp, _vp, _f64]),
    "amg_par_csr_hybrid_gs": (C.c_int, [_vp, _vp, _vp, _vp, _i64]),
    "amg_par_csr_hybrid_gs_backward": (C.c_int, [_vp, _vp, _vp, _vp, _i64]),
    "amg_par_csr_residual_norm": (C.c_int, [_vp, _vp, _vp, _pf64]),
    "amg_par_csr_matmat": (C.c_int, [_vp, _vp, C.POINTER(_vp)]),
    "amg_par_csr_destroy": (C.c_int, [_vp]),
    "amg_options_default": (C.c_int, [C.c_int, C.POINTER(Options)]),
    "amg_solver_setup": (C.c_int, [_vp, C.POINTER(Options), C.POINTER(_vp)]),
    "amg_solver_num_levels": (C.c_int, [_vp, C.POINTER(_i32)]),
    "amg_solver_level_info": (C.c_int, [_vp, _i32, C.POINTER(LevelInfo)]),
    "amg_solver_level_matrix": (C.c_int, [_vp, _i32, _i32, C.POINTER(_vp)]),
    "amg_solver_level_split": (C.c_int, [_vp, _i32, C.POINTER(_i32)]),
    "amg_solver_cycle": (C.c_int, [_vp, _vp, _vp]),
    "amg_solver_solve": (C.c_int, [_vp, _vp, _vp, _i32, _f64, _pf64, C.POINTER(_i32)]),
    "amg_solver_pcg": (C.c_int, [_vp, _vp, _vp, _i32, _f64, _pf64, C.POINTER(_i32)]),
    "amg_solver_set_graph": (C.c_int, [_vp, _i32]),
    "amg_solver_get_graph": (C.c_int, [_vp, C.POINTER(_i32)]),
    "amg_solver_cycle_timeline": (C.c_int, [_vp, _vp, _vp, _i32, _i32, C.POINTER(C.c_double), C.c_char_p, _i32,
                                            C.POINTER(_i32), C.POINTER(_i32)]),
    "amg_solver_destroy": (C.c_int, [_vp]),
    "amg_vector_uniform": (C.c_int, [_vp, _i64, _i64, C.c_uint64, _vp]),
    "amg_vector_copy": (C.c_int, [_vp, _i64, _vp, _vp]),
    "amg_vector_read": (C.c_int, [_vp, _i64, _vp, _vp, _i64]),
    "amg_device_malloc": (C.c_int, [_vp, _i64, C.POINTER(_vp)]),
    "amg_device_free": (C.c_int, [_vp, _vp]),
    "amg_memcpy": (C.c_int, [_vp, _vp, _vp, _i64]),
    "amg_memset_async": (C.c_int, [_vp, _vp, C.c_int, _i64]),
    "amg_event_create": (C.c_int, [_vp, C.POINTER(_vp)]),
    "amg_event_record": (C.c_int, [_vp]),
    "amg_event_elapsed_ms": (C.c_int, [_vp, _vp, C.POINTER(C.c_float)]),
    "amg_event_destroy": (C.c_int, [_vp]),
    "amg_host_hierarchy_build": (C.c_int, [C.c_int, C.c_int, ALLTOALLV_FN, _vp, _i64, _i64, _i64,
                                           _pi64, _pi64, _pf64, C.POINTER(Options),
                                           C.POINTER(_vp)]),
    "amg_host_hierarchy_num_levels": (C.c_int, [_vp, C.POINTER(_i32)]),
    "amg_host_hierarchy_level_size": (C.c_int, [_vp, _i32, _i32, _pi64]),
    "amg_host_hierarchy_level_export": (C.c_int, [_vp, _i32, _i32, _pi64, _pi64, _pf64]),
    "amg_host_hierarchy_level_split": (C.c_int, [_vp, _i32, C.POINTER(_i32)]),
    "amg_host_hierarchy_coarse_inverse": (C.c_int, [_vp, _pf64]),
    "amg_host_hierarchy_destroy": (C.c_int, [_vp]),
    "amg_host_csr_graph_laplacian": (C.c_int, [C.c_int, C.c_int, _i64, _i64, C.c_uint64, C.POINTER(_vp)]),
    "amg_host_csr_read": (C.c_int, [C.c_int, C.c_int, C.c_char_p, C.POINTER(_vp)]),
    "amg_host_csr_write": (C.c_int, [C.c_int, C.c_int, ALLTOALLV_FN, _vp, _vp, C.c_char_p]),
    "amg_host_csr_reorder": (C.c_int, [C.c_int, C.c_int, ALLTOALLV_FN, _vp, _vp, C.c_int, C.POINTER(_vp),
                                       _pi64]),
    "amg_host_csr_size": (C.c_int, [_vp, _pi64]),
    "amg_host_csr_export": (C.c_int, [_vp, _pi64, _pi64, _pf64]),
    "amg_host_csr_destroy": (C.c_int, [_vp]),
}

_lib = None


def lib():
    """Load libraptor_amd.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(lib_path):
            raise ImportError(
                f"{lib_path} not found: build it with `python -c 'import __graft_entry__ as g; "
                "g.build()'` (hipcc --offload-arch=gfx950); raptor_amd has no fallback path")
        L = C.CDLL(lib_path)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int):
    if rc != AMG_OK:
        msg = lib().amg_last_error()
        raise AmgError(rc, msg.decode() if msg else "")
