"""The C-ABI library loads and exports every symbol include/raptor_amd.h declares; the
Python mirror binds all of them; without a GPU the product refuses to run (no fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "raptor_amd.h")).read()
    return sorted(set(re.findall(r"\b(amg_[a-z0-9_]+)\s*\(", txt)) - {"amg_alltoallv_fn"})


def test_library_exports_every_declared_symbol():
    from raptor_amd import _lib

    L = ctypes.CDLL(_lib.lib_path)
    syms = header_symbols()
    assert len(syms) >= 35
    missing = [s for s in syms if not hasattr(L, s)]
    assert missing == []
    assert sorted(_lib.SIGNATURES) == syms  # the Python mirror binds exactly the header


def test_version_and_error_string():
    from raptor_amd import _lib

    L = _lib.lib()
    assert L.amg_version() == 100
    opt = _lib.Options()
    assert L.amg_options_default(99, ctypes.byref(opt)) == 1  # AMG_ERR_INVALID
    assert b"preset" in L.amg_last_error()
    assert L.amg_options_default(0, ctypes.byref(opt)) == 0
    assert opt.coarsen == 1 and abs(opt.jacobi_omega - 2.0 / 3.0) < 1e-16


def test_no_gpu_means_loud_failure():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import raptor_amd as ra

    with pytest.raises(RuntimeError):
        ra.Context(0)


def test_oracle_is_not_linked_by_the_product():
    import subprocess

    from raptor_amd import _lib

    out = subprocess.run(["ldd", _lib.lib_path], capture_output=True, text=True).stdout
    assert "oracle" not in out
    pat = re.compile(r"^\s*(from\s+oracle|import\s+oracle)|liboracle|amg_oracle\.h|orc_[a-z_]+\(",
                     re.M)
    for d in ("raptor_amd", os.path.join("raptor_amd", "csrc")):
        for f in os.listdir(os.path.join(ROOT, d)):
            if f.endswith((".py", ".cpp", ".hip", ".hpp", "Makefile")):
                src = open(os.path.join(ROOT, d, f)).read()
                assert not pat.search(src), f
