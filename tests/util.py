"""Test helpers: host<->device copies on the context stream, oracle conversions, contexts.

AMG_TEST_NATIVE=1 runs the GPU tests on torch-free contexts (raptor_amd.Context.native):
device buffers and copies go through the C-ABI, so the library binds the ROCm HIP runtime
and RCCL it was built against -- the runtime bench.py times -- instead of torch's bundled
copies (tests/test_gpu_native_runtime.py runs the bit-exact suite that way)."""
import os

import numpy as np


def native_mode() -> bool:
    return os.environ.get("AMG_TEST_NATIVE") == "1"


def make_ctx(device=0):
    """A context of the suite's mode (torch stream, or native)."""
    import raptor_amd as ra

    return ra.Context.native(device) if native_mode() else ra.Context(device)


def loopback_ctx(rank, nranks, world, device=0):
    import raptor_amd as ra

    return ra.Context.loopback(rank, nranks, world, device, native=native_mode())


def to_dev(ctx, a):
    a = np.ascontiguousarray(a, np.float64)
    if getattr(ctx, "is_native", False):
        import raptor_amd as ra

        return ra.DeviceVector(ctx, a.size).copy_from(a)
    import torch

    with torch.cuda.stream(ctx.stream):
        t = torch.from_numpy(a).to(ctx.torch_device, non_blocking=False)
    ctx.stream.synchronize()
    return t


def to_host(ctx, t):
    ctx.synchronize()
    if getattr(ctx, "is_native", False):
        return t.numpy()
    return t.detach().cpu().numpy().copy()


def oracle_levels(O, ml):
    """Oracle Csr triples (A_l, P_l, R_l) exported from a product hierarchy (1 rank)."""
    levels = []
    for l in range(ml.num_levels):
        mats = []
        for w in "APR":
            if w != "A" and l == ml.num_levels - 1:
                mats.append(None)
                continue
            M = ml.level_matrix(l, w)
            rp, col, val = M.export()
            mats.append(O.Csr.from_arrays(rp.size - 1, M.info["n_global_cols"], rp, col, val))
        levels.append(tuple(mats))
    return levels


def same_csr(a, b):
    a = a.tocsr()
    b = b.tocsr()
    return (a.shape == b.shape and np.array_equal(a.indptr, b.indptr)
            and np.array_equal(a.indices, b.indices) and np.array_equal(a.data, b.data))
