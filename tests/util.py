"""Test helpers: host<->device copies on the context stream, oracle conversions."""
import numpy as np


def to_dev(ctx, a):
    import torch

    with torch.cuda.stream(ctx.stream):
        t = torch.from_numpy(np.ascontiguousarray(a, np.float64)).to(ctx.torch_device, non_blocking=False)
    ctx.stream.synchronize()
    return t


def to_host(ctx, t):
    ctx.synchronize()
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
