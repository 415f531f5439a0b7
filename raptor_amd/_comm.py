"""Setup-time host exchange for multi-rank runs: the ``amg_alltoallv_fn`` callback of the
C-ABI implemented with ``torch.distributed.all_to_all_single`` on a gloo group.

Only the AMG setup (halo plans, ghost rows, coarse numbering) goes
through here.  The solve-time halo exchange is RCCL inside libraptor_amd.so."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import ALLTOALLV_FN


def make_exchange(group, nranks: int):
    import torch
    import torch.distributed as dist

    def _cb(user, send, sbytes, recv, rbytes):
        try:
            sb = [int(sbytes[r]) for r in range(nranks)]
            rb = [int(rbytes[r]) for r in range(nranks)]
            st, rt = sum(sb), sum(rb)
            if st:
                src = np.ctypeslib.as_array(C.cast(send, C.POINTER(C.c_uint8)), shape=(st,))
                inp = torch.from_numpy(src.copy())
            else:
                inp = torch.empty(0, dtype=torch.uint8)
            out = torch.empty(rt, dtype=torch.uint8)
            dist.all_to_all_single(out, inp, rb, sb, group=group)
            if rt:
                dst = np.ctypeslib.as_array(C.cast(recv, C.POINTER(C.c_uint8)), shape=(rt,))
                dst[:] = out.numpy()
            return 0
        except Exception as e:  # never let an exception unwind through C
            import sys

            print(f"raptor_amd exchange failed: {e!r}", file=sys.stderr)
            return 1

    return ALLTOALLV_FN(_cb)
