"""Setup wall time and phase timers (AMG_TIMING=1) of the 7-pt PMIS hierarchy on 1 rank and on
N loopback ranks (threads sharing this GPU), for SURVEY.md 8f row f1.

    AMG_TIMING=1 python scripts/setup_ranks.py 256 8 [boxes]

Prints one JSON line: setup seconds per rank count.  The phase timers go to stderr (rank 0)."""
import json
import os
import sys
import threading
import time
import uuid

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import raptor_amd as ra  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    boxes = (2, 2, 2) if (len(sys.argv) > 3 and sys.argv[3] == "boxes") else None
    dims = (n, n, n)
    out = {"dims": dims, "ranks": N, "boxes": boxes}
    ctx = ra.Context(0)
    A = ra.par_stencil_grid(ctx, "7pt", dims, boxes=boxes)
    t = time.perf_counter()
    ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
    out["setup_1rank_s"] = time.perf_counter() - t
    out["levels"] = ml.num_levels
    print(f"[setup_ranks] 1 rank {out['setup_1rank_s']:.2f}s", file=sys.stderr, flush=True)
    del ml, A
    world = "sr-" + uuid.uuid4().hex
    st = [None] * N
    errs = []

    def rank(r):
        try:
            c = ra.Context.loopback(r, N, world)
            Ar = ra.par_stencil_grid(c, "7pt", dims, boxes=boxes)
            t0 = time.perf_counter()
            mr = ra.ParRugeStubenSolver(coarsen="pmis").setup(Ar)
            st[r] = time.perf_counter() - t0
            del mr, Ar
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=rank, args=(r,)) for r in range(N)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=900)
    if errs:
        raise errs[0]
    out[f"setup_{N}rank_s"] = max(st)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
