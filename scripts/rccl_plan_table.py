"""Per-level RCCL plan of one V-cycle on N ranks, from the real halo plans.

    python scripts/rccl_plan_table.py [7pt|sa27|g3sub] [N] [nx ny nz] [bx by bz]

Builds the hierarchy the bench runs at --gpus N (default: 7-pt 512^3 on 2 x 2 x 2 boxes, 8
ranks) with N in-process loopback ranks on this GPU -- the same halo plans, replication
decision and setup code as N RCCL processes -- and reads every level operator's plan (peers,
halo entries received, entries sent; amg_matrix_info).  Per cycle the halo
exchanges are:
  Jacobi cycle: level 0 -- pre-Jacobi (+ norm), residual, post-Jacobi on A_0; levels >= 1 --
  residual and post-Jacobi on A_l (the first sweep from x = 0 needs no halo); every level --
  R_l r and P_l e;
  hybrid-GS cycle: forward and backward sweep plus the residual on A_l, R_l r, P_l e.
One exchange = one ncclGroupStart/End with a send and a receive per peer.  Replicated levels
(<= replicate_below global rows) exchange nothing; the cycle then allgathers the padded
restricted residual once, and the norm allgathers one double per rank.  Prints one JSON object
(per level, per rank min / max) and a markdown table on stderr."""
import json
import os
import sys
import threading
import uuid

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import raptor_amd as ra  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "7pt"
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dims = tuple(int(v) for v in sys.argv[3:6]) if len(sys.argv) > 5 else (512, 512, 512)
    boxes = tuple(int(v) for v in sys.argv[6:9]) if len(sys.argv) > 8 else (2, 2, 2)
    world = "plan-" + uuid.uuid4().hex
    res = [None] * N
    errs = []

    def rank(r):
        try:
            c = ra.Context.loopback(r, N, world, native=True)
            if cfg == "g3sub":
                A = ra.par_graph_laplacian(c, 1225, 1225, seed=1)
                A, _ = A.reorder("rcm")
                ml = ra.ParSmoothedAggregationSolver().setup(A)
            elif cfg == "sa27":
                A = ra.par_stencil_grid(c, "27pt", dims, boxes=boxes)
                ml = ra.ParSmoothedAggregationSolver().setup(A)
            else:
                A = ra.par_stencil_grid(c, "7pt", dims, boxes=boxes)
                ml = ra.ParRugeStubenSolver(coarsen="pmis").setup(A)
            out = []
            for l in range(ml.num_levels):
                li = ml.level_info(l)
                e = {"level": l, "n_global": li["n_global"], "nnz_global": li["nnz_global"],
                     "n_local": li["n_local"], "replicated": li["n_local"] == li["n_global"] and N > 1}
                for w in "APR":
                    if w != "A" and l == ml.num_levels - 1:
                        continue
                    inf = ml.level_matrix(l, w + "_cycle").info  # the operators the cycle runs
                    e[w] = {"peers": inf["n_neighbors"], "recv": inf["n_halo"], "send": inf["n_send"]}
                out.append(e)
            res[r] = out
            del ml, A
        except BaseException as ex:  # noqa: BLE001
            errs.append((r, ex))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(N)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0][1]
    gs = cfg in ("sa27", "g3sub")
    nlev = len(res[0])
    table = []
    tot = {"groups": 0, "msgs_max": 0, "bytes_max": 0}
    for l in range(nlev):
        row = {k: res[0][l][k] for k in ("level", "n_global", "nnz_global", "replicated")}
        # halo applications per cycle of each operator (module docstring)
        apps = {"A": (3 if gs else (3 if l == 0 else 2)), "P": 1, "R": 1}
        if l == nlev - 1:
            apps = {"A": 0}
        for w, k in apps.items():
            peers = [r[l][w]["peers"] for r in res]
            send = [r[l][w]["send"] for r in res]
            recv = [r[l][w]["recv"] for r in res]
            active = k if max(peers) > 0 else 0
            row[w] = {"per_cycle": active, "peers_min": min(peers), "peers_max": max(peers),
                      "send_bytes_max": 8 * max(send), "recv_bytes_max": 8 * max(recv)}
            tot["groups"] += active
            tot["msgs_max"] += active * 2 * max(peers)
            tot["bytes_max"] += active * 8 * max(send)
        table.append(row)
    rep = [t["level"] for t in table if t["replicated"]]
    out = {"config": cfg, "ranks": N, "dims": dims, "boxes": boxes, "levels": table,
           "per_cycle": dict(tot, replicated_from_level=rep[0] if rep else None,
                             allgathers=(1 if rep else 0) + 1 + 1,
                             what="groups: ncclGroupStart/End halo exchanges; msgs_max / bytes_max: "
                                  "sends + receives / bytes sent by the busiest rank, summed over "
                                  "exchanges; allgathers: replicated-tail b (if any) + coarse b + "
                                  "the norm")}
    print(json.dumps(out))
    print(f"| level | rows | op | per cycle | peers | sent / exchange (max rank) | received |", file=sys.stderr)
    print("|---|---|---|---|---|---|---|", file=sys.stderr)
    for t in table:
        for w in "APR":
            if w in t:
                v = t[w]
                print(f"| {t['level']}{' (repl.)' if t['replicated'] else ''} | {t['n_global']} | {w} | "
                      f"{v['per_cycle']} | {v['peers_min']}-{v['peers_max']} | "
                      f"{v['send_bytes_max'] / 1e6:.3f} MB | {v['recv_bytes_max'] / 1e6:.3f} MB |", file=sys.stderr)
    print(f"per cycle: {tot['groups']} exchanges, busiest rank {tot['msgs_max']} messages, "
          f"{tot['bytes_max'] / 1e6:.2f} MB sent", file=sys.stderr)


if __name__ == "__main__":
    main()
