"""Modelled N = 8 cycle time of configs[3] (7-pt 512^3, 2x2x2 boxes) per coarse-level policy
(VERDICT r5 "next" 6).  Inputs, both measured:

  * the per-rank halo plans of every level of the 512^3 / 8-rank hierarchy
    (scripts/rccl_plan_table.py 7pt 8 -> profiles/r5/r5c_rccl_plan_7pt_512_8ranks.json):
    exchanges per cycle, peers and the busiest rank's bytes per exchange;
  * the in-graph time of every operation of the 1-GPU 256^3 cycle (bench.py cycle_timeline):
    one rank of 512^3 / 8 holds a 256^3 box, and its level-l share has the rows of the 256^3
    hierarchy's level l (profiles/r5/r5c: 5.14 M vs 5.16 M rows on level 1, 1.08 M vs 1.09 M on
    level 2), so the distributed level-l work per rank is the 1-GPU level-l time.

Model per level and cycle (distributed): t = compute_l + e_l * (alpha + bytes_l / beta) for the
exchanges that cannot hide (coarse levels: the interior rows finish before the halo arrives);
levels 0-2 overlap the exchange with the interior rows, so only max(0, exchange
- interior) is added there.  A replicated level costs the whole level's compute on every rank:
the 1-GPU time of the 256^3 level of the same row count (coarse levels are launch-latency
bound), no exchange, plus one allgather of the level's right-hand side at the transition.
Every policy adds the coarse allgather and the norm allreduce (2 alpha).  alpha = latency of
one grouped RCCL send/recv round over xGMI (10 and 20 us bracket it), beta = 50 GB/s per peer
(a third of one xGMI link).  Levels the measured plan replicated get, distributed, the four
exchanges of the level above with few-KB messages.

usage: python scripts/r6/comm_model.py PLAN.json BENCH_7PT.json
"""
import json
import math
import re
import sys

BETA = 50e3  # bytes per us per peer


def level_compute(bench):
    """{level: us per cycle} from the bench's in-graph timeline (cycle_timeline.ops)."""
    t = {}
    for op in bench["cycle_timeline"]["ops"]:
        m = re.match(r"L(\d+) ", op["op"])
        t[int(m.group(1))] = t.get(int(m.group(1)), 0.0) + op["us"]
    return t


def matched(comp, rows1, n):
    """1-GPU time of the 256^3 level whose row count is nearest n (log scale): a replicated
    512^3 level is the whole level on one GPU, and the coarse levels are launch-latency
    bound, so its cost follows the level of the same size, not 8 x the same index."""
    k = min(rows1, key=lambda q: abs(math.log(max(1, rows1[q]) / max(1, n))))
    return comp.get(k, 0.0)


def model(plan, comp, rep_level, alpha, rows1, overlap_levels=3):
    # every policy: the coarsest level's allgather of b and the norm's allreduce
    total = 2 * alpha
    rows = []
    for L in plan["levels"]:
        l = L["level"]
        c1 = comp.get(l, 0.0)
        if rep_level is not None and l >= rep_level:
            t = matched(comp, rows1, L["n_global"])
            ex = 0.0
            if l == rep_level:  # the transition's allgather of b_l (padded slots)
                ex = alpha + 8.0 * L["n_global"] / 8 / BETA
            rows.append((l, L["n_global"], "replicated", round(t, 1), round(ex, 1)))
            total += t + ex
            continue
        ex = 0.0
        if L.get("replicated"):
            # replicated in the measured plan: distributed, it would post the exchanges of the
            # level above (2 for A, 1 for P, 1 for R) with messages of a few KB
            ex = 4 * (alpha + 4096 / BETA)
        for w in "APR":
            e = L.get(w)
            if not e or not e["per_cycle"]:
                continue
            one = alpha + max(e["send_bytes_max"], e["recv_bytes_max"]) / max(1, e["peers_max"]) / BETA
            ex += e["per_cycle"] * one
        hidden = min(ex, 0.5 * c1) if l < overlap_levels else 0.0  # interior rows ~ half the op time
        t = c1 + ex - hidden
        rows.append((l, L["n_global"], "distributed", round(c1, 1), round(ex - hidden, 1)))
        total += t
    return total, rows


def main(plan_path, bench_path):
    plan = json.load(open(plan_path))
    bench = json.load(open(bench_path))
    comp = level_compute(bench)
    rows1 = dict(enumerate(bench["config"]["level_rows"]))
    t1 = bench["cycle_timeline"]["sum_us"]
    levels = {L["level"]: L["n_global"] for L in plan["levels"]}
    print(f"1-GPU 256^3 cycle (in-graph timeline): {t1:.0f} us")
    print("| policy | replicated from | alpha us | modelled N=8 cycle us | efficiency |")
    print("|---|---|---|---|---|")
    for name, thr in [("distributed to the coarsest", 0), ("replicate_below 65,536 (default)", 65536),
                      ("replicate_below 262,144", 262144), ("replicate_below 2,097,152", 2097152)]:
        rep = None
        if thr:
            rep = min((l for l, n in levels.items() if l > 0 and n <= thr), default=None)
        for alpha in (10.0, 20.0):
            t, _ = model(plan, comp, rep, alpha, rows1)
            print(f"| {name} | {'level ' + str(rep) if rep is not None else '-'} | {alpha:.0f} | {t:.0f} | {t1 / t:.2f} |")
    t, rows = model(plan, comp, min(l for l, n in levels.items() if l > 0 and n <= 65536), 15.0, rows1)
    print("\nper level at alpha = 15 us, default policy (level, rows, kind, compute us, exposed exchange us):")
    for r in rows:
        print(" ", r)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
