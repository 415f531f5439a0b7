#!/bin/bash
# round-3 probe l: same-box A/B of the round-2 end tree (_r2tree, commit 612f21f, built here)
# against the current tree, the driver's bench command, alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="--steps 20 --warmup 5 --no-cpu-baseline"
for v in 1 2; do
  timeout -k 10 300 python bench.py $B > gpurun_out/r3l_cur_$v.json 2> gpurun_out/r3l_cur_$v.err || { tail -20 gpurun_out/r3l_cur_$v.err; exit 1; }
  (cd _r2tree && timeout -k 10 300 python bench.py $B > ../gpurun_out/r3l_r2_$v.json 2> ../gpurun_out/r3l_r2_$v.err) || { tail -20 gpurun_out/r3l_r2_$v.err; exit 1; }
done
python - <<'PY'
import json
for f in ("r3l_cur_1", "r3l_r2_1", "r3l_cur_2", "r3l_r2_2"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    k = {r["level"]: 0 for r in d.get("vcycle_kernels", [])}
    print(f, d["value"], d["ms_per_step"], "setup", d["config"].get("setup_s"), "csr", d["roofline"]["avg_launch_ms"],
          " ".join(f"L{r['level']}:{r['op'][:5]}={r['us']}" for r in d.get("vcycle_kernels", [])[:12]))
PY
echo probe-ok
