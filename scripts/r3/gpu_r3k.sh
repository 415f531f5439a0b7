#!/bin/bash
# round-3 batch k: the sa27 and g3sub configs with the round-3 setup (device formats, staged
# copies, overlap), setup phase timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in sa27 g3sub; do
  AMG_TIMING=1 timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3k_$cfg.json 2> gpurun_out/r3k_$cfg.err || { tail -20 gpurun_out/r3k_$cfg.err; exit 1; }
done
python - <<'PY'
import json
for f in ("r3k_sa27", "r3k_g3sub"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], "setup_s", d["config"].get("setup_s"))
PY
echo batch-ok
