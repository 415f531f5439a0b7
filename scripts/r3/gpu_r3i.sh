#!/bin/bash
# round-3 probe i: V-cycle rate after overlapped setup with device-built formats (batch h:
# 193 vs 751 V-cycles/s without overlap) -- repeat, stream probe, kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="--steps 30 --warmup 3 --no-cpu-baseline --spmv-reps 5"
for v in a b; do
  timeout -k 10 300 python bench.py $B > gpurun_out/r3i_ovl_$v.json 2> gpurun_out/r3i_ovl_$v.err || { tail -20 gpurun_out/r3i_ovl_$v.err; exit 1; }
done
AMG_FMT_STREAM=ctx timeout -k 10 300 python bench.py $B > gpurun_out/r3i_ctxstream.json 2> gpurun_out/r3i_ctxstream.err || { tail -20 gpurun_out/r3i_ctxstream.err; exit 1; }
timeout -k 10 300 python bench.py $B --no-graph > gpurun_out/r3i_nograph.json 2> gpurun_out/r3i_nograph.err || { tail -20 gpurun_out/r3i_nograph.err; exit 1; }
python - <<'PY'
import json
for f in ("r3i_ovl_a", "r3i_ovl_b", "r3i_ctxstream", "r3i_nograph"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], "setup_s", d["config"].get("setup_s"))
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3i_prof -o r3i -- python3 $GRAFT_REPO_ROOT/bench.py $B > $GRAFT_REPO_ROOT/gpurun_out/r3i_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3i_prof.log; exit 1; }
echo probe-ok
