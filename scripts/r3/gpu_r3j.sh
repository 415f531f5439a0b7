#!/bin/bash
# round-3 probe j: V-cycle rate after the overlapped setup with KMP_BLOCKTIME=0 (library default)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="--steps 30 --warmup 3 --no-cpu-baseline --spmv-reps 5"
for v in a b c; do
  timeout -k 10 300 python bench.py $B > gpurun_out/r3j_$v.json 2> gpurun_out/r3j_$v.err || { tail -20 gpurun_out/r3j_$v.err; exit 1; }
done
python - <<'PY'
import json
for f in ("r3j_a", "r3j_b", "r3j_c"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], "setup_s", d["config"].get("setup_s"))
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3j_prof -o r3j -- python3 $GRAFT_REPO_ROOT/bench.py $B > $GRAFT_REPO_ROOT/gpurun_out/r3j_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3j_prof.log; exit 1; }
echo probe-ok
