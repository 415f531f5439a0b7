#!/bin/bash
# round-3 batch g: GPU suite with staged host<->device copies; setup timing A/B
# (staged copies on / off) for 7-pt 256^3
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r3g_tests.log 2>&1 || { tail -40 gpurun_out/r3g_tests.log; exit 1; }
tail -3 gpurun_out/r3g_tests.log
AMG_TIMING=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3g_7pt.json 2> gpurun_out/r3g_7pt.err || { tail -20 gpurun_out/r3g_7pt.err; exit 1; }
AMG_STAGED_COPY=0 AMG_TIMING=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3g_7pt_nostage.json 2> gpurun_out/r3g_7pt_nostage.err || { tail -20 gpurun_out/r3g_7pt_nostage.err; exit 1; }
AMG_SETUP_OVERLAP=0 AMG_TIMING=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3g_7pt_noovl.json 2> gpurun_out/r3g_7pt_noovl.err || { tail -20 gpurun_out/r3g_7pt_noovl.err; exit 1; }
python - <<'PY'
import json
for f in ("r3g_7pt", "r3g_7pt_nostage", "r3g_7pt_noovl"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], "setup_s", d["config"].get("setup_s"))
PY
echo batch-ok
