#!/bin/bash
# round-3 batch f: GPU suite (RCCL graph policy, overlapped format builds, device-resident A*P),
# setup timing with the format builds overlapped and not (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1 || { tail -40 gpurun_out/r3f_tests.log; exit 1; }
tail -3 gpurun_out/r3f_tests.log
AMG_TIMING=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3f_7pt.json 2> gpurun_out/r3f_7pt.err || { tail -20 gpurun_out/r3f_7pt.err; exit 1; }
AMG_SETUP_OVERLAP=0 AMG_TIMING=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3f_7pt_noovl.json 2> gpurun_out/r3f_7pt_noovl.err || { tail -20 gpurun_out/r3f_7pt_noovl.err; exit 1; }
python - <<'PY'
import json
for f in ("r3f_7pt", "r3f_7pt_noovl"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], "setup_s", d["config"].get("setup_s"))
PY
echo batch-ok
