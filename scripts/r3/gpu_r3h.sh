#!/bin/bash
# round-3 batch h: device-built formats (formats.hip) -- the GPU suite incl. the byte-identity
# test against the host builders, setup timing (device formats on / off), then the 512^3 test
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r3h_tests.log 2>&1 || { tail -40 gpurun_out/r3h_tests.log; exit 1; }
tail -3 gpurun_out/r3h_tests.log
AMG_TIMING=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3h_7pt.json 2> gpurun_out/r3h_7pt.err || { tail -20 gpurun_out/r3h_7pt.err; exit 1; }
AMG_DEVICE_FORMATS=0 AMG_TIMING=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3h_7pt_hostfmt.json 2> gpurun_out/r3h_7pt_hostfmt.err || { tail -20 gpurun_out/r3h_7pt_hostfmt.err; exit 1; }
AMG_SETUP_OVERLAP=0 AMG_TIMING=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3h_7pt_noovl.json 2> gpurun_out/r3h_7pt_noovl.err || { tail -20 gpurun_out/r3h_7pt_noovl.err; exit 1; }
python - <<'PY'
import json
for f in ("r3h_7pt", "r3h_7pt_hostfmt", "r3h_7pt_noovl"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], "setup_s", d["config"].get("setup_s"))
PY
AMG_TEST_REPORT_DIR=gpurun_out timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_gpu_zfull_512.py > gpurun_out/r3h_512.log 2>&1 || { tail -40 gpurun_out/r3h_512.log; exit 1; }
tail -6 gpurun_out/r3h_512.log
echo batch-ok
