#!/bin/bash
# round-3 batch: GPU tests (not the 512^3 one), setup timing, slab benches, per-kernel PMC
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r3b_tests.log 2>&1 || { tail -30 gpurun_out/r3b_tests.log; exit 1; }
tail -3 gpurun_out/r3b_tests.log
AMG_TIMING=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3b_7pt.json 2> gpurun_out/r3b_7pt.err || exit 1
timeout -k 10 300 python bench.py --grid 512,512,64 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3b_512x512x64.json 2> gpurun_out/r3b_512x512x64.err || exit 1
timeout -k 10 300 python bench.py --grid 256,256,512 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/r3b_256x256x512.json 2> gpurun_out/r3b_256x256x512.err || exit 1
ROUND=r3b bash scripts/gpu_pmc_vcycle.sh > gpurun_out/r3b_pmc.log 2>&1 || { tail gpurun_out/r3b_pmc.log; exit 1; }
echo batch-ok
