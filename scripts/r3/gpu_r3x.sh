#!/bin/bash
# Round 3 probe x: chain walk of the split GS sweep from a per-lane LDS queue (gs_chain_kernel)
# -- the GS kernel-path tests, then sa27 / g3sub bench lines (default, and AMG_GS_SPLIT=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernel_paths.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "hybrid_gs or sa_gs or sa_restriction or sa27_npl16" > gpurun_out/r3x_tests.log 2>&1 || { tail -40 gpurun_out/r3x_tests.log; exit 1; }
tail -2 gpurun_out/r3x_tests.log
ROUND=r3x VARIANTS="lds:;ell:AMG_GS_SPLIT=0" CONFIGS="g3sub sa27" bash scripts/gpu_envab.sh
