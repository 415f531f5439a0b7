#!/bin/bash
# Round 3 probe u: split hybrid-GS sweeps (KM_GSACC block pass + chain walk) --
# the GS kernel-path tests, then same-box A/B: split (default, >= 16384 rows) vs one-kernel
# sliced ELL (AMG_GS_SPLIT=0) vs split on every level (AMG_GS_SPLIT_MIN=0) on sa27 and g3sub
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernel_paths.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "hybrid_gs or sa_gs or sa_restriction or sa27_npl16" > gpurun_out/r3u_tests.log 2>&1 || { tail -40 gpurun_out/r3u_tests.log; exit 1; }
tail -2 gpurun_out/r3u_tests.log
ROUND=r3u VARIANTS="split:;ell:AMG_GS_SPLIT=0;splitall:AMG_GS_SPLIT_MIN=0" CONFIGS="g3sub sa27" bash scripts/gpu_envab.sh
