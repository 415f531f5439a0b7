#!/bin/bash
# Round 3 probe m: uniform-stencil template rows (variant bit 512) -- the template / GS
# kernel-path tests against the oracle, then same-box A/B against the per-template tables
# (AMG_TPL_MASTER=0) on sa27 and 7-pt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernel_paths.py -x -v --timeout 240 --timeout-method thread \
  -k "template or gs or sa27_npl16 or vcycle_paths" > gpurun_out/r3m_tests.log 2>&1 || { tail -30 gpurun_out/r3m_tests.log; exit 1; }
tail -3 gpurun_out/r3m_tests.log
ROUND=r3m VARIANTS="master:;generic:AMG_TPL_MASTER=0;master2:" CONFIGS="sa27 7pt" bash scripts/gpu_envab.sh
