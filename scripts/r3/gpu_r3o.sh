#!/bin/bash
# Round 3 probe o: uniform-stencil rows with split per-row LDS reads (ds_read_b64, not
# ds_read2st64_b64) -- kernel-path tests; then same-box A/B: sa27 / 7-pt default, and the block
# kernels' row sums as single ds_read_b64 (libraptor_amd_alt.so, AMG_ROWSUM_SPLIT=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernel_paths.py -x -v --timeout 240 --timeout-method thread \
  -k "template or gs or sa27_npl16 or vcycle_paths" > gpurun_out/r3o_tests.log 2>&1 || { tail -30 gpurun_out/r3o_tests.log; exit 1; }
tail -2 gpurun_out/r3o_tests.log
ALT="RAPTOR_AMD_LIB=$GRAFT_REPO_ROOT/raptor_amd/libraptor_amd_alt.so"
ROUND=r3o VARIANTS="def:;split:$ALT;def2:;split2:$ALT" CONFIGS="7pt sa27" bash scripts/gpu_envab.sh
