#!/bin/bash
# Round 3 probe r: plain-CSR kernel with the near-diagonal x window in LDS (AMG_PLAIN_XWIN=256)
# -- plain-CSR format tests (bit-exact vs oracle), TA counters, then same-box A/B against the
# gather-only kernel (libraptor_amd_alt.so, AMG_PLAIN_XWIN=0) on the 7-pt bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_paths.py tests/test_gpu_multirank.py tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread \
  -k "formats_bit_exact or plain or csr" > gpurun_out/r3r_tests.log 2>&1 || { tail -40 gpurun_out/r3r_tests.log; exit 1; }
tail -2 gpurun_out/r3r_tests.log
TAG=r3r_pmc_win bash scripts/gpu_plain_pmc_ta.sh || exit 1
ALT="RAPTOR_AMD_LIB=$GRAFT_REPO_ROOT/raptor_amd/libraptor_amd_alt.so"
ROUND=r3r VARIANTS="win:;gather:$ALT;win2:;gather2:$ALT" CONFIGS="7pt" bash scripts/gpu_envab.sh
