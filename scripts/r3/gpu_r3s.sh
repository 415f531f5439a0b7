#!/bin/bash
# Round 3 probe s: 32-byte x-tile lines (512 per tile; AMG_TILE_LINE=4, the new default) --
# the whole -m gpu suite except the 512^3 test, then same-box A/B against 64-byte lines
# (libraptor_amd_alt.so, AMG_TILE_LINE=8) on 7-pt, sa27 and g3sub
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_zfull_512.py > gpurun_out/r3s_tests.log 2>&1 || { tail -40 gpurun_out/r3s_tests.log; exit 1; }
tail -2 gpurun_out/r3s_tests.log
ALT="RAPTOR_AMD_LIB=$GRAFT_REPO_ROOT/raptor_amd/libraptor_amd_alt.so"
ROUND=r3s VARIANTS="half:;full:$ALT;half2:;full2:$ALT" CONFIGS="7pt" bash scripts/gpu_envab.sh || exit 1
ROUND=r3s VARIANTS="half:;full:$ALT" CONFIGS="sa27 g3sub" bash scripts/gpu_envab.sh
