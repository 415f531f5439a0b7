#!/bin/bash
# Round 3 probe t: x-tile line width chosen per operator (32 B where it cuts >= 10 % of the
# row blocks, else 64 B) -- the -m gpu suite except the 512^3 test, then same-box A/B: auto vs
# AMG_TILE_LINE=8 (all 64 B) vs AMG_TILE_LINE=4 (all 32 B) on 7-pt, sa27, g3sub
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_zfull_512.py > gpurun_out/r3t_tests.log 2>&1 || { tail -40 gpurun_out/r3t_tests.log; exit 1; }
tail -2 gpurun_out/r3t_tests.log
ROUND=r3t VARIANTS="auto:;l64:AMG_TILE_LINE=8;l32:AMG_TILE_LINE=4;auto2:" CONFIGS="7pt sa27" bash scripts/gpu_envab.sh || exit 1
ROUND=r3t VARIANTS="auto:;l64:AMG_TILE_LINE=8" CONFIGS="g3sub" bash scripts/gpu_envab.sh
