#!/bin/bash
# Round 3 probe v: split GS sweeps by average row length (>= 12 entries) --
# the -m gpu suite except the 512^3 test, then same-box A/B: default vs AMG_GS_SPLIT=0 vs
# every level split on g3sub and sa27, and the default 7-pt bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_zfull_512.py > gpurun_out/r3v_tests.log 2>&1 || { tail -40 gpurun_out/r3v_tests.log; exit 1; }
tail -2 gpurun_out/r3v_tests.log
ROUND=r3v VARIANTS="npr12:;ell:AMG_GS_SPLIT=0;all:AMG_GS_SPLIT_NPR=0" CONFIGS="g3sub sa27" bash scripts/gpu_envab.sh || exit 1
ROUND=r3v VARIANTS="default:" CONFIGS="7pt" bash scripts/gpu_envab.sh
