#!/bin/bash
# Jacobi template LDS with an ntpl-entry 1/a_ii table (libraptor_amd) vs the 256-entry one
# (lib_ab_old): template/march parity, then same-box A/B of the level operators.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "template or march or vcycle" --timeout 120 --timeout-method thread > gpurun_out/pd_tests.log 2>&1 || { tail -30 gpurun_out/pd_tests.log; exit 1; }
tail -1 gpurun_out/pd_tests.log
LIBS="libraptor_amd lib_ab_old" VARS=170 bash scripts/gpu_libab.sh
