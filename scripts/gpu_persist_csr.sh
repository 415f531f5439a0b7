#!/bin/bash
# Persistent x-tile CSR kernel (variant bit 64): parity tests, then same-box A/B of the
# default kernel (42) against the persistent one (106) on the level operators, for the
# 6-wave (libraptor_amd) and 5-wave (lib_ab_w5) builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "persistent" --timeout 120 --timeout-method thread > gpurun_out/pcsr_tests.log 2>&1 || { tail -30 gpurun_out/pcsr_tests.log; exit 1; }
tail -1 gpurun_out/pcsr_tests.log
LIBS="libraptor_amd lib_ab_w5" VARS=42,106 bash scripts/gpu_libab.sh
