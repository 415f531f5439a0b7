#!/bin/bash
# Same-box A/B of the template-kernel window batch (AMG_TPL_BATCH build knob): parity of the
# batched builds on the template tests, then level-operator timings per build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in lib_ab_b8 lib_ab_b4; do
  RAPTOR_AMD_LIB=$PWD/raptor_amd/$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "template" --timeout 120 --timeout-method thread > gpurun_out/batch_tests_$lib.log 2>&1 || { tail -30 gpurun_out/batch_tests_$lib.log; exit 1; }
  tail -1 gpurun_out/batch_tests_$lib.log
done
LIBS="libraptor_amd lib_ab_b8 lib_ab_b4" VARS=42 bash scripts/gpu_libab.sh
