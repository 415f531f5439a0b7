#!/bin/bash
# Round 3 probe n: rotated uniform-stencil rows + padded GS-chain stage -- kernel-path tests,
# then same-box variants on sa27 / 7-pt: default, persistent / marching 27-pt windows, and the
# exec-masked build (libraptor_amd_alt.so, AMG_TPL_MASK_BRANCH=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernel_paths.py -x -v --timeout 240 --timeout-method thread \
  -k "template or gs or sa27_npl16 or vcycle_paths" > gpurun_out/r3n_tests.log 2>&1 || { tail -30 gpurun_out/r3n_tests.log; exit 1; }
tail -2 gpurun_out/r3n_tests.log
ROUND=r3n VARIANTS="def:;persist:AMG_TPL_WIDE_PERSIST=1;march:AMG_TPL_MARCH_WIDE=1;maskbr:RAPTOR_AMD_LIB=$GRAFT_REPO_ROOT/raptor_amd/libraptor_amd_alt.so;def2:" CONFIGS="sa27" bash scripts/gpu_envab.sh || exit 1
ROUND=r3n VARIANTS="def:;maskbr:RAPTOR_AMD_LIB=$GRAFT_REPO_ROOT/raptor_amd/libraptor_amd_alt.so" CONFIGS="7pt" bash scripts/gpu_envab.sh
