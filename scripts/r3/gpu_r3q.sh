#!/bin/bash
# Round 3 probe q: global value dictionary for rectangular x-tile operators (variant bit 1024)
# -- dictionary / format-identity / SA kernel-path tests, then same-box A/B on sa27 (AMG_GD=0 =
# 8-byte values) and the 7-pt line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_paths.py tests/test_gpu_formats.py -x -v --timeout 240 --timeout-method thread \
  -k "dictionary or formats_equal or sa_ or template_window or gs" > gpurun_out/r3q_tests.log 2>&1 || { tail -40 gpurun_out/r3q_tests.log; exit 1; }
tail -2 gpurun_out/r3q_tests.log
ROUND=r3q VARIANTS="gd:;values:AMG_GD=0;gd2:;values2:AMG_GD=0" CONFIGS="sa27" bash scripts/gpu_envab.sh || exit 1
ROUND=r3q VARIANTS="def:" CONFIGS="7pt g3sub" bash scripts/gpu_envab.sh
