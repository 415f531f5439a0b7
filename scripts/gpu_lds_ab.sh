#!/bin/bash
# Template-kernel LDS without the Jacobi-only 1/a_ii table outside Jacobi (8 SpMV workgroups
# per CU instead of 7): gpu tests, same-box A/B against the previous build, bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lds_tests.log 2>&1 || { tail -30 gpurun_out/lds_tests.log; exit 1; }
tail -1 gpurun_out/lds_tests.log
LIBS="libraptor_amd lib_ab_old" VARS=42 bash scripts/gpu_libab.sh
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/lds_bench.json 2> gpurun_out/lds_bench.err || { tail gpurun_out/lds_bench.err; exit 1; }
cat gpurun_out/lds_bench.json
