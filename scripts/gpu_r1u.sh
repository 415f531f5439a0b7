#!/bin/bash
# Round-end evidence after making the z-marching template kernel the default: gpu tests,
# smoke, then the round profile (PMC traffic passes, bench line, rocprofv3 stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r1u_tests.log 2>&1 || { tail -30 gpurun_out/r1u_tests.log; exit 1; }
tail -1 gpurun_out/r1u_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1u_smoke.log 2>&1 || { tail gpurun_out/r1u_smoke.log; exit 1; }
tail -1 gpurun_out/r1u_smoke.log
ROUND=r1u bash scripts/gpu_round_profile.sh
