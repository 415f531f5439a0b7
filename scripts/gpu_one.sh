#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T='tests/test_gpu_multirank.py::test_multirank_vcycle_bit_exact'
timeout -k 10 300 python -u -m pytest "$T" -q -k "rep-deep or rep-all" --timeout 120 --timeout-method thread > gpurun_out/one_a.log 2>&1; echo "tail graph on: rc=$?"
grep -E "Error|passed|failed" gpurun_out/one_a.log | head -8
AMG_TAIL_GRAPH=0 timeout -k 10 300 python -u -m pytest "$T" -q -k "rep-deep or rep-all" --timeout 120 --timeout-method thread > gpurun_out/one_b.log 2>&1; echo "tail graph off: rc=$?"
grep -E "Error|passed|failed" gpurun_out/one_b.log | head -8
