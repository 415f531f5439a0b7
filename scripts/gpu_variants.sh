#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python scripts/spmv_variants.py 256 0,1,2,3 > gpurun_out/variants.log 2>&1 || { tail -20 gpurun_out/variants.log; exit 1; }
cat gpurun_out/variants.log | grep -v amdgpu.ids
AMG_KERNEL_VARIANT=3 timeout -k 10 600 python -m pytest tests -x -q -m "gpu and not slow" > gpurun_out/tv3.log 2>&1; rc=$?; tail -2 gpurun_out/tv3.log; [ $rc -eq 0 ] || exit $rc
AMG_KERNEL_VARIANT=1 timeout -k 10 600 python -m pytest tests -x -q -m "gpu and not slow" > gpurun_out/tv1.log 2>&1; rc=$?; tail -2 gpurun_out/tv1.log; exit $rc
