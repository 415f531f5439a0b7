#!/bin/bash
# z-marching template kernel (variant bit 128): parity tests (march first, then the whole gpu
# suite), same-process A/B of the level operators (42 default vs 170 = 42|128), and the
# bench with and without it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "march" --timeout 120 --timeout-method thread > gpurun_out/march_tests.log 2>&1 || { tail -30 gpurun_out/march_tests.log; exit 1; }
tail -1 gpurun_out/march_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/march_alltests.log 2>&1 || { tail -30 gpurun_out/march_alltests.log; exit 1; }
tail -1 gpurun_out/march_alltests.log
timeout -k 10 300 python scripts/spmv_variants.py 256 42,170 > gpurun_out/march_variants.txt 2>&1 || { tail -20 gpurun_out/march_variants.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/march_variants.txt
for v in 170 42; do
  AMG_KERNEL_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/march_bench_$v.json 2> gpurun_out/march_bench_$v.err || { tail gpurun_out/march_bench_$v.err; exit 1; }
  python -c "
import json; d = json.load(open('gpurun_out/march_bench_$v.json')); r = d['roofline']; print('var $v', d['value'], r['avg_launch_ms'], r['achieved'], r['frac'])"
done
