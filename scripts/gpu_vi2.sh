#!/bin/bash
# VI A/B per level (interleaved, HIP events) + HBM FETCH for the level-0 SpMV with and without VI
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python scripts/spmv_variants.py 256 0,8,6,14 > gpurun_out/vi_variants.txt 2>&1 || { tail gpurun_out/vi_variants.txt; exit 1; }
cat gpurun_out/vi_variants.txt
for v in 0 8; do
  AMG_KERNEL_VARIANT=$v timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/vi_fetch_$v -o run -- python scripts/pmc_levels.py 256 > gpurun_out/vi_fetch_$v.log 2>&1 || { tail -5 gpurun_out/vi_fetch_$v.log; exit 1; }
done
for v in 0 8; do echo "== variant $v"; python scripts/pmc_fetch.py gpurun_out/vi_fetch_$v/run_counter_collection.csv; done
