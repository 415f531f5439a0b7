#!/bin/bash
# Per-cycle-kernel HBM traffic: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 --pmc passes over scripts/pmc_vcycle.py, then profiles-ready JSON.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-r3}
CFG=${CFG:-7pt}  # sa27: configs[2]'s cycle operations (hybrid GS sweeps)
[ "$CFG" != 7pt ] && R=${R}_$CFG
for pass in FETCH_SIZE WRITE_SIZE; do
  AMG_PMC_OPS=gpurun_out/${R}_pmc_vcycle_ops.json timeout -k 10 -s KILL 300 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/${R}_vpmc_$pass -o run -- python scripts/pmc_vcycle.py 256 $CFG > gpurun_out/${R}_vpmc_$pass.log 2>&1 || { tail -5 gpurun_out/${R}_vpmc_$pass.log; exit 1; }
done
python scripts/pmc_vcycle_traffic.py gpurun_out/${R}_vpmc gpurun_out/${R}_pmc_vcycle_ops.json gpurun_out/${R}_pmc_vcycle_kernels.json
