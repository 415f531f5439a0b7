#!/bin/bash
# separate rocprofv3 --pmc passes (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share
# a pass; no --pmc together with -s/-r or trace domains)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-pmc}
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/${TAG}_$name -o run -- python scripts/pmc_levels.py 256 > gpurun_out/${TAG}_$name.log 2>&1 || { tail -5 gpurun_out/${TAG}_$name.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_trace -o run -- python scripts/pmc_levels.py 256 > gpurun_out/${TAG}_trace.log 2>&1 || exit 1
ls gpurun_out/${TAG}_*
