#!/bin/bash
# CSR block kernel variant A/B only (interleaved, HIP events).  VARS=comma list
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-var}
timeout -k 10 600 python scripts/spmv_variants.py 256 ${VARS:-8,10} > gpurun_out/${TAG}_variants.txt 2>&1 || { tail gpurun_out/${TAG}_variants.txt; exit 1; }
cat gpurun_out/${TAG}_variants.txt
