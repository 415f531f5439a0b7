#!/bin/bash
# Parity suite, CSR variant A/B, and the three benches (7pt, sa27, g3sub) without CPU baseline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r1o}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 600 python scripts/spmv_variants.py 256 ${VARS:-8,10} > gpurun_out/${TAG}_variants.txt 2>&1 || { tail gpurun_out/${TAG}_variants.txt; exit 1; }
cat gpurun_out/${TAG}_variants.txt
for cfg in ${CFGS:-7pt sa27 g3sub}; do
  timeout -k 10 500 python bench.py --config $cfg --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_$cfg.json 2> gpurun_out/${TAG}_$cfg.err || { tail gpurun_out/${TAG}_$cfg.err; exit 1; }
  grep "V-cycles in" gpurun_out/${TAG}_$cfg.err
done
