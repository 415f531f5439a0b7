#!/bin/bash
# hybrid-GS iteration: parity tests, then sa27 256^3 and g3sub benches under a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-gsq}
timeout -k 10 900 python -m pytest tests -q -m gpu -k "level_kernels or vcycle or graph or multirank or pcg" > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
for cfg in sa27 g3sub; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$cfg -o run -- python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_$cfg.json 2> gpurun_out/${TAG}_$cfg.err || { tail gpurun_out/${TAG}_$cfg.err; exit 1; }
  grep -E "V-cycles in" gpurun_out/${TAG}_$cfg.err
  python scripts/trace_summary.py gpurun_out/${TAG}_$cfg/run_kernel_trace.csv > gpurun_out/${TAG}_${cfg}_trace.txt; grep -E "hybrid_gs|csr_stream" gpurun_out/${TAG}_${cfg}_trace.txt | head -14
done
