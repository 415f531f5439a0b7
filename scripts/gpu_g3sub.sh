#!/bin/bash
# BASELINE config 5 substitute: unstructured graph Laplacian (1.5M rows), SA + hybrid GS,
# RCM-reordered and random numbering, bench + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config g3sub --steps 20 --warmup 3 --no-cpu-baseline --no-reorder > gpurun_out/g3_rand.json 2> gpurun_out/g3_rand.err || { tail gpurun_out/g3_rand.err; exit 1; }
grep -E "setup|V-cycles" gpurun_out/g3_rand.err; cut -c1-300 gpurun_out/g3_rand.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g3_prof -o run -- python bench.py --config g3sub --steps 20 --warmup 3 --cpu-seconds 15 > gpurun_out/g3_rcm.json 2> gpurun_out/g3_rcm.err || { tail gpurun_out/g3_rcm.err; exit 1; }
grep -E "setup|V-cycles" gpurun_out/g3_rcm.err; cat gpurun_out/g3_rcm.json
python scripts/trace_summary.py gpurun_out/g3_prof/run_kernel_trace.csv > gpurun_out/g3_trace_summary.txt; head -25 gpurun_out/g3_trace_summary.txt
