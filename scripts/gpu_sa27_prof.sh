#!/bin/bash
# sa27 (BASELINE configs[2]) kernel trace: where the SA + hybrid-GS V-cycle spends its time.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r1q}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_sa27prof -o run -- python bench.py --config sa27 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_sa27prof.json 2> gpurun_out/${TAG}_sa27prof.err || { tail gpurun_out/${TAG}_sa27prof.err; exit 1; }
python scripts/trace_summary.py gpurun_out/${TAG}_sa27prof/run_kernel_trace.csv > gpurun_out/${TAG}_sa27_trace.txt
python scripts/cycle_breakdown.py gpurun_out/${TAG}_sa27prof/run_kernel_trace.csv 12 > gpurun_out/${TAG}_sa27_cycle.txt
head -30 gpurun_out/${TAG}_sa27_trace.txt
