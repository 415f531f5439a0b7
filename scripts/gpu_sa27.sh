#!/bin/bash
# BASELINE config 3: 27-pt anisotropic SA + hybrid GS, bench + kernel trace (128^3 then 256^3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config sa27 --grid 128,128,128 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sa27_128.json 2> gpurun_out/sa27_128.err || { tail gpurun_out/sa27_128.err; exit 1; }
grep setup gpurun_out/sa27_128.err; cut -c1-200 gpurun_out/sa27_128.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sa27_prof -o run -- python bench.py --config sa27 --steps 10 --warmup 2 --cpu-seconds 15 > gpurun_out/sa27_256.json 2> gpurun_out/sa27_256.err || { tail gpurun_out/sa27_256.err; exit 1; }
grep setup gpurun_out/sa27_256.err; cat gpurun_out/sa27_256.json
python scripts/trace_summary.py gpurun_out/sa27_prof/run_kernel_trace.csv > gpurun_out/sa27_trace_summary.txt; head -25 gpurun_out/sa27_trace_summary.txt
