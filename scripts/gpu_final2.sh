#!/bin/bash
# Final round-end check: gpu suite, smoke, the default bench line with rocprofv3 stats, and
# the sa27 bench (march gated off for its 3078-double window).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=r1v
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || { tail -30 gpurun_out/${R}_tests.log; exit 1; }
tail -1 gpurun_out/${R}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { tail gpurun_out/${R}_smoke.log; exit 1; }
tail -1 gpurun_out/${R}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { tail gpurun_out/${R}_bench.err; exit 1; }
cat gpurun_out/${R}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- python bench.py --no-cpu-baseline > gpurun_out/${R}_prof.log 2>&1 || exit 1
python scripts/trace_summary.py gpurun_out/${R}_prof/run_kernel_trace.csv > gpurun_out/${R}_trace_summary.txt
timeout -k 10 600 python bench.py --config sa27 --cpu-seconds 15 > gpurun_out/${R}_sa27_bench.json 2> gpurun_out/${R}_sa27_bench.err || { tail gpurun_out/${R}_sa27_bench.err; exit 1; }
cat gpurun_out/${R}_sa27_bench.json
