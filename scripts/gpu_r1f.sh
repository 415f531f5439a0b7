#!/bin/bash
# Re-entry check: gpu parity suite, bench with/without value-indexed blocks, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r1f}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
AMG_KERNEL_VARIANT=0 timeout -k 10 400 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_novi.json 2> gpurun_out/${TAG}_novi.err || { tail gpurun_out/${TAG}_novi.err; exit 1; }
grep "V-cycles in" gpurun_out/${TAG}_novi.err
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --cpu-seconds 10 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
grep "V-cycles in" gpurun_out/${TAG}_bench.err; cut -c1-300 gpurun_out/${TAG}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { tail gpurun_out/${TAG}_prof.err; exit 1; }
python scripts/trace_summary.py gpurun_out/${TAG}_prof/run_kernel_trace.csv > gpurun_out/${TAG}_trace.txt; head -30 gpurun_out/${TAG}_trace.txt
