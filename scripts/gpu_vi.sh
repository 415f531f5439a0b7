#!/bin/bash
# value-indexed CSR: parity tests, then 7pt 256^3 bench with and without VI (+ kernel trace)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-vi}
timeout -k 10 900 python -m pytest tests -q -m gpu -x > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
AMG_KERNEL_VARIANT=0 timeout -k 10 400 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_novi.json 2> gpurun_out/${TAG}_novi.err || { tail gpurun_out/${TAG}_novi.err; exit 1; }
grep "V-cycles in" gpurun_out/${TAG}_novi.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_7pt.json 2> gpurun_out/${TAG}_7pt.err || { tail gpurun_out/${TAG}_7pt.err; exit 1; }
grep "V-cycles in" gpurun_out/${TAG}_7pt.err; cut -c1-400 gpurun_out/${TAG}_7pt.json
python scripts/trace_summary.py gpurun_out/${TAG}_prof/run_kernel_trace.csv > gpurun_out/${TAG}_trace.txt; head -24 gpurun_out/${TAG}_trace.txt
