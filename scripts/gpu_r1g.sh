#!/bin/bash
# Branch-free CSR block kernel: parity suite, variant A/B (new vs old kernel), bench + trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r1g}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 600 python scripts/spmv_variants.py 256 8,14 > gpurun_out/${TAG}_variants.txt 2>&1 || { tail gpurun_out/${TAG}_variants.txt; exit 1; }
cat gpurun_out/${TAG}_variants.txt
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --cpu-seconds 10 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
grep "V-cycles in" gpurun_out/${TAG}_bench.err; cut -c1-200 gpurun_out/${TAG}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || { tail gpurun_out/${TAG}_prof.err; exit 1; }
python scripts/trace_summary.py gpurun_out/${TAG}_prof/run_kernel_trace.csv > gpurun_out/${TAG}_trace.txt; head -24 gpurun_out/${TAG}_trace.txt
