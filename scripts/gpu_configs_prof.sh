#!/bin/bash
# BASELINE configs[2] (sa27) and configs[4] (G3_circuit substitute): bench line with CPU
# baseline, then rocprofv3 --kernel-trace --stats of the same command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-r1s}
for cfg in sa27 g3sub; do
  timeout -k 10 600 python bench.py --config $cfg --steps 20 --warmup 3 --cpu-seconds 15 > gpurun_out/${R}_${cfg}_bench.json 2> gpurun_out/${R}_${cfg}_bench.err || { tail gpurun_out/${R}_${cfg}_bench.err; exit 1; }
  grep "V-cycles in" gpurun_out/${R}_${cfg}_bench.err
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_${cfg}_prof -o run -- python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${R}_${cfg}_prof.log 2>&1 || { tail gpurun_out/${R}_${cfg}_prof.log; exit 1; }
  python scripts/trace_summary.py gpurun_out/${R}_${cfg}_prof/run_kernel_trace.csv > gpurun_out/${R}_${cfg}_trace_summary.txt
done
