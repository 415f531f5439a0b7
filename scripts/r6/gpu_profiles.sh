#!/bin/bash
# Round-6 profiles on one MI355X (outputs under gpurun_out/, copied to profiles/r6 by hand):
#  1. PMC FETCH_SIZE / WRITE_SIZE passes (separate runs) over every cycle operation of the sa27
#     and g3sub hierarchies (the SA definition changed: new formats) and of 7-pt -> the
#     pmc_vcycle_kernels*.json files bench.py reads for its traffic column;
#  2. rocprofv3 --kernel-trace --stats of the default bench command (7-pt), its summary.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-s6p}
for CFG in ${PMC_CONFIGS:-sa27 g3sub 7pt}; do
  for pass in FETCH_SIZE WRITE_SIZE; do
    AMG_PMC_OPS=gpurun_out/${R}_${CFG}_pmc_ops.json timeout -k 10 -s KILL 300 rocprofv3 --pmc $pass --output-format csv \
      -d gpurun_out/${R}_${CFG}_vpmc_$pass -o run -- python scripts/pmc_vcycle.py 256 $CFG \
      > gpurun_out/${R}_${CFG}_vpmc_$pass.log 2>&1 || { tail -5 gpurun_out/${R}_${CFG}_vpmc_$pass.log; exit 1; }
  done
  python scripts/pmc_vcycle_traffic.py gpurun_out/${R}_${CFG}_vpmc gpurun_out/${R}_${CFG}_pmc_ops.json \
    gpurun_out/${R}_pmc_vcycle_kernels_${CFG}.json || exit 1
  echo "pmc $CFG done"
done
if [ -z "$NO_TRACE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- \
    python bench.py --no-cpu-baseline > gpurun_out/${R}_prof_bench.json 2> gpurun_out/${R}_prof_bench.err || { tail gpurun_out/${R}_prof_bench.err; exit 1; }
  python scripts/trace_summary.py gpurun_out/${R}_prof/run_kernel_trace.csv > gpurun_out/${R}_trace_summary.txt
  cp gpurun_out/${R}_prof/run_kernel_stats.csv gpurun_out/${R}_kernel_stats.csv
  head -14 gpurun_out/${R}_trace_summary.txt
fi
echo profiles-done
