#!/bin/bash
# rocprofv3 --kernel-trace --stats of the bench command per config (round 6, final tree): the
# summaries the bench lines' in-graph roofline is cross-checked against (outputs under gpurun_out/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-s6r}
for cfg in ${CONFIGS:-sa27 g3sub}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof_$cfg -o run -- \
    python bench.py --config $cfg --no-cpu-baseline $EXTRA > gpurun_out/${R}_prof_bench_$cfg.json 2> gpurun_out/${R}_prof_bench_$cfg.err || { tail gpurun_out/${R}_prof_bench_$cfg.err; exit 1; }
  python scripts/trace_summary.py gpurun_out/${R}_prof_$cfg/run_kernel_trace.csv > gpurun_out/${R}_trace_summary_$cfg.txt
  cp gpurun_out/${R}_prof_$cfg/run_kernel_stats.csv gpurun_out/${R}_kernel_stats_$cfg.csv
  head -8 gpurun_out/${R}_trace_summary_$cfg.txt
done
echo traces-done
