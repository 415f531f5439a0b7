#!/bin/bash
# Round-2 profiles on one MI355X: copy-ceiling probe, rocprofv3 --kernel-trace --stats of the
# bench command, and the FETCH_SIZE / WRITE_SIZE passes (separate runs) of the level kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-r2}
if [ -x scripts/probe/copy_probe ]; then
  timeout -k 10 120 scripts/probe/copy_probe > gpurun_out/${R}_copy_probe.txt 2>&1 || exit 1
  cat gpurun_out/${R}_copy_probe.txt
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/${R}_prof.log 2>&1 || { tail gpurun_out/${R}_prof.log; exit 1; }
python scripts/trace_summary.py gpurun_out/${R}_prof/run_kernel_trace.csv > gpurun_out/${R}_trace_summary.txt
head -12 gpurun_out/${R}_trace_summary.txt
if [ -z "$NO_PMC" ]; then
  for pass in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 300 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/${R}_pmc_$pass -o run -- python scripts/pmc_levels.py 256 > gpurun_out/${R}_pmc_$pass.log 2>&1 || { tail -5 gpurun_out/${R}_pmc_$pass.log; exit 1; }
  done
  python scripts/pmc_traffic.py gpurun_out/${R}_pmc gpurun_out/${R}_pmc_traffic.json
  python scripts/pmc_traffic.py gpurun_out/${R}_pmc gpurun_out/${R}_pmc_traffic_tpl.json tpl_march_kernel\<0
fi
