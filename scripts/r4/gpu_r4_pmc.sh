#!/bin/bash
# round-4 PMC re-take on the final tree: per-cycle-kernel FETCH_SIZE /
# WRITE_SIZE (separate passes) for bench.py's vcycle_kernels table, and the level-0 plain-CSR
# SpMV traffic for roofline.traffic; then the kernel-trace summary of the bench command.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4p}
ROUND=$R bash scripts/gpu_pmc_vcycle.sh || exit 1
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/${R}_pmc_$pass -o run -- python scripts/pmc_levels.py 256 > gpurun_out/${R}_pmc_$pass.log 2>&1 || { tail -5 gpurun_out/${R}_pmc_$pass.log; exit 1; }
done
python scripts/pmc_traffic.py gpurun_out/${R}_pmc gpurun_out/${R}_pmc_traffic.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_prof.log 2>&1 || { tail gpurun_out/${R}_prof.log; exit 1; }
python scripts/trace_summary.py gpurun_out/${R}_prof/run_kernel_trace.csv > gpurun_out/${R}_trace_summary.txt
head -30 gpurun_out/${R}_trace_summary.txt
echo pmc-done
