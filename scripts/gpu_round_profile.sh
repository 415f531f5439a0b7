#!/bin/bash
# Round evidence on one MI355X: bench line, rocprofv3 kernel stats of the same command,
# separate PMC passes (FETCH_SIZE / WRITE_SIZE / TCC hit) on the level kernels.
# Outputs land in gpurun_out/; copy what is judged into profiles/ (see profiles/README.md).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-r1}
timeout -k 10 300 bash scripts/gpu_pmc.sh > gpurun_out/${R}_pmc.log 2>&1 || { tail gpurun_out/${R}_pmc.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/${R}_pmc_levels.txt
python scripts/pmc_traffic.py gpurun_out/pmc gpurun_out/${R}_pmc_traffic.json || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 15 --traffic-json gpurun_out/${R}_pmc_traffic.json > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${R}_prof.log 2>&1 || exit 1
python scripts/trace_summary.py gpurun_out/${R}_prof/run_kernel_trace.csv > gpurun_out/${R}_trace_summary.txt
cat gpurun_out/${R}_bench.json
head -20 gpurun_out/${R}_trace_summary.txt
