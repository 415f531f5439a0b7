#!/bin/bash
# End-of-round bench line (default command, PMC traffic from profiles/pmc_level0_spmv.json,
# STREAM-copy ceiling) followed by the sa27 / g3sub config profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-r1t}
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 15 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { tail gpurun_out/${R}_bench.err; exit 1; }
cat gpurun_out/${R}_bench.json
ROUND=$R bash scripts/gpu_configs_prof.sh
