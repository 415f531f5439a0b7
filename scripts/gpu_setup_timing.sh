#!/bin/bash
# setup phase timing (AMG_TIMING=1) for the three single-GPU bench configs
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in 7pt sa27 g3sub; do
  AMG_TIMING=1 timeout -k 10 400 python bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --spmv-reps 5 > gpurun_out/setup_$cfg.json 2> gpurun_out/setup_$cfg.err || { tail gpurun_out/setup_$cfg.err; exit 1; }
  echo "== $cfg"; grep -E "\[amg\]|setup|built" gpurun_out/setup_$cfg.err
done
