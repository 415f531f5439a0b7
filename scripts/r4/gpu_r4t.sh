#!/bin/bash
# x-tile line width on the round-4 tree: per-operator rule (default) vs every operator at 32 B
# (AMG_TILE_LINE=4) vs every operator at 64 B (AMG_TILE_LINE=8), same box, twice.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4t}
for i in 1 2; do
  ROUND=${R}_$i CONFIGS="7pt sa27" VARIANTS="rule:;all32:AMG_TILE_LINE=4;all64:AMG_TILE_LINE=8" BENCH_ARGS="--steps 20 --warmup 5" bash scripts/gpu_envab.sh || exit 1
done
