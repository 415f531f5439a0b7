#!/bin/bash
# round-4 final evidence in one call: PMC re-take on this tree (FETCH_SIZE / WRITE_SIZE passes
# + kernel trace of the bench command), the g3sub split-everywhere A/B, then the final bench
# lines (7-pt with the CPU baseline, sa27, g3sub, N=2 / N=8 shared-GPU rehearsals).  Each step
# time-limited; a timeout or crash ends the script.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4m}
R=${R}p bash scripts/r4/gpu_r4_pmc.sh || exit 1
R=${R}l bash scripts/r4/gpu_r4l.sh || exit 1
NO_TESTS=1 R=${R}z bash scripts/r4/gpu_r4c.sh || exit 1
R=${R}n bash scripts/r4/gpu_r4n.sh || exit 1
echo r4m-done
