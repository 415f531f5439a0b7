#!/bin/bash
# round-4 final tree: the whole -m gpu suite (slow tests included), then smoke, the bench lines
# and the N=2 / N=8 rehearsals.  Each step time-limited; a timeout or crash ends the script.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4z}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  --durations=10 > gpurun_out/${R}_tests.log 2>&1
rc=$?
grep -oE "(PASSED|FAILED|ERROR|SKIPPED)" gpurun_out/${R}_tests.log | sort | uniq -c
tail -3 gpurun_out/${R}_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit 1
NO_TESTS=1 R=${R}b bash scripts/r4/gpu_r4c.sh
