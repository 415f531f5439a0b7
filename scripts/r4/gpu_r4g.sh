#!/bin/bash
# round-4 GPU suite, part 1: every -m gpu test except the slow full-size ones, one process,
# per-test time limit; progress streams into gpurun_out (one line per test).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4g}
SEL=${SEL:-gpu and not slow}
timeout -k 10 1080 python -u -m pytest tests -m "$SEL" -x -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider --durations=15 ${KSEL:+-k "$KSEL"} ${EXTRA_ARGS} > gpurun_out/${R}_tests.log 2>&1
rc=$?
grep -oE "(PASSED|FAILED|ERROR|SKIPPED)" gpurun_out/${R}_tests.log | sort | uniq -c
tail -25 gpurun_out/${R}_tests.log
echo "tests rc=$rc"
