#!/bin/bash
# round-4 GPU suite, part 1: every -m gpu test except the slow full-size ones, one process,
# per-test time limit; the log is kept short (tail) in gpurun_out.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4g}
timeout -k 10 1080 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider --durations=15 > /tmp/t.log 2>&1
rc=$?
grep -v "amdgpu.ids" /tmp/t.log | tail -c 40000 > gpurun_out/${R}_tests.log
tail -40 gpurun_out/${R}_tests.log
echo "tests rc=$rc"
