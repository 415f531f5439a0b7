#!/bin/bash
# GPU box: the gpu-marked test suite (one process), then stop.  PYTEST_K selects (-k).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-t}
K=()
[ -n "$PYTEST_K" ] && K=(-k "$PYTEST_K")
timeout -k 10 1100 python -m pytest tests -q -m gpu "${K[@]}" ${PYTEST_ARGS} > gpurun_out/tests_$TAG.log 2>&1; rc=$?
tail -30 gpurun_out/tests_$TAG.log
exit $rc
