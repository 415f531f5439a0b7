#!/bin/bash
# GPU box: parity tests (incl. full size) + bench.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-q}
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/tgpu_$TAG.log 2>&1; rc=$?
tail -4 gpurun_out/tgpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
