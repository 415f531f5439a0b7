#!/bin/bash
# GPU box: bench + rocprofv3 kernel stats + full-size parity.  Each GPU step has its own
# time limit; any failure ends the script (no retries).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r1}
echo "bench $(date)"
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
echo "rocprof $(date)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || exit $?
echo "full-size parity $(date)"
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -k full_size > gpurun_out/tfull_$TAG.log 2>&1 || exit $?
tail -3 gpurun_out/tfull_$TAG.log
echo "done $(date)"
