#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_fz.log 2>&1 || { tail -30 gpurun_out/tests_fz.log; exit 1; }
tail -1 gpurun_out/tests_fz.log
for rep in 1 2; do for f in 1 0; do
  AMG_FUSE_ZERO=$f timeout -k 10 400 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/fz_$f.json 2> gpurun_out/fz_$f.err || { tail gpurun_out/fz_$f.err; exit 1; }
  echo "fuse=$f $(grep 'V-cycles in' gpurun_out/fz_$f.err)"
done; done
