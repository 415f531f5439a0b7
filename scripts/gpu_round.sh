#!/bin/bash
# Round-2 check on one MI355X: gpu tests (verbose, per-test timeout), smoke, the default bench
# line.  ROUND names the output files under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-r2}
TESTS=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || { tail -40 gpurun_out/${R}_tests.log; exit 1; }
tail -1 gpurun_out/${R}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { tail gpurun_out/${R}_smoke.log; exit 1; }
tail -1 gpurun_out/${R}_smoke.log
timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { tail gpurun_out/${R}_bench.err; exit 1; }
cat gpurun_out/${R}_bench.json
