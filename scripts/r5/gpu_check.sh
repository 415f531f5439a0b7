#!/bin/bash
# Round-5 check on one MI355X: selected (or all) -m gpu tests, the default bench line, and
# optionally one rocprofv3 --pmc pass over scripts/pmc_vcycle.py with no manual teardown
# (the facade's atexit hook).  R names the outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r5}
TESTS=${TESTS:-tests}
if [ "$TESTS" != none ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread --durations=40 > gpurun_out/${R}_tests.log 2>&1 || { tail -60 gpurun_out/${R}_tests.log; exit 1; }
  tail -3 gpurun_out/${R}_tests.log
fi
for cfg in ${BENCH_CONFIGS:-7pt}; do
  timeout -k 10 300 python bench.py --config $cfg $BENCH_ARGS > gpurun_out/${R}_bench_$cfg.json 2> gpurun_out/${R}_bench_$cfg.err || { tail gpurun_out/${R}_bench_$cfg.err; exit 1; }
  head -c 600 gpurun_out/${R}_bench_$cfg.json; echo
done
if [ -n "$PMC_TEARDOWN" ]; then
  timeout -k 10 -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${R}_pmcexit -o run -- python scripts/pmc_vcycle.py 256 > gpurun_out/${R}_pmcexit.log 2>&1
  echo "pmc_vcycle under rocprofv3 --pmc, no manual teardown: exit $?"
fi
echo check-done
