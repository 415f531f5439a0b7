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
# extra bench lines under an environment: EXTRA_BENCH="tag:cfg:NAME=VAL ..." (build-time knobs)
for spec in $EXTRA_BENCH; do
  IFS=':' read -r tag cfg kv <<< "$spec"
  env $kv timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline $BENCH_ARGS > gpurun_out/${R}_bench_${cfg}_$tag.json 2> gpurun_out/${R}_bench_${cfg}_$tag.err || { tail gpurun_out/${R}_bench_${cfg}_$tag.err; exit 1; }
  head -c 300 gpurun_out/${R}_bench_${cfg}_$tag.json; echo
done
for cfg in $TIMING_CONFIGS; do  # setup phase timers (AMG_TIMING=1, rank 0 to stderr)
  AMG_TIMING=1 timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 3 > gpurun_out/${R}_timing_$cfg.json 2> gpurun_out/${R}_timing_$cfg.err || { tail gpurun_out/${R}_timing_$cfg.err; exit 1; }
  grep -c "\[amg\]" gpurun_out/${R}_timing_$cfg.err
done
if [ -n "$AB_CONFIG" ]; then  # in-process A/B of run-time knobs (scripts/ab_env.py); AB_SETTINGS: ;-separated
  IFS=';' read -ra SETS <<< "$AB_SETTINGS"
  timeout -k 10 400 python scripts/ab_env.py $AB_CONFIG "${SETS[@]}" > gpurun_out/${R}_ab_$AB_CONFIG.json 2> gpurun_out/${R}_ab_$AB_CONFIG.err || { tail gpurun_out/${R}_ab_$AB_CONFIG.err; exit 1; }
  cat gpurun_out/${R}_ab_$AB_CONFIG.err | tail -4
fi
for spec in $PLAN; do  # per-level RCCL plan of a cycle (scripts/rccl_plan_table.py): cfg:N
  IFS=':' read -r cfg nr <<< "$spec"
  timeout -k 10 400 python scripts/rccl_plan_table.py $cfg $nr > gpurun_out/${R}_plan_${cfg}_$nr.json 2> gpurun_out/${R}_plan_${cfg}_$nr.md || { tail gpurun_out/${R}_plan_${cfg}_$nr.md; exit 1; }
  tail -2 gpurun_out/${R}_plan_${cfg}_$nr.md
done
if [ -n "$N2" ]; then
  CONFIGS="$N2" R=$R bash scripts/r5/gpu_n2_rehearsal.sh || exit 1
fi
if [ -n "$PHASES" ]; then  # x-tile block kernel phase trace (diagnostic build)
  RAPTOR_AMD_LIB=raptor_amd/libraptor_amd_phase.so timeout -k 10 300 python scripts/csr_phase_trace.py > gpurun_out/${R}_phases.json 2> gpurun_out/${R}_phases.err || { tail gpurun_out/${R}_phases.err; exit 1; }
  tail -c 300 gpurun_out/${R}_phases.json; echo
fi
if [ -n "$PMC_TEARDOWN" ]; then
  timeout -k 10 -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${R}_pmcexit -o run -- python scripts/pmc_vcycle.py 256 > gpurun_out/${R}_pmcexit.log 2>&1
  echo "pmc_vcycle under rocprofv3 --pmc, no manual teardown: exit $?"
fi
echo check-done
