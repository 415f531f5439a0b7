#!/bin/bash
# Round-6 final check on one MI355X (outputs under gpurun_out/${R}_*, copied to profiles/r6 by
# hand): the whole -m gpu suite, smoke(), the opt-in 512^3 eight-RCCL-process case at the default
# replicate_below, and the three bench lines (the default one with its CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-s6z}
if [ -z "$NO_SUITE" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    --durations=30 > gpurun_out/${R}_tests.log 2>&1 || { tail -60 gpurun_out/${R}_tests.log; exit 1; }
  tail -3 gpurun_out/${R}_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { tail gpurun_out/${R}_smoke.log; exit 1; }
  tail -2 gpurun_out/${R}_smoke.log
fi
if [ -n "$RCCL_512" ]; then
  mkdir -p gpurun_out/${R}_512
  AMG_TEST_RCCL_512=1 AMG_TEST_REPORT_DIR=gpurun_out/${R}_512 timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_zfull_512.py -k rccl -m gpu -x -v --timeout 900 --timeout-method thread \
    > gpurun_out/${R}_512_rccl.log 2>&1 || { tail -40 gpurun_out/${R}_512_rccl.log; exit 1; }
  tail -3 gpurun_out/${R}_512_rccl.log
fi
for cfg in ${BENCH_CONFIGS:-7pt sa27 g3sub}; do
  extra=""
  [ "$cfg" != 7pt ] && extra="--no-cpu-baseline"
  timeout -k 10 400 python bench.py --config $cfg $extra > gpurun_out/${R}_bench_$cfg.json 2> gpurun_out/${R}_bench_$cfg.err || { tail gpurun_out/${R}_bench_$cfg.err; exit 1; }
  head -c 400 gpurun_out/${R}_bench_$cfg.json; echo
done
for tol in $DROP7; do  # 7-pt with a coarse drop tolerance (time to solution; not the default)
  timeout -k 10 400 python bench.py --config 7pt --no-cpu-baseline --drop-tol $tol > gpurun_out/${R}_bench_7pt_drop$tol.json 2> gpurun_out/${R}_bench_7pt_drop$tol.err || { tail gpurun_out/${R}_bench_7pt_drop$tol.err; exit 1; }
  head -c 300 gpurun_out/${R}_bench_7pt_drop$tol.json; echo
done
echo final-done
