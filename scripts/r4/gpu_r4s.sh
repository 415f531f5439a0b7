#!/bin/bash
# (Record of a round-4 A/B: the knobs it exercises were removed after this measurement.)
# (1) long-row sums software-pipelined (AMG_ROWSUM_PIPE, default build) vs the 16-ahead build
# (raptor_amd/lib_ab_nopipe.so); (2) the one-shot fused template GS sweep (AMG_GS_FUSED=1) vs
# the acc + chain pair.  Parity tests first (both GS forms; full-size 27-pt with the fused
# sweep), then same-box A/Bs.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4s}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "vcycle_paths or restriction_paths or sa27_npl16 or test_gpu_parity or hybrid_gs or sa_gs" > gpurun_out/${R}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${R}_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit 1
AMG_GS_FUSED=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "full_size_27pt or full_size_sa27" > gpurun_out/${R}_tests_full.log 2>&1
rc=$?; tail -3 gpurun_out/${R}_tests_full.log; echo "full tests (fused) rc=$rc"
[ $rc -ne 0 ] && exit 1
for i in 1 2; do
  ROUND=${R}f_$i CONFIGS=sa27 VARIANTS="pair:AMG_GS_FUSED=0;fused:AMG_GS_FUSED=1" BENCH_ARGS="--steps 20 --warmup 5" bash scripts/gpu_envab.sh || exit 1
done
for i in 1 2; do
  ROUND=${R}_$i CONFIGS="sa27 7pt g3sub" ALT=raptor_amd/lib_ab_nopipe.so BENCH_ARGS="--steps 20 --warmup 5" bash scripts/gpu_ab.sh || exit 1
done
