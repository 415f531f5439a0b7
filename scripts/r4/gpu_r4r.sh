#!/bin/bash
# (Record of a round-4 A/B: the knobs it exercises were removed after this measurement.)
# LDS-DMA window loads for the one-shot 27-pt window kernels (AMG_TPL_GLDS): parity tests on
# both paths, then a same-box sa27 A/B (default vs AMG_TPL_GLDS=1), twice.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4r}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "sa27_npl16 or template_window or hybrid_gs_template" > gpurun_out/${R}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${R}_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit 1
AMG_TPL_GLDS=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "full_size_27pt or full_size_sa27" > gpurun_out/${R}_tests_full.log 2>&1
rc=$?; tail -3 gpurun_out/${R}_tests_full.log; echo "full tests rc=$rc"
[ $rc -ne 0 ] && exit 1
for i in 1 2; do
  ROUND=${R}_$i CONFIGS=sa27 VARIANTS="reg:;glds:AMG_TPL_GLDS=1" BENCH_ARGS="--steps 20 --warmup 5" bash scripts/gpu_envab.sh || exit 1
done
