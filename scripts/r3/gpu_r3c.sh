#!/bin/bash
# round-3 batch c: GPU tests (device setup on N ranks), per-kernel PMC (fixed segments), 512^3
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1 || { tail -40 gpurun_out/r3c_tests.log; exit 1; }
tail -3 gpurun_out/r3c_tests.log
ROUND=r3c bash scripts/gpu_pmc_vcycle.sh > gpurun_out/r3c_pmc.log 2>&1 || { tail gpurun_out/r3c_pmc.log; exit 1; }
cat gpurun_out/r3c_pmc.log
AMG_TRACE_BLOCKS=1 timeout -k 10 300 python bench.py --grid 512,512,64 --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3c_slab_blocks.json 2> gpurun_out/r3c_slab_blocks.err || exit 1
AMG_TPL_MARCH_WIDE=1 timeout -k 10 300 python bench.py --grid 512,512,64 --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3c_slab_marchwide.json 2> gpurun_out/r3c_slab_marchwide.err || exit 1
AMG_TEST_REPORT_DIR=gpurun_out timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_gpu_zfull_512.py > gpurun_out/r3c_512.log 2>&1 || { tail -40 gpurun_out/r3c_512.log; exit 1; }
tail -15 gpurun_out/r3c_512.log
# the N=2 bench path with the box partition (both ranks on this one GPU, RCCL over sockets):
# a path check, not a scaling number
AMG_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3c_n2_boxes.json 2> gpurun_out/r3c_n2_boxes.err || { tail -20 gpurun_out/r3c_n2_boxes.err; exit 1; }
echo batch-ok
