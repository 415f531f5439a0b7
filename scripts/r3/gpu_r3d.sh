#!/bin/bash
# round-3 batch d: the 512^3 configs[3] test, the N=2 box-partition bench rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
AMG_TEST_REPORT_DIR=gpurun_out timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_gpu_zfull_512.py > gpurun_out/r3d_512.log 2>&1 || { tail -40 gpurun_out/r3d_512.log; exit 1; }
tail -15 gpurun_out/r3d_512.log
AMG_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/r3d_n2_boxes.json 2> gpurun_out/r3d_n2_boxes.err || { tail -20 gpurun_out/r3d_n2_boxes.err; exit 1; }
echo batch-ok
