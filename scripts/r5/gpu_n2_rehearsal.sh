#!/bin/bash
# N = 2 rehearsal on a 1-GPU box (both ranks on device 0, RCCL over its socket transport;
# AMG_BENCH_SHARED_GPU=1): bench.py --gpus 2 under torch.distributed.run, for CONFIG.  Not a
# scaling measurement: it checks the multi-rank path end to end (gs_split on every rank,
# hipgraph on every rank, graph vs eager cycles).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r5}
for cfg in ${CONFIGS:-g3sub}; do
  port=$((29500 + RANDOM % 400))
  AMG_BENCH_SHARED_GPU=1 timeout -k 10 ${LIMIT:-400} python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --config $cfg --steps 10 --warmup 2 --spmv-reps 5 $BENCH_ARGS \
    > gpurun_out/${R}_n2_$cfg.json 2> gpurun_out/${R}_n2_$cfg.err || { tail -30 gpurun_out/${R}_n2_$cfg.err; exit 1; }
  head -c 400 gpurun_out/${R}_n2_$cfg.json; echo
done
echo n2-done
