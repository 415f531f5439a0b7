#!/bin/bash
# N-rank rehearsal of the driver's scaling bench on a 1-GPU box: bench.py --gpus N under
# torch.distributed.run, every rank on device 0 (AMG_BENCH_SHARED_GPU=1, RCCL over its socket
# transport).  Not a scaling measurement: it checks that the multi-rank bench path runs end to
# end on this tree (device setup, replicated coarse levels, captured cycles on every rank).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-s6n}
for spec in ${RUNS:-7pt:8 7pt:2 g3sub:8}; do
  IFS=':' read -r cfg np <<< "$spec"
  port=$((29500 + RANDOM % 400))
  # heartbeat (the box kills a command silent for 180 s; the bench is bounded by LIMIT below)
  ( while true; do sleep 60; echo "[rehearsal] $cfg N=$np still running $(date +%T)"; done ) & hb=$!
  AMG_BENCH_SHARED_GPU=1 timeout -k 10 ${LIMIT:-500} python -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus $np --config $cfg --steps 5 --warmup 2 --spmv-reps 3 $BENCH_ARGS \
    > gpurun_out/${R}_n${np}_$cfg.json 2> gpurun_out/${R}_n${np}_$cfg.err || { kill $hb; tail -30 gpurun_out/${R}_n${np}_$cfg.err; exit 1; }
  kill $hb
  head -c 300 gpurun_out/${R}_n${np}_$cfg.json; echo
done
echo rehearsal-done
