#!/bin/bash
# 2 RCCL ranks on one GPU (per-rank NCCL_HOSTID, socket transport), V-cycles with hipGraph
# capture: Python faulthandler + NCCL_DEBUG to locate a crash.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
PORT=29617
for r in 0 1; do
  RANK=$r WORLD_SIZE=2 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT NCCL_HOSTID=dbg-$r \
  NCCL_SOCKET_IFNAME=lo GLOO_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 NCCL_DEBUG=${NCCL_DEBUG:-WARN} AMG_TRACE_RCCL=1 OMP_NUM_THREADS=2 \
  timeout -k 5 120 python -X faulthandler tests/rccl_worker.py \
    '{"kind": "7pt", "dims": [16, 15, 18], "coarsen": "pmis", "smoother": "jacobi", "rep": 0, "graph": true}' \
    /tmp/dbg > gpurun_out/rccl_dbg_$r.log 2>&1 &
done
wait
for r in 0 1; do echo "== rank $r"; grep -v "^$" gpurun_out/rccl_dbg_$r.log | tail -40; done
