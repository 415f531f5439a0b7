#!/bin/bash
# round-3 probe e: whole-cycle RCCL graph replays on the torch-free ROCm 7.2 runtime
#   1. solve (fused-norm cycles) with each multi-rank replay synchronised (AMG_RCCL_GRAPH_SYNC=1)
#   2. plain cycles replayed back to back, one synchronisation at the end
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
export AMG_TRACE_RCCL=1 AMG_RCCL_GRAPH=1 NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1
AMG_RCCL_GRAPH_SYNC=1 timeout -k 10 90 tests/cxx/build/cxx_driver ranks 2 graph tests/golden/cxx_7pt24_hist.txt > gpurun_out/r3e_graph_sync.log 2>&1 || { echo "sync solve rc=$?"; tail -20 gpurun_out/r3e_graph_sync.log; exit 1; }
tail -3 gpurun_out/r3e_graph_sync.log
AMG_CXX_GRAPH_MULT=4 timeout -k 10 60 tests/cxx/build/cxx_driver ranks 2 graph tests/golden/cxx_7pt24_hist.txt > gpurun_out/r3e_graph_b2b.log 2>&1 || { echo "b2b rc=$?"; tail -20 gpurun_out/r3e_graph_b2b.log; exit 1; }
tail -3 gpurun_out/r3e_graph_b2b.log
echo probe-ok
