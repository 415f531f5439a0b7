#!/bin/bash
# Attribution of the N-rank rehearsal's per-operation floor: N ranks on
# this one GPU (AMG_BENCH_SHARED_GPU=1, RCCL over its socket transport), eager and graph
# cycles, two problem sizes, with the cgroup's CPU throttling counters (cpu.stat:
# nr_throttled, throttled_usec, usage_usec) read around each run.  A floor that does not
# move with the problem size and comes with heavy throttling is the box's CPU quota feeding
# 8 processes' RCCL proxy threads, not the product.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r5}
out=gpurun_out/${R}_n8_attrib.txt
: > $out
for N in ${NS:-8}; do
  for grid in ${GRIDS:-"64,64,128 128,128,256"}; do
    for mode in eager graph; do
      extra=""; [ $mode = eager ] && extra="--no-graph"
      port=$((29500 + RANDOM % 400))
      s0=$(cat /sys/fs/cgroup/cpu.stat | tr '\n' ' ')
      t0=$(date +%s.%N)
      AMG_BENCH_SHARED_GPU=1 RAPTOR_AMD_MESH_KEY=attrib$port timeout -k 10 ${LIMIT:-300} python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $N --master-addr 127.0.0.1 --master-port $port bench.py --gpus $N --grid $grid \
        --steps 5 --warmup 1 --quick $extra > gpurun_out/${R}_n${N}_${grid}_$mode.json 2> gpurun_out/${R}_n${N}_${grid}_$mode.err || { tail -20 gpurun_out/${R}_n${N}_${grid}_$mode.err; exit 1; }
      t1=$(date +%s.%N)
      s1=$(cat /sys/fs/cgroup/cpu.stat | tr '\n' ' ')
      echo "N=$N grid=$grid mode=$mode wall=$(python -c "print(round($t1-$t0,1))")s line=$(cat gpurun_out/${R}_n${N}_${grid}_$mode.json)" | tee -a $out
      echo "   cpu.stat before: $s0" | tee -a $out
      echo "   cpu.stat after:  $s1" | tee -a $out
    done
  done
done
echo "quota: $(cat /sys/fs/cgroup/cpu.max)" | tee -a $out
echo attrib-done
