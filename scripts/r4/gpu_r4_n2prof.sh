#!/bin/bash
# N=2 rehearsal (both ranks on this GPU, RCCL socket transport) under rocprofv3 --kernel-trace,
# graph replay vs eager cycles: per rank, the per-cycle split of compute / RCCL-only / idle
# time (scripts/rank_idle.py).  Each rank is its own `rocprofv3 -- python bench.py` process
# (no launcher under the profiler); they meet over the Unix-socket mesh keyed by MASTER_PORT.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4n}
for mode in graph eager; do
  extra=""; [ $mode = eager ] && extra="--no-graph"
  port=$((29600 + RANDOM % 300))
  for r in 0 1; do
    RANK=$r WORLD_SIZE=2 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port AMG_BENCH_SHARED_GPU=1 \
      timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${R}_${mode}_$r -o run -- \
      python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 $extra \
      > gpurun_out/${R}_${mode}_$r.json 2> gpurun_out/${R}_${mode}_$r.err &
  done
  wait
  for r in 0 1; do
    f=$(ls gpurun_out/${R}_${mode}_$r/*kernel_trace.csv 2>/dev/null | head -1)
    echo "== $mode rank $r: $(head -c 200 gpurun_out/${R}_${mode}_$r.json)"
    [ -n "$f" ] && python scripts/rank_idle.py "$f" 8 | tee gpurun_out/${R}_${mode}_${r}_idle.txt
  done
done
echo n2prof-done
