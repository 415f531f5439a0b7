#!/bin/bash
# round 4 check: ring-kernel parity tests, graph probes, torch-free bench lines (7pt, sa27,
# N=2 rehearsal).  Each GPU step under its own limit; a timeout / crash ends the script.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4b}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/${R}_$name.log 2>&1
  local rc=$?
  echo "$name: exit $rc :: $(tail -c 400 gpurun_out/${R}_$name.log | tr '\n' ' ')"
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit 1; fi
  return 0
}
run ringtests 600 python -u -m pytest tests/test_gpu_kernel_paths.py -x -q --timeout 300 --timeout-method thread -k "ring or window_lanes or hybrid_gs_template or sa_gs_vcycle"
run bench7 400 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 8
cp gpurun_out/${R}_bench7.log gpurun_out/${R}_bench7.txt
run sa27 400 python bench.py --config sa27 --steps 20 --warmup 5 --cpu-seconds 6
run sa27_noring 400 env AMG_TPL_RING=0 AMG_GS_RING=0 python bench.py --config sa27 --steps 20 --warmup 5 --no-cpu-baseline
run bench7_noring 400 env AMG_TPL_RING=0 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run bench7_pair 400 env AMG_CSR_PAIR=1 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
run n2 400 env AMG_BENCH_SHARED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5
R=$R bash scripts/gpu_graph_probe.sh
