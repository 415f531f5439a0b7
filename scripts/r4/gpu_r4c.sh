#!/bin/bash
# round-4 checkpoint on one MI355X: the whole -m gpu suite (incl. the 512^3 and full-size
# tests), smoke, the driver's bench command, sa27 / g3sub lines, and N=2 / N=8 box-partition
# rehearsals (every rank on this GPU, RCCL socket transport, torch-free ranks replaying
# captured cycles).  Each step under its own limit; a timeout or crash ends the script.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4c}
step() {  # step <name> <seconds> <cmd...>: stdout -> <name>.out, stderr -> <name>.err
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/${R}_$name.out 2> gpurun_out/${R}_$name.err
  local rc=$?
  echo "$name: exit $rc :: $(tail -c 300 gpurun_out/${R}_$name.out | tr '\n' ' ')"
  [ $rc -ne 0 ] && tail -c 1500 gpurun_out/${R}_$name.err
  if [ $rc -ge 124 ]; then echo "stopping after $name"; exit 1; fi
  return 0
}
if [ -z "$NO_TESTS" ]; then
  step tests 1100 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread -p no:cacheprovider
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --gpus 1 --steps 20 --warmup 5
step sa27 400 python bench.py --config sa27 --steps 20 --warmup 5 --cpu-seconds 8
step g3sub 400 python bench.py --config g3sub --steps 20 --warmup 5 --cpu-seconds 8
step n2 400 env AMG_BENCH_SHARED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5
step n8 900 env AMG_BENCH_SHARED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --steps 5 --warmup 2 --no-cpu-baseline --spmv-reps 3
if [ -n "$WITH_SETUP" ]; then
  step setup8 600 env AMG_TIMING=1 python -u scripts/setup_ranks.py 256 8 boxes
fi
python - <<'PY'
import json, os
R = os.environ.get("R", "r4c")
for f in ("bench", "sa27", "g3sub", "n2", "n8"):
    try:
        line = [l for l in open(f"gpurun_out/{R}_{f}.out") if l.startswith("{")][-1]
        d = json.loads(line)
        print(f, d["value"], d["ms_per_step"], "graph", d["config"].get("hipgraph_all_ranks"), "roofline",
              d["roofline"]["frac"], "rt", d.get("runtime"), "cpu", (d.get("cpu_baseline") or {}).get("value"))
    except Exception as e:
        print(f, "no line", e)
PY
echo r4c-done
