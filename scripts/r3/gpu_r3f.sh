#!/bin/bash
# round-3 final check (r3f: after the LDS-queue chain walk; + sa27 kernel stats) on one MI355X: the whole -m gpu suite (incl. the 512^3 test), smoke, the
# driver's bench command, sa27 / g3sub lines, the N=2 box-partition rehearsal (both ranks on this
# GPU), and rocprofv3 --kernel-trace --stats of the bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r3f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 880 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || { tail -40 gpurun_out/${R}_tests.log; exit 1; }
tail -2 gpurun_out/${R}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { tail gpurun_out/${R}_smoke.log; exit 1; }
tail -1 gpurun_out/${R}_smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { tail gpurun_out/${R}_bench.err; exit 1; }
for cfg in sa27 g3sub; do
  timeout -k 10 600 python bench.py --config $cfg --steps 20 --warmup 5 > gpurun_out/${R}_$cfg.json 2> gpurun_out/${R}_$cfg.err || { tail gpurun_out/${R}_$cfg.err; exit 1; }
done
AMG_BENCH_SHARED_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --spmv-reps 5 > gpurun_out/${R}_n2_boxes.json 2> gpurun_out/${R}_n2_boxes.err || { tail -20 gpurun_out/${R}_n2_boxes.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_prof.log 2>&1 || { tail gpurun_out/${R}_prof.log; exit 1; }
python scripts/trace_summary.py gpurun_out/${R}_prof/run_kernel_trace.csv > gpurun_out/${R}_trace_summary.txt
export R; python - <<'PY'
import json
import os
R = os.environ.get("R", "r3z")
for f in (f"{R}_bench", f"{R}_sa27", f"{R}_g3sub", f"{R}_n2_boxes"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], d["ms_per_step"], "setup_s", d["config"].get("setup_s"), "roofline", d["roofline"]["frac"],
          "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY

# sa27 kernel stats: the split GS sweep's pass (csr_block_kernel<4, ...>) and chain walk
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_sa27prof -o run -- python bench.py --config sa27 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${R}_sa27prof.log 2>&1 || { tail gpurun_out/${R}_sa27prof.log; exit 1; }
python scripts/trace_summary.py gpurun_out/${R}_sa27prof/run_kernel_trace.csv > gpurun_out/${R}_sa27_trace_summary.txt
echo final-ok
