#!/bin/bash
# round-3 final check, short form (r3f: no N=2 rehearsal or rocprof: after the LDS-queue chain walk; + sa27 kernel stats) on one MI355X: the whole -m gpu suite (incl. the 512^3 test), smoke, the
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
for f in bench sa27 g3sub; do python -c "import json,sys; d=json.load(open('gpurun_out/${R}_'+sys.argv[1]+'.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d['config'].get('setup_s'), d['roofline']['frac'])" $f; done
echo final-ok
