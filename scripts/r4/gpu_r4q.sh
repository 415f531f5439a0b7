#!/bin/bash
# sa27 per-cycle-kernel PMC traffic (FETCH_SIZE / WRITE_SIZE passes over every operation of
# bench.py --config sa27's table), then the sa27 bench line with those counters attached.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4q}
CFG=sa27 ROUND=$R bash scripts/gpu_pmc_vcycle.sh || exit 1
cp gpurun_out/${R}_sa27_pmc_vcycle_kernels.json profiles/pmc_vcycle_kernels_sa27.json
timeout -k 10 300 python bench.py --config sa27 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_sa27.json 2> /tmp/b.err || { tail -5 /tmp/b.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/${R}_sa27.json'))
print('sa27', d['value'])
for r in d['vcycle_kernels']: print('  ', r['level'], r['op'], r['us'], r['stored_bytes'], r.get('traffic'), r.get('traffic_over_stored'), r.get('traffic_stale'))"
