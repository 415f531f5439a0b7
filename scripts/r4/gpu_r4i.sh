#!/bin/bash
# plain-CSR roofline leg A/B (pipelined persistent kernel vs one workgroup per block), then the
# round-4 PMC re-take on this tree (scripts/r4/gpu_r4_pmc.sh).  Each step time-limited.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4i}
for v in 1 0 1 0; do
  AMG_PLAIN_PIPE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${R}_pipe$v.json 2> /tmp/b.err || { tail -5 /tmp/b.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${R}_pipe$v.json')); r=d['roofline']
print('pipe=$v', d['value'], 'plain ms', r.get('avg_launch_ms'), 'frac', r['frac'], 'achieved', r['achieved'])"
done
[ -n "$NO_PMC" ] && exit 0
R=${R}p bash scripts/r4/gpu_r4_pmc.sh
