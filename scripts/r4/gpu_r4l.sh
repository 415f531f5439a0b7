#!/bin/bash
# g3sub: split hybrid-GS sweeps on every level (AMG_GS_SPLIT_NPR=0) vs the default rule (rows of
# >= 12 entries: level 0, 5.5 per row, keeps the one-kernel sweep), alternating runs.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4l}
for i in 1 2; do
  for v in default 0; do
    ev="AMG_NOTHING=0"; [ $v = 0 ] && ev="AMG_GS_SPLIT_NPR=0"
    env $ev timeout -k 10 300 python bench.py --config g3sub --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_npr${v}_$i.json 2> /tmp/b.err || { tail -5 /tmp/b.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/${R}_npr${v}_$i.json'))
print('npr=$v', d['value'], d['ms_per_step'], [(k['level'], k['op'].split()[0], k['us']) for k in d['vcycle_kernels'] if 'GS' in k['op']])"
  done
done
