#!/bin/bash
# same-box A/B of the round-4 kernel changes (alternating runs): the pipelined plain-CSR
# roofline kernel (AMG_PLAIN_PIPE) and the two-deep template GS chain walk
# (AMG_GS_CHAIN_DEEP) on sa27 / g3sub.  Each run time-limited; a failure ends the script.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4k}
run() {  # run <tag> <env> <bench args...>
  local tag=$1 ev=$2; shift 2
  env $ev timeout -k 10 300 python bench.py "$@" --no-cpu-baseline > gpurun_out/${R}_$tag.json 2> /tmp/b.err || { tail -5 /tmp/b.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${R}_$tag.json')); r=d['roofline']
gs=[(k['level'], k['op'].split()[0], k['us']) for k in d['vcycle_kernels'] if 'GS' in k['op']]
print('$tag', d['value'], d['ms_per_step'], 'plain', r.get('avg_launch_ms'), r['frac'], gs)"
}
for i in 1 2; do
  run 7pt_pipe1_$i AMG_PLAIN_PIPE=1 --steps 10 --warmup 3
  run 7pt_pipe0_$i AMG_PLAIN_PIPE=0 --steps 10 --warmup 3
done
for cfg in sa27 g3sub; do
  for i in 1 2; do
    run ${cfg}_deep1_$i AMG_GS_CHAIN_DEEP=1 --config $cfg --steps 20 --warmup 5
    run ${cfg}_deep0_$i AMG_GS_CHAIN_DEEP=0 --config $cfg --steps 20 --warmup 5
  done
done
echo r4k-done
