#!/bin/bash
# round-4 evidence: N=2 rehearsal idle split (graph vs eager), setup timing 1 vs 8 loopback
# ranks, kernel-trace summaries of the 7-pt and g3sub bench commands.  Each step time-limited;
# a timeout or crash ends the script.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4f}
R=${R}n bash scripts/r4/gpu_r4_n2prof.sh > gpurun_out/${R}_n2prof.txt 2>&1; rc=$?
tail -40 gpurun_out/${R}_n2prof.txt; [ $rc -ne 0 ] && exit 1
AMG_TIMING=1 timeout -k 10 600 python -u scripts/setup_ranks.py 256 8 boxes > gpurun_out/${R}_setup8.json 2> gpurun_out/${R}_setup8.err
rc=$?; echo "setup8 rc=$rc $(cat gpurun_out/${R}_setup8.json)"; [ $rc -ge 124 ] && exit 1
for cfg in 7pt g3sub; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_prof_$cfg -o run -- python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_prof_$cfg.json 2> gpurun_out/${R}_prof_$cfg.err || { tail gpurun_out/${R}_prof_$cfg.err; exit 1; }
  python scripts/trace_summary.py gpurun_out/${R}_prof_$cfg/run_kernel_trace.csv > gpurun_out/${R}_${cfg}_trace_summary.txt
  head -25 gpurun_out/${R}_${cfg}_trace_summary.txt
done
for v in 1 0 1 0; do
  AMG_GS_CHAIN_BUCKETS=$v timeout -k 10 300 python bench.py --config g3sub --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_g3sub_b$v.json 2> /tmp/g.err || { tail -5 /tmp/g.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${R}_g3sub_b$v.json')); print('g3sub buckets=$v', d['value'], d['ms_per_step'], [(r['level'], r['op'][:6], r['us']) for r in d['vcycle_kernels'] if 'GS' in r['op']])"
done
echo r4f-done
