#!/bin/bash
# ring-kernel parity on MI355X: the template-path tests (plane ring, windows, march), the GS
# template sweeps (fused ring and the acc + chain pair) and the SA V-cycle; logs kept small
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4d}
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernel_paths.py -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider --tb=short --maxfail=6 -k "ring or window_lanes or hybrid_gs_template or sa_gs_vcycle" > /tmp/t.log 2>&1
rc=$?
grep -v "amdgpu.ids" /tmp/t.log | tail -c 60000 > gpurun_out/${R}_tests.log
tail -30 gpurun_out/${R}_tests.log
echo "tests rc=$rc"
[ $rc -ge 124 ] && exit 1
for leg in 7pt:ring 7pt:noring sa27:ring sa27:noring sa27:nogsring; do
  cfg=${leg%%:*}; v=${leg##*:}
  case $v in noring) ev="AMG_TPL_RING=0";; nogsring) ev="AMG_GS_RING=0";; *) ev="AMG_NOTHING=0";; esac
  env $ev timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_${cfg}_$v.json 2> /tmp/b.err || { tail -c 2000 /tmp/b.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${R}_${cfg}_$v.json'))
print('$leg', d['value'], d['ms_per_step'], d['runtime'], d['config']['hipgraph'], d['roofline']['frac'])
for r in d['vcycle_kernels']: print('   ', r['level'], r['op'], r['us'], r['frac'])"
done
