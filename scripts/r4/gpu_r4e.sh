#!/bin/bash
# A/B of the batched uniform-stencil window reads (AMG_TPL_MASTER_EB / AMG_TPL_GS_EB build
# knobs: libraptor_amd.so = batched, lib_ab_eb0.so = scheduler's order) x plane ring on/off,
# after the template-path parity tests of the default library.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4e}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernel_paths.py -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider --tb=short --maxfail=4 -k "ring or window_lanes or hybrid_gs_template or sa_gs_vcycle or master or uniform" > /tmp/t.log 2>&1
rc=$?
grep -v "amdgpu.ids" /tmp/t.log | tail -c 30000 > gpurun_out/${R}_tests.log
tail -5 gpurun_out/${R}_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit 1
for lib in libraptor_amd lib_ab_eb0; do
for leg in 7pt:ring 7pt:noring sa27:ring sa27:noring; do
  cfg=${leg%%:*}; v=${leg##*:}
  case $v in noring) ev="AMG_TPL_RING=0";; *) ev="AMG_NOTHING=0";; esac
  out=gpurun_out/${R}_${lib}_${cfg}_$v.json
  env $ev RAPTOR_AMD_LIB=raptor_amd/$lib.so timeout -k 10 400 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > $out 2> /tmp/b.err || { tail -c 2000 /tmp/b.err; exit 1; }
  python -c "
import json; d=json.load(open('$out'))
print('$lib $leg', d['value'], d['ms_per_step'])
for r in d['vcycle_kernels'][:5]: print('   ', r['level'], r['op'], r['us'], r['frac'])"
done; done
