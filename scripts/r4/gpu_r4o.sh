#!/bin/bash
# template GS chain walk in 16-row batches (whole 128-byte lines): its tests, then same-box
# A/B against the 8-row build (raptor_amd/lib_ab_u8.so) on sa27, then its counters.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4o}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "hybrid_gs or sa_gs or sa27 or full_size_27pt or vcycle_bit_exact" > gpurun_out/${R}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${R}_tests.log; echo "tests rc=$rc"
[ $rc -ne 0 ] && exit 1
for i in 1 2; do
  for lib in libraptor_amd lib_ab_u8; do
    RAPTOR_AMD_LIB=raptor_amd/$lib.so timeout -k 10 300 python bench.py --config sa27 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${R}_${lib}_$i.json 2> /tmp/b.err || { tail -5 /tmp/b.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/${R}_${lib}_$i.json'))
print('$lib', d['value'], d['ms_per_step'], [(k['level'], k['op'].split()[0], k['us']) for k in d['vcycle_kernels'] if 'GS' in k['op']])"
  done
done
R=${R}n bash scripts/r4/gpu_r4n.sh
