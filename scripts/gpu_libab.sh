#!/bin/bash
# Same-box A/B of library builds (RAPTOR_AMD_LIB): CSR-kernel variant timings per build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for lib in ${LIBS:-libraptor_amd lib_ab_head lib_ab_nopad}; do
    echo "== $lib (rep $rep)"
    RAPTOR_AMD_LIB=$PWD/raptor_amd/$lib.so timeout -k 10 300 python scripts/spmv_variants.py 256 ${VARS:-10} > gpurun_out/ab_${lib}_$rep.txt 2>&1 || { tail gpurun_out/ab_${lib}_$rep.txt; exit 1; }
    grep -v amdgpu.ids gpurun_out/ab_${lib}_$rep.txt
  done
done
