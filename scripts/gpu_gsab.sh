#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do for lib in lib_ab_new lib_ab_head; do
  echo "== $lib"; RAPTOR_AMD_LIB=$PWD/raptor_amd/$lib.so timeout -k 10 300 python scripts/gs_time.py 256 27pt 2>&1 | grep -v amdgpu.ids || exit 1
done; done
