#!/bin/bash
# SQ counters + kernel stats of the level-0 template kernels (scripts/dev/tpl_probe.py) with
# uniform-stencil rows (default) and with the per-template tables (AMG_TPL_MASTER=0); separate
# --pmc passes, no tracing with counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-tplsq2}
for v in master generic; do
  if [ $v = generic ]; then export AMG_TPL_MASTER=0; else unset AMG_TPL_MASTER; fi
  i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
              "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" \
              "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/${TAG}_${v}_p$i -o run -- python scripts/dev/tpl_probe.py 256 > gpurun_out/${TAG}_${v}_p$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_${v}_p$i.log; exit 1; }
    python scripts/pmc_generic.py gpurun_out/${TAG}_${v}_p$i/run_counter_collection.csv > gpurun_out/${TAG}_${v}_p$i.txt
  done
done
head -14 gpurun_out/${TAG}_*_p*.txt
