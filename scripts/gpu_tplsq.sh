#!/bin/bash
# SQ counters + kernel stats of the level-0 template kernels (scripts/dev/tpl_probe.py) for the
# default library and $ALT (separate --pmc passes, no tracing with counters)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-tplsq}
for v in default alt; do
  if [ $v = alt ]; then export RAPTOR_AMD_LIB=$GRAFT_REPO_ROOT/$ALT; else unset RAPTOR_AMD_LIB; fi
  i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
              "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/${TAG}_${v}_p$i -o run -- python scripts/dev/tpl_probe.py 256 > gpurun_out/${TAG}_${v}_p$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_${v}_p$i.log; exit 1; }
    python scripts/pmc_generic.py gpurun_out/${TAG}_${v}_p$i/run_counter_collection.csv > gpurun_out/${TAG}_${v}_p$i.txt
  done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${v}_trace -o run -- python scripts/dev/tpl_probe.py 256 > gpurun_out/${TAG}_${v}_trace.log 2>&1 || exit 1
done
head -12 gpurun_out/${TAG}_*_p*.txt
