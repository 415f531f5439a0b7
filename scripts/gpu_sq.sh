#!/bin/bash
# SQ stall / LDS / TA counters on the level operators (separate --pmc passes, no tracing)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-sq}
timeout -k 10 120 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1 || true
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" \
            "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python scripts/pmc_levels.py 256 > gpurun_out/${TAG}_p$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python scripts/pmc_generic.py gpurun_out/${TAG}_p1/run_counter_collection.csv > gpurun_out/${TAG}_p1.txt
python scripts/pmc_generic.py gpurun_out/${TAG}_p2/run_counter_collection.csv > gpurun_out/${TAG}_p2.txt
python scripts/pmc_generic.py gpurun_out/${TAG}_p3/run_counter_collection.csv > gpurun_out/${TAG}_p3.txt
head -14 gpurun_out/${TAG}_p1.txt gpurun_out/${TAG}_p2.txt gpurun_out/${TAG}_p3.txt
