#!/bin/bash
# SQ / TA / TCP / TCC counters of the plain-CSR roofline kernel (scripts/dev/plain_probe.py),
# one --pmc pass each, no tracing with counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-plainpmc}
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM" \
            "TA_BUSY_avr TA_BUSY_max TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum" \
            "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python scripts/dev/plain_probe.py 256 > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/${TAG}_p$i.log; exit 1; }
  python scripts/pmc_generic.py gpurun_out/${TAG}_p$i/run_counter_collection.csv > gpurun_out/${TAG}_p$i.txt
  grep -E "kernel |csr_plain" gpurun_out/${TAG}_p$i.txt
done
