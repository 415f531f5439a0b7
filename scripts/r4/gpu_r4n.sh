#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of sa27's level-0 GS kernels (separate passes) and their times
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${R:-r4n}
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/${R}_gs_$pass -o run -- python scripts/pmc_gs27.py 256 > gpurun_out/${R}_gs_$pass.log 2>&1 || { tail -5 gpurun_out/${R}_gs_$pass.log; exit 1; }
done
python scripts/pmc_generic.py gpurun_out/${R}_gs_FETCH_SIZE/run_counter_collection.csv gpurun_out/${R}_gs_WRITE_SIZE/run_counter_collection.csv | tee gpurun_out/${R}_gs_pmc.txt
