#!/bin/bash
# persistent vs one-shot row-template kernel (AMG_TPL_PERSIST), same box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-pers}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for rep in 1 2; do
  for p in 1 0; do
    AMG_TPL_PERSIST=$p timeout -k 10 300 python scripts/spmv_variants.py 256 42 > gpurun_out/${T}_p${p}_$rep.txt 2>&1 || { tail -20 gpurun_out/${T}_p${p}_$rep.txt; exit 1; }
    echo "persist=$p rep $rep"; grep A0 gpurun_out/${T}_p${p}_$rep.txt
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
python -c "
import json; d = json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['roofline']['avg_launch_ms'], d['roofline']['achieved'], d['roofline']['frac'])"
