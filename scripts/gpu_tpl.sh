#!/bin/bash
# row-template kernel: GPU tests, per-level A/B against the CSR block kernel (variant 42 =
# templates + VI + XCD, 10 = VI + XCD), window vs global x loads, and short benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-tpl}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q ${TESTK:+-k "$TESTK"} --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
timeout -k 10 300 python scripts/spmv_variants.py 256 42,10 > gpurun_out/${T}_var_win.txt 2>&1 || { tail -20 gpurun_out/${T}_var_win.txt; exit 1; }
AMG_TPL_WINDOW=0 timeout -k 10 300 python scripts/spmv_variants.py 256 42,10 > gpurun_out/${T}_var_glob.txt 2>&1 || { tail -20 gpurun_out/${T}_var_glob.txt; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_win.json 2> gpurun_out/${T}_bench_win.err || exit 1
AMG_TPL_WINDOW=0 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench_glob.json 2> gpurun_out/${T}_bench_glob.err || exit 1
cat gpurun_out/${T}_var_win.txt gpurun_out/${T}_var_glob.txt
python -c "
import json
for f in ('win', 'glob'):
    d = json.load(open('gpurun_out/${T}_bench_' + f + '.json'))
    print(f, d['value'], d['roofline']['avg_launch_ms'], d['roofline']['achieved'], d['roofline']['frac'])
"
