#!/bin/bash
# Same-box A/B: the default library and an alternative build (RAPTOR_AMD_LIB=$ALT) on the bench
# configs in $CONFIGS; bench lines under gpurun_out/${R}_{default,alt}_{cfg}.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-ab}
for cfg in ${CONFIGS:-7pt}; do
  for v in default alt; do
    if [ $v = alt ]; then export RAPTOR_AMD_LIB=$GRAFT_REPO_ROOT/$ALT; else unset RAPTOR_AMD_LIB; fi
    timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline $BENCH_ARGS > gpurun_out/${R}_${v}_${cfg}.json 2> gpurun_out/${R}_${v}_${cfg}.err || { tail gpurun_out/${R}_${v}_${cfg}.err; exit 1; }
    python - "$v" "$cfg" gpurun_out/${R}_${v}_${cfg}.json <<'PY'
import json, sys
d = json.load(open(sys.argv[3]))
t = " ".join(f"L{k['level']}:{k['op'].split()[0]}={k['us']}" for k in d["vcycle_kernels"])
print(sys.argv[1], sys.argv[2], d["value"], "csr", d["roofline"]["avg_launch_ms"], "stored", d["roofline_stored"]["avg_launch_ms"], t)
PY
  done
done
