#!/bin/bash
# Same-box A/B over environment settings: VARIANTS="name1:VAR=1 VAR2=0;name2:..." (';'
# separated, empty setting = defaults) on the bench configs in $CONFIGS; bench lines under
# gpurun_out/${ROUND}_{name}_{cfg}.json and one summary line per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${ROUND:-envab}
IFS=';' read -ra VS <<< "${VARIANTS:-default:}"
for cfg in ${CONFIGS:-7pt}; do
  for v in "${VS[@]}"; do
    name=${v%%:*}; settings=${v#*:}
    env $settings timeout -k 10 400 python bench.py --config $cfg --no-cpu-baseline $BENCH_ARGS > gpurun_out/${R}_${name}_${cfg}.json 2> gpurun_out/${R}_${name}_${cfg}.err || { tail gpurun_out/${R}_${name}_${cfg}.err; exit 1; }
    python - "$name" "$cfg" gpurun_out/${R}_${name}_${cfg}.json <<'PY'
import json, sys
d = json.load(open(sys.argv[3]))
t = " ".join(f"L{k['level']}:{k['op'].split()[0]}={k['us']}" for k in d["vcycle_kernels"] if k["level"] <= 1)
print(sys.argv[1], sys.argv[2], d["value"], "csr", d["roofline"]["avg_launch_ms"], "stored", d["roofline_stored"]["avg_launch_ms"], t)
PY
  done
done
