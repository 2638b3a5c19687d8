#!/bin/bash
# Layout / variant A/B on the GPU box: step time per scenario for each variant (tools/variants.py).
# Usage: bash tools/gpu_ab.sh TAG "SCENARIOS" VARIANT...
set -u
TAG=$1; SCNS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p "$OUT"
for S in $SCNS; do
  timeout -k 10 400 python3 "$R/tools/variants.py" run "$@" --scenario "$S" --rounds 3 > "$OUT/$S.log" 2>&1 || { echo "STOP $S"; exit 1; }
  python3 - "$OUT/$S.log" "$S" <<'PY'
import json, sys
t = open(sys.argv[1]).read(); j = json.loads(t[t.index("{"):t.rindex("}") + 1])
print(sys.argv[2], {k: round(v["ms_per_step_min"] * 1000, 2) for k, v in j["variants"].items()}, "us/step")
PY
done
