#!/bin/bash
# Variant A/B at a given batch size (GPU box): bash tools/gpu_ab_envs.sh TAG ENVS "SCENARIOS" VARIANT...
set -u
TAG=$1; ENVS=$2; SCNS=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p "$OUT"
for S in $SCNS; do
  timeout -k 10 400 python3 "$R/tools/variants.py" run "$@" --scenario "$S" --envs "$ENVS" --rounds 3 > "$OUT/${S}_$ENVS.log" 2>&1 || { echo "STOP $S"; exit 1; }
  python3 - "$OUT/${S}_$ENVS.log" "$S" "$ENVS" <<'PY'
import json, sys
t = open(sys.argv[1]).read(); j = json.loads(t[t.index("{"):t.rindex("}") + 1])
print(sys.argv[2], sys.argv[3], {k: round(v["ms_per_step_min"] * 1000, 2) for k, v in j["variants"].items()}, "us/step")
PY
done
