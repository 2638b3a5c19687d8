#!/bin/bash
# Per-variant SQ instruction counters of the step kernel (GPU box): one rocprofv3 --pmc pass per
# variant library built by tools/variants.py (e.g. the role ablations: `variants.py build r0:D2D_ABL=1@role_ablation ...`,
# tools/patches/role_ablation.patch).
# Usage: bash tools/role_pmc.sh TAG...   -> gpurun_out/role_pmc/<TAG>/..., summary on stdout
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/role_pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for T in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-include-regex d2d_step_kernel -T --output-format csv -d "$OUT/$T" -o pmc \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -- \
    python3 "$R/tools/variants.py" run "$T" --rounds 1 --steps 40 --warmup 300 > "$OUT/$T.log" 2>&1 || { echo "STOP $T"; exit 1; }
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, os, sys
import numpy as np
out, tags = sys.argv[1], sys.argv[2:]
for t in tags:
    d = {}
    for f in glob.glob(os.path.join(out, t, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    med = {k: float(np.median(v[len(v) // 2:])) for k, v in d.items()}
    w = med.get("SQ_WAVES", 1.0)
    print(t, {k: round(v / (w / 4.0)) for k, v in sorted(med.items()) if k != "SQ_WAVES"}, "per workgroup")
PY
