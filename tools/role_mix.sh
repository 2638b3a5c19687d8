#!/bin/bash
# VALU instruction mix of the step kernel per variant library (tools/variants.py builds, e.g. the
# role ablations: `variants.py build r0:D2D_ABL=1@role_ablation ...`,
# tools/patches/role_ablation.patch): one rocprofv3 --pmc pass per variant.  The difference base - variant is
# the skipped role's share.  Usage: [SCN=scenario] bash tools/role_mix.sh TAG...  -> gpurun_out/role_mix/<TAG>/...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/role_mix${SCN:+_$SCN}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for T in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-include-regex d2d_step_kernel -T --output-format csv -d "$OUT/$T" -o pmc \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 \
          SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU -- \
    python3 "$R/tools/variants.py" run "$T" --rounds 1 --steps 40 --warmup 300 --scenario "${SCN:-corridor}" > "$OUT/$T.log" 2>&1 || { echo "STOP $T"; exit 1; }
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, os, sys
import numpy as np
out, tags = sys.argv[1], sys.argv[2:]
for t in tags:
    d = {}
    for f in glob.glob(os.path.join(out, t, "**", "*counter_collection.csv"), recursive=True):
        per = {}
        for r in csv.DictReader(open(f)):
            per[(r["Counter_Name"], r["Dispatch_Id"])] = per.get((r["Counter_Name"], r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
        for (k, _), v in per.items():
            d.setdefault(k, []).append(v)
    med = {k: float(np.median(v[len(v) // 2:])) / 1024.0 for k, v in d.items()}  # per SIMD
    oth = med["SQ_INSTS_VALU"] - sum(med[k] for k in med if k.startswith("SQ_INSTS_VALU_"))
    print(t, {k.replace("SQ_INSTS_", ""): round(v) for k, v in sorted(med.items())}, "OTHER", round(oth), "per SIMD")
PY
