#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of tools/ubench_traffic.hip's known-byte kernels (GPU box), one rocprofv3
# --pmc pass per counter, then the measured / algorithmic ratio per kernel and access width.
# Usage: bash tools/ubench_traffic.sh TAG [envs]   -> gpurun_out/ubench_traffic_TAG/
set -u
TAG=${1:-r05}
N=${2:-65536}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ubench_traffic_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
B=$R/tools/ubench_traffic
[ -x "$B" ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o "$B" "$R/tools/ubench_traffic.hip" || exit 1
"$B" "$N" > "$OUT/bytes.json" || exit 1
cd /tmp
timeout -s KILL 60 rocprofv3 -T --output-format csv -d "$OUT/fetch" -o fetch --pmc FETCH_SIZE -- "$B" "$N" > "$OUT/fetch.log" 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 -T --output-format csv -d "$OUT/write" -o write --pmc WRITE_SIZE -- "$B" "$N" > "$OUT/write.log" 2>&1 || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys
out = sys.argv[1]
want = json.load(open(os.path.join(out, "bytes.json")))
res = {"envs": want["envs"]}
for ctr, key in (("FETCH_SIZE", "read"), ("WRITE_SIZE", "write")):
    per = {}
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == ctr:
                per.setdefault(r["Kernel_Name"].split("(")[0], []).append(float(r["Counter_Value"]) * 1024.0)
    for k, v in per.items():
        v = sorted(v)[len(v) // 2]  # median over the 5 launches
        w = want.get(k, {}).get(key)
        if w:
            res.setdefault(k, {})[ctr] = {"measured_bytes": v, "algorithmic_bytes": w, "ratio": v / w}
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(out, "traffic_calibration.json"), "w"), indent=1)
PY
