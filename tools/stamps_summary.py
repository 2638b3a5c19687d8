#!/usr/bin/env python3
"""Print the per-role phase-A / total cycle summary of gpurun_out/stamps*.json."""
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps*.json")):
    for r in json.load(open(f)):
        print(f, r["envs"], "w2_by_simd_share", r.get("w2_by_simd_share"))
        for w in range(4):
            d = r[f"wave{w}"]
            print(f"  w{w} phaseA {d['phase1']}  total {d['total']}")
