#!/usr/bin/env python3
"""Per-launch HBM-side traffic of the step kernel from rocprofv3 PMC passes (tools/profile.sh).

    python tools/traffic.py gpurun_out/prof_TAG [--out profiles/traffic_corridor_65536.json]

FETCH_SIZE / WRITE_SIZE are KB per dispatch.  MI355X_MICROARCH.md (HBM, gfx950): FETCH_SIZE reports
half of the bytes of wide coalesced reads -> doubled; WRITE_SIZE is exact for streaming stores.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os

import numpy as np


def counter(d, name, kernel="d2d_step_kernel"):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == name and kernel in row["Kernel_Name"]:
                vals.append(float(row["Counter_Value"]))
    return np.array(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--out", default=None)
    ap.add_argument("--envs", type=int, default=65536)
    a = ap.parse_args()
    fetch = counter(os.path.join(a.prof_dir, "pmc_fetch"), "FETCH_SIZE")
    write = counter(os.path.join(a.prof_dir, "pmc_write"), "WRITE_SIZE")
    assert len(fetch) and len(write), "no FETCH_SIZE / WRITE_SIZE rows for d2d_step_kernel"
    # skip the first launches (episodes have not ended yet: no auto-reset traffic)
    f = np.median(fetch[len(fetch) // 2:]) * 1024.0 * 2.0
    w = np.median(write[len(write) // 2:]) * 1024.0
    res = {"kernel": "d2d_step_kernel", "envs": a.envs, "bytes_per_launch": f + w,
           "fetch_bytes_corrected": f, "write_bytes": w, "bytes_per_env_step": (f + w) / a.envs,
           "launches": [int(len(fetch)), int(len(write))],
           "note": "median over the second half of the profiled launches; FETCH_SIZE x2 (gfx950)"}
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
