#!/usr/bin/env python3
"""Per-step HBM-side traffic of the step path from rocprofv3 PMC passes (tools/profile.sh).

    python tools/traffic.py gpurun_out/prof_TAG [--out profiles/traffic_corridor_65536.json]

One env step is one d2d_step_kernel launch plus its share of the periodic d2d_fill_kernel: the
bytes of both kernels over the second half of the profiled dispatches, divided by the number of
step-kernel launches there.  FETCH_SIZE / WRITE_SIZE are KB per dispatch.  MI355X_MICROARCH.md
(HBM, gfx950): FETCH_SIZE reports half of the bytes of wide coalesced reads -> doubled; WRITE_SIZE
is exact for streaming stores.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os



def counter(d, name):
    """[(dispatch id, kernel, value)] of the d2d kernels, in dispatch order"""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == name and row["Kernel_Name"].startswith("d2d_"):
                rows.append((int(row["Dispatch_Id"]), row["Kernel_Name"], float(row["Counter_Value"])))
    return sorted(rows)


def per_step(rows):
    """bytes per step over the second half of the launches: (step + fill kernels) / step launches"""
    rows = rows[len(rows) // 2:]
    steps = sum(1 for _, k, _ in rows if k.startswith("d2d_step_kernel"))
    step_b = sum(v for _, k, v in rows if k.startswith("d2d_step_kernel"))
    fill_b = sum(v for _, k, v in rows if k.startswith("d2d_fill_kernel"))
    return (step_b + fill_b) * 1024.0 / max(steps, 1), step_b * 1024.0 / max(steps, 1), steps


def per_buffer(fd, read_meas, write_meas):
    """Bytes per env-step by buffer: the 650 B of the roofline plus what the
    auto-reset adds at fd episodes finished per env-step, against the measured read / write bytes."""
    rd = {"state (32 fp64 SoA fields)": 256.0, "t + flags (int32)": 8.0, "action (2 f32)": 8.0,
          "episode counter (int32, every step)": 4.0,
          "finished episodes: reset-cache tag + accumulators (4 + 64 B)": 68.0 * fd,
          "fill kernel: cache tags / episode counters, every 16th step (8 B / 16)": 0.5}
    wr = {"state (32 fp64 SoA fields; the spawn state for envs that reset)": 256.0, "t + flags": 8.0,
          "obs row (27 f32)": 108.0, "reward (f32)": 4.0, "terminated + truncated (u8)": 2.0,
          "finished episodes: episode counter + terminal obs row + 7 accumulators (4 + 108 + 56 B)": 168.0 * fd,
          "fill kernel: reset-cache obs row + flags + tag (108 + 4 + 4 B) per finished episode": 116.0 * fd}
    r_alg, w_alg = sum(rd.values()), sum(wr.values())
    return {"done_frac": fd, "read": rd, "write": wr, "read_attributed": r_alg, "write_attributed": w_alg,
            "read_measured": read_meas, "write_measured": write_meas,
            "unattributed": (read_meas - r_alg) + (write_meas - w_alg),
            "note": "650 B algorithmic (272 read + 378 write) + the auto-reset's per-episode bytes at the bench's "
                    "episode rate; measured = FETCH_SIZE x 2 / WRITE_SIZE per env-step. The joint sweep's "
                    "scratch spill (40 B each way, round 5 until the LDS stash) is gone"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--out", default=None)
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--done-frac", type=float, default=None,
                    help="episodes finished per env-step (the bench line's episodes: finished / sum_len); "
                         "adds the per-buffer table")
    ap.add_argument("--source", default=None, help="the committed PMC CSVs the figures come from")
    ap.add_argument("--commit", default=None, help="the commit the profile was taken on")
    a = ap.parse_args()
    fetch = counter(os.path.join(a.prof_dir, "pmc_fetch"), "FETCH_SIZE")
    write = counter(os.path.join(a.prof_dir, "pmc_write"), "WRITE_SIZE")
    assert len(fetch) and len(write), "no FETCH_SIZE / WRITE_SIZE rows for the d2d kernels"
    # second half only: by then episodes end and the fill kernel runs (auto-reset traffic)
    f, f_step, nf = per_step(fetch)
    w, w_step, nw = per_step(write)
    f, f_step = 2.0 * f, 2.0 * f_step
    res = {"kernel": "d2d_step_kernel + d2d_fill_kernel share", "envs": a.envs, "bytes_per_launch": f + w,
           "fetch_bytes_corrected": f, "write_bytes": w, "bytes_per_env_step": (f + w) / a.envs,
           "step_kernel_only_bytes": f_step + w_step, "step_launches": [nf, nw],
           "note": "per step = (step + fill kernel bytes) / step launches over the second half of the "
                   "profiled launches; FETCH_SIZE x2 (gfx950)"}
    if a.done_frac is not None:
        res["per_buffer"] = per_buffer(a.done_frac, f / a.envs, w / a.envs)
    if a.source:
        res["source"] = a.source
    if a.commit:
        res["commit"] = a.commit
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
