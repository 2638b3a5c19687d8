#!/usr/bin/env python3
"""VALU-issue summary of the step kernel from a rocprofv3 SQ counter pass (tools/profile.sh's
pmc_sq): per SIMD per launch, VALU wave-instructions, the cycles the SIMD spent issuing VALU work and
the wave lifetime.  bench.py reads the JSON into its "valu" object (the kernel's actual bound: fp64
VALU issue, DESIGN.md "What bounds it").

    python tools/valu.py profiles/r01/v10/pmc_sq.csv --out profiles/valu_corridor_65536.json
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics
from collections import defaultdict

SIMDS = 256 * 4  # MI355X: 256 CUs x 4 SIMDs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", default="d2d_step_kernel")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(a.csv)):
        if a.kernel in r["Kernel_Name"]:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    med = {k: statistics.median(v.values()) / SIMDS for k, v in per.items()}
    # SQ_WAVE_CYCLES and SQ_ACTIVE_INST_VALU count in units of 4 cycles (quad-cycles); SQ_WAVE_CYCLES
    # sums the lifetimes of the SIMD's waves
    waves = med["SQ_WAVES"]
    life = med["SQ_WAVE_CYCLES"] * 4.0 / waves
    active = med["SQ_ACTIVE_INST_VALU"] * 4.0
    out = {"kernel": a.kernel, "source": a.csv, "simds": SIMDS, "waves_per_simd": waves,
           "valu_insts_per_simd": med["SQ_INSTS_VALU"], "valu_active_cycles_per_simd": active,
           "wave_lifetime_cycles": life, "valu_busy_frac": active / life,
           "note": "per SIMD per launch, median over dispatches; busy = VALU-issue cycles / wave lifetime"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
