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
    ap.add_argument("--mix", nargs="*", default=[],
                    help="counter CSVs of the VALU-mix passes (tools/profile.sh pmc_mix, pmc_mix2)")
    ap.add_argument("--util", default=None,
                    help="counter CSV of the lane-utilisation pass (tools/profile.sh pmc_util)")
    ap.add_argument("--envs", type=int, default=65536, help="envs per launch (per-env-step figures)")
    ap.add_argument("--commit", default=None, help="the commit the profile was taken on")
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(float))
    util = defaultdict(lambda: defaultdict(float))
    for f, dst in [(f, per) for f in [a.csv, *a.mix]] + ([(a.util, util)] if a.util else []):
        for r in csv.DictReader(open(f)):
            if a.kernel in r["Kernel_Name"]:
                dst[r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
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
    if a.commit:
        out["commit"] = a.commit
    if a.mix:
        # wave-instructions per SIMD per launch by class; each wave instruction covers 64 lanes
        cls = ["FMA_F64", "ADD_F64", "MUL_F64", "TRANS_F64", "INT32", "INT64", "CVT",
               "FMA_F32", "ADD_F32", "MUL_F32", "TRANS_F32"]
        mix = {c: med.get("SQ_INSTS_VALU_" + c) for c in cls if ("SQ_INSTS_VALU_" + c) in med}
        tot = med["SQ_INSTS_VALU"]
        mix["other"] = tot - sum(v for v in mix.values() if v is not None)
        per_env = SIMDS * 64.0 / a.envs  # wave-instructions per SIMD -> lane-instructions per env-step
        f64 = 2.0 * mix["FMA_F64"] + mix["ADD_F64"] + mix["MUL_F64"]
        out["mix_per_simd"] = mix
        out["mix_frac"] = {c: v / tot for c, v in mix.items()}
        out["fp64_flops_per_env_step_issued"] = f64 * per_env  # (2 FMA + ADD + MUL) x 64 lanes / env
        out["fp64_trans_per_env_step"] = mix["TRANS_F64"] * per_env
        if "SQ_INSTS_VALU_FLOPS_FP64" in med:
            # the hardware's own fp64 flop counter counts per wave-instruction (FMA = 2), like the
            # SQ_INSTS_VALU_* classes above, not per lane: x 64 lanes per env-step, it agrees with the
            # instruction-derived figure (round 4 printed it without the x 64: "123")
            out["fp64_flops_per_env_step_counter"] = med["SQ_INSTS_VALU_FLOPS_FP64"] * per_env
        out["salu_per_simd"] = med.get("SQ_INSTS_SALU")
        if util:
            # lanes a VALU instruction actually computes for (exec mask): thread-cycles over 64 x the
            # VALU-issue cycles of the same pass (rocprofiler's VALUUtilization).  The Brent
            # continuation runs with few active lanes, so the issued-lane fp64 figure overstates the
            # useful work; x this fraction estimates the active-lane figure (assuming the fp64
            # instructions' lane occupancy is the VALU average)
            um = {k: statistics.median(v.values()) for k, v in util.items()}
            frac = um["SQ_THREAD_CYCLES_VALU"] / (um["SQ_ACTIVE_INST_VALU"] * 64.0)
            out["valu_lane_util"] = frac
            out["fp64_flops_per_env_step_active_est"] = out["fp64_flops_per_env_step_issued"] * frac
            out["util_source"] = a.util
        out["mix_sources"] = a.mix
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
