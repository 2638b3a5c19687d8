#!/usr/bin/env python3
"""CPU analysis of the Brent searches a K1 path wave runs (no GPU): steady-state lane positions
from the C oracle (the bench's workload: random U(-1,1) actions, auto-reset, W warmup steps), then
per search scipy's fminbound step sequence (_optimize.py:2251-2398) with its decisions logged:

  kind / dev   the golden-march table kind and the first step whose decision differs (the search
               resumes brent_step there: the "continuation")
  decisions    per continuation step: parabolic or golden, new probe better (le) or worse

and per wave of 64 consecutive slots: lanes in continuation, max / sum of continuation steps, so
lane utilisation and packing alternatives can be priced before writing kernel code.

    python tools/brent_lanes.py [--scenario corridor] [--envs 4096] [--warmup 300]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]

GOLD = 0.3819660112501051
SQRT_EPS = 1.4832396974191326e-08


def fminbound_log(f, x1, x2, xatol=1e-6, maxfun=500):
    a, b = x1, x2
    fulc = a + GOLD * (b - a)
    nfc = xf = fulc
    rat = e = 0.0
    x = xf
    fx = f(x)
    num = 1
    ffulc = fnfc = fx
    xm = 0.5 * (a + b)
    tol1 = SQRT_EPS * abs(xf) + xatol / 3.0
    tol2 = 2.0 * tol1
    log = []  # (par, le, plain worse, speculation possible before the step) per step
    while abs(xf - xm) > (tol2 - 0.5 * (b - a)):
        spec_ok = (nfc != xf) and (fulc != xf) and (fulc != nfc)
        golden = True
        par = False
        if abs(e) > tol1:
            golden = False
            r = (xf - nfc) * (fx - ffulc)
            q = (xf - fulc) * (fx - fnfc)
            p = (xf - fulc) * q - (xf - nfc) * r
            q = 2.0 * (q - r)
            if q > 0.0:
                p = -p
            q = abs(q)
            r = e
            e = rat
            if (abs(p) < abs(0.5 * q * r)) and (p > q * (a - xf)) and (p < q * (b - xf)):
                rat = (p + 0.0) / q
                x = xf + rat
                par = True
                if ((x - a) < tol2) or ((b - x) < tol2):
                    si = np.sign(xm - xf) + ((xm - xf) == 0)
                    rat = tol1 * si
            else:
                golden = True
        if golden:
            e = (a - xf) if xf >= xm else (b - xf)
            rat = GOLD * e
        si = np.sign(rat) + (rat == 0)
        x = xf + si * max(abs(rat), tol1)
        fu = f(x)
        num += 1
        le = fu <= fx
        plain_worse = (not le) and not (fu <= fnfc) and not (fu <= ffulc)
        if le:
            if x >= xf:
                a = xf
            else:
                b = xf
            fulc, ffulc = nfc, fnfc
            nfc, fnfc = xf, fx
            xf, fx = x, fu
        else:
            if x < xf:
                a = x
            else:
                b = x
            if (fu <= fnfc) or (nfc == xf):
                fulc, ffulc = nfc, fnfc
                nfc, fnfc = x, fu
            elif (fu <= ffulc) or (fulc == xf) or (fulc == nfc):
                fulc, ffulc = x, fu
        if log:  # the previous step's "better" speculation held iff it was better and this step is golden
            log[-1] = log[-1][:4] + (log[-1][1] and not par,)
        log.append((par, le, plain_worse, spec_ok, False))
        xm = 0.5 * (a + b)
        tol1 = SQRT_EPS * abs(xf) + xatol / 3.0
        tol2 = 2.0 * tol1
        if num >= maxfun:
            break
    return xf, log


def table_dev(log, kind_len):
    """kind (step 0: better -> 1, worse -> 0) and the first step k >= 1 whose decision is not
    'golden, better' (the table's), capped at the table length."""
    kind = 1 if log and log[0][1] else 0
    n = kind_len[kind]
    for k in range(1, min(len(log), n)):
        par, le = log[k][:2]
        if par or not le:
            return kind, k
    return kind, min(len(log), n)


def spec_iterations(steps, mode="worse"):
    """Wave-loop passes a lane needs for `steps` (log entries) when every pass evaluates the step's
    probe AND, speculatively, the next step's probe under the assumption that this step's new probe
    is "plain worse" (not better, no nfc / fulc update: the next probe then depends on the bracket
    alone); a pass whose assumption holds completes two steps."""
    it = k = 0
    prev_better = False
    while k < len(steps):
        par, le, pw, ok, bg = steps[k]
        it += 1
        w_hit = ok and pw
        b_hit = bg
        if mode == "worse":
            hit = w_hit
        elif mode == "better":
            hit = b_hit
        elif mode == "predict":   # the previous step's outcome picks the speculation
            hit = b_hit if prev_better else w_hit
        else:                     # both (three probes per pass)
            hit = w_hit or b_hit
        hit = hit and k + 1 < len(steps)
        prev_better = steps[k + 1][1] if hit else le
        k += 2 if hit else 1
    return it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default="corridor")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import oracle

    import drone2d_amd  # noqa: F401
    from drone2d_amd.config import ENV_TRAIN_CONFIG, make_cfg
    from drone2d_amd.env import build_scenarios

    kw = dict(ENV_TRAIN_CONFIG, scenario=args.scenario)
    scn = build_scenarios(kw)[0]
    sc = scn.to_c()
    b = oracle.OracleBatch(make_cfg(dict(kw)), [sc], args.envs)
    b.reset(12345)
    rng = np.random.default_rng(1000)
    for _ in range(args.warmup):
        b.step(rng.uniform(-1, 1, (args.envs, 2)).astype(np.float32), nthreads=8)
    st, _ = b.get_state()
    px, py = st[0], st[1]
    L = float(scn.path.length)

    def fdist(p):
        def f(u):
            x, y = oracle.path_eval(sc, u)
            dx, dy = x - p[0], y - p[1]
            return math.sqrt(dx * dx + dy * dy)
        return f

    # table lengths: forced marches (kind 0: worse then better; kind 1: always better)
    def forced_len(kind):
        a, bb = -10.0, L + 10.0
        fulc = a + GOLD * (bb - a)
        xf = nfc = fulc
        e = 0.0
        k = 0
        xm = 0.5 * (a + bb)
        tol1 = SQRT_EPS * abs(xf) + 1e-6 / 3.0
        while abs(xf - xm) > (2 * tol1 - 0.5 * (bb - a)) and k < 48:
            e = (a - xf) if xf >= xm else (bb - xf)
            rat = GOLD * e
            x = xf + (np.sign(rat) + (rat == 0)) * max(abs(rat), tol1)
            le = not (kind == 0 and k == 0)
            if le:
                if x >= xf:
                    a = xf
                else:
                    bb = xf
                xf = x
            else:
                if x < xf:
                    a = x
                else:
                    bb = x
            k += 1
            xm = 0.5 * (a + bb)
            tol1 = SQRT_EPS * abs(xf) + 1e-6 / 3.0
        return k

    kind_len = [forced_len(0), forced_len(1)]
    rows = []
    for i in range(args.envs):
        _, log = fminbound_log(fdist((px[i], py[i])), -10.0, L + 10.0)
        kind, dev = table_dev(log, kind_len)
        cont = log[dev:] if dev < len(log) else []
        # trailing run of golden-worse steps in the continuation
        tail = 0
        for par, le, *_ in reversed(cont):
            if par or le:
                break
            tail += 1
        rows.append(dict(n=len(log), kind=kind, dev=dev, cont=len(cont), tail=tail,
                         par=sum(x[0] for x in cont), gw=sum((not x[0]) and (not x[1]) for x in cont),
                         **{f"cont_{m}": spec_iterations(cont, m) for m in ("worse", "better", "predict", "both")},
                         **{f"full_{m}": spec_iterations(log, m) for m in ("worse", "better", "predict", "both")}))
    C = np.array([r["cont"] for r in rows])
    T = np.array([r["tail"] for r in rows])
    waves = C.reshape(-1, 64)
    tails = T.reshape(-1, 64)
    lanes = (waves > 0).sum(1)
    wmax = waves.max(1)
    wsum = waves.sum(1)
    # alternatives (wave-steps of continuation per 64 envs)
    pair_max = np.maximum(waves[0::2].max(1), waves[1::2].max(1))  # two waves pooled -> one (if <= 64 lanes)
    pooled_ok = (lanes[0::2] + lanes[1::2]) <= 64
    # pooled with refill (lanes pull the next search when done): ~max(longest, ceil(sum / 64))
    refill = np.maximum(pair_max, np.ceil((wsum[0::2] + wsum[1::2]) / 64.0))
    notail = (waves - tails).max(1)
    res = {
        "scenario": args.scenario, "envs": args.envs, "warmup": args.warmup, "table_len": kind_len,
        "steps_mean": float(np.mean([r["n"] for r in rows])), "steps_max": int(max(r["n"] for r in rows)),
        "kind0_frac": float(np.mean([r["kind"] == 0 for r in rows])),
        "dev_mean": float(np.mean([r["dev"] for r in rows])),
        "cont_lane_frac": float((C > 0).mean()), "cont_mean_active": float(C[C > 0].mean()) if (C > 0).any() else 0.0,
        "wave_cont_max_mean": float(wmax.mean()), "wave_cont_lanes_mean": float(lanes.mean()),
        "lane_util": float(wsum.sum() / (64.0 * wmax.sum())),
        "pooled_two_waves_wave_steps_per_64": float(pair_max.mean() / 2), "pooled_fits_64_frac": float(pooled_ok.mean()),
        "pooled_refill_wave_steps_per_64": float(refill.mean() / 2),
        "tail_mean_active": float(T[C > 0].mean()) if (C > 0).any() else 0.0,
        "wave_max_without_golden_tail": float(notail.mean()),
        "par_frac_of_cont": float(sum(r["par"] for r in rows) / max(1, C.sum())),
        "golden_worse_frac_of_cont": float(sum(r["gw"] for r in rows) / max(1, C.sum())),
        # speculative next-probe evaluation (spec_iterations): wave-max passes of the continuation
        # (tables) and of the whole search (no tables: the fresh curriculum's plain search)
        "wave_full_max_mean": float(np.array([r["n"] for r in rows]).reshape(-1, 64).max(1).mean()),
        **{f"wave_{p}_max_spec_{m}": float(np.array([r[f"{p}_{m}"] for r in rows]).reshape(-1, 64).max(1).mean())
           for p in ("cont", "full") for m in ("worse", "better", "predict", "both")},
    }
    print(json.dumps(res, indent=1))
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
