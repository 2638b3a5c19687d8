#!/usr/bin/env python3
"""CPU estimate (no GPU) of a decision-trie generalisation of the golden-march tables.

While fminbound takes golden steps, its probes depend only on the decisions taken so far: per step
"better" (fu <= fx) or one of the three "worse" updates (the probe replaces nfc, fulc, or neither).
The round-6 tables hold two such decision strings (kind 0 / kind 1).  A trie holds many: a search
marches while its decisions stay golden and its decision string stays inside the trie, and resumes
brent_step at the first node the trie lacks (or at its first parabolic step).

The trie is grown from searches at one set of steady-state positions (train: other seed / warm-ups)
and scored on the bench's positions (test), per wave of 64 slots: the max over lanes of march steps
and of brent_step steps, against the two-string tables.

    python tools/brent_trie.py [--scenario S_corridor] [--envs 4096] [--nodes 64,256,1024]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
from collections import Counter

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle")]

GOLD = 0.3819660112501051
SQRT_EPS = 1.4832396974191326e-08


def search(f, x1, x2, xatol=1e-6, maxfun=500):
    """scipy 1.15.3 fminbound; per step (parabolic, decision 0 better / 1 nfc / 2 fulc / 3 none)."""
    a, b = x1, x2
    fulc = a + GOLD * (b - a)
    nfc = xf = fulc
    rat = e = 0.0
    fx = f(xf)
    num = 1
    ffulc = fnfc = fx
    xm = 0.5 * (a + b)
    tol1 = SQRT_EPS * abs(xf) + xatol / 3.0
    tol2 = 2.0 * tol1
    log = []
    while abs(xf - xm) > (tol2 - 0.5 * (b - a)):
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
        if fu <= fx:
            dec = 0
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
                dec = 1
                fulc, ffulc = nfc, fnfc
                nfc, fnfc = x, fu
            elif (fu <= ffulc) or (fulc == xf) or (fulc == nfc):
                dec = 2
                fulc, ffulc = x, fu
            else:
                dec = 3
        log.append((par, dec))
        xm = 0.5 * (a + b)
        tol1 = SQRT_EPS * abs(xf) + xatol / 3.0
        tol2 = 2.0 * tol1
        if num >= maxfun:
            break
    return log


def golden_prefix(log):
    """decision strings of the golden prefix: node keys before each golden step."""
    keys = [()]
    for par, dec in log:
        if par:
            break
        keys.append(keys[-1] + (dec,))
    return keys  # keys[k] = node before step k (k <= number of golden steps)


def march_len(log, nodes):
    """steps a search marches through a trie holding `nodes`: the first step k that is parabolic or
    whose node is missing stops it (steps are re-checked per node)."""
    key = ()
    for k, (par, dec) in enumerate(log):
        if par or key not in nodes:
            return k
        key = key + (dec,)
    return len(log)


def positions(scn, sc, kw, envs, seed, warmups):
    import oracle
    from drone2d_amd.config import make_cfg
    b = oracle.OracleBatch(make_cfg(dict(kw)), [sc], envs)
    b.reset(seed)
    rng = np.random.default_rng(seed + 1)
    out = []
    done = 0
    for w in sorted(warmups):
        for _ in range(w - done):
            b.step(rng.uniform(-1, 1, (envs, 2)).astype(np.float32), nthreads=8)
        done = w
        st, _ = b.get_state()
        out.append(np.stack([st[0], st[1]], 1))
    return np.concatenate(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default="S_corridor")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--nodes", default="64,128,256,512,1024,4096")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import oracle

    import drone2d_amd  # noqa: F401
    from drone2d_amd.config import ENV_TRAIN_CONFIG
    from drone2d_amd.env import build_scenarios

    kw = dict(ENV_TRAIN_CONFIG, scenario=args.scenario)
    scn = build_scenarios(kw)[0]
    sc = scn.to_c()
    L = float(scn.path.length)

    def logs_at(P):
        res = []
        for px, py in P:
            def f(u, px=px, py=py):
                x, y = oracle.path_eval(sc, u)
                return math.sqrt((x - px) ** 2 + (y - py) ** 2)
            res.append(search(f, -10.0, L + 10.0))
        return res

    train = logs_at(positions(scn, sc, kw, args.envs, 777, [50, 150, 250, 400]))
    test = logs_at(positions(scn, sc, kw, args.envs, 12345, [300]))

    cnt = Counter()
    for lg in train:
        for key in golden_prefix(lg):
            cnt[key] += 1
    # the round-6 tables: kind 0 = (1, 0, 0, ...), kind 1 = (0, 0, ...), 48 steps each
    two = {()} | {(1,) + (0,) * k for k in range(48)} | {(0,) * (k + 1) for k in range(48)}

    def score(nodes):
        m = np.array([march_len(lg, nodes) for lg in test])
        n = np.array([len(lg) for lg in test])
        c = n - m
        M, Cc = m.reshape(-1, 64).max(1), c.reshape(-1, 64).max(1)
        return dict(nodes=len(nodes), march_mean=float(m.mean()), cont_mean=float(c.mean()),
                    wave_march_max=float(M.mean()), wave_cont_max=float(Cc.mean()),
                    cont_lane_frac=float((c > 0).mean()))

    n = np.array([len(lg) for lg in test])
    golden_all = np.array([len(golden_prefix(lg)) - 1 for lg in test])
    res = {"scenario": args.scenario, "envs": args.envs, "steps_mean": float(n.mean()),
           "wave_steps_max": float(n.reshape(-1, 64).max(1).mean()),
           "golden_prefix_mean": float(golden_all.mean()),
           "golden_prefix_wave_min": float(golden_all.reshape(-1, 64).min(1).mean()),
           "distinct_train_nodes": len(cnt), "two_strings": score(two), "trie": []}
    ranked = [k for k, _ in cnt.most_common()]
    for N in [int(x) for x in args.nodes.split(",")]:
        # most-visited nodes; a node is useful only with its parent, and visit counts never grow
        # along a path, so the top-N set is prefix-closed up to ties
        res["trie"].append(score(set(ranked[:N])))
    print(json.dumps(res, indent=1))
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
