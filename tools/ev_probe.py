"""Diagnostic: wall time per step of a 20-step eager window (after 5 warm-up steps) with the bench's
HIP event pair around it, without events, and with the start event recorded before the window
(alternating rounds, corridor, 65 536 envs).  python tools/ev_probe.py (GPU box)"""
import statistics, sys, time
sys.path.insert(0, ".")
import torch
import drone2d_amd as d2
from drone2d_amd import shard
from drone2d_amd.config import ENV_TRAIN_CONFIG
n = 65536
kw = dict(ENV_TRAIN_CONFIG, scenario="corridor")
venv = shard.make_shard_venv(n, 0, 1, device=torch.device("cuda", 0), seed=12345, with_info=False, **kw)
g = torch.Generator(device="cuda").manual_seed(1000)
bank = [torch.rand(n, 2, device="cuda", generator=g) * 2 - 1 for _ in range(16)]
venv.reset()
stream = torch.cuda.current_stream()
for k in range(400):
    venv.step(bank[k % 16])
torch.cuda.synchronize()
res = {"events": [], "none": [], "early_start": []}
for r in range(12):
    for mode in res:
        for k in range(5):
            venv.step(bank[k % 16])
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if mode == "early_start":
            s.record(stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "events":
            s.record(stream)
        for k in range(20):
            venv.step(bank[k % 16])
        if mode != "none":
            e.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e6 / 20
        res[mode].append(wall)
for m, v in res.items():
    print(m, "us/step median %.2f min %.2f" % (statistics.median(v), min(v)))
