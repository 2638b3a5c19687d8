"""Diagnostic (not product): does stepping the 65 536 envs as two independent 32 768-env shards on two
streams (one captured graph with two branches) hide the step kernel's tail?  Compares ms per step of
one handle against two handles (global env ids, the same envs) for the given scenarios."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: F401,E402
from drone2d_amd import shard  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402

MIXED = ["perpendicular", "parallel", "S_parallel", "corridor", "S_corridor", "large", "impossible"]
N, GLEN, WARM, STEPS = 65536, 256, 300, 2048


def run(scn, parts):
    kw = dict(ENV_TRAIN_CONFIG, scenario=MIXED if scn == "mixed" else scn)
    dev = torch.device("cuda", 0)
    envs = [shard.make_shard_venv(N, r, parts, device=dev, seed=12345, with_info=False, **kw) for r in range(parts)]
    g = torch.Generator(device=dev).manual_seed(1000)
    bank = [torch.rand(N, 2, device=dev, generator=g) * 2 - 1 for _ in range(16)]
    n = N // parts
    banks = [[b[r * n:(r + 1) * n].contiguous() for b in bank] for r in range(parts)]
    for e in envs:
        e.reset()
    main = torch.cuda.current_stream(dev)
    streams = [torch.cuda.Stream(dev) for _ in range(parts)]
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        cap = torch.cuda.current_stream(dev)
        for r in range(parts):
            streams[r].wait_stream(cap)
            with torch.cuda.stream(streams[r]):
                for k in range(GLEN):
                    envs[r].step(banks[r][k % 16])
        for r in range(parts):
            cap.wait_stream(streams[r])
    torch.cuda.synchronize()
    for _ in range(max(1, WARM // GLEN)):
        gr.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(STEPS // GLEN):
        gr.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for e in envs:
        e.close()
    return dt / STEPS * 1e6


for scn in sys.argv[1:] or ["corridor", "mixed"]:
    one = run(scn, 1)
    two = run(scn, 2)
    four = run(scn, 4)
    print(f"{scn}: us/step one handle {one:.2f}, two streams {two:.2f}, four streams {four:.2f}", flush=True)
