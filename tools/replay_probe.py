"""Diagnostic (not product): where the driver's short bench line (20 timed steps after 5 warm-up
steps) loses against the steady state.  Builds the bench's batch, captures one 20-step graph (as
bench.py does for --steps 20), runs the bench's clock warm-up and 5 eager warm-up steps, then
replays the graph R times: per replay the host wall time (synchronize on both sides) and the HIP
event time on the launch stream.  Replay 1 is the bench's timed region; later replays show the
same graph once it is warm and the episodes older."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
import drone2d_amd  # noqa: E402,F401
from drone2d_amd import shard  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402

n, L, W, R = 65536, 20, 5, int(sys.argv[1]) if len(sys.argv) > 1 else 8
kw = dict(ENV_TRAIN_CONFIG, scenario="corridor")
dev = torch.device("cuda", 0)
venv = shard.make_shard_venv(n, 0, 1, device=dev, seed=12345, with_info=False, **kw)
g = torch.Generator(device=dev).manual_seed(1000)
bank = [(torch.rand(n, 2, device=dev, generator=g) * 2 - 1).contiguous() for _ in range(16)]
venv.reset()
stream = torch.cuda.current_stream(dev)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    for k in range(L):
        venv.step(bank[k % 16])
torch.cuda.synchronize()
bench._upload_graphs([graph], stream)
spin = shard.make_shard_venv(n, 0, 1, device=dev, seed=777, with_info=False, **kw)
spin.reset()
torch.cuda.synchronize()
t_w = time.perf_counter()
k = 0
while (time.perf_counter() - t_w) < 0.1:
    for _ in range(16):
        spin.step(bank[k % 16])
        k += 1
    torch.cuda.synchronize()
spin.close()
for k in range(W):
    venv.step(bank[k % 16])
out = []
for r in range(R):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    graph.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    out.append({"replay": r + 1, "wall_us_per_step": wall * 1e6 / L, "event_us_per_step": e0.elapsed_time(e1) * 1e3 / L})
print(json.dumps(out, indent=0))
