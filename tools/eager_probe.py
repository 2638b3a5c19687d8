"""Diagnostic (GPU box): host cost of an eager ``Drone2dVecEnv.step`` at 65 536 corridor envs.  The
eager loop is host-bound when a step's Python + ctypes + launch time exceeds the step kernel's
~28 us; prints ms per step for the current ``step`` and for the round-4 host path (a c_void_p per
pointer, ``torch.cuda.current_stream`` per call), and each host piece's cost alone."""
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import drone2d_amd as d2  # noqa: E402
from drone2d_amd.config import ENV_TRAIN_CONFIG  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
venv = d2.Drone2dVecEnv(n, seed=0, with_info=False, **dict(ENV_TRAIN_CONFIG, scenario="corridor"))
venv.reset()
bank = [torch.rand(n, 2, device="cuda") * 2 - 1 for _ in range(8)]


def old_step(v, actions):  # the round-4 host path, for comparison
    a = v._prep_actions(actions)
    v._k ^= 1
    b = v._bufs[v._k]
    v._check(v._lib.d2d_step(v._h, v._ptr(a), v._ptr(b["obs"]), v._ptr(b["rew"]), v._ptr(b["term"]),
                             v._ptr(b["trunc"]), v._ptr(b["info"]) if v.with_info else None, v._ptr(b["tobs"]),
                             v._stream()), "d2d_step")
    v._last_actions = a


def loop(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        fn(bank[k & 7])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / steps * 1e6, (t2 - t0) / steps * 1e6


def piece(fn, reps=20000):
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


for _ in range(300):
    venv.step(bank[0])
out = {"envs": n}
for r in range(3):
    for name, fn in (("new", venv.step), ("old", lambda a: old_step(venv, a))):
        host, wall = loop(fn, 2000)
        out.setdefault(name, []).append({"host_us": round(host, 2), "wall_us": round(wall, 2)})
a = bank[0]
out["pieces_us"] = {
    "prep_actions": piece(lambda: venv._prep_actions(a)),
    "fast_check": piece(lambda: type(a) is torch.Tensor and a.dtype is torch.float32 and a.is_cuda
                        and a.shape == venv._act_shape and a.get_device() == venv.device.index and a.is_contiguous()),
    "current_stream": piece(lambda: venv._stream()),
    "raw_stream": piece(lambda: venv._raw_stream(venv.device.index)) if venv._raw_stream else None,
    "c_void_p_x7": piece(lambda: [venv._ptr(a) for _ in range(7)]),
    "event_record": piece(lambda: torch.cuda.Event(enable_timing=True).record(), 2000),
}
torch.cuda.synchronize()
print(json.dumps(out), flush=True)
