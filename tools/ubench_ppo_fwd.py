"""Diagnostic (not product): time d2d_ppo_rollout_step (the fused rollout forward) and the
minibatch forward / backward at several batch sizes with HIP events, to separate a launch's fixed
latency from its per-workgroup cost.  Prints one JSON line per (kernel, n).  --stamps (with
D2D_PPO_LIB pointing at a -DD2D_PPO_STAMPS build, `python tools/ubench_ppo_fwd.py build`): the
forward's phase times per wave (s_memtime cycles from the workgroup's first stamp)."""
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from drone2d_amd import abi  # noqa: E402
from drone2d_amd.ppo import ActorCritic, D2DPPORollout, ManualStep, PPOConfig  # noqa: E402


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / reps


if len(sys.argv) > 1 and sys.argv[1] == "build":
    import subprocess

    from drone2d_amd import _build

    out = os.path.join(REPO, "tools", "_abl", "libd2d_ppo_stamps.so")
    subprocess.run([_build.hipcc(), *_build.PPO_FLAGS, "-DD2D_PPO_STAMPS", "-I", os.path.join(REPO, "include"),
                    _build.PPO_SRC, "-o", out], check=True)
    print("built", out)
    sys.exit(0)
STAMPS = "--stamps" in sys.argv
pol = ActorCritic().cuda()
man = ManualStep(pol, PPOConfig(), "cuda")
lib, st = man.lib, torch.cuda.current_stream().cuda_stream
for n in (4096, 16384, 32768, 65536):
    T = 16
    obs = torch.rand(n, 27, device="cuda")
    bufs = {k: torch.empty(T * n * d, device="cuda") for k, d in (("obs", 27), ("act", 2), ("logp", 1), ("val", 1))}
    noise = torch.randn(n, 2, device="cuda")
    act_env = torch.empty(n, 2, device="cuda")
    r = D2DPPORollout(n=n, t=3, T=T, info_dim=abi.INFO_DIM, info_totrew=abi.INFO_TOTREW, gamma=0.99,
                      gae_lambda_gamma=0.9405, obs=obs.data_ptr(), noise=noise.data_ptr(),
                      log_std=pol.log_std.data_ptr(), obs_buf=bufs["obs"].data_ptr(), act_buf=bufs["act"].data_ptr(),
                      logp_buf=bufs["logp"].data_ptr(), val_buf=bufs["val"].data_ptr(), act_env=act_env.data_ptr())
    r.t = 0
    wp = man.weight_ptrs()
    if STAMPS:
        import numpy as np

        nb = (n + 63) // 64
        sbuf = torch.zeros(nb * 4 * 8, dtype=torch.int64, device="cuda")
        lib.d2d_ppo_debug_stamps.argtypes = [C.c_void_p]
        for _ in range(3):
            lib.d2d_ppo_rollout_step(C.byref(r), wp, st)
        lib.d2d_ppo_debug_stamps(C.c_void_p(sbuf.data_ptr()))
        lib.d2d_ppo_rollout_step(C.byref(r), wp, st)
        torch.cuda.synchronize()
        lib.d2d_ppo_debug_stamps(None)
        a = sbuf.cpu().numpy().reshape(nb, 4, 8).astype(np.int64)
        t0 = a[:, :, 0].min(1)[:, None]
        rel = a[:, :, :7] - t0[:, :, None]
        print(json.dumps({"stamps_n": n, "phase_cycles_median_per_wave": np.median(rel, 0).astype(int).tolist(),
                          "p90_end": int(np.percentile(rel[:, :, 6], 90))}), flush=True)
    us = timed(lambda: lib.d2d_ppo_rollout_step(C.byref(r), wp, st))
    print(json.dumps({"kernel": "rollout_step", "n": n, "us": round(us, 2), "workgroups": (n + 63) // 64}), flush=True)
    if STAMPS and n == 32768:  # the fused gradient kernel's phases
        M = n
        rollout = (torch.rand(M, 27, device="cuda"), torch.randn(M, 2, device="cuda"),
                   torch.randn(M, device="cuda") - 3, torch.randn(M, device="cuda"), torch.randn(M, device="cuda"))
        idx = torch.randperm(M, device="cuda")
        acc = {k: torch.zeros((), device="cuda") for k in ("policy_loss", "value_loss", "entropy", "clip_fraction")}
        man.fused = True
        for _ in range(3):
            man.grad(idx, rollout, acc)
        rows = lib.d2d_ppo_fused_rows(M)
        sbuf = torch.zeros(2 * rows * 4 * 8, dtype=torch.int64, device="cuda")
        lib.d2d_ppo_debug_stamps(C.c_void_p(sbuf.data_ptr()))
        man.grad(idx, rollout, acc)
        torch.cuda.synchronize()
        lib.d2d_ppo_debug_stamps(None)
        a = sbuf.cpu().numpy().reshape(2 * rows, 4, 8).astype(np.int64)
        rel = a - a[:, :, :1].min(1)[:, None, :]
        print(json.dumps({"fused_stamps_m": M, "rows": rows,
                          "phase_cycles_median_per_wave": np.median(rel, 0).astype(int).tolist(),
                          "end_p90": int(np.percentile(rel[:, :, 7], 90)), "end_max": int(rel[:, :, 7].max())}),
              flush=True)
    # the minibatch forward + backward on n rollout rows
    M = n
    rollout = (torch.rand(M, 27, device="cuda"), torch.randn(M, 2, device="cuda"), torch.randn(M, device="cuda") - 3,
               torch.randn(M, device="cuda"), torch.randn(M, device="cuda"))
    idx = torch.randperm(M, device="cuda")
    acc = {k: torch.zeros((), device="cuda") for k in ("policy_loss", "value_loss", "entropy", "clip_fraction")}
    us = timed(lambda: man.grad(idx, rollout, acc))
    print(json.dumps({"kernel": "minibatch_grad (fwd+bwd+wgrad+reduce)", "n": M, "us": round(us, 2)}), flush=True)
