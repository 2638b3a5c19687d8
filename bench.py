#!/usr/bin/env python3
"""Benchmark: env-steps/s of the batched Drone2dEnv step at 65 536 envs per MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]     (N > 1: starts its N ranks itself)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" = one ``d2d_step`` (libdrone2d_hip.so) over all envs of a GPU: thrust -> Chipmunk-
equivalent 3-body/6-joint solve -> collision -> 3-nearest sensing -> Brent closest point ->
27-dim obs -> reward/termination -> in-kernel auto-reset.  Workload (BASELINE.json configs[2]):
65 536 envs per GPU on the ``corridor`` test scenario (18 circles), U(-1,1) float32 actions
pre-generated on the device (a bank of 16, cycled), inputs resident in HBM before timing.  The timed
loop launches every step from Python (``venv.step``, the SB3 adapter's path; ~5.5 us of host work
per call, GPU-bound at ~26 us); ``--graph`` replays the steps captured as hipGraphs instead.  Either
way every step runs the full kernel on fresh state.  Eager is the default because it measured
faster: 2.39-2.42 G vs 2.31-2.36 G env-steps/s for 20 timed steps after 5 warm-up steps, alternating
on one box, and 2.451-2.457 G vs 2.446-2.452 G for 2 000 steps (profiles/r06/short/): a graph's
kernel nodes cost ~0.8 us more per step on this ROCm.
Multi-GPU: one process per GPU, each with its own 65 536 envs (weak scaling, global env ids), no
collective in the step; the episode statistics are all-reduced once per timed interval (RCCL).

Prints ONE JSON line (rank 0).  ``roofline.achieved`` = 650 algorithmic bytes per env-step x envs
per launch / mean step time on the device (HIP events on the launch stream around the timed
steps: one pair around the eager loop, one per graph replay with --graph); ``cpu_baseline`` = the C
oracle (a scalar port of the same algorithm) timed on this host's cores on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "env-steps/sec at 65 536 parallel envs; 1/2/4/8 MI355X scaling"
ENVS_PER_GPU = 65536
SCENARIO = "corridor"
BYTES_PER_ENV_STEP = 650   # DESIGN.md "Algorithmic bytes": 272 read + 378 written, info off
INFO_BYTES = 48            # --info: the f32 [N, 12] info row per env-step
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFS = 78.6       # MI355X fp64 vector peak (the co-bound reported alongside)
ACTION_BANK = 16
# BASELINE.json configs[4]: env i gets scenario i mod 7 in this order
MIXED = ["perpendicular", "parallel", "S_parallel", "corridor", "S_corridor", "large", "impossible"]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--warmup", type=int, default=300,
                   help="untimed steps; ~4 mean episode lengths, so the timed loop sees the steady-state mix "
                        "of envs (the first episodes after reset all start at the spawn boxes)")
    p.add_argument("--envs", type=int, default=ENVS_PER_GPU)
    p.add_argument("--scenario", default=SCENARIO,
                   help="test scenario name, NAME_free (no obstacles: configs[1]), 'mixed' (configs[4]) or "
                        "'curriculum' (the fresh training curriculum: a new device-generated scenario per episode)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget (s)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--clock-warmup-ms", type=float, default=100.0,
                   help="device clock warm-up before the warmup steps: the step kernels on a separate "
                        "throwaway batch (the measured envs are untouched); 0 disables")
    p.add_argument("--info", action="store_true",
                   help="also write the per-env info rows (f32 [N, 12], what the SB3 adapter reads): +48 B/env-step")
    p.add_argument("--graph", action="store_true",
                   help="replay the steps captured as hipGraphs instead of launching each step from Python")
    p.add_argument("--eager", action="store_true", help="(the default) launch every step from Python")
    p.add_argument("--exact-trig", action="store_true",
                   help="the exact-trig library build (Drone2dVecEnv(exact_trig=True): fdlibm sin / cos / "
                        "atan2, the reference's bearing sequence; bit-identical to the oracle's exact build)")
    return p.parse_args()


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """``--gpus N`` (N > 1) without a launcher: start the N ranks ourselves, one process per GPU,
    as children under ``torch.distributed.run`` (rendezvous on 127.0.0.1) -- the reference's
    process fan-out (main.py:183-190, SubprocVecEnv) -- and return the launcher's exit status.
    Nothing here touches the GPU (``device_count`` does not initialise HIP on this image), so the
    children start from a clean process; the parent never execs."""
    import subprocess

    backend = os.environ.get("D2D_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and args.gpus > ndev:
        print(f"bench.py: --gpus {args.gpus} but only {ndev} HIP device(s) are visible "
              f"(RCCL needs one device per rank; D2D_BENCH_BACKEND=gloo rehearses on fewer)", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL)
    return subprocess.call(cmd, env=env)


def setup_dist(args):
    from drone2d_amd import shard

    # RCCL ("nccl") between GPUs; D2D_BENCH_BACKEND=gloo rehearses the multi-rank path with every
    # rank on the one GPU of a single-GPU box (RCCL refuses two ranks on one device)
    backend = os.environ.get("D2D_BENCH_BACKEND", "nccl")
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        # refuse rather than report a world the run did not have (n_gpus is the world that stepped)
        print(f"bench.py: launched with WORLD_SIZE={world_env} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank, world, local = shard.init_process_group_from_env(backend)
    if world == 1 or backend != "nccl":
        torch.cuda.set_device(local % torch.cuda.device_count())
    return rank, world, local


def _upload_graphs(graphs, stream):
    """hipGraphUpload each instantiated graph (its first replay then does not pay the upload); the
    symbol comes from the HIP runtime torch loaded (through libdrone2d_hip.so's dependency tree)."""
    try:
        from drone2d_amd import _native
        import ctypes as C

        up = _native.load().hipGraphUpload
        up.restype, up.argtypes = C.c_int, [C.c_void_p, C.c_void_p]
        for g in graphs:
            up(C.c_void_p(g.raw_cuda_graph_exec()), C.c_void_p(stream.cuda_stream))
        torch.cuda.synchronize()
    except (AttributeError, RuntimeError, OSError):
        pass


def sysfs_card(dev_index: int):
    """The DRM sysfs directory of HIP device ``dev_index``, matched by its PCI address (None when not
    found, e.g. no amdgpu sysfs in a container)."""
    import glob

    try:
        p = torch.cuda.get_device_properties(dev_index)
        want = "%04x:%02x:%02x." % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    except (RuntimeError, AttributeError, AssertionError):
        return None
    for d in sorted(glob.glob("/sys/class/drm/card*/device")):
        if os.path.basename(os.path.realpath(d)).lower().startswith(want):
            return d
    return None


def gpu_clock(card):
    """The shader clock right now, read from sysfs (file reads only): the current level of
    ``pp_dpm_sclk`` (the line marked '*') and the hwmon ``freq1_input`` (sclk, Hz).  None if neither
    is readable."""
    import glob
    import re

    if card is None:
        return None
    out = {}
    t0 = time.perf_counter()
    try:
        for line in open(os.path.join(card, "pp_dpm_sclk")):
            if "*" in line:
                m = re.search(r"(\d+)\s*[Mm][Hh]z", line)
                if m:
                    out["pp_dpm_sclk_mhz"] = float(m.group(1))
    except OSError:
        pass
    for f in sorted(glob.glob(os.path.join(card, "hwmon", "hwmon*", "freq1_input"))):
        try:
            out["hwmon_sclk_mhz"] = int(open(f).read().strip()) / 1e6
            break
        except (OSError, ValueError):
            pass
    if out:
        out["read_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
    return out or None


def valu_budget(bytes_per_launch: float, valu: dict, clk: dict | None, frac: float = 0.40) -> dict:
    """The VALU-issue budget that ``frac`` of the HBM roof implies (DESIGN.md "What bounds K1"): the
    launch must last bytes / (frac x peak); at the profiled busy fraction and cycles per VALU
    instruction (``valu``: the committed VALU profile) and this run's shader clock (``clk``: the
    line's ``gpu_clock``), that leaves this many VALU wave-instructions per SIMD per launch."""
    t = bytes_per_launch / (frac * HBM_PEAK_GBS * 1e9)
    mhz, src = None, None
    for key in ("after_timed", "before_timed"):
        c = (clk or {}).get(key) or {}
        if c.get("pp_dpm_sclk_mhz"):
            mhz, src = float(c["pp_dpm_sclk_mhz"]), f"sysfs pp_dpm_sclk ({key})"
            break
    if mhz is None:
        mhz, src = 2100.0, "assumed 2.1 GHz (sysfs clock unreadable)"
    cpi = valu["valu_active_cycles_per_simd"] / valu["valu_insts_per_simd"]
    budget = t * mhz * 1e6 * valu["valu_busy_frac"] / cpi
    return {"roof_frac": frac, "launch_us": t * 1e6, "clock_mhz": mhz, "clock_source": src,
            "busy_frac": valu["valu_busy_frac"], "cycles_per_valu": cpi, "valu_per_simd_budget": budget,
            "valu_per_simd_profiled": valu["valu_insts_per_simd"],
            "cut_needed_frac": 1.0 - budget / valu["valu_insts_per_simd"]}


def barrier_sync(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def cpu_info() -> dict:
    """The host's CPU budget: the affinity set, the cgroup CPU quota (if any), the CPU model."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(round(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"affinity_cores": aff, "cgroup_quota_cores": quota, "cpu_model": model}


def cpu_baseline(args, kwargs):
    """Time the C oracle on a bounded sample of the same workload (test infrastructure).

    Threads: one per core of the affinity set (BASELINE.md / SURVEY 8(d): 1 core and all cores;
    D2D_CPU_THREADS overrides); ``cores`` is the thread count actually used.  When a cgroup CPU
    quota grants fewer CPUs than the affinity set holds, the same sample is also timed with one
    thread per granted CPU (``quota_threads`` / ``quota_threads_value``): the all-cores threads then
    time-slice inside the quota."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle

    import drone2d_amd as d2  # noqa: F401
    from drone2d_amd.config import make_cfg
    from drone2d_amd.env import build_scenarios

    oracle.build()
    info = cpu_info()
    threads = info["affinity_cores"]
    if os.environ.get("D2D_CPU_THREADS"):
        threads = max(1, int(os.environ["D2D_CPU_THREADS"]))
    threads = min(threads, 256)  # d2d_oracle.c's per-call thread bound
    quota = info["cgroup_quota_cores"]
    qthreads = quota if (quota and quota < threads) else None
    n = args.envs
    scn = [s.to_c() for s in build_scenarios(kwargs)]
    b = oracle.OracleBatch(make_cfg(dict(kwargs)), scn, n)
    b.reset(0)
    rng = np.random.default_rng(0)
    act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    t0 = time.perf_counter()
    b.step(act, nthreads=threads)  # one step to size the sample
    one = time.perf_counter() - t0
    steps = max(1, min(20000, int(args.cpu_seconds / max(one, 1e-6))))
    t0 = time.perf_counter()
    for _ in range(steps):
        b.step(act, nthreads=threads)
    dt = time.perf_counter() - t0
    # the same batch on one core (1 core and all cores), a shorter sample
    t1 = time.perf_counter()
    steps1 = 0
    while steps1 < 1 or (time.perf_counter() - t1 < args.cpu_seconds / 4 and steps1 < 20000):
        b.step(act, nthreads=1)
        steps1 += 1
    dt1 = time.perf_counter() - t1
    extra = {}
    if qthreads:
        tq = time.perf_counter()
        for _ in range(steps):
            b.step(act, nthreads=qthreads)
        extra = {"quota_threads": qthreads, "quota_threads_value": n * steps / (time.perf_counter() - tq)}
    b.close()
    return {"value": n * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "single_core_value": n * steps1 / dt1, **extra, **info,
            "sample": f"C oracle (oracle/d2d_oracle.c, scalar fp64 port of the reference step), "
                      f"{n} envs x {steps} steps of {args.scenario} with auto-reset, {threads} threads "
                      f"({info['affinity_cores']} cores in the affinity set, {info['cpu_model']}), "
                      f"{dt:.1f} s; single core: {steps1} steps, {dt1:.1f} s"}


def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    import drone2d_amd  # noqa: F401  (registers the package as drone2d_amd)
    from drone2d_amd import shard
    from drone2d_amd.config import ENV_TRAIN_CONFIG

    rank, world, local = setup_dist(args)

    if args.scenario == "curriculum":
        # the reference's training distribution: every reset on its own device-generated scenario,
        # stages 1-5 on the device step clock (starts at stage 1, stage 5 after 2 M global steps)
        kwargs = dict(ENV_TRAIN_CONFIG, mode="curriculum", scenario="curriculum", sim_num=0)
    else:
        kwargs = dict(ENV_TRAIN_CONFIG, scenario=MIXED if args.scenario == "mixed" else args.scenario)
    dev = torch.device("cuda", torch.cuda.current_device())
    n = args.envs
    # this rank's block of a global batch of world x n envs (global env ids, no step collective)
    venv = shard.make_shard_venv(n * world, rank, world, device=dev, seed=12345, with_info=args.info,
                                 exact_trig=args.exact_trig, **kwargs)
    # one global action bank (seed 1000) sliced by rank: a run of world x n envs in one process
    # steps exactly the same envs with exactly the same actions (global env ids below)
    g = torch.Generator(device=dev).manual_seed(1000)
    bank = [(torch.rand(n * world, 2, device=dev, generator=g) * 2 - 1)[rank * n:(rank + 1) * n].contiguous()
            for _ in range(ACTION_BANK)]
    venv.reset()
    stream = torch.cuda.current_stream(dev)

    # The timed steps replay captured HIP graphs: one graph of all args.steps steps (longer runs: a
    # 256-step graph replayed + one graph of the remainder).  The graphs are captured and uploaded
    # BEFORE the warmup, so the warmup steps run right before the timed region (no idle GPU, no
    # host-side capture in between) and the timed region holds as few replay boundaries as possible.
    glen = args.steps if args.steps <= 512 else 256
    reps, rem = divmod(args.steps, glen)
    graph = tail = None
    hipgraph = args.graph and not args.eager
    if hipgraph:
        def capture(n_steps):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for k in range(n_steps):
                    venv.step(bank[k % ACTION_BANK])
            return g
        if reps:
            graph = capture(glen)
        if rem:
            tail = capture(rem)
        torch.cuda.synchronize()
        _upload_graphs([g for g in (graph, tail) if g is not None], stream)

    # Device clock warm-up (not part of the measured run: the measured envs are untouched).  An idle
    # MI355X starts ~10-13 % below its sustained clock and ramps over tens of ms (GRBM_GUI_ACTIVE per
    # ns of the first vs the later step launches, profiles/r04/final1/pmc_clk.csv), which a 20-step
    # run would measure instead of the kernel: 31.4 vs 29.0 us per step (profiles/r04/clock/).  So
    # the same step kernels first run for --clock-warmup-ms on a separate, throwaway batch of this
    # rank's size; fp64 GEMMs instead do not raise the clock (31.4 us).
    card = sysfs_card(dev.index)
    clk = {"card": os.path.basename(os.path.dirname(card)) if card else None, "at_start": gpu_clock(card)}
    if args.clock_warmup_ms > 0:
        spin = shard.make_shard_venv(n * world, rank, world, device=dev, seed=777, with_info=args.info, **kwargs)
        spin.reset()
        torch.cuda.synchronize()
        t_w = time.perf_counter()
        k = 0
        while (time.perf_counter() - t_w) * 1e3 < args.clock_warmup_ms:
            for _ in range(16):
                spin.step(bank[k % ACTION_BANK])
                k += 1
            torch.cuda.synchronize()
        spin.close()
    for k in range(args.warmup):
        venv.step(bank[k % ACTION_BANK])
    venv.episode_stats(clear=True)
    torch.cuda.synchronize()
    clk["before_timed"] = gpu_clock(card)

    # eager: one event pair around the whole loop (an event record per step is a queue marker of a
    # few us each on the GPU side: it measured 35 instead of 28 us per step, tools/eager_probe.py)
    segs = (reps + (1 if rem else 0)) if hipgraph else 1
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(segs)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(segs)]
    barrier_sync(world)
    t0 = time.perf_counter()
    if hipgraph:
        for r in range(reps):
            starts[r].record(stream)
            graph.replay()
            ends[r].record(stream)
        if rem:
            starts[reps].record(stream)
            tail.replay()
            ends[reps].record(stream)
    else:
        starts[0].record(stream)
        for k in range(args.steps):
            venv.step(bank[k % ACTION_BANK])
        ends[0].record(stream)
    n_timed = args.steps
    barrier_sync(world)
    wall = time.perf_counter() - t0
    clk["after_timed"] = gpu_clock(card)

    # episode statistics of the interval: the one RCCL all-reduce (timed separately)
    stats = venv.episode_stats(clear=True)
    torch.cuda.synchronize()
    t_ar = 0.0
    if world > 1:
        t1 = time.perf_counter()
        shard.allreduce_stats(stats)  # the one RCCL collective: 8 doubles per logging interval
        torch.cuda.synchronize()
        t_ar = time.perf_counter() - t1
    # device time of the timed steps (HIP events on the launch stream) per step
    kern_ms = float(np.sum([s.elapsed_time(e) for s, e in zip(starts, ends)])) / n_timed

    wall_t = torch.tensor([wall], dtype=torch.float64, device=dev)
    kern_ranks, dev_ranks = [kern_ms], [dev.index]
    if world > 1:
        dist.all_reduce(wall_t, op=dist.ReduceOp.MAX)
        parts = [None] * world
        dist.all_gather_object(parts, (kern_ms, dev.index))
        kern_ranks = [float(k) for k, _ in parts]
        dev_ranks = [int(d) for _, d in parts]
    wall = float(wall_t.item())
    kern_ms = max(kern_ranks)

    if rank == 0:
        total_steps = n * world * n_timed
        value = total_steps / wall
        bytes_env = BYTES_PER_ENV_STEP + (INFO_BYTES if args.info else 0)
        achieved = bytes_env * n / (kern_ms * 1e-3) / 1e9
        st = stats.cpu().numpy()
        traffic = traffic_src = None
        tag = f"{args.scenario}_{n}" + ("_info" if args.info else "")
        tf = os.path.join(REPO, "profiles", f"traffic_{tag}.json")
        if os.path.exists(tf):
            tj = json.load(open(tf))
            traffic = tj.get("bytes_per_launch")
            # PMC bytes come from a committed rocprofv3 pass, not from this run: say which
            traffic_src = {"profile": os.path.relpath(tf, REPO), "pmc": tj.get("source"), "commit": tj.get("commit")}
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": n_timed,
            "warmup": args.warmup,
            "clock_warmup_ms": args.clock_warmup_ms,
            "ms_per_step": wall * 1e3 / n_timed,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"{args.scenario}, {n} envs per GPU, U(-1,1) f32 actions, in-kernel auto-reset",
                       "envs_per_gpu": n, "total_envs": n * world, "scenario": args.scenario,
                       "parallelism": f"env-shard x{world}", "hipgraph": hipgraph,
                       "outputs": "obs f32[N,27], reward f32, terminated/truncated u8, terminal obs"
                                  + (", info f32[N,12]" if args.info else " (info rows off)")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": ("d2d_step_kernel + d2d_fill_kernel (every 16th step, filling every 3rd) per "
                                    "step, graph replay" if hipgraph else
                                    "d2d_step_kernel + d2d_fill_kernel (every 48th step) per step, eager"),
                         "kernel_ms": kern_ms,
                         "bytes_per_env_step": bytes_env},
            "episodes": {"finished": float(st[1]), "mean_return": float(st[0] / max(st[1], 1)),
                         "success": float(st[2]), "fails": float(st[3]), "collisions": float(st[4]),
                         "sum_ape": float(st[5]), "sum_len": float(st[6]),
                         "allreduce_ms": t_ar * 1e3},
            # the multi-rank evidence: ranks that stepped, the collective's backend, each rank's
            # device time per step (the line's kernel_ms is their max)
            "ranks": world, "backend": (dist.get_backend() if world > 1 else None),
            "kernel_ms_per_rank": kern_ranks,
            # HIP device of each rank (RCCL: one per rank; the gloo rehearsal shares one GPU)
            "device_per_rank": dev_ranks,
            # rank 0's shader clock (sysfs) at start, right before and right after the timed window:
            # tells a slow box or an unramped clock apart from a slower kernel
            "gpu_clock": clk,
        }
        vf = os.path.join(REPO, "profiles", f"valu_{tag}.json")
        if os.path.exists(vf):
            # the kernel's actual bound (fp64 VALU issue), from the committed rocprofv3 SQ pass
            v = json.load(open(vf))
            line["valu"] = {k: v[k] for k in ("valu_insts_per_simd", "valu_active_cycles_per_simd",
                                              "wave_lifetime_cycles", "valu_busy_frac", "source")}
            line["valu"]["profile"] = os.path.relpath(vf, REPO)
            line["valu"]["commit"] = v.get("commit")
            line["valu"]["valu_budget_for_40pct"] = valu_budget(bytes_env * n, v, clk)
            if v.get("fp64_flops_per_env_step_issued"):
                # the fp64 co-roofline: fp64 flops per env-step from the committed
                # rocprofv3 VALU-mix pass x the env-steps this run's kernel did per second
                fl = float(v["fp64_flops_per_env_step_issued"])
                tfs = fl * n / (kern_ms * 1e-3) / 1e12
                line["roofline"]["fp64"] = {
                    "bound": "fp64 vector", "achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                    "frac": tfs / FP64_PEAK_TFS, "flops_per_env_step": fl,
                    "flops_per_env_step_counter": v.get("fp64_flops_per_env_step_counter"),
                    "valu_issue_busy_frac": v["valu_busy_frac"], "mix_frac": v.get("mix_frac"),
                    "source": v.get("mix_sources"), "commit": v.get("commit"),
                    "note": "flops = (2 FMA + ADD + MUL) f64 wave-instructions x 64 lanes per env-step "
                            "(issued lanes); the kernel is bound by VALU issue, of which fp64 arithmetic "
                            "is the mix_frac share"}
                if v.get("valu_lane_util"):
                    # the same over active lanes only (SQ_THREAD_CYCLES_VALU / 64 x SQ_ACTIVE_INST_VALU):
                    # the Brent continuation issues with few lanes active
                    ua = float(v["valu_lane_util"])
                    line["roofline"]["fp64"].update({
                        "valu_lane_util": ua, "achieved_active_lanes": tfs * ua,
                        "frac_active_lanes": tfs * ua / FP64_PEAK_TFS,
                        "flops_per_env_step_active_est": v.get("fp64_flops_per_env_step_active_est")})
        if args.scenario == "curriculum":
            line["config"]["workload"] = (f"fresh training curriculum (a new device-generated scenario per episode, "
                                          f"stage from the device step clock), {n} envs per GPU, U(-1,1) f32 "
                                          f"actions, in-kernel auto-reset")
            line["kernel_note"] = "per step: step kernel + scenario generator (K5) + queue clear + fill/16"
        elif not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(args, kwargs)
        print(json.dumps(line), flush=True)
    venv.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
