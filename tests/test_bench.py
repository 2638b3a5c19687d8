"""bench.py's multi-rank path, rehearsed on one GPU.

The driver runs ``bench.py`` under ``torch.distributed.run`` with one rank per GPU over RCCL; a
one-GPU box cannot host two RCCL ranks on one device, so ``D2D_BENCH_BACKEND=gloo`` runs the same
code path (global env ids, the sliced global action bank, the episode-statistics all-reduce, the
max-over-ranks timing) with both ranks on cuda:0.  Two ranks of n envs step exactly the envs of one
process with 2n envs, so the reduced episode statistics must be the one-process run's.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "48", "--warmup", "16", "--no-cpu-baseline"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _line(out: str) -> dict:
    rows = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert rows, out[-2000:]
    return json.loads(rows[-1])


def _run(cmd, env):
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    return _line(r.stdout)


@pytest.mark.gpu
def test_bench_two_ranks_match_one_process():
    env = dict(os.environ, D2D_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                "--envs", "4096", *ARGS], env)
    one = _run([sys.executable, "bench.py", "--envs", "8192", *ARGS], env)
    assert two["n_gpus"] == 2 and two["ranks"] == 2 and two["backend"] == "gloo"
    assert len(two["kernel_ms_per_rank"]) == 2 and two["roofline"]["kernel_ms"] == max(two["kernel_ms_per_rank"])
    assert one["ranks"] == 1 and one["backend"] is None
    assert two["config"]["total_envs"] == one["config"]["total_envs"] == 8192
    e1, e2 = one["episodes"], two["episodes"]
    assert e1["finished"] > 0
    for k in ("finished", "success", "fails", "collisions", "sum_len"):
        assert e2[k] == e1[k], k
    # float sums: per-env accumulators are identical, the reduction order differs (two blocks)
    assert e2["mean_return"] == pytest.approx(e1["mean_return"], rel=1e-9)
    assert e2["sum_ape"] == pytest.approx(e1["sum_ape"], rel=1e-9)


@pytest.mark.gpu
def test_bench_gpus_flag_launches_its_ranks():
    """``python bench.py --gpus 2`` with no launcher starts its two ranks itself:
    the line reports the world that stepped, and the reduced episode statistics are one process's."""
    env = dict(os.environ, D2D_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    two = _run([sys.executable, "bench.py", "--gpus", "2", "--envs", "4096", *ARGS], env)
    one = _run([sys.executable, "bench.py", "--envs", "8192", *ARGS], env)
    assert two["n_gpus"] == two["ranks"] == 2 and two["backend"] == "gloo"
    assert len(two["device_per_rank"]) == 2
    assert two["config"]["total_envs"] == 8192
    for k in ("finished", "success", "fails", "collisions", "sum_len"):
        assert two["episodes"][k] == one["episodes"][k], k


def test_bench_refuses_world_mismatch():
    """Under a launcher whose world differs from --gpus the bench exits non-zero before any GPU work."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *ARGS], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_bench_refuses_more_gpus_than_devices():
    """RCCL needs one device per rank: --gpus 4 on a host with fewer visible devices is refused."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "D2D_BENCH_BACKEND")}
    env["HIP_VISIBLE_DEVICES"] = env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", *ARGS], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "HIP device" in r.stderr
