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


def test_gpu_clock_reads_sysfs(tmp_path):
    """The line's ``gpu_clock``: the current pp_dpm_sclk level (the '*' line) and hwmon freq1_input,
    plus how long the reads took; None when neither file is readable (no GPU / no amdgpu sysfs)."""
    sys.path.insert(0, REPO)
    import bench

    card = tmp_path / "device"
    (card / "hwmon" / "hwmon3").mkdir(parents=True)
    (card / "pp_dpm_sclk").write_text("0: 500Mhz\n1: 1600Mhz\n2: 2316Mhz *\n")
    (card / "hwmon" / "hwmon3" / "freq1_input").write_text("2316000000\n")
    c = bench.gpu_clock(str(card))
    assert c.pop("read_ms") >= 0.0 and c == {"pp_dpm_sclk_mhz": 2316.0, "hwmon_sclk_mhz": 2316.0}
    (card / "pp_dpm_sclk").write_text("0: 500Mhz\n1: 2100Mhz\n")  # no current level marked
    c = bench.gpu_clock(str(card))
    assert c.pop("read_ms") >= 0.0 and c == {"hwmon_sclk_mhz": 2316.0}
    assert bench.gpu_clock(str(tmp_path / "nothing")) is None and bench.gpu_clock(None) is None


def test_valu_budget_for_40pct():
    """valu_budget: 40 % of 8 TB/s at 650 B x 65 536 is a 13.312 us launch; at 2.316 GHz, 84.4 % busy
    and 4.15 cycles per VALU instruction that is ~6.27 k VALU per SIMD (DESIGN.md "What bounds K1");
    without a readable clock it assumes 2.1 GHz and says so."""
    sys.path.insert(0, REPO)
    import bench

    v = {"valu_active_cycles_per_simd": 44556.09375, "valu_insts_per_simd": 10727.45849609375,
         "valu_busy_frac": 0.8443313720606864}
    b = bench.valu_budget(650 * 65536, v, {"before_timed": {"pp_dpm_sclk_mhz": 2000.0},
                                           "after_timed": {"pp_dpm_sclk_mhz": 2316.0}})
    assert abs(b["launch_us"] - 13.312) < 1e-9 and b["clock_mhz"] == 2316.0 and "after_timed" in b["clock_source"]
    assert abs(b["valu_per_simd_budget"] - 6267.36) < 0.1
    assert abs(b["cut_needed_frac"] - (1 - 6267.36 / 10727.458)) < 1e-4
    b = bench.valu_budget(650 * 65536, v, None)
    assert b["clock_mhz"] == 2100.0 and "assumed" in b["clock_source"]
