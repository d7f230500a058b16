"""bench.py --gpus N starts and verifies N ranks (the driver's BENCH command
form `python bench.py --gpus N` as well as torchrun's).

CPU: the launch decision and the child command.  GPU: 2 ranks over gloo on
the one-GPU box against 1 rank — n_gpus, the process group and the global
model's hash (the sharded round is bit-identical at every world size)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_needs_launch_without_torchrun_env():
    assert bench.needs_launch(1, env={}) is False
    assert bench.needs_launch(8, env={}) is True


def test_needs_launch_inside_torchrun():
    assert bench.needs_launch(4, env={"WORLD_SIZE": "4"}) is False
    assert bench.needs_launch(1, env={"WORLD_SIZE": "1"}) is False
    with pytest.raises(SystemExit):
        bench.needs_launch(8, env={"WORLD_SIZE": "1"})


def test_launch_command_is_torchrun_child():
    cmd = bench.launch_command(["--gpus", "8", "--steps", "3"], 8, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    i = cmd.index("--master-addr")
    assert cmd[i + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    assert os.path.samefile(cmd[-5], os.path.join(ROOT, "bench.py"))


def _bench(gpus, extra=()):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--steps", "1", "--warmup", "1",
           "--config", "C3", "--clients", "16", "--no-cpu-baseline", *extra]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_two_gloo_ranks_equal_one(cuda):
    one = _bench(1)
    two = _bench(2, ["--backend", "gloo"])
    print("\n[bench --gpus 1]", {k: one[k] for k in ("value", "n_gpus", "global_sha256")})
    print("[bench --gpus 2 gloo]", {k: two[k] for k in ("value", "n_gpus", "process_group", "global_sha256")})
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["process_group"] == {"backend": "gloo", "world_size": 2}
    assert two["global_sha256"] == one["global_sha256"]
    assert two["attackers_selected"] == one["attackers_selected"] == []


def test_cpu_baseline_every_aggregator():
    """cpu_baseline reports a local-update time and the
    aggregate-ms of every hot-path aggregator, for any defense (TINY model,
    small budget)."""
    from flr.models.multimodal import TINY, num_params
    P = num_params(TINY)
    out = bench.cpu_baseline(TINY, P, 8, "trimmed_mean", 1, 4, 2, 4, budget_s=2.0)
    assert set(out["aggregate_ms"]) == {"fedavg", "krum", "trimmed_mean", "median", "krum_trimmed_mean"}
    assert all(v > 0 for v in out["aggregate_ms"].values())
    assert out["aggregate_ms_this_defense"] == out["aggregate_ms"]["trimmed_mean"]
    assert out["value"] == pytest.approx(1.0 / (8 * out["local_update_s_per_client"]
                                                + out["aggregate_ms"]["trimmed_mean"] * 1e-3))
    assert out["kind"] == "port" and out["cores"] >= 1
