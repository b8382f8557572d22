"""bench.py's multi-GPU harness: ``--gpus N`` is authoritative (self-launch of N ranks when no
torchrun environment is present; a mismatch with torchrun's WORLD_SIZE is an error), and the
CPU baseline runs on the host-core share the process actually has."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _bench(args, env_extra=None, timeout=120):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, cwd=REPO,
                          capture_output=True, text=True, timeout=timeout)


def test_gpus_must_match_torchrun_world_size():
    r = _bench(["--gpus", "2"], {"WORLD_SIZE": "3"})
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr and "--gpus 2" in r.stderr, r.stderr[-2000:]


def test_host_cpu_share_is_recorded():
    import bench
    cores, aff, quota, src = bench.host_cpu_share()
    assert aff == len(os.sched_getaffinity(0)) and 1 <= cores <= aff
    assert quota is None or cores <= max(1, int(quota))
    assert isinstance(src, str) and src


def test_launcher_command_line(monkeypatch):
    """Without WORLD_SIZE, --gpus N > 1 re-runs bench.py under torch.distributed.run with N
    ranks on 127.0.0.1 and exits with the child's status (the child is not started here)."""
    import bench
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return R()

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "3"])
    a = bench.parse_args(["--gpus", "8", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.launch_ranks_if_needed(a)
    assert e.value.code == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"] and cmd[-5].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    # a single GPU, or an existing torchrun world, does not launch anything
    bench.launch_ranks_if_needed(bench.parse_args(["--gpus", "1"]))
    monkeypatch.setenv("WORLD_SIZE", "8")
    bench.launch_ranks_if_needed(a)


@pytest.mark.gpu
def test_bench_self_launches_two_ranks(gpu):
    """The driver's command shape: `bench.py --gpus 2` with no torchrun wrapper starts two
    ranks (rehearsed over gloo with both on cuda:0 -- RCCL refuses two ranks on one device)
    and rank 0 prints one JSON line with n_gpus 2 and the all-gather exchange."""
    r = _bench(["--gpus", "2", "--dist-backend", "gloo", "--device-index", "0", "--steps", "2", "--warmup", "1",
                "--no-cpu-baseline", "--alt-precision", "none", "--no-extra"], timeout=400)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 128 and res["config"]["parallelism"] == "dp2"
    ex = res["config"]["exchange"]
    assert ex["collective"] == "gloo all_gather_into_tensor([pooled | logits])" and ex["collectives_per_step"] == 1
    assert ex["ms_per_step"] is not None and ex["ms_per_step"] > 0
    assert res["config"]["num_classes"] == 200 and res["value"] > 0


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_extra_labels_state_what_runs(world):
    """every ``extra.*.workload`` names exactly what ran at N ranks.  C3 is a
    1-GPU config (a per-rank replica beyond N = 1); C5 is configs[4] (256 over 4 GPUs): exact
    4-rank groups at N = 4k (two of them at N = 8), 64-image shards of its layout below 4."""
    import bench
    for rank in range(world):
        granks, gw, label = bench.extra_layout("c3", world, rank)
        assert granks is None and gw == world
        if world == 1:
            assert "configs[2] (1 GPU)" in label
        else:
            assert "per-rank replica" in label and f"{world * 128} images per step" in label
        granks, gw, label = bench.extra_layout("c5", world, rank)
        if world % 4 == 0:
            assert gw == 4 and "configs[4] exactly" in label and f"{world // 4} independent 4-rank group" in label
            assert f"{world * 64} images per step" in label
            if world == 8:
                assert granks == list(range(4 * (rank // 4), 4 * (rank // 4) + 4)) and rank in granks
            else:
                assert granks is None
        else:
            assert gw == world and granks is None and "shards of BASELINE configs[4]'s layout" in label
            assert "256 images over 4 GPUs" in label and "exactly" not in label
