"""bench.py's launch contract on CPU (no GPU is touched): `--gpus N` (N > 1) outside torchrun
starts torchrun as a child process (shown by --dry-run), a WORLD_SIZE that differs from --gpus is
refused, and one GPU runs in-process with the golden self-check on."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=120)


def test_multi_gpu_request_spawns_torchrun_child():
    r = _run(["--gpus", "8", "--steps", "20", "--warmup", "5", "--dry-run"])
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    cmd = plan["cmd"]
    assert plan["launch"] == "torchrun child"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "127.0.0.1" in cmd
    assert cmd[cmd.index("--gpus") + 1] == "8" and "--dry-run" not in cmd
    assert cmd[-6:] == ["--gpus", "8", "--steps", "20", "--warmup", "5"]


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "8", "--dry-run"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE 4" in r.stderr


def test_single_gpu_runs_in_process_with_verification():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan == {"launch": "in-process", "world": 1, "n_gpus": 1, "config": "c3",
                    "theta": 0.5, "verify": True}
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan["world"] == 4 and plan["config"] == "c4" and plan["verify"] is True


def test_single_process_multi_gpu_stays_in_process():
    """--single-process: one process, one engine handle over the N GPUs (bh_create_multi), no
    torchrun child; refused under torchrun."""
    r = _run(["--gpus", "8", "--single-process", "--dry-run"])
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan["launch"].startswith("single process") and plan["n_gpus"] == 8
    assert plan["world"] == 1 and plan["config"] == "c4" and plan["verify"] is True
    r = _run(["--gpus", "4", "--single-process", "--dry-run"],
             {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "torchrun" in r.stderr
