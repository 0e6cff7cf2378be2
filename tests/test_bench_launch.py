"""bench.py's launch contract on CPU (no GPU is touched): `--gpus N` (N > 1) outside torchrun
starts torchrun as a child process (shown by --dry-run), a WORLD_SIZE that differs from --gpus is
refused, and one GPU runs in-process with the golden self-check on."""
import json
import os
import subprocess
import sys
import time

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
    torchrun (the measuring process is a child of the watchdog parent); refused under torchrun."""
    r = _run(["--gpus", "8", "--single-process", "--dry-run"])
    assert r.returncode == 0, r.stderr
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan["launch"].startswith("single process") and plan["n_gpus"] == 8
    assert plan["world"] == 1 and plan["config"] == "c4" and plan["verify"] is True
    r = _run(["--gpus", "4", "--single-process", "--dry-run"],
             {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "torchrun" in r.stderr


_DUMMY_WORKER = """
import sys, time
sys.path.insert(0, sys.argv[1])
import bench
bench.set_phase("collective")
bench.start_heartbeat(1, lambda: None, period=0.2)
time.sleep(120)
"""

_DUMMY_LAUNCHER = """
import subprocess, sys, time
sys.path.insert(0, sys.argv[1])
import bench
# a worker in a session of its own, as torchrun starts its ranks
subprocess.Popen([sys.executable, "-c", sys.argv[2], sys.argv[1]], start_new_session=True)
bench.set_phase("timed")
bench.start_heartbeat(0, lambda: None, period=0.2)
time.sleep(120)
"""


def _alive(pid):
    try:
        with open(f"/proc/{pid}/status") as fh:
            return fh.read().split("State:")[1].split()[0] != "Z"
    except OSError:
        return False


def test_watchdog_ends_a_hung_child_and_reports_heartbeats(capsys):
    """bench.py's parent watchdog (run_child) against a child that never finishes -- a launcher
    that starts a 'rank' in a session of its own (as torchrun does) and both sleep: past the
    deadline the parent kills the launcher's group and every rank that wrote a heartbeat, and
    prints one JSON line with "error": "timeout" and each rank's last phase; status 5."""
    sys.path.insert(0, ROOT)
    import bench
    t0 = time.monotonic()
    rc = bench.run_child([sys.executable, "-c", _DUMMY_LAUNCHER, ROOT, _DUMMY_WORKER],
                         dict(os.environ), 3.0, "dummy", 2)
    elapsed = time.monotonic() - t0
    assert rc == 5 and elapsed < 40, (rc, elapsed)
    line = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1])
    assert line["error"] == "timeout" and line["deadline_s"] == 3.0 and line["value"] is None
    beats = {b["rank"]: b for b in line["heartbeats"]}
    assert beats[0]["phase"] == "timed" and beats[1]["phase"] == "collective", beats
    time.sleep(0.5)
    for b in beats.values():
        assert not _alive(b["pid"]), f"rank {b['rank']} (pid {b['pid']}) survived the watchdog"


def test_watchdog_reports_a_child_that_fails_without_a_line(capsys):
    sys.path.insert(0, ROOT)
    import bench
    rc = bench.run_child([sys.executable, "-c", "import sys; sys.exit(7)"], dict(os.environ),
                         30.0, "dummy", 2)
    assert rc == 7
    line = json.loads([ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")][-1])
    assert line["error"] == "child exited with 7"


_PARENT = """
import os, sys
sys.path.insert(0, sys.argv[1])
import bench
bench.run_child([sys.executable, "-c",
                 "import os, sys, time; open(sys.argv[1], 'w').write(str(os.getpid())); time.sleep(120)",
                 sys.argv[2]], dict(os.environ), 120.0, "dummy", 2)
"""


def test_watchdog_child_dies_with_the_parent(tmp_path):
    """Whoever runs the bench may kill its parent outright (SIGKILL): the measuring child must
    not outlive it on the GPUs -- it gets SIGTERM from the kernel (PR_SET_PDEATHSIG)."""
    import signal
    pidfile = tmp_path / "child.pid"
    parent = subprocess.Popen([sys.executable, "-c", _PARENT, ROOT, str(pidfile)])
    for _ in range(200):
        if pidfile.exists() and pidfile.read_text():
            break
        time.sleep(0.05)
    child = int(pidfile.read_text())
    assert _alive(child)
    parent.send_signal(signal.SIGKILL)
    parent.wait(timeout=10)
    for _ in range(100):
        if not _alive(child):
            break
        time.sleep(0.05)
    assert not _alive(child), "the child outlived the killed watchdog parent"
