#!/usr/bin/env python3
"""Benchmark: body-steps/s of the reference's PhysicsEngine.step() (BHA:405-439) on MI355X.

Workload (BASELINE.json metric "body-steps/sec at N=1e6, theta=0.5"): configuration C3, two
colliding galaxy disks (NBodyPanel.kt:83-100 scaled: 8e5 + 2e5 bodies, seeds 1/2), theta 0.5,
dt 0.005, G 80, eps^2 1, merge rule on.  One step = the full reference step: two tree builds,
two force evaluations, kick-drift-kick, merge.  Inputs are resident in HBM before timing.

Multi-GPU (one rank per GPU): the north-star configuration C4 (1e7-body uniform cloud, total
fixed: strong scaling; `--config c3x` = weak scaling, 1e6 two-disk bodies per GPU).  The state is
replicated; each rank builds a locally essential tree (only the cells its bodies can open, plus
the top from every rank's cell values), evaluates and integrates its Hilbert-ordered lane range,
and the new positions are all-gathered by RCCL over xGMI inside the engine.
  * `python bench.py --gpus N` (N > 1) outside torchrun starts `python -m torch.distributed.run
    --nproc-per-node N ... bench.py ...` as a CHILD process before anything touches the GPU and
    exits with its status (`--dry-run` prints that command); inside torchrun, WORLD_SIZE must
    equal --gpus, and RCCL's own communicator size (ncclCommCount) must equal it too.
  * After the timed region every rank checks itself (`--verify`, on by default): the engine is
    reset to a committed golden configuration -- C4 x 10 steps on N > 1 GPUs (the north-star
    scene through the sharded path), C3 x 10 steps on one GPU -- and the SHA-256 of every final
    SoA field must equal tests/golden/digests.json (made by the CPU oracle) on every rank; a
    mismatch prints the line with "verify" and exits non-zero.

Prints ONE JSON line on rank 0 (see the driver contract in the task statement).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "barnes-hut-n-body_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_VEC_PEAK_TF = 78.6  # MI355X FP64 vector peak (FMA = 2 flop), AMD spec sheet (not in the guide)
FP64_NOFMA_PEAK_TF = 39.3  # the same issue rate without FMA: -ffp-contract=off (bit-exactness)
# k_direct's inner loop per interaction (gfx950 ISA of direct.hip, fast path): 33 fp64 VALU
# instructions (11 mul, 7 add, 15 fma/fmac) + 1 v_rsq_f64; one wave64 fp64 instruction per CU
# per clock (the 78.6 TF peak = 256 CU x 2.4 GHz x 64 lanes x 2)
DIRECT_VALU_PER_INTERACTION = 34
N_CU = 256
FLOP_PER_INTERACTION = 20  # SURVEY §8d convention: one point force (BHA:250-259), sqrt/div = 1
NODE_BYTES = 32        # one fp64 node record (comX, comY, mass, next/meta) — SURVEY §8d
BODY_EVAL_BYTES = 40   # body read (x, y, m) + acceleration write (ax, ay) per evaluation
KDK_BYTES_PER_EVAL = 32  # SURVEY §8d's 64 B of KDK per body-step, half per evaluation


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (default: WORLD_SIZE under torchrun, else 1); N > 1 outside "
                         "torchrun launches torchrun as a child process")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default=None,
                    help="c3 (default on one GPU), c4 (default on N>1 GPUs: strong scaling of "
                         "the north-star 1e7 cloud), c3x (weak scaling: 1e6 bodies per GPU), "
                         "c2, c5 (theta=0 all-pairs), c1_code, c1_baseline")
    ap.add_argument("--theta", type=float, default=None, help="default 0.5 (c5: 0.0)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-counters", action="store_true",
                    help="skip the V-bar / lane-efficiency counting walks on the timed state")
    ap.add_argument("--no-events", action="store_true",
                    help="diagnostic: no HIP events in the timed region (no kernel times)")
    ap.add_argument("--cpu-steps", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--verify", dest="verify", action="store_true", default=None,
                    help="golden-digest self-check after the timed region (default on)")
    ap.add_argument("--no-verify", dest="verify", action="store_false")
    ap.add_argument("--no-single-gpu", action="store_true",
                    help="N > 1: skip rank 0's one-GPU run of the same workload")
    ap.add_argument("--no-drop-in", action="store_true",
                    help="skip the one-step-per-call leg (the front-end's call pattern)")
    ap.add_argument("--drop-in-calls", type=int, default=40)
    ap.add_argument("--dry-run", action="store_true",
                    help="print the launch plan (the torchrun child command for N > 1) and exit")
    ap.add_argument("--single-process", action="store_true",
                    help="N > 1: one process, one engine handle over the N GPUs "
                         "(bh_create_multi: a host thread per GPU, RCCL communicators made "
                         "in-process) -- the front-end's own way to drive N GPUs -- instead "
                         "of torchrun with one process per GPU")
    ap.add_argument("--devices", default=None,
                    help="--single-process rehearsal on fewer GPUs: the handle's device list, "
                         "e.g. 0,0 (a repeated device exchanges by device-to-device copies, "
                         "not RCCL)")
    ap.add_argument("--deadline", type=float, default=600.0,
                    help="N > 1: seconds the parent waits for the measuring child (torchrun, or "
                         "the --single-process child) before it kills it and prints one JSON "
                         "line with \"error\": \"timeout\" and every rank's last heartbeat")
    return ap.parse_args()


def _free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


# ---- the parent's watchdog (N > 1) ------------------------------------------------------
# The reference's join always returns (BHA:408, 426); a multi-GPU run can hang instead -- a rank
# that returned early leaves its peers in a collective.  The engine bounds its own waits
# (BH_COMM_TIMEOUT_S, set below the deadline for the child) and aborts its communicators; the
# parent, which never touches the GPU, bounds the whole run: past the deadline it ends the child
# and every rank it knows of, and prints one JSON line with each rank's last heartbeat.
HEARTBEAT_ENV = "BH_BENCH_HEARTBEAT"
_phase = {"name": "start"}


def set_phase(name):
    _phase["name"] = name


def start_heartbeat(rank, engine_fn, period=1.0):
    """Rank side: every `period` s write <$BH_BENCH_HEARTBEAT>/rank<R>.json -- pid, phase, and
    the engine's progress (bh_progress of every member: API calls, collectives, last site,
    busy / failed flags), read from a daemon thread while the main thread is inside a call."""
    d = os.environ.get(HEARTBEAT_ENV)
    if not d:
        return
    path = os.path.join(d, f"rank{rank}.json")
    t0 = time.monotonic()

    def beat():
        while True:
            rec = {"rank": rank, "pid": os.getpid(), "phase": _phase["name"],
                   "elapsed_s": round(time.monotonic() - t0, 1)}
            try:
                eng = engine_fn()
                if eng is not None:
                    rec["progress"] = [eng.member(r).progress()
                                       for r in range(max(1, eng.multi_world()))]
            except Exception as exc:  # noqa: BLE001 - diagnostics only
                rec["progress_error"] = repr(exc)[:200]
            try:
                with open(path + ".tmp", "w") as fh:
                    json.dump(rec, fh)
                os.replace(path + ".tmp", path)
            except OSError:
                return
            time.sleep(period)
    threading.Thread(target=beat, daemon=True).start()


def read_heartbeats(d):
    out = []
    for name in sorted(os.listdir(d)) if d and os.path.isdir(d) else []:
        if name.startswith("rank") and name.endswith(".json"):
            try:
                with open(os.path.join(d, name)) as fh:
                    out.append(json.load(fh))
            except (OSError, ValueError):
                pass
    return out


def _kill_group(pid, sig):
    try:
        os.killpg(pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def _die_with_parent():
    """(preexec_fn) the child gets SIGTERM when this process dies -- killed by whoever runs the
    bench -- so torchrun stops its workers instead of leaving them on the GPUs."""
    try:
        import ctypes
        ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
    except Exception:  # noqa: BLE001 - best effort
        pass


def run_child(cmd, env, deadline, what, n_gpus=None):
    """Run `cmd` relaying its stdout; past `deadline` seconds end it -- SIGTERM (torchrun then
    stops its workers), SIGKILL 15 s later to it and to every rank that wrote a heartbeat, with
    that rank's process group (torchrun starts each worker in a session of its own) -- and print
    one JSON line {"error": "timeout", "heartbeats": [...]}; returns the child's status (5 on a
    timeout).  A child that fails without printing a bench line gets an error line too.  The
    child stays in this process's group and dies with it (PR_SET_PDEATHSIG)."""
    hb_dir = tempfile.mkdtemp(prefix="bh_bench_hb_")
    env = dict(env)
    env[HEARTBEAT_ENV] = hb_dir
    # the ranks give up on a collective before the parent gives up on them
    env.setdefault("BH_COMM_TIMEOUT_S", str(max(10, int(deadline / 3))))
    t0 = time.monotonic()
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1,
                            preexec_fn=_die_with_parent)
    saw_line = threading.Event()

    def relay():
        for line in proc.stdout:
            sys.stdout.write(line)
            sys.stdout.flush()
            if line.startswith("{") and '"metric"' in line:
                saw_line.set()
    rt = threading.Thread(target=relay, daemon=True)
    rt.start()
    try:
        rc = proc.wait(timeout=deadline)
    except subprocess.TimeoutExpired:
        beats = read_heartbeats(hb_dir)
        proc.terminate()
        try:
            proc.wait(timeout=15)
        except subprocess.TimeoutExpired:
            proc.kill()
        for b in beats:  # the workers torchrun started in sessions of their own
            if isinstance(b.get("pid"), int) and b["pid"] != os.getpid():
                _kill_group(b["pid"], signal.SIGKILL)
                try:
                    os.kill(b["pid"], signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
        try:
            proc.wait(timeout=10)
        except subprocess.TimeoutExpired:
            pass
        rt.join(timeout=5)
        print(json.dumps({"metric": None, "value": None, "error": "timeout", "launch": what,
                          "n_gpus": n_gpus, "deadline_s": deadline,
                          "elapsed_s": round(time.monotonic() - t0, 1),
                          "heartbeats": beats}), flush=True)
        shutil.rmtree(hb_dir, ignore_errors=True)
        return 5
    rt.join(timeout=30)
    if rc != 0 and not saw_line.is_set():
        print(json.dumps({"metric": None, "value": None, "error": f"child exited with {rc}",
                          "launch": what, "n_gpus": n_gpus,
                          "heartbeats": read_heartbeats(hb_dir)}), flush=True)
    shutil.rmtree(hb_dir, ignore_errors=True)
    return rc


def _child_env():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver
    return env


def spawn_torchrun(args) -> int:
    """`--gpus N` (N > 1) without torchrun: run the same command under torch.distributed.run as
    a child process -- nothing in this process has touched the GPU, and no exec replaces it --
    relaying the child's output (rank 0 prints the JSON line) and returning its exit status,
    under the watchdog (run_child)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)]
    cmd += [a for a in sys.argv[1:] if a != "--dry-run"]
    if args.dry_run:
        print(json.dumps({"launch": "torchrun child", "cmd": cmd, "deadline_s": args.deadline}),
              flush=True)
        return 0
    return run_child(cmd, _child_env(), args.deadline, "torchrun", args.gpus)


def spawn_single_process(args) -> int:
    """`--gpus N --single-process`: the one-handle run in a child process under the watchdog."""
    cmd = [sys.executable, os.path.abspath(__file__)] + [a for a in sys.argv[1:]
                                                         if a != "--dry-run"]
    env = _child_env()
    env["BH_BENCH_CHILD"] = "1"
    return run_child(cmd, env, args.deadline, "single process", args.gpus)


def committed_traffic(config, kernel):
    """HBM bytes per launch of `kernel` on this workload from the committed PMC summary
    (profiles/hbm_traffic.json, rocprofv3 FETCH_SIZE / WRITE_SIZE passes summarised by
    tools/summarize_profile.py), or None."""
    path = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    try:
        with open(path) as fh:
            return json.load(fh).get(config, {}).get(kernel)
    except (OSError, ValueError):
        return None


class ClockSampler:
    """GPU clock / activity during the timed region, sampled by amdsmi from a host thread
    (the GPU is matched by PCI bus id).  Silent no-op where amdsmi is unavailable."""

    def __init__(self, device):
        self.samples = []
        self._stop = None
        self._h = None
        try:
            import amdsmi
            import torch
            amdsmi.amdsmi_init()
            props = torch.cuda.get_device_properties(device)
            want = getattr(props, "pci_bus_id", None)
            handles = amdsmi.amdsmi_get_processor_handles()
            for h in handles:
                bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)
                if want is None or int(bdf.split(":")[1], 16) == int(want):
                    self._h = h
                    break
            self._amdsmi = amdsmi
        except Exception as exc:  # noqa: BLE001 - diagnostics only
            self.error = repr(exc)[:200]

    def _read(self):
        a = self._amdsmi
        c = a.amdsmi_get_clock_info(self._h, a.AmdSmiClkType.SYS)
        return c.get("clk"), c.get("max_clk")

    def start(self):
        if self._h is None:
            return
        import threading
        self._stop = threading.Event()

        def run():
            while not self._stop.is_set():
                try:
                    self.samples.append(self._read())
                except Exception:  # noqa: BLE001
                    return
                self._stop.wait(0.002)
        self._t = threading.Thread(target=run, daemon=True)
        self._t.start()

    def stop(self):
        if self._stop is None:
            return None
        self._stop.set()
        self._t.join()
        clk = [c for c, _ in self.samples if isinstance(c, (int, float))]
        if not clk:
            return None
        clk.sort()
        return {"samples": len(clk), "min_mhz": clk[0], "median_mhz": clk[len(clk) // 2],
                "max_mhz": clk[-1], "max_clk_mhz": self.samples[-1][1]}


def traversal_counters(bh_amd, params, device, arrs):
    """Counting walk (bh_compute_accelerations with visits) on a copy of `arrs` in a separate
    engine: V-bar, point-force contributions, lane efficiency, force-block lane use."""
    import numpy as np
    probe = bh_amd.Engine(params, device=device)
    probe.reset_bodies(*arrs)
    _, _, vis = probe.compute_accelerations(visits=True)
    c = probe.traversal_counters()
    probe.close()
    n = len(vis)
    return {
        "bodies": n,
        "vbar": float(np.mean(vis)) if n else 0.0,
        "contrib_per_body": c["lane_contrib"] / n if n else 0.0,
        "lane_efficiency": c["lane_visits"] / (64.0 * c["wave_iters"]) if c["wave_iters"] else 0.0,
        "force_block_lane_use": (c["lane_contrib"] + n) / (64.0 * c["wave_blocks"])
        if c["wave_blocks"] else 0.0,
        "wave_iters_per_wave": c["wave_iters"] / c["waves"] if c["waves"] else 0.0,
        "blocks_per_wave": c["wave_blocks"] / c["waves"] if c["waves"] else 0.0,
        "lane_contrib": c["lane_contrib"],
    }


def scene_for(config, world):
    """(arrays, scene name, scaling): c3x = weak scaling (1e6 bodies per GPU of the two-disk
    geometry), every other config is a fixed total (strong scaling over GPUs)."""
    from bh_amd import scenes
    if config == "c3x":
        name = f"c3x{world}" if world > 1 else "c3"
        return scenes.config_scene(name), name, "weak"
    return scenes.config_scene(config), config, "strong"


WORKLOAD_DESC = {
    "c3": "two colliding galaxy disks (8e5 r=300 + 2e5 r=100 y=160 vx=-50), N=1e6",
    "c2": "Kepler disk N=1e5 (BodyFactory.makeKeplerDisk, seed 3)",
    "c4": "uniform cloud N=1e7 over 2400x800, m=0.5 (the north-star configuration)",
    "c1_code": "defaultBodies(): two galaxy disks 10000 + 2500",
    "c1_baseline": "BASELINE 'R' scene: two galaxy disks 2 x 1000",
    "c5": "uniform cloud N=262144, theta=0: direct all-pairs sum in tree leaf order",
}


GOLDEN = os.path.join(ROOT, "tests", "golden", "digests.json")
FIELDS = ("x", "y", "vx", "vy", "m")


def _sha(a) -> str:
    import numpy as np
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<f8").tobytes()).hexdigest()


def verify_leg(bh_amd, eng, case, arrs, dist, rank, world):
    """Reset the engine to the golden configuration `case` of tests/golden/digests.json, run its
    steps in one bh_step call and compare the SHA-256 of every final SoA field (little-endian
    fp64, caller order) with the oracle's; the digests of all ranks are compared as well."""
    with open(GOLDEN) as fh:
        want = json.load(fh)[case]
    t0 = time.perf_counter()
    eng.set_params(bh_amd.default_params(theta=want["theta"]))
    eng.reset_bodies(*arrs)
    eng.step(want["steps"])
    state = eng.get_bodies()
    mine = {"n": len(state[0])}
    mine.update({f: _sha(a) for f, a in zip(FIELDS, state)})
    match = mine["n"] == want["n"] and all(mine[f] == want[f] for f in FIELDS)
    agree = True
    if eng.multi_world() > 1:  # one handle over several GPUs: every member's replica
        for r in range(1, eng.multi_world()):
            st = eng.member(r).get_bodies()
            agree = agree and all(_sha(a) == mine[f] for f, a in zip(FIELDS, st))
    if world > 1:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        agree = all(g == gathered[0] for g in gathered)
        match = match and all(g["n"] == want["n"] and all(g[f] == want[f] for f in FIELDS)
                              for g in gathered)
    return {"case": case, "steps": want["steps"], "n": want["n"], "digest_match": bool(match),
            "ranks_agree": bool(agree), "ranks": max(world, eng.multi_world()),
            "bad_fields": [f for f in FIELDS if mine[f] != want[f]],
            "seconds": round(time.perf_counter() - t0, 3),
            "source": "tests/golden/digests.json (SHA-256 of the CPU oracle's final state)"}


def available_processors():
    """The reference's worker count, Runtime.getRuntime().availableProcessors() (BHA:292, used
    at BHA:377 and 470): the CPUs this process may run on, bounded by the cgroup CPU quota the
    way a container-aware JVM bounds it.  Returns (count, details)."""
    import math
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as fh:
                q, period = fh.read().split()[:2]
            if q != "max":
                quota = max(1, math.ceil(int(q) / int(period)))
        except (OSError, ValueError):
            pass
    count = min(affinity, quota) if quota else affinity
    return count, {"os_cpu_count": os.cpu_count(), "sched_affinity": affinity,
                   "cgroup_cpu_quota": quota}


def cpu_baseline_leg(args, arrs, scene_name, direct):
    """The reference CPU path, restated in C (oracle/bh_oracle.c: serial pointer-tree build,
    `threads` workers on an atomic body queue, BHA:359-395), on a bounded sample of the same
    workload, timed on this host's cores with the reference's own thread policy
    (availableProcessors(), BHA:292)."""
    res = _cpu_baseline(args, arrs, scene_name, direct)
    res["host"] = args._cpu_host
    res["thread_policy"] = ("availableProcessors() (BHA:292): sched affinity bounded by the "
                            "cgroup CPU quota" if not args.cpu_threads else "--cpu-threads")
    return res


def _cpu_baseline(args, arrs, scene_name, direct):
    import numpy as np
    import oracle
    avail, host = available_processors()
    args._cpu_host = host
    threads = args.cpu_threads or avail
    n0 = len(arrs[0])
    if direct:
        # theta = 0: one evaluation of a body subsample through the oracle's tree walk (every
        # leaf visited), scaled to body-steps/s (2 evaluations per step)
        ref = oracle.Oracle(*arrs, theta=0.0, threads=threads)
        sample = np.arange(0, n0, max(1, n0 // 4096), dtype=np.int64)
        c0 = time.perf_counter()
        ref.accelerations(subset=sample)
        c1 = time.perf_counter()
        ref.close()
        return {"value": round(len(sample) / (2.0 * (c1 - c0)), 1), "unit": "body-steps/s",
                "cores": threads, "kind": "port",
                "sample": f"one theta=0 evaluation of {len(sample)} of {n0} bodies (every leaf of "
                          f"the tree) with the C restatement (oracle/bh_oracle.c), scaled by 2 "
                          f"evaluations per step; includes the serial tree build",
                "seconds": round(c1 - c0, 3)}
    if n0 > 2_000_000:
        # C4-sized: a full CPU step takes minutes, so one evaluation is timed in its two parts --
        # the serial tree build of all bodies and the walk of every 128th body -- and one step
        # is extrapolated as 2 x (build + walk of all bodies)
        ref = oracle.Oracle(*arrs, theta=args.theta, threads=threads)
        sample = np.arange(0, n0, 128, dtype=np.int64)
        c0 = time.perf_counter()
        ref.accelerations(subset=sample)
        c1 = time.perf_counter()
        t_build, t_walk_sample = ref.last_timing()
        ref.close()
        step_s = 2.0 * (t_build + t_walk_sample * n0 / len(sample))
        return {"value": round(n0 / step_s, 1), "unit": "body-steps/s", "cores": threads,
                "kind": "port",
                "sample": f"{scene_name} ({n0} bodies), one evaluation with the C restatement "
                          f"(oracle/bh_oracle.c): serial tree build of all bodies "
                          f"{t_build:.2f} s, walk of every 128th body ({len(sample)} bodies, "
                          f"{threads} workers) {t_walk_sample:.3f} s; one step extrapolated as "
                          f"2 x (build + walk of all bodies) = {step_s:.1f} s",
                "seconds": round(c1 - c0, 3)}
    ref = oracle.Oracle(*arrs, theta=args.theta, threads=threads)
    ref.step(1)  # same first step the GPU warmup took; bounded sample follows
    c0 = time.perf_counter()
    ref.step(args.cpu_steps)
    c1 = time.perf_counter()
    nb = ref.num_bodies()
    ref.close()
    return {"value": round(nb * args.cpu_steps / (c1 - c0), 1), "unit": "body-steps/s",
            "cores": threads, "kind": "port",
            "sample": f"{args.cpu_steps} full step(s) of {scene_name} ({nb} bodies) with the C "
                      f"restatement of the reference CPU path (oracle/bh_oracle.c: serial "
                      f"pointer-tree build, {threads} workers on an atomic body queue)",
            "seconds": round(c1 - c0, 3)}


def single_gpu_leg(bh_amd, params, device, arrs, steps, warmup):
    """Rank 0 of a multi-GPU run: the same workload on its one GPU with the single-GPU engine
    (a reference point for the driver's scaling curve; the N = 1 bench line runs C3)."""
    eng = bh_amd.Engine(params, device=device)
    eng.reset_bodies(*arrs)
    if warmup > 0:
        eng.step(warmup)
    n0 = eng.num_bodies()
    eng.synchronize()
    t0 = time.perf_counter()
    eng.step(steps)
    eng.synchronize()
    el = time.perf_counter() - t0
    n1 = eng.num_bodies()
    eng.close()
    return {"value": round(0.5 * (n0 + n1) * steps / el, 1), "unit": "body-steps/s",
            "ms_per_step": round(1e3 * el / max(steps, 1), 4), "n_gpus": 1,
            "note": "rank 0's GPU alone, single-GPU engine, same scene / steps / warmup"}


def drop_in_leg(eng, steps, warmup=5):
    """The front-end's own call pattern (NBodyPanel.kt:290-293 tick() -> engine.step(), then
    paintComponent reads every body, NBodyPanel.kt:302-306): one bh_step(1) call per frame.
    Timed on the engine's current state (after the batched timed region), three ways:
    step only; step + bh_get_bodies into pageable numpy arrays (the plain copying ABI);
    step + bh_map_bodies (the engine's pinned caller-order mirror, written by the step itself
    while its last build overlaps -- what the JNI shim reads)."""
    import numpy as np
    out = {"calls": steps, "steps_per_call": 1}

    def timed(fn):
        for _ in range(warmup):
            fn()
        eng.synchronize()
        n0 = eng.num_bodies()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        eng.synchronize()
        el = time.perf_counter() - t0
        return 1e3 * el / steps, 0.5 * (n0 + eng.num_bodies()) * steps / el

    def step_only():
        eng.step(1)

    bufs = [np.empty(eng.num_bodies(), dtype=np.float64) for _ in range(5)]
    for a in bufs:
        a.fill(0.0)  # a caller's own, resident buffers (no first-touch page faults in the timing)

    def step_copy():
        eng.step(1)
        eng.get_bodies(out=bufs)

    ms, v = timed(step_only)
    out.update(ms_per_step=round(ms, 4), value=round(v, 1))
    ms, v = timed(step_copy)
    out.update(ms_per_step_with_get_bodies=round(ms, 4), value_with_get_bodies=round(v, 1))
    if hasattr(eng, "set_mirror"):
        eng.set_mirror(True)
        sink = np.zeros(1)

        def step_map():
            eng.step(1)
            x, y, vx, vy, m = eng.map_bodies()
            sink[0] += x[-1] + m[0]  # touch the mapped arrays (the caller reads them)

        ms, v = timed(step_map)
        eng.set_mirror(False)
        out.update(ms_per_step_with_mirror=round(ms, 4), value_with_mirror=round(v, 1))
    out["note"] = ("one bh_step(1) call per frame as the Swing front-end does; 'with_get_bodies' "
                   "adds the 40 B/body caller-order copy-out (bh_get_bodies) into the caller's "
                   "own resident pageable arrays; "
                   "'with_mirror' reads the pinned mirror the step fills asynchronously")
    return out


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    single_proc = args.single_process and args.gpus is not None and args.gpus > 1
    if single_proc and env_world is not None and int(env_world) > 1:
        print("bench.py: --single-process runs in one process, not under torchrun",
              file=sys.stderr)
        sys.exit(2)
    if env_world is None and args.gpus is not None and args.gpus > 1 and not single_proc:
        sys.exit(spawn_torchrun(args))  # before anything touches the GPU
    if single_proc and not os.environ.get("BH_BENCH_CHILD") and not args.dry_run:
        sys.exit(spawn_single_process(args))  # (the watchdog's child)
    world = int(env_world) if env_world is not None else 1
    if args.gpus is None:
        args.gpus = world
    # n_gpus: GPUs measured; world: processes (torchrun ranks)
    n_gpus = args.gpus if single_proc else world
    if args.gpus != n_gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: refusing to measure a "
              f"different number of GPUs than asked", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config is None:  # BASELINE's metric on one GPU; the north-star cloud on N > 1
        args.config = "c3" if n_gpus == 1 else "c4"
    if args.theta is None:
        args.theta = 0.0 if args.config == "c5" else 0.5
    direct = args.theta == 0.0
    if args.verify is None:
        args.verify = True
    if args.dry_run:
        print(json.dumps({"launch": "single process, one handle over the GPUs" if single_proc
                          else "in-process", "world": world, "n_gpus": n_gpus,
                          "config": args.config, "theta": args.theta, "verify": args.verify}),
              flush=True)
        return

    import numpy as np
    import torch
    import torch.distributed as dist

    import bh_amd

    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    holder = {"eng": None}
    start_heartbeat(rank, lambda: holder["eng"])
    set_phase("engine")
    torch.cuda.set_device(local_rank)

    params = bh_amd.default_params(theta=args.theta)
    rccl = None
    if world > 1:
        uid = [bh_amd.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng = bh_amd.Engine(params, device=local_rank, rank=rank, world=world, unique_id=uid[0])
        nr, ur = eng.comm_ranks()
        views = [None] * world
        dist.all_gather_object(views, [nr, ur])
        rccl = {"comm_count": nr, "user_ranks": [v[1] for v in views]}
        if any(v[0] != world for v in views) or sorted(v[1] for v in views) != list(range(world)):
            if rank == 0:
                print(f"bench.py: RCCL communicator {views} does not span the {world} ranks",
                      file=sys.stderr)
            sys.exit(3)
    elif single_proc:
        # one handle over GPUs 0..N-1 (the decomposition at every body count: bench sizes are the
        # point), in-process RCCL communicators
        os.environ.setdefault("BH_MULTI_MIN_BODIES", "0")
        devs = ([int(d) for d in args.devices.split(",")] if args.devices
                else list(range(n_gpus)))
        if len(devs) != n_gpus:
            print(f"bench.py: --devices lists {len(devs)} devices for --gpus {n_gpus}",
                  file=sys.stderr)
            sys.exit(2)
        eng = bh_amd.Engine(params, devices=devs)
        nr, ur = eng.comm_ranks()
        members = [eng.member(r).comm_ranks() for r in range(eng.multi_world())]
        repeated = len(set(devs)) < len(devs)
        rccl = {"comm_count": nr, "user_ranks": [m[1] for m in members], "devices": devs,
                "communicators": "device-to-device copies (a device listed twice)" if repeated
                else "ncclCommInitAll, one per GPU, one host thread each"}
        if eng.multi_world() != n_gpus or (not repeated and any(m[0] != n_gpus for m in members)):
            print(f"bench.py: the handle's RCCL communicators {members} do not span {n_gpus} GPUs",
                  file=sys.stderr)
            sys.exit(3)
    else:
        eng = bh_amd.Engine(params, device=local_rank)
        # the drop-in leg reads the pinned mirror: its stream is made now, right after the
        # engine's own streams and before the counter probe's (hardware queues go out in stream
        # creation order), and the mirror stays off until that leg
        eng.set_mirror(True)
        eng.set_mirror(False)

    holder["eng"] = eng
    arrs, scene_name, scaling = scene_for(args.config, n_gpus)
    n0 = len(arrs[0])

    set_phase("warmup")
    eng.reset_bodies(*arrs)
    if args.warmup > 0:
        eng.step(args.warmup)
    n_start = eng.num_bodies()
    # V-bar and the lane counters on the state the timed region starts from (a copy in a
    # separate engine: the timed state is untouched)
    cnt_start = None
    if not direct and not args.no_counters and rank == 0:
        cnt_start = traversal_counters(bh_amd, params, local_rank, eng.get_bodies())

    clocks = ClockSampler(local_rank) if rank == 0 else None
    set_phase("timed")
    eng.set_profiling(not args.no_events)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.synchronize()
    if clocks:
        clocks.start()
    t0 = time.perf_counter()
    eng.step(args.steps)  # blocks until the device work is complete
    eng.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    clock_stats = clocks.stop() if clocks else None
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    n_end = eng.num_bodies()
    trav_ms, trav_launches = eng.traverse_kernel_ms()
    samples = eng.traverse_kernel_samples()
    phases = eng.last_timings()
    eng.set_profiling(False)
    per_rank = None
    if world > 1:
        mine = {k: round(v / max(args.steps, 1), 3) for k, v in phases.items()}
        mine["let"] = eng.let_stats()  # sharded builds: LET / full builds, subset, LET nodes
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        per_rank = gathered
    elif single_proc:
        per_rank = []
        for r in range(eng.multi_world()):
            m = eng.member(r)
            mine = {k: round(v / max(args.steps, 1), 3) for k, v in m.last_timings().items()}
            mine["let"] = m.let_stats()
            per_rank.append(mine)
    cnt_end = None
    if not direct and not args.no_counters and rank == 0:
        cnt_end = traversal_counters(bh_amd, params, local_rank, eng.get_bodies())

    bodies = 0.5 * (n_start + n_end)  # the merge rule can remove a handful of bodies
    value = bodies * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / max(args.steps, 1)
    kstats = {}
    if len(samples):
        ss = np.sort(samples)
        kstats = {"min": round(float(ss[0]), 4), "median": round(float(np.median(ss)), 4),
                  "max": round(float(ss[-1]), 4)}

    # Roofline of the dominant kernel.  Both paths are bound by fp64 VALU issue: the flop
    # figure is SURVEY §8d's 20 flop per point-force interaction (BHA:250-259, the IEEE sqrt
    # and each division counted as one flop; the criterion's compare work is not counted).
    if direct:
        bodies_per_launch = bodies / n_gpus
        flops_per_launch = FLOP_PER_INTERACTION * bodies_per_launch * (bodies - 1)
        kernel = "k_direct"
        ips = flops_per_launch / FLOP_PER_INTERACTION / (trav_ms * 1e-3) if trav_ms > 0 else 0
        extra = {"interactions_per_s": round(ips)}
        if clock_stats and clock_stats.get("median_mhz"):
            # the instruction-issue ceiling of this exact sequence at the measured clock
            ceil = N_CU * clock_stats["median_mhz"] * 1e6 * 64 / DIRECT_VALU_PER_INTERACTION
            extra["valu_issue_ceiling"] = {
                "valu_per_interaction": DIRECT_VALU_PER_INTERACTION,
                "clock_mhz": clock_stats["median_mhz"],
                "interactions_per_s": round(ceil),
                "frac": round(ips / ceil, 4)}
    else:
        kernel = "k_traverse" if n_gpus == 1 else "k_traverse (one rank's 4 rounds, 2 streams)"
        cs = [c for c in (cnt_start, cnt_end) if c]
        contrib = float(np.mean([c["contrib_per_body"] for c in cs])) if cs else 0.0
        vbar = float(np.mean([c["vbar"] for c in cs])) if cs else 0.0
        # world > 1: one timed interval spans a rank's 4 round launches (its 1 / world of the
        # bodies), from the first round's start to the last even round's end on its stream
        bodies_per_launch = bodies / n_gpus
        flops_per_launch = FLOP_PER_INTERACTION * contrib * bodies_per_launch
        node_bytes = (NODE_BYTES * vbar + BODY_EVAL_BYTES) * bodies_per_launch
        # the bytes a launch must move at least: every node record a wave's cursor stops at,
        # once per wave (one scalar load feeds its 64 lanes), + each body's read and kick
        stops_per_wave = float(np.mean([c["wave_iters_per_wave"] for c in cs])) if cs else 0.0
        waves_per_launch = bodies_per_launch / 64.0
        unique_bytes = (NODE_BYTES * stops_per_wave * waves_per_launch
                        + (BODY_EVAL_BYTES + KDK_BYTES_PER_EVAL) * bodies_per_launch)
        unique_gbs = unique_bytes / (trav_ms * 1e-3) / 1e9 if trav_ms > 0 else 0.0
        extra = {
            "contrib_per_body_eval": round(contrib, 2),
            "vbar_nodes_per_body_eval": round(vbar, 2),
            "counted_on": "copies of the state at the start and the end of the timed region",
            "lane_efficiency": round(float(np.mean([c["lane_efficiency"] for c in cs])), 4)
            if cs else None,
            "force_block_lane_use": round(float(np.mean([c["force_block_lane_use"] for c in cs])), 4)
            if cs else None,
            "hbm_model": {
                "model": "32 B x cursor stops per wave (one wave-uniform scalar load per node "
                         "record, shared by 64 lanes) + 40 B per body-evaluation (x, y, m read, "
                         "ax, ay) + 32 B KDK per body-evaluation (64 B per body-step)",
                "cursor_stops_per_wave": round(stops_per_wave, 1),
                "bytes_per_launch": round(unique_bytes),
                "gbs": round(unique_gbs, 1),
                "frac_of_hbm_peak": round(unique_gbs / HBM_PEAK_GBS, 4),
                "hbm_peak_gbs": HBM_PEAK_GBS,
                "per_lane_node_bytes_gbs": round(node_bytes / (trav_ms * 1e-3) / 1e9, 1)
                if trav_ms > 0 else 0,
                "note": "SURVEY 8d's (32 V-bar + 40) B per body counts each lane's node reads; "
                        "per wave a record is read once, so the honest HBM demand is the "
                        "wave-unique figure (bytes_per_launch); the kernel is bound by fp64 "
                        "VALU issue, and the counters (traffic) measure what HBM delivers",
            },
        }
    achieved = flops_per_launch / (trav_ms * 1e-3) / 1e12 if trav_ms > 0 else 0.0
    tr = committed_traffic(scene_name, kernel)
    traffic = tr.get("hbm_bytes_per_launch") if tr else None
    roofline = {
        "bound": "fp64_valu",
        "achieved": round(achieved, 3),
        "peak": FP64_VEC_PEAK_TF,
        "unit": "TFLOP/s",
        "frac": round(achieved / FP64_VEC_PEAK_TF, 4),
        "frac_of_nofma_ceiling": round(achieved / FP64_NOFMA_PEAK_TF, 4),
        "flop_convention": "20 flop per point-force contribution (SURVEY 8d); peak 78.6 TF "
                           "counts FMA as 2, the FMA-free ceiling (-ffp-contract=off, needed "
                           "for bit-exactness) is 39.3 TF",
        "traffic": traffic,
        "traffic_source": tr.get("source") if tr else None,
        "hbm_measured_gbs": round(traffic / (trav_ms * 1e-3) / 1e9, 1)
        if traffic and trav_ms > 0 else None,
        "hbm_measured_frac_of_peak": round(traffic / (trav_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        if traffic and trav_ms > 0 else None,
        "kernel": kernel,
        "kernel_ms": dict(avg=round(trav_ms, 4), **kstats),
        "launches": trav_launches,
        "flops_per_launch": round(flops_per_launch),
        "gpu_clock": clock_stats,
    }
    roofline.update(extra)

    # rank 0's extra legs; the other ranks wait at the next collective
    set_phase("extra legs")
    drop_in = None
    if n_gpus == 1 and not args.no_drop_in:
        drop_in = drop_in_leg(eng, args.drop_in_calls)
        drop_in["ms_per_step_batched"] = round(ms_per_step, 4)
    single = None
    if rank == 0 and n_gpus > 1 and not args.no_single_gpu:
        single = single_gpu_leg(bh_amd, params, local_rank, arrs, args.steps, args.warmup)
    cpu_baseline = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu_baseline = cpu_baseline_leg(args, arrs, scene_name, direct)

    verify = None
    if world > 1:
        dist.barrier()  # rank 0's extra legs are done: the verify leg's collectives start together
    if args.verify:
        set_phase("verify")
        from bh_amd import scenes
        case = "c4_k10" if n_gpus > 1 else "c3_k10"
        golden_scene = "c4" if n_gpus > 1 else "c3"
        varrs = arrs if scene_name == golden_scene else scenes.config_scene(golden_scene)
        verify = verify_leg(bh_amd, eng, case, varrs, dist, rank, world)

    if rank == 0:
        line = {
            "metric": "body-steps/sec at N=1e6, theta=0.5; achieved HBM GB/s vs roofline"
            if args.config == "c3" else f"body-steps/sec ({scene_name}, theta={args.theta})",
            "value": round(value, 1),
            "unit": "body-steps/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded BodyFactory scenes generated in-process)",
            "config": {
                "workload": f"{scene_name}: {WORKLOAD_DESC.get(args.config, args.config)}",
                "n_bodies": int(n_start),
                "theta": args.theta,
                "dt": params.dt,
                "G": params.G,
                "soft2": params.soft2,
                "root": "2400x800",
                "evals_per_step": 2,
                "parallelism": f"replicated state, build sharded as locally essential trees, "
                               f"force sharded x{n_gpus} "
                               + ("(device-to-device copies: a device listed twice)"
                                  if rccl and "copies" in str(rccl.get("communicators", ""))
                                  else "(RCCL all-gather)")
                               + (", one process: one handle over the GPUs (bh_create_multi)"
                                  if single_proc else ", one process per GPU")
                if n_gpus > 1 else "single GPU",
            },
            "phase_ms": {k: round(v, 3) for k, v in phases.items()},
            "roofline": roofline,
            "cpu_baseline": cpu_baseline,
            "verify": verify,
        }
        if drop_in is not None:
            line["drop_in"] = drop_in
        if rccl is not None:
            line["rccl"] = rccl
        if single is not None:
            line["single_gpu_same_workload"] = single
        if per_rank is not None:
            line["per_rank_phase_ms_per_step"] = per_rank
        print(json.dumps(line), flush=True)
    set_phase("done")
    holder["eng"] = None
    eng.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if verify is not None and not (verify["digest_match"] and verify["ranks_agree"]):
        if rank == 0:
            print(f"bench.py: VERIFY FAILED: {verify}", file=sys.stderr)
        sys.exit(4)


if __name__ == "__main__":
    main()
