#!/usr/bin/env python3
"""Benchmark: body-steps/s of the reference's PhysicsEngine.step() (BHA:405-439) on MI355X.

Workload (BASELINE.json metric "body-steps/sec at N=1e6, theta=0.5"): configuration C3, two
colliding galaxy disks (NBodyPanel.kt:83-100 scaled: 8e5 + 2e5 bodies, seeds 1/2), theta 0.5,
dt 0.005, G 80, eps^2 1, merge rule on.  One step = the full reference step: two tree builds,
two force evaluations, kick-drift-kick, merge.  Inputs are resident in HBM before timing.

Multi-GPU (torchrun, one rank per GPU): the north-star configuration C4 (1e7-body uniform cloud,
total fixed: strong scaling; `--config c3x` = weak scaling, 1e6 two-disk bodies per GPU).  The
state is replicated; each rank builds a locally essential tree (only the cells its bodies can
open, plus the top from every rank's cell values), evaluates and integrates its Hilbert-ordered
lane range, and the new positions are all-gathered by RCCL over xGMI inside the engine.

Prints ONE JSON line on rank 0 (see the driver contract in the task statement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "barnes-hut-n-body_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP64_VEC_PEAK_TF = 78.6  # MI355X FP64 vector peak (FMA = 2 flop), AMD spec sheet (not in the guide)
FP64_NOFMA_PEAK_TF = 39.3  # the same issue rate without FMA: -ffp-contract=off (bit-exactness)
FLOP_PER_INTERACTION = 20  # SURVEY §8d convention: one point force (BHA:250-259), sqrt/div = 1
NODE_BYTES = 32        # one fp64 node record (comX, comY, mass, next/meta) — SURVEY §8d
BODY_EVAL_BYTES = 40   # body read (x, y, m) + acceleration write (ax, ay) per evaluation


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
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
    return ap.parse_args()


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


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.config is None:  # BASELINE's metric on one GPU; the north-star cloud on N > 1
        args.config = "c3" if world == 1 else "c4"
    if args.theta is None:
        args.theta = 0.0 if args.config == "c5" else 0.5
    direct = args.theta == 0.0
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    import numpy as np
    import torch
    import torch.distributed as dist

    import bh_amd

    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local_rank)

    params = bh_amd.default_params(theta=args.theta)
    if world > 1:
        uid = [bh_amd.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng = bh_amd.Engine(params, device=local_rank, rank=rank, world=world, unique_id=uid[0])
    else:
        eng = bh_amd.Engine(params, device=local_rank)

    arrs, scene_name, scaling = scene_for(args.config, world)
    n0 = len(arrs[0])

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
        bodies_per_launch = bodies / world
        flops_per_launch = FLOP_PER_INTERACTION * bodies_per_launch * (bodies - 1)
        kernel = "k_direct"
        extra = {"interactions_per_s": round(flops_per_launch / FLOP_PER_INTERACTION /
                                             (trav_ms * 1e-3)) if trav_ms > 0 else 0}
    else:
        kernel = "k_traverse"
        cs = [c for c in (cnt_start, cnt_end) if c]
        contrib = float(np.mean([c["contrib_per_body"] for c in cs])) if cs else 0.0
        vbar = float(np.mean([c["vbar"] for c in cs])) if cs else 0.0
        # world > 1: one launch per round evaluates 1 / (world * rounds) of the bodies
        bodies_per_launch = bodies / (world * (bh_amd.SHARD_ROUNDS if world > 1 else 1))
        flops_per_launch = FLOP_PER_INTERACTION * contrib * bodies_per_launch
        node_bytes = (NODE_BYTES * vbar + BODY_EVAL_BYTES) * bodies_per_launch
        extra = {
            "contrib_per_body_eval": round(contrib, 2),
            "vbar_nodes_per_body_eval": round(vbar, 2),
            "counted_on": "copies of the state at the start and the end of the timed region",
            "lane_efficiency": round(float(np.mean([c["lane_efficiency"] for c in cs])), 4)
            if cs else None,
            "force_block_lane_use": round(float(np.mean([c["force_block_lane_use"] for c in cs])), 4)
            if cs else None,
            "node_stream_gbs": round(node_bytes / (trav_ms * 1e-3) / 1e9, 1) if trav_ms > 0 else 0,
            "node_stream_note": "(32 V-bar + 40) B per body: served by the scalar cache / L2, "
                                "not HBM (one record feeds 64 lanes)",
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
        "kernel": kernel,
        "kernel_ms": dict(avg=round(trav_ms, 4), **kstats),
        "launches": trav_launches,
        "flops_per_launch": round(flops_per_launch),
        "gpu_clock": clock_stats,
    }
    roofline.update(extra)

    cpu_baseline = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and direct:
        # theta = 0: one evaluation of a body subsample through the oracle's tree walk (every
        # leaf visited), scaled to body-steps/s (2 evaluations per step)
        import oracle
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        ref = oracle.Oracle(*arrs, theta=0.0, threads=threads)
        sample = np.arange(0, n0, max(1, n0 // 4096), dtype=np.int64)
        c0 = time.perf_counter()
        ref.accelerations(subset=sample)
        c1 = time.perf_counter()
        cpu_baseline = {
            "value": round(len(sample) / (2.0 * (c1 - c0)), 1),
            "unit": "body-steps/s",
            "cores": threads,
            "kind": "port",
            "sample": f"one theta=0 evaluation of {len(sample)} of {n0} bodies (every leaf of the "
                      f"tree) with the C restatement (oracle/bh_oracle.c), scaled by 2 "
                      f"evaluations per step; includes the serial tree build",
            "seconds": round(c1 - c0, 3),
        }
        ref.close()
    elif rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        ref = oracle.Oracle(*arrs, theta=args.theta, threads=threads)
        ref.step(1)  # same first step the GPU warmup took; bounded sample follows
        c0 = time.perf_counter()
        ref.step(args.cpu_steps)
        c1 = time.perf_counter()
        cpu_baseline = {
            "value": round(ref.num_bodies() * args.cpu_steps / (c1 - c0), 1),
            "unit": "body-steps/s",
            "cores": threads,
            "kind": "port",
            "sample": f"{args.cpu_steps} full step(s) of {scene_name} ({ref.num_bodies()} bodies) "
                      f"with the C restatement of the reference CPU path (oracle/bh_oracle.c: "
                      f"serial pointer-tree build, {threads} workers on an atomic body queue)",
            "seconds": round(c1 - c0, 3),
        }
        ref.close()

    if rank == 0:
        line = {
            "metric": "body-steps/sec at N=1e6, theta=0.5; achieved HBM GB/s vs roofline"
            if args.config == "c3" else f"body-steps/sec ({scene_name}, theta={args.theta})",
            "value": round(value, 1),
            "unit": "body-steps/s",
            "n_gpus": world,
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
                               f"force sharded x{world} (RCCL all-gather)"
                if world > 1 else "single GPU",
            },
            "phase_ms": {k: round(v, 3) for k, v in phases.items()},
            "roofline": roofline,
            "cpu_baseline": cpu_baseline,
        }
        if per_rank is not None:
            line["per_rank_phase_ms_per_step"] = per_rank
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
