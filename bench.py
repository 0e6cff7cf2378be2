#!/usr/bin/env python3
"""Benchmark: body-steps/s of the reference's PhysicsEngine.step() (BHA:405-439) on MI355X.

Workload (BASELINE.json metric "body-steps/sec at N=1e6, theta=0.5"): configuration C3, two
colliding galaxy disks (NBodyPanel.kt:83-100 scaled: 8e5 + 2e5 bodies, seeds 1/2), theta 0.5,
dt 0.005, G 80, eps^2 1, merge rule on.  One step = the full reference step: two tree builds,
two force evaluations, kick-drift-kick, merge.  Inputs are resident in HBM before timing.

Multi-GPU (torchrun, one rank per GPU): weak scaling — each rank adds 1e6 bodies to the same
two-disk geometry (c3x<N>), state is replicated, force evaluation is sharded over ranks by
Morton range and accelerations are all-gathered by RCCL over xGMI inside the engine.

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
FP64_VEC_PEAK_TF = 78.6  # MI355X FP64 vector peak, AMD spec sheet (not in the local guide)
FLOP_PER_INTERACTION = 20  # SURVEY §8d C5 convention (sqrt and divisions counted as 1)
NODE_BYTES = 32        # one fp64 node record (comX, comY, mass, s2/next) — SURVEY §8d
BODY_EVAL_BYTES = 40   # body read (x, y, m) + acceleration write (ax, ay) per evaluation


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c3",
                    help="c3 (default), c2, c4, c5 (theta=0 all-pairs), c1_code, c1_baseline")
    ap.add_argument("--theta", type=float, default=None, help="default 0.5 (c5: 0.0)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0)
    return ap.parse_args()


def measured_traffic(config, kernel):
    """HBM bytes per launch of `kernel` from the committed PMC summary of this workload
    (profiles/hbm_traffic.json, written from rocprofv3 FETCH_SIZE/WRITE_SIZE passes by
    tools/summarize_profile.py), or None."""
    path = os.path.join(ROOT, "profiles", "hbm_traffic.json")
    try:
        with open(path) as fh:
            ent = json.load(fh).get(config, {}).get(kernel)
    except (OSError, ValueError):
        return None, None
    if not ent:
        return None, None
    return ent.get("hbm_bytes_per_launch"), ent.get("source")


def measured_valu_busy(config, kernel):
    """VALU-busy fraction of `kernel` on this workload from the committed SQ counter summary
    (profiles/valu_busy.json, written by tools/summarize_sq.py), or None: the traversal is
    fp64-VALU bound, so this is its efficiency figure next to the HBM roofline."""
    try:
        with open(os.path.join(ROOT, "profiles", "valu_busy.json")) as fh:
            ent = json.load(fh).get(config, {}).get(kernel)
    except (OSError, ValueError):
        return None
    return ent


def scene_for(config, world):
    from bh_amd import scenes
    if config == "c3" and world > 1:
        return scenes.config_scene(f"c3x{world}"), f"c3x{world}"
    return scenes.config_scene(config), config


WORKLOAD_DESC = {
    "c3": "two colliding galaxy disks (8e5 r=300 + 2e5 r=100 y=160 vx=-50), N=1e6",
    "c2": "Kepler disk N=1e5 (BodyFactory.makeKeplerDisk, seed 3)",
    "c4": "uniform cloud N=1e7 over 2400x800, m=0.5",
    "c1_code": "defaultBodies(): two galaxy disks 10000 + 2500",
    "c1_baseline": "BASELINE 'R' scene: two galaxy disks 2 x 1000",
    "c5": "uniform cloud N=262144, theta=0: direct all-pairs sum in tree leaf order",
}


def main():
    args = parse()
    if args.theta is None:
        args.theta = 0.0 if args.config == "c5" else 0.5
    direct = args.theta == 0.0
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
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

    arrs, scene_name = scene_for(args.config, world)
    n0 = len(arrs[0])

    # V-bar: mean non-empty nodes visited per body per evaluation on this scene,
    # counted by the engine on a separate instance so the timed state is untouched.
    vbar = lane_eff = 0.0
    if not direct:
        probe = bh_amd.Engine(params, device=local_rank)
        probe.reset_bodies(*arrs)
        _, _, vis = probe.compute_accelerations(visits=True)
        vbar = float(np.mean(vis)) if len(vis) else 0.0
        lane_visits, wave_iters, waves = probe.traversal_stats()
        lane_eff = lane_visits / (64.0 * wave_iters) if wave_iters else 0.0
        probe.close()
        del probe

    eng.reset_bodies(*arrs)
    if args.warmup > 0:
        eng.step(args.warmup)
    n_start = eng.num_bodies()

    eng.set_profiling(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.synchronize()
    t0 = time.perf_counter()
    eng.step(args.steps)  # blocks until the device work is complete
    eng.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    n_end = eng.num_bodies()
    trav_ms, trav_launches = eng.traverse_kernel_ms()
    phases = eng.last_timings()
    eng.set_profiling(False)

    bodies = 0.5 * (n_start + n_end)  # the merge rule can remove a handful of bodies
    value = bodies * args.steps / elapsed
    ms_per_step = 1e3 * elapsed / max(args.steps, 1)

    # Roofline of the dominant kernel: algorithmic bytes (traversal) or flops (theta = 0
    # all-pairs) per launch / its average duration on the engine's stream.
    bodies_per_launch = bodies / world
    if direct:
        flops_per_launch = FLOP_PER_INTERACTION * bodies_per_launch * (bodies - 1)
        achieved = flops_per_launch / (trav_ms * 1e-3) / 1e12 if trav_ms > 0 else 0.0
        roofline = {
            "bound": "valu",
            "achieved": round(achieved, 2),
            "peak": FP64_VEC_PEAK_TF,
            "unit": "TFLOP/s",
            "frac": round(achieved / FP64_VEC_PEAK_TF, 4),
            "traffic": measured_traffic(scene_name, "k_direct")[0],
            "kernel": "k_direct",
            "kernel_avg_ms": round(trav_ms, 4),
            "launches": trav_launches,
            "flops_per_launch": round(flops_per_launch),
            "interactions_per_s": round(flops_per_launch / FLOP_PER_INTERACTION / (trav_ms * 1e-3))
            if trav_ms > 0 else 0,
        }
    else:
        bytes_per_launch = (NODE_BYTES * vbar + BODY_EVAL_BYTES) * bodies_per_launch
        achieved = bytes_per_launch / (trav_ms * 1e-3) / 1e9 if trav_ms > 0 else 0.0
        roofline = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": measured_traffic(scene_name, "k_traverse")[0],
            "traffic_source": measured_traffic(scene_name, "k_traverse")[1],
            "kernel": "k_traverse",
            # N > 1: per evaluation (BH_SHARD_ROUNDS launches overlapped with the all-gathers)
            "kernel_avg_ms": round(trav_ms, 4),
            "launches": trav_launches,
            "rounds_per_eval": bh_amd.SHARD_ROUNDS if world > 1 else 1,
            "vbar_nodes_per_body_eval": round(vbar, 2),
            "valu_busy": (measured_valu_busy(scene_name, "k_traverse") or {}).get("valu_busy"),
            "wave_lane_efficiency": round(lane_eff, 4),
            "bytes_per_launch": round(bytes_per_launch),
        }

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
            if args.config == "c3" else f"body-steps/sec ({args.config}, theta={args.theta})",
            "value": round(value, 1),
            "unit": "body-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
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
                "parallelism": f"replicated state, force sharded x{world} (RCCL all-gather)"
                if world > 1 else "single GPU",
            },
            "phase_ms": {k: round(v, 3) for k, v in phases.items()},
            "roofline": roofline,
            "cpu_baseline": cpu_baseline,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
