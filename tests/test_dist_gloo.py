"""The multi-GPU exchange protocol, multi-process on CPU (torch.distributed / gloo, world 2 and 3).

bh_create_dist engines (engine.cpp evaluate / evaluate_let / sync_velocities, let.hip) keep the
state replicated and, per force evaluation, either build a locally essential tree and exchange
2 MB cell tables plus 16 B positions per body (owner kick), or build the full tree and exchange
accelerations; velocities follow before every full build.  tests/let_mirror.py runs exactly
that protocol -- the same pieces (bh_shard_range), the same in-place round layout
(bh_gather_slot), the same cell tables and halo rule -- with gloo in place of RCCL and the
pure-Python tree in place of the HIP kernels, one process per rank.  Every rank's final state
after two bh_step calls (LET builds, the full build that ends each call, merges, jitter,
out-of-root bodies) must equal the C oracle's serial PhysicsEngine.step() (BHA:405-439) bit for
bit.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

FIELDS = ("x", "y", "vx", "vy", "m")
PARAMS = dict(G=80.0, dt=0.005, theta=0.5, soft2=1.0, width_px=2400, height_px=800,
              merge_max_mass=4000.0, merge_min_dist=8.0)
CALLS = (3, 2)


COLL_ACC, COLL_POS, COLL_VEL, COLL_TABLE, COLL_FLAGS, COLL_VMAX = 1, 2, 3, 4, 5, 7


def check_log(log, world, n0, n_min, calls):
    """The collective sequence of a rank (bh_collective_log entries: API call, site, bytes) for
    a reset and bh_step calls of k steps each, LET from the second build on: per call the
    evaluations' exchanges in order, then the LET-status agreement and the velocity gather.
    Sizes: only the call's pieces matter (bodies removed by a call's merges change the next
    call's sizes; the byte counts are checked for internal consistency: every round of a
    per-body exchange carries the same size within a call, the table 32 (65536 + 1) B a rank)."""
    from let_mirror import _rounds
    R = _rounds()
    table_bytes = 32 * 65537 * world
    calls_seen = sorted({c for c, _, _ in log})
    assert calls_seen == list(range(2, 2 + len(calls))), calls_seen  # reset = API call 1
    boxes = False
    for ci, k in enumerate(calls):
        got = [(s, b) for c, s, b in log if c == 2 + ci]
        want_sites = []
        for step in range(k):
            for kick in ("drift", "kick"):
                if ci == 0 and step == 0 and kick == "drift":
                    want_sites += [COLL_ACC] * R  # the first (full) build
                    boxes = True
                    continue
                want_sites += [COLL_TABLE] + [COLL_POS] * R
                if kick == "drift" and boxes:
                    want_sites.append(COLL_VMAX)
        want_sites += [COLL_FLAGS] + [COLL_VEL] * R
        assert [s for s, _ in got] == want_sites, (ci, [s for s, _ in got])
        per_body = {b for s, b in got if s in (COLL_ACC, COLL_POS, COLL_VEL)}
        assert len(per_body) == 1  # R rounds of `sub` bodies a rank, 16 B each: >= n bodies
        b = per_body.pop()
        assert b % (16 * world) == 0 and R * b >= 16 * n_min
        assert R * b < 16 * (n0 + R * world * 256)  # (padded pieces)
        assert {b for s, b in got if s == COLL_TABLE} == {table_bytes}
        assert {b for s, b in got if s == COLL_FLAGS} == {8}
        assert {b for s, b in got if s == COLL_VMAX} <= {8 * world}
        boxes = True  # (valid again after a compaction: recomputed at the call's end)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def scene():
    """Two galaxy disks (NBodyPanel.kt:83-100, 2200 + 700 bodies: every rank owns lanes at
    world 3) plus: five light bodies inside the big disk's merge radius (merges in the first
    step), a coincident pair and a pair 4e-4 apart (the h < 1e-3 jitter, BHA:146-151), two
    bodies outside the root (BHA:126), and a cluster of negative masses (mass-0 cells,
    BHA:189-192)."""
    from bh_amd import scenes
    x, y, vx, vy, m = scenes.two_disks(2200, 700)
    ex = [1203.0, 1200.0, 1195.5, 1201.0, 1206.0, 700.0, 700.0, 1500.0, 1500.0004, -40.0, 2600.0]
    ey = [400.0, 405.0, 398.0, 393.5, 404.0, 650.0, 650.0, 120.0, 119.9997, 300.0, 900.0]
    ex += list(2000.0 + 3.0 * np.arange(8) % 9)
    ey += list(700.0 + np.arange(8) // 3 * 2.5)
    k = len(ex)
    em = [0.5] * 11 + [-0.4] * 8
    return (np.concatenate([x, ex]), np.concatenate([y, ey]), np.concatenate([vx, np.zeros(k)]),
            np.concatenate([vy, np.zeros(k)]), np.concatenate([m, em]))


def _worker(rank, world, port, out_dir, params=None):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "barnes-hut-n-body_amd"), os.path.dirname(__file__)]
    from let_mirror import MirrorRank

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    mr = MirrorRank(params or PARAMS, rank, world, dist)
    mr.reset_bodies(*scene())
    for k in CALLS:
        mr.step(k)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), *mr.get_bodies())
    with open(os.path.join(out_dir, f"stats{rank}.json"), "w") as fh:
        json.dump(dict(mr.stats, log=mr.log), fh)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,merge", [(2, True), (3, True), (2, False), (3, False)])
def test_exchange_protocol_matches_the_reference_step(tmp_path, world, merge):
    """Every rank of a world-2/3 gloo group runs the engine's exchange protocol (LET builds,
    table and position all-gathers, velocity syncs, replicated merge rule) with and without the
    merge rule; every rank's final state equals the oracle's bit for bit."""
    import bh_amd  # noqa: F401  (the engine library's host-only shard layout must load)
    import oracle

    params = dict(PARAMS, merge_min_dist=8.0 if merge else 0.0)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), params), nprocs=world, join=True)
    arrs = scene()
    ref = oracle.Oracle(*arrs, threads=1, **params)
    for k in CALLS:
        ref.step(k)
    want = ref.get_bodies()
    if merge:
        assert len(want[0]) < len(arrs[0])  # the merge rule removed bodies
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npz")
        stats = json.load(open(tmp_path / f"stats{r}.json"))
        # the first build after the reset is full, every later one a LET build (fewer than
        # BH_LET_REFRESH); the velocities are gathered at the end of every call
        assert stats["let"] == 2 * sum(CALLS) - 1 and stats["full"] == 1
        assert stats["vel_syncs"] == len(CALLS)
        check_log(stats["log"], world, n0=len(arrs[0]), n_min=len(want[0]), calls=CALLS)
        assert stats["log"] == json.load(open(tmp_path / "stats0.json"))["log"]
        assert stats["merged"] == len(arrs[0]) - len(want[0])
        # every rank owns bodies; at world 3 a rank builds a part of the scene only
        assert 0 < stats["max_subset"] <= len(arrs[0])
        if world == 3:
            assert stats["max_subset"] < len(arrs[0]), stats
        for k, name in enumerate(FIELDS):
            a = got[f"arr_{k}"]
            assert a.shape == want[k].shape, f"rank {r}: {name} length"
            bad = np.flatnonzero(a.view(np.int64) != want[k].view(np.int64))
            assert len(bad) == 0, f"rank {r}: {name} differs at {bad[:5]}"


def test_morton_order_matches_tree_preorder():
    """The slot order the pieces are cut from is the tree's leaf pre-order (child 0..3 =
    ascending Morton digit, BHA:73-81)."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from let_mirror import Geometry
    from bh_amd import scenes
    x, y, *_ = scenes.uniform(64, 1.0, seed=2)
    perm = np.argsort(Geometry(2400, 800).keys(x, y, np.zeros(64, dtype=bool)), kind="stable")
    cx0, cy0 = 1200.0, 400.0
    q = [(x[i] >= cx0) + 2 * (y[i] >= cy0) for i in perm]
    assert q == sorted(q)
