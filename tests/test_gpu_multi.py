"""One PhysicsEngine handle over several GPUs (bh_create_multi / bh_create_multi_list, multi.cpp).

The reference's step() fans its force evaluation out over worker threads and joins them
(computeAccelerations, BarnesHutAlg.kt:374-395, inside runBlocking, :408, :426); the front-end
holds ONE PhysicsEngine (NBodyPanel.kt:103) and steps it per frame (:290-293).  The multi-device
handle is that object over GPUs: member engines -- the ranks of the multi-GPU decomposition --
each on its own host thread, the caller's thread running member 0.  On this one-GPU box the
members share device 0 (a device listed twice exchanges by device-to-device copies: RCCL refuses
two ranks per device); a one-member handle on an in-process RCCL communicator covers the RCCL
path (BH_MULTI_EXCHANGE=rccl).  Every state is compared bit for bit with the oracle or the
single-GPU engine, and every member's collective log (bh_collective_log: the order in which a
rank issues its all-gathers / all-reduces) must be identical -- a mismatch is what would hang
the first real 8-GPU run.
"""
import numpy as np
import pytest

import bh_amd
import oracle
from bh_amd import scenes
from conftest import bits_equal
from test_gpu_parity import FIELDS, _assert_arrays_equal, _frames_scene, _let_scene

pytestmark = pytest.mark.gpu

SITES = {1: "acc", 2: "pos", 3: "vel", 4: "table", 5: "flags", 6: "settings", 7: "vmax"}


@pytest.fixture(autouse=True)
def _decompose_small_scenes(monkeypatch):
    # below BH_MULTI_MIN_BODIES a multi-device handle steps on one GPU; these scenes are small
    monkeypatch.setenv("BH_MULTI_MIN_BODIES", "0")


def _logs_agree(eng):
    """Every member's collective log, asserted identical; returns member 0's."""
    logs = [eng.member(r).collective_log() for r in range(eng.multi_world())]
    for r, lg in enumerate(logs[1:], 1):
        assert lg.shape == logs[0].shape and np.array_equal(lg, logs[0]), \
            f"member {r} issued another collective sequence: {_first_diff(logs[0], lg)}"
    return logs[0]


def _first_diff(a, b):
    n = min(len(a), len(b))
    for i in range(n):
        if not np.array_equal(a[i], b[i]):
            return f"entry {i}: {a[i].tolist()} vs {b[i].tolist()}"
    return f"lengths {len(a)} vs {len(b)}"


def _count(log, site):
    return int(np.sum(log[:, 1] == site)) if len(log) else 0


def _single(params, arrs, calls):
    eng = bh_amd.Engine(params, device=0)
    eng.reset_bodies(*arrs)
    for k in calls:
        eng.step(k)
    want = eng.get_bodies()
    quads = eng.get_quads()
    eng.close()
    return want, quads


def test_multi_handle_frames_match_the_oracle():
    """The front-end's pattern on a 3-member handle (device 0 three times): one step() per
    frame, every body read back through the handle's pinned mirror and bh_get_bodies,
    getTreeForDebug().visitQuads every few frames -- including frames whose last step's merge
    rule removed a body, where getTreeForDebug builds a fresh tree whose jitter moves bodies
    (BHA:146-151, 329-332, 526) in every replica alike -- frame by frame bit-identical to the
    oracle, and the members' collective sequences identical."""
    arrs = _frames_scene()
    p = bh_amd.default_params(theta=0.5)
    eng = bh_amd.Engine(p, devices=[0, 0, 0])
    assert eng.multi_world() == 3
    eng.set_mirror(True)
    eng.reset_bodies(*arrs)
    ref = oracle.Oracle(*arrs, theta=0.5)
    fresh_after_merge = 0
    for f in range(24):
        n_before = eng.num_bodies()
        eng.step(1)
        ref.step(1)
        want = ref.get_bodies()
        _assert_arrays_equal(eng.map_bodies(), want, f"frame {f} mirror")
        _assert_arrays_equal(eng.get_bodies(), want, f"frame {f}")
        removed_now = eng.num_bodies() < n_before
        if f % 3 == 1 or removed_now:
            wq = ref.quads()
            for u, v in zip(eng.get_quads(), wq):
                assert bits_equal(u, v), f"frame {f} quads"
            fresh_after_merge += int(removed_now)
            want = ref.get_bodies()  # a fresh tree jitters the bodies (BHA:146-151)
            _assert_arrays_equal(eng.get_bodies(), want, f"frame {f} after quads")
            _assert_arrays_equal(eng.map_bodies(), want, f"frame {f} mirror after quads")
    assert eng.num_bodies() < len(arrs[0])
    assert fresh_after_merge >= 1, "no frame exercised getTreeForDebug after a removal"
    log = _logs_agree(eng)
    assert _count(log, 4) > 0 and _count(log, 2) > 0 and _count(log, 3) >= 24, \
        {SITES[k]: _count(log, k) for k in SITES}
    eng.close()
    ref.close()


@pytest.mark.parametrize("devices,scene,theta", [
    ([0, 0], "c2", 0.5), ([0, 0, 0, 0], "jitter", 0.5), ([0] * 8, "cloud", 0.5),
    ([0, 0, 0], "outside", 0.7)])
def test_multi_handle_equals_single_gpu(devices, scene, theta):
    """Batched calls (4 then 3 steps) through the handle: state and lastTree quads equal the
    single-GPU engine's bit for bit at 2, 3, 4 and 8 members; identical collective logs."""
    arrs = _let_scene(scene)
    params = bh_amd.default_params(theta=theta, merge_min_dist=0.0 if scene == "jitter" else 8.0)
    want, want_q = _single(params, arrs, (4, 3))
    eng = bh_amd.Engine(params, devices=devices)
    eng.reset_bodies(*arrs)
    for k in (4, 3):
        eng.step(k)
    got = eng.get_bodies()
    for k, name in enumerate(FIELDS):
        assert bits_equal(got[k], want[k]), name
    for u, v in zip(eng.get_quads(), want_q):
        assert bits_equal(u, v), "lastTree quads"
    log = _logs_agree(eng)
    st = eng.let_stats()
    assert st["let_builds"] == 13 and st["full_builds"] == 1, st
    assert _count(log, 4) == 13 and _count(log, 5) == 2, {SITES[k]: _count(log, k) for k in SITES}
    eng.close()


def test_collective_logs_agree_across_branches():
    """The branches that decide which collectives a rank issues, through one 4-member handle:
    a reset, the LET builds inside a call and its end-of-call velocity sync, the refresh full
    build of a 40-build call, a rank-local LET guard (injected on member 2 only) that every
    rank replays, a subset overflow after a reset to 4x the bodies (every rank replays),
    getTreeForDebug after a call whose last step merged, BH_LET-off full evaluations, theta = 0
    -- every member's log identical after each, and the state equal to the single-GPU engine."""
    small = scenes.uniform(50_000, 0.5, seed=21)
    big = scenes.uniform(200_000, 0.5, seed=22)
    heavy = _frames_scene()
    params = bh_amd.default_params(theta=0.5)
    eng = bh_amd.Engine(params, devices=[0, 0, 0, 0])
    single = bh_amd.Engine(params, device=0)

    def both(fn):
        fn(eng)
        fn(single)
        lg = _logs_agree(eng)
        want = single.get_bodies()
        got = eng.get_bodies()
        for k, name in enumerate(FIELDS):
            assert bits_equal(got[k], want[k]), name
        return lg

    both(lambda e: (e.reset_bodies(*small), e.step(3)))
    lg = both(lambda e: e.step(20))  # 40 builds: a refresh full build inside the call
    assert eng.let_stats()["full_builds"] >= 2
    eng.member(2).debug_inject(1)    # rank 2's next LET build trips its guard
    before = eng.member(0).let_stats()["overflows"]
    lg = both(lambda e: e.step(2))
    for r in range(4):
        assert eng.member(r).let_stats()["overflows"] == before + 1, r
    lg = both(lambda e: (e.reset_bodies(*big), e.step(2)))
    assert eng.let_stats()["overflows"] >= before + 2
    both(lambda e: (e.reset_bodies(*heavy), e.step(2)))
    for _ in range(12):  # until a call's last step merges: getTreeForDebug builds afresh
        n0 = eng.num_bodies()
        both(lambda e: e.step(1))
        if eng.num_bodies() < n0:
            break
    assert eng.num_bodies() < len(heavy[0])
    q_multi, q_single = eng.get_quads(), single.get_quads()
    for u, v in zip(q_multi, q_single):
        assert bits_equal(u, v), "quads after a merge"
    both(lambda e: e.step(2))  # ... and the next steps from the jittered state
    p0 = bh_amd.default_params(theta=0.0)
    both(lambda e: (e.set_params(p0), e.step(1)))  # theta = 0: full builds, accelerations
    eng.close()
    single.close()


def test_multi_handle_let_off_and_theta0(monkeypatch):
    """BH_LET=0: every build full and replicated, the accelerations all-gathered (site 1), at
    theta 0.5 and 0 -- 3 members, state equal to the oracle, identical logs."""
    monkeypatch.setenv("BH_LET", "0")
    arrs = scenes.config_scene("c1_code")
    for theta in (0.5, 0.0):
        eng = bh_amd.Engine(bh_amd.default_params(theta=theta), devices=[0, 0, 0])
        eng.reset_bodies(*arrs)
        eng.step(3)
        ref = oracle.Oracle(*arrs, theta=theta)
        ref.step(3)
        want = ref.get_bodies()
        got = eng.get_bodies()
        for k, name in enumerate(FIELDS):
            assert bits_equal(got[k], want[k]), f"theta {theta}: {name}"
        log = _logs_agree(eng)
        assert _count(log, 1) == 6 * bh_amd.SHARD_ROUNDS and _count(log, 4) == 0, log
        eng.close()
        ref.close()


@pytest.mark.parametrize("let", ["0", "1"])
def test_multi_handle_on_in_process_rccl(let, monkeypatch):
    """The handle's RCCL path: a communicator made in this process by ncclCommInitAll (one rank
    on this one-GPU box), the settings check run by the member's thread, the round all-gathers
    and (BH_LET=1) the table all-gathers and status all-reduce over RCCL -- bit-identical to the
    oracle, and the member's log holds the settings check."""
    monkeypatch.setenv("BH_MULTI_EXCHANGE", "rccl")
    monkeypatch.setenv("BH_LET", let)
    arrs = scenes.config_scene("c1_code")
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), devices=[0])
    assert eng.multi_world() == 1 and eng.comm_ranks() == (1, 0)
    eng.reset_bodies(*arrs)
    eng.step(3)
    ref = oracle.Oracle(*arrs, theta=0.5)
    ref.step(3)
    want = ref.get_bodies()
    got = eng.get_bodies()
    for k, name in enumerate(FIELDS):
        assert bits_equal(got[k], want[k]), name
    log = eng.member(0).collective_log()
    assert _count(log, 6) == 1
    assert _count(log, 4 if let == "1" else 1) > 0
    eng.close()
    ref.close()


def test_small_body_lists_step_on_one_gpu(monkeypatch):
    """Below BH_MULTI_MIN_BODIES the handle steps the body list with the single-GPU engine
    (the reference's min(cores, n) workers, BHA:377): reset to a small list -> one member,
    reset to a large one -> the decomposition; the states equal the oracle's either way and the
    settings (params, mirror) follow across the switch."""
    monkeypatch.setenv("BH_MULTI_MIN_BODIES", "10000")
    small = scenes.config_scene("c1_baseline")  # 2 000 bodies
    large = scenes.config_scene("c1_code")      # 12 500 bodies
    p = bh_amd.default_params(theta=0.5)
    eng = bh_amd.Engine(p, devices=[0, 0])
    eng.set_mirror(True)
    for arrs, world in ((small, 1), (large, 2), (small, 1)):
        eng.set_params(bh_amd.default_params(theta=0.6))
        eng.reset_bodies(*arrs)
        assert eng.multi_world() == world
        eng.step(2)
        ref = oracle.Oracle(*arrs, theta=0.6)
        ref.step(2)
        _assert_arrays_equal(eng.map_bodies(), ref.get_bodies(), f"world {world}")
        ref.close()
    eng.close()


def test_let_selection_bound_with_fast_movers():
    """The LET selection scans only the slot blocks whose box (their bodies' cells at the last
    full build) widened by the displacement bound since (max speed x dt per drift, every rank's
    maximum exchanged, plus the jitter) reaches a built cell.  Streams of fast bodies (up to 3
    depth-8 cells per step) cross every rank's region, and a few run off the root and come back;
    4 members over 24 steps (two refresh-free calls of 12): the state equals the single-GPU
    engine's bit for bit -- a body the bound missed would be left out of a subset."""
    rng = np.random.default_rng(91)
    x, y, vx, vy, m = (a.copy() for a in scenes.uniform(120_000, 0.5, seed=90))
    k = 3000
    sx, sy = rng.uniform(0, 2400, k), rng.uniform(0, 800, k)
    ang = rng.uniform(0, 2 * np.pi, k)
    sp = rng.uniform(500.0, 5600.0, k)  # 5600 px/unit x 0.005 = 28 px = 3 cells per step
    arrs = (np.concatenate([x, sx]), np.concatenate([y, sy]),
            np.concatenate([vx, sp * np.cos(ang)]), np.concatenate([vy, sp * np.sin(ang)]),
            np.concatenate([m, np.full(k, 0.5)]))
    params = bh_amd.default_params(theta=0.5, merge_min_dist=0.0)
    want, want_q = _single(params, arrs, (12, 12))
    eng = bh_amd.Engine(params, devices=[0, 0, 0, 0])
    eng.reset_bodies(*arrs)
    for kk in (12, 12):
        eng.step(kk)
    got = eng.get_bodies()
    for j, name in enumerate(FIELDS):
        assert bits_equal(got[j], want[j]), name
    log = _logs_agree(eng)
    assert _count(log, 7) > 0  # the speed bounds were exchanged
    eng.close()


@pytest.mark.parametrize("world,merge", [(2, True), (3, False)])
def test_collective_sequence_equals_the_protocol_mirror(tmp_path, world, merge):
    """The engine's recorded collective sequence (every member's bh_collective_log: API call,
    site, bytes) equals, entry by entry, the one the CPU protocol mirror issues over gloo for the
    same scene and calls (tests/let_mirror.py, one process per rank) -- the sequence the CPU suite
    checks (test_dist_gloo.check_log) is the engine's own, and so are the final states."""
    import json
    import torch.multiprocessing as mp
    import test_dist_gloo as tg

    params = dict(tg.PARAMS, merge_min_dist=8.0 if merge else 0.0)
    mp.spawn(tg._worker, args=(world, tg._free_port(), str(tmp_path), params), nprocs=world,
             join=True)
    eng = bh_amd.Engine(bh_amd.default_params(**params), devices=[0] * world)
    eng.reset_bodies(*tg.scene())
    for k in tg.CALLS:
        eng.step(k)
    got = eng.get_bodies()
    log = _logs_agree(eng)[:, :3].tolist()
    for r in range(world):
        st = json.load(open(tmp_path / f"stats{r}.json"))
        assert log == st["log"], f"rank {r}: {_first_diff(np.array(log), np.array(st['log']))}"
        mine = np.load(tmp_path / f"rank{r}.npz")
        for k, name in enumerate(FIELDS):
            assert bits_equal(got[k], mine[f"arr_{k}"]), f"rank {r}: {name}"
    eng.close()
