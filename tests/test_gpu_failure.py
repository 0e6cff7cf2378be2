"""A rank-local failure in a multi-rank decomposition must end every rank's call, bounded in time.

The reference's force pass fans out over worker threads and joins them (computeAccelerations,
BarnesHutAlg.kt:374-395, inside runBlocking, :408, :426): the join always returns.  A decomposition
over GPUs can hang instead -- one rank returns early between collectives and its peers wait
forever in the next all-gather or barrier.  These tests make one member fail host-side
(bh_debug_inject 100 + k: before its k-th next collective; 200 + k: before its k-th next group
barrier) and check that
  * the handle's call returns an error within a bounded time, and every member refuses further
    calls (BH_E_COMM) -- no member is left waiting, and none steps on alone;
  * bh_reset_bodies recovers (new RCCL communicators for an aborted handle), and the next steps
    are bit-identical to the oracle;
  * a group barrier whose peer never arrives gives up after BH_COMM_TIMEOUT_S (a subprocess with a
    3 s limit).
"""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import bh_amd
import oracle
from bh_amd import scenes
from test_gpu_parity import FIELDS, _assert_arrays_equal

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _decompose_small_scenes(monkeypatch):
    monkeypatch.setenv("BH_MULTI_MIN_BODIES", "0")


def _scene():
    return scenes.two_disks(30000, 6000)


def _oracle_after(arrs, theta, steps):
    ref = oracle.Oracle(*arrs, theta=theta)
    ref.step(steps)
    want = ref.get_bodies()
    ref.close()
    return want


def _fail_then_recover(eng, victim, what, arrs, want):
    """Inject `what` on member `victim`, step until the call fails (bounded), check that every
    member refuses, then reset and step 4: bit-identical to `want` (the oracle after 4 steps)."""
    world = eng.multi_world()
    eng.reset_bodies(*arrs)
    eng.step(2)  # (LET builds, tables, rounds, velocity exchange: every site once)
    eng.member(victim).debug_inject(what)
    t0 = time.monotonic()
    with pytest.raises(bh_amd.BhError) as ei:
        for _ in range(4):  # (a late k may lie beyond one call's collectives)
            eng.step(2)
    elapsed = time.monotonic() - t0
    assert elapsed < 60.0, f"the failing call took {elapsed:.1f} s"
    assert ei.value.rc in (bh_amd.BH_E_COMM, bh_amd.BH_E_DEVICE), ei.value
    for r in range(world):
        pr = eng.member(r).progress()
        assert pr["failed"] and not pr["busy"], (r, pr)
    with pytest.raises(bh_amd.BhError) as ei2:  # the handle refuses until bh_reset_bodies
        eng.step(1)
    assert ei2.value.rc == bh_amd.BH_E_COMM, ei2.value
    with pytest.raises(bh_amd.BhError):
        eng.get_bodies()
    eng.reset_bodies(*arrs)
    for r in range(world):
        assert not eng.member(r).progress()["failed"], r
    eng.collective_log_clear()
    eng.step(4)
    _assert_arrays_equal(eng.get_bodies(), want, f"after recovering from {what}")
    logs = [eng.member(r).collective_log() for r in range(world)]
    for r in range(1, world):
        assert np.array_equal(logs[r], logs[0]), f"member {r}: another collective sequence"
    return elapsed


@pytest.mark.parametrize("what", [100, 101, 104, 109, 200, 203, 211])
def test_injected_member_failure_ends_every_member(what):
    """A 3-member handle on device 0 (in-process group: device-to-device copies, host barriers):
    member 1 fails before its k-th next collective (100 + k) or barrier (200 + k).  Members 0
    and 2 are released from their barriers by the group's abort -- the call returns an error,
    every member refuses the next call, and after bh_reset_bodies the state is the oracle's."""
    arrs = _scene()
    want = _oracle_after(arrs, 0.5, 4)
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), devices=[0, 0, 0])
    _fail_then_recover(eng, 1, what, arrs, want)
    eng.close()


@pytest.mark.parametrize("what", [100, 102, 105])
def test_injected_failure_on_in_process_rccl(what, monkeypatch):
    """The handle's RCCL path (one-rank communicator from ncclCommInitAll on this one-GPU box):
    the failing member aborts its communicator (ncclCommAbort); bh_reset_bodies makes a new one
    (ncclCommInitAll again), and the next steps run over RCCL bit-identically to the oracle."""
    monkeypatch.setenv("BH_MULTI_EXCHANGE", "rccl")
    monkeypatch.setenv("BH_LET", "1")
    arrs = _scene()
    want = _oracle_after(arrs, 0.5, 4)
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), devices=[0])
    assert eng.multi_world() == 1 and eng.comm_ranks() == (1, 0)
    _fail_then_recover(eng, 0, what, arrs, want)
    assert eng.comm_ranks() == (1, 0)  # a fresh communicator
    assert not eng.member(0).progress()["comm_aborted"]
    eng.close()


_PEER_NEVER_ARRIVES = r"""
import sys, threading, time
sys.path.insert(0, sys.argv[1])
import numpy as np
import bh_amd
from bh_amd import scenes
arrs = scenes.two_disks(20000, 4000)
g = bh_amd.LocalGroup(2)
p = bh_amd.default_params(theta=0.5)
e = [bh_amd.Engine(p, device=0, rank=r, local_group=g) for r in range(2)]
for m in e:
    m.reset_bodies(*arrs)
t0 = time.monotonic()
try:
    e[0].step(1)          # rank 1 never calls: rank 0's first barrier must give up
    print("NO-ERROR"); sys.exit(1)
except bh_amd.BhError as x:
    waited = time.monotonic() - t0
    assert x.rc == bh_amd.BH_E_COMM and "BH_COMM_TIMEOUT_S" in str(x), x
try:
    e[1].step(1)          # the group is aborted: the late rank refuses at once
    print("NO-ERROR-1"); sys.exit(1)
except bh_amd.BhError as x:
    assert x.rc == bh_amd.BH_E_COMM, x
for m in e:               # recovery: both reset, both step together
    m.reset_bodies(*arrs)
err = []
def run(m):
    try:
        m.step(2)
    except Exception as x:
        err.append(x)
th = [threading.Thread(target=run, args=(m,)) for m in e]
[t.start() for t in th]
[t.join() for t in th]
assert not err, err
a, b = e[0].get_bodies(), e[1].get_bodies()
assert all(np.array_equal(u.view(np.int64), v.view(np.int64)) for u, v in zip(a, b))
single = bh_amd.Engine(p, device=0)
single.reset_bodies(*arrs)
single.step(2)
w = single.get_bodies()
assert all(np.array_equal(u.view(np.int64), v.view(np.int64)) for u, v in zip(a, w))
print("WAITED %.2f" % waited)
"""


def test_group_barrier_gives_up_when_a_peer_never_arrives():
    """Two in-process ranks; rank 0 steps, rank 1 never does.  With BH_COMM_TIMEOUT_S=3 rank 0's
    first barrier gives up after ~3 s (BH_E_COMM, naming the limit), rank 1 then refuses at once
    (the group is aborted), and after both reset they step together, equal to one GPU."""
    env = dict(os.environ, BH_COMM_TIMEOUT_S="3", BH_LET="1")
    r = subprocess.run([sys.executable, "-c", _PEER_NEVER_ARRIVES,
                        os.path.join(ROOT, "barnes-hut-n-body_amd")],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    waited = float(r.stdout.split("WAITED")[1])
    assert 2.5 < waited < 30.0, waited


def test_calls_during_an_async_step_are_refused():
    """A call begun by bh_step_begin owns the handle until bh_step_end: the
    calls that fan out over the members or change engine state -- bh_synchronize,
    bh_set_profiling, bh_debug_inject, bh_collective_log_clear, bh_step, bh_last_removed -- are
    refused with BH_E_STATE from another thread; the call's result is unaffected."""
    arrs = _scene()
    eng = bh_amd.Engine(bh_amd.default_params(theta=0.5), devices=[0, 0])
    eng.set_mirror(True, buffers=2)
    eng.reset_bodies(*arrs)
    eng.step(1)
    eng.map_bodies()
    eng.step_begin(3)
    lib, h = eng._lib, eng._h
    refused = {
        "bh_synchronize": lib.bh_synchronize(h),
        "bh_set_profiling": lib.bh_set_profiling(h, 1),
        "bh_debug_inject": lib.bh_debug_inject(h, 1),
        "bh_collective_log_clear": lib.bh_collective_log_clear(h),
        "bh_step": lib.bh_step(h, 1),
        "bh_last_removed": lib.bh_last_removed(h, None, 0, None),
    }
    assert int(lib.bh_num_bodies(h)) == -1
    eng.step_end()
    assert all(v == bh_amd.BH_E_STATE for v in refused.values()), refused
    want = _oracle_after(arrs, 0.5, 4)
    _assert_arrays_equal(eng.get_bodies(), want, "after the async call")
    eng.close()


@pytest.mark.parametrize("exchange", ["copy", "rccl"])
def test_injection_sweep_never_hangs(exchange, monkeypatch):
    """Every injection point of a 2-step call: a member fails before each of its collectives
    (100 + k) and, in-process, before each of its group barriers (200 + k) in turn -- the call
    always raises within seconds, every member refuses the next call, and after the reset two
    steps equal the single-GPU engine's.  (3 members on device 0 for 'copy'; the one-rank RCCL
    handle for 'rccl'.)"""
    if exchange == "rccl":
        monkeypatch.setenv("BH_MULTI_EXCHANGE", "rccl")
        monkeypatch.setenv("BH_LET", "1")
        devices = [0]
    else:
        devices = [0, 0, 0]
    arrs = scenes.two_disks(8000, 2000)
    p = bh_amd.default_params(theta=0.5)
    single = bh_amd.Engine(p, device=0)
    single.reset_bodies(*arrs)
    single.step(2)
    want = single.get_bodies()
    single.close()
    eng = bh_amd.Engine(p, devices=devices)
    eng.reset_bodies(*arrs)
    eng.collective_log_clear()
    eng.step(2)  # how many collectives a 2-step call issues from a reset
    n_coll = len(eng.member(0).collective_log())
    assert n_coll > 0
    points = [100 + k for k in range(0, n_coll)]
    if exchange == "copy":
        points += [200 + k for k in range(0, 2 * n_coll, 2)]
    victim = len(devices) - 1
    failed = 0
    for what in points:
        eng.reset_bodies(*arrs)
        eng.member(victim).debug_inject(what)
        t0 = time.monotonic()
        try:
            eng.step(2)
            tripped = False
        except bh_amd.BhError as err:
            tripped = True
            assert err.rc in (bh_amd.BH_E_COMM, bh_amd.BH_E_DEVICE), (what, err)
        assert time.monotonic() - t0 < 60.0, what
        if not tripped:  # (fewer barriers than that in the call: the fault stays armed)
            continue
        failed += 1
        for r in range(eng.multi_world()):
            assert eng.member(r).progress()["failed"], (what, r)
        with pytest.raises(bh_amd.BhError):
            eng.step(1)
        eng.reset_bodies(*arrs)
        eng.step(2)
        _assert_arrays_equal(eng.get_bodies(), want, f"after the fault {what}")
    assert failed >= n_coll, (failed, n_coll)
    eng.close()
