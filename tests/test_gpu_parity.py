"""GPU parity: the HIP engine (through the C-ABI) vs the CPU oracle on identical inputs.

The bar is bit-identity of every fp64 word (positions, velocities, masses, accelerations,
per-body node-visit counts): the reference is strict IEEE binary64 (JVM >= 17) and the engine
reproduces its tree, criterion, summation order and expression order exactly.  The
north-star tolerance (<= 1e-6 relative position drift after 100 steps) is therefore met with
margin 0; where NaN can arise (zero-mass bodies), NaN payloads are compared as "both NaN".
"""
import numpy as np
import pytest

import bh_amd
import oracle
from bh_amd import scenes
from conftest import bits_equal

pytestmark = pytest.mark.gpu

FIELDS = ("x", "y", "vx", "vy", "m")


def _pair(arrs, **kw):
    theta = kw.pop("theta", 0.5)
    p = bh_amd.default_params(theta=theta, **kw)
    eng = bh_amd.Engine(p, device=0)
    eng.reset_bodies(*arrs)
    eng.initial = arrs  # for a second engine on the same start (a build may jitter positions)
    ref = oracle.Oracle(*arrs, theta=theta, **kw)
    return eng, ref


def _production_walk(eng):
    """Accelerations of the production walk (paired force blocks, no counters) on a fresh
    engine from the same start: a second build on `eng` would see jittered positions."""
    e2 = bh_amd.Engine(eng.params, device=0)
    e2.reset_bodies(*eng.initial)
    fx, fy = e2.compute_accelerations()
    e2.close()
    return fx, fy


def _assert_state_equal(eng, ref, nan_ok=False):
    got, want = eng.get_bodies(), ref.get_bodies()
    assert len(got[0]) == len(want[0]), f"N: engine {len(got[0])} vs oracle {len(want[0])}"
    for k, name in enumerate(FIELDS):
        if nan_ok:
            assert np.array_equal(got[k], want[k], equal_nan=True), name
        else:
            bad = np.flatnonzero(got[k].view(np.int64) != want[k].view(np.int64))
            assert bad.size == 0, f"{name}: {bad.size} words differ, first at {bad[:5]}"


def _assert_acc_equal(eng, ref, nan_ok=False):
    """Accelerations and visit counts vs the oracle.  The engine evaluates twice on the same
    tree: the production walk (no counters: paired force blocks) and the counting walk."""
    fx, fy = _production_walk(eng)
    ax, ay, vis = eng.compute_accelerations(visits=True)
    rax, ray, rvis = ref.accelerations(visits=True)
    if nan_ok:
        assert np.array_equal(fx, rax, equal_nan=True) and np.array_equal(fy, ray, equal_nan=True)
    else:
        assert bits_equal(fx, rax) and bits_equal(fy, ray), "production walk differs"
    if nan_ok:
        assert np.array_equal(ax, rax, equal_nan=True)
        assert np.array_equal(ay, ray, equal_nan=True)
    else:
        assert bits_equal(ax, rax), f"ax differs at {np.flatnonzero(ax.view(np.int64) != rax.view(np.int64))[:5]}"
        assert bits_equal(ay, ray)
    assert np.array_equal(vis, rvis), "node-visit counts differ"
    _assert_state_equal(eng, ref, nan_ok=nan_ok)  # the jitter's mutation must match too
    return vis


def test_two_body_known_answer():
    # a1 = G m2 d / (|d|^2 + eps^2)^{3/2}: d = (3, 4), |d|^2 + 1 = 26
    arrs = (np.array([100.0, 103.0]), np.array([100.0, 104.0]), np.zeros(2), np.zeros(2),
            np.array([1.0, 2.0]))
    eng, ref = _pair(arrs, merge_min_dist=0.0)
    ax, ay = eng.compute_accelerations()
    rax, ray = ref.accelerations()
    assert bits_equal(ax, rax) and bits_equal(ay, ray)
    k = 80.0 / 26.0 ** 1.5
    np.testing.assert_allclose(ax, [k * 2 * 3, -k * 1 * 3], rtol=1e-14)
    np.testing.assert_allclose(ay, [k * 2 * 4, -k * 1 * 4], rtol=1e-14)


@pytest.mark.parametrize("theta", [0.0, 0.2, 0.3, 0.5, 1.0, 1.6])
def test_theta_sweep_accelerations(theta):
    arrs = scenes.two_disks(2500, 700)
    eng, ref = _pair(arrs, theta=theta)
    _assert_acc_equal(eng, ref)


def test_c1_baseline_100_steps():
    """BASELINE 'R' scene, 2 x 1000 bodies, theta 0.5: 100 full steps, bit-identical."""
    arrs = scenes.config_scene("c1_baseline")
    eng, ref = _pair(arrs, theta=0.5)
    eng.step(100)
    ref.step(100)
    _assert_state_equal(eng, ref)


def test_c1_code_default_scene():
    """The code's defaultBodies() (12 500 bodies) at the code's theta 0.30, 10 steps."""
    arrs = scenes.config_scene("c1_code")
    eng, ref = _pair(arrs, theta=0.30)
    eng.step(10)
    ref.step(10)
    _assert_state_equal(eng, ref)


def test_jitter_coincident_and_near_bodies():
    """Exact duplicates and pairs closer than 1e-3 force the h < 1e-3 jitter (BHA:146-151),
    which mutates positions and drops bodies from the tree; replayed in index order."""
    rng = np.random.default_rng(7)
    base = scenes.uniform(3000, 1.0, seed=11)
    x, y, vx, vy, m = (a.copy() for a in base)
    # 40 exact duplicates of existing bodies, 40 near pairs (2e-4 apart), a 6-fold stack
    dup = rng.choice(3000, 40, replace=False)
    near = rng.choice(3000, 40, replace=False)
    ex = np.concatenate([x[dup], x[near] + 2e-4, np.full(6, 1234.5678)])
    ey = np.concatenate([y[dup], y[near] - 1.5e-4, np.full(6, 321.0123)])
    n_extra = len(ex)
    x = np.concatenate([x, ex])
    y = np.concatenate([y, ey])
    vx = np.concatenate([vx, np.zeros(n_extra)])
    vy = np.concatenate([vy, np.zeros(n_extra)])
    m = np.concatenate([m, np.full(n_extra, 1.0)])
    perm = rng.permutation(len(x))  # interleave so insertion order matters
    arrs = tuple(a[perm] for a in (x, y, vx, vy, m))
    eng, ref = _pair(arrs, theta=0.5, merge_min_dist=0.0)
    _assert_acc_equal(eng, ref)
    eng.step(3)
    ref.step(3)
    _assert_state_equal(eng, ref)


def test_bodies_outside_root_cell():
    """Bodies outside [cx-h, cx+h) are never inserted (BHA:126) but still feel and integrate."""
    arrs = scenes.uniform(500, 1.0, seed=5)
    x = np.concatenate([arrs[0], [-3.0, 2402.0, 1200.0 + 1202.0, 1200.0 - 1202.0, 600.0]])
    y = np.concatenate([arrs[1], [400.0, 400.0, 100.0, 100.0, -802.0 - 1e-9]])
    k = 5
    arrs = (x, y, np.concatenate([arrs[2], np.zeros(k)]), np.concatenate([arrs[3], np.zeros(k)]),
            np.concatenate([arrs[4], np.full(k, 3.0)]))
    eng, ref = _pair(arrs, theta=0.5)
    _assert_acc_equal(eng, ref)
    eng.step(5)
    ref.step(5)
    _assert_state_equal(eng, ref)


def test_every_body_outside_the_root_cell():
    """No body inside the root cell: the tree is empty, every body feels no force and just
    drifts (BHA:126, 216); also after a live geometry change that puts them all outside."""
    n = 300
    rng = np.random.default_rng(8)
    x = rng.uniform(2500.0, 2600.0, n)  # x >= cx + h = 2402
    y = rng.uniform(0.0, 800.0, n)
    arrs = (x, y, rng.uniform(-5, 5, n), rng.uniform(-5, 5, n), np.full(n, 2.0))
    eng, ref = _pair(arrs, theta=0.5)
    ax, ay = eng.compute_accelerations()
    rax, ray = ref.accelerations()
    assert bits_equal(ax, rax) and bits_equal(ay, ray) and not np.any(ax)
    eng.step(3)
    ref.step(3)
    _assert_state_equal(eng, ref)


def test_merge_rule():
    """Heavy bodies (m > 4000) absorb bodies with d^2 < 64 (BHA:463-532): 7.9 eaten, 8.1 not;
    a heavy absorbed by a later heavy carries its grown mass; N shrinks."""
    bx = [1000.0, 1007.9, 1008.1, 1000.0, 1003.0, 1500.0, 1504.0, 1200.0, 1200.5]
    by = [400.0, 400.0, 400.0, 406.0, 403.0, 300.0, 300.0, 200.0, 200.0]
    bm = [5000.0, 1.0, 1.0, 2.0, 4500.0, 10.0, 9000.0, 3.0, 4001.0]
    field = scenes.uniform(300, 0.5, seed=9)
    arrs = (np.concatenate([bx, field[0]]), np.concatenate([by, field[1]]),
            np.concatenate([np.zeros(9), field[2]]), np.concatenate([np.zeros(9), field[3]]),
            np.concatenate([bm, field[4]]))
    eng, ref = _pair(arrs, theta=0.5, dt=0.0)  # dt = 0: positions fixed, pure merge
    eng.step(1)
    ref.step(1)
    _assert_state_equal(eng, ref)
    assert eng.num_bodies() < len(arrs[0])
    eng2, ref2 = _pair(arrs, theta=0.5)
    eng2.step(20)
    ref2.step(20)
    _assert_state_equal(eng2, ref2)


@pytest.mark.parametrize("crowd", [400, 6000])
def test_merge_rule_long_candidate_lists(crowd):
    """More candidate pairs than the LDS replay holds (1024 / 2048): the bitmap-ordered replay
    (integrate.hip replay_large).  Three heavy bodies inside one crowd -- the first absorbs the
    second, whose grown mass it then carries -- plus a heavy in a second crowd; dt = 0 isolates
    the rule, then full steps."""
    rng = np.random.default_rng(crowd)
    r = 7.9 * np.sqrt(rng.random(crowd))
    phi = 2 * np.pi * rng.random(crowd)
    cx = np.concatenate([1000.0 + r * np.cos(phi), 1600.0 + r[: crowd // 3] * np.sin(phi[: crowd // 3])])
    cy = np.concatenate([400.0 + r * np.sin(phi), 300.0 + r[: crowd // 3] * np.cos(phi[: crowd // 3])])
    cm = rng.uniform(0.1, 3.0, len(cx))
    hx = [1000.0, 1003.0, 1001.0, 1600.0]
    hy = [400.0, 401.0, 399.0, 300.0]
    hm = [5000.0, 4500.0, 9000.0, 6000.0]
    field = scenes.uniform(500, 0.5, seed=13)
    x = np.concatenate([cx, hx, field[0]])
    y = np.concatenate([cy, hy, field[1]])
    m = np.concatenate([cm, hm, field[4]])
    perm = rng.permutation(len(x))  # heavies and victims interleaved in list order
    arrs = tuple(a[perm] for a in (x, y, np.zeros(len(x)), np.zeros(len(x)), m))
    eng, ref = _pair(arrs, theta=0.5, dt=0.0)
    eng.step(1)
    ref.step(1)
    _assert_state_equal(eng, ref)
    assert eng.num_bodies() < len(x) - crowd
    eng2, ref2 = _pair(arrs, theta=0.5)
    eng2.step(3)
    ref2.step(3)
    _assert_state_equal(eng2, ref2)


def test_merge_rule_more_pairs_than_the_mailbox():
    """A crowd of 520 heavy bodies (m > mergeMaxMass) within a 20 x 20 box: every heavy sees
    ~180 others closer than mergeMinDist, ~9e4 candidate pairs against a mailbox of
    max(65 536, 2 N) -- the call is replayed from its snapshot with a grown mailbox, and the
    list (more heavies than the bitmap replay takes) is sorted by the one-workgroup radix
    sort, so the rule (BHA:478-520) holds for any number of pairs: bit-identical to the
    oracle, with light bodies around and several steps per call."""
    rng = np.random.default_rng(77)
    nh = 520
    hx = 1000.0 + 20.0 * rng.random(nh)
    hy = 400.0 + 20.0 * rng.random(nh)
    hm = rng.uniform(4001.0, 6000.0, nh)
    field = scenes.uniform(3000, 0.5, seed=17)
    x = np.concatenate([hx, field[0]])
    y = np.concatenate([hy, field[1]])
    m = np.concatenate([hm, field[4]])
    perm = rng.permutation(len(x))
    arrs = tuple(a[perm] for a in (x, y, np.zeros(len(x)), np.zeros(len(x)), m))
    d2 = (hx[:, None] - x[None, :]) ** 2 + (hy[:, None] - y[None, :]) ** 2
    assert (d2 < 64.0).sum() - nh > max(65_536, 2 * len(x))  # the first step overflows
    eng, ref = _pair(arrs, theta=0.5)
    eng.step(3)
    ref.step(3)
    _assert_state_equal(eng, ref)
    assert eng.num_bodies() < len(x) - nh // 2
    removed = eng.last_removed()
    assert len(removed) == len(x) - eng.num_bodies()


@pytest.mark.parametrize("wh", [(640, 480), (800, 600), (1366, 768), (1920, 1080),
                                (2560, 1440), (3840, 2160), (5120, 2880), (7680, 4320)])
def test_jitter_replay_across_screen_geometries(wh):
    """Main.kt:11-12 sets the root cell from the screen size, which moves the jitter depth J
    (h < 1e-3, BHA:146-151) and the cell centres.  Coincident, 1e-4 / 5e-4 / 9e-4-apart pairs
    and coincident triples at random places: the serial replay of every depth-J cell never
    reports an unsupported geometry (BH_E_STATE) and the state is bit-identical over 3 steps."""
    W, H = wh
    rng = np.random.default_rng(W * 7 + H)
    base = scenes.uniform(1500, 1.0, seed=W + H, width_px=W, height_px=H)
    k = 60
    px = rng.uniform(0.0, W, k)
    py = rng.uniform(0.0, H, k)
    sep = rng.choice([0.0, 1e-4, 5e-4, 9e-4], k)
    ang = rng.uniform(0.0, 2 * np.pi, k)
    ex = np.concatenate([px, px + sep * np.cos(ang), px[:10]])
    ey = np.concatenate([py, py + sep * np.sin(ang), py[:10]])
    x = np.concatenate([base[0], ex])
    y = np.concatenate([base[1], ey])
    m = np.concatenate([base[4], np.full(len(ex), 1.0)])
    perm = rng.permutation(len(x))
    arrs = tuple(a[perm] for a in (x, y, np.zeros(len(x)), np.zeros(len(x)), m))
    eng, ref = _pair(arrs, theta=0.5, width_px=W, height_px=H, merge_min_dist=0.0)
    eng.step(3)  # raises BhError(BH_E_STATE) if the replay met an unsupported geometry
    ref.step(3)
    _assert_state_equal(eng, ref)


@pytest.mark.parametrize("n", [0, 1, 2])
def test_tiny_and_empty(n):
    arrs = tuple(a[:n] for a in scenes.uniform(4, 2.0, seed=1))
    eng, ref = _pair(arrs)
    eng.step(3)
    ref.step(3)
    _assert_state_equal(eng, ref)


def test_zero_and_negative_mass():
    arrs = [a.copy() for a in scenes.uniform(400, 1.0, seed=3)]
    arrs[4][[5, 17]] = 0.0     # a = 0/0 for these (NaN), skipped as nodes
    arrs[4][[9]] = -2.0        # visited as a leaf, excluded from parents' COM (BHA:189-192)
    eng, ref = _pair(tuple(arrs), merge_min_dist=0.0)
    _assert_acc_equal(eng, ref, nan_ok=True)


def test_other_screen_geometry():
    """Config.WIDTH_PX/HEIGHT_PX = a 1920x1080 screen (Main.kt:11-12): root h = 962, so the
    jitter depth is 20 instead of 21."""
    arrs = scenes.two_disks(1500, 400)
    eng, ref = _pair(arrs, theta=0.5, width_px=1920, height_px=1080)
    _assert_acc_equal(eng, ref)
    eng.step(5)
    ref.step(5)
    _assert_state_equal(eng, ref)


def test_live_config_changes_between_steps():
    """theta / DT / G are read live at every step (PNL:247-260); theta 0 in between switches to
    the all-pairs kernel and back (the Hilbert lane map is rebuilt after it)."""
    arrs = scenes.two_disks(1500, 400)
    eng, ref = _pair(arrs, theta=0.5)
    for theta, dt, G in ((0.5, 0.005, 80.0), (0.9, 0.01, 60.0), (0.0, 0.005, 80.0),
                         (0.3, -0.005, 80.0)):
        eng.set_params(bh_amd.default_params(theta=theta, dt=dt, G=G))
        ref.set_params(oracle.params(theta=theta, dt=dt, G=G))
        eng.step(2)
        ref.step(2)
    _assert_state_equal(eng, ref)


def test_quads_match_visit_quads():
    arrs = scenes.two_disks(800, 200)
    eng, ref = _pair(arrs, theta=0.5, merge_min_dist=0.0)
    eng.step(1)
    ref.step(1)
    got = eng.get_quads()
    want = ref.quads()
    for g, w in zip(got, want):
        assert bits_equal(g, w)


def test_deterministic_rerun():
    arrs = scenes.config_scene("c1_code")
    a = bh_amd.Engine(bh_amd.default_params(theta=0.5))
    a.reset_bodies(*arrs)
    a.step(3)
    b = bh_amd.Engine(bh_amd.default_params(theta=0.5))
    b.reset_bodies(*arrs)
    b.step(3)
    for u, v in zip(a.get_bodies(), b.get_bodies()):
        assert bits_equal(u, v)


def test_c2_kepler_1e5_100_steps():
    """C2 (Kepler disk, 1e5 bodies, theta 0.5) over the north star's 100 steps (SURVEY §8d
    parity runs: K = 100 for C1/C2): positions, velocities and masses bit-identical, i.e.
    zero drift against the <= 1e-6 bound."""
    arrs = scenes.config_scene("c2")
    eng, ref = _pair(arrs, theta=0.5)
    eng.step(100)
    ref.step(100)
    _assert_state_equal(eng, ref)


def test_c3_1e6_full_size_sampled():
    """The bench workload (two colliding disks, N = 1e6, theta 0.5): one evaluation, every
    body's acceleration and visit count against the oracle; then one full step."""
    arrs = scenes.config_scene("c3")
    eng, ref = _pair(arrs, theta=0.5)
    vis = _assert_acc_equal(eng, ref)
    assert vis.mean() > 10
    eng.step(1)
    ref.step(1)
    _assert_state_equal(eng, ref)


def _assert_sampled_evaluation(arrs, theta, stride):
    """Engine: every body's acceleration (and visit count unless theta = 0); oracle: its own
    serial tree, then the walk of every `stride`-th body; the sampled bodies bit-identical."""
    eng, ref = _pair(arrs, theta=theta)
    sample = np.arange(0, len(arrs[0]), stride, dtype=np.int64)
    if theta == 0.0:  # the all-pairs kernel (no visit counts on that path)
        ax, ay = eng.compute_accelerations()
        rax, ray = ref.accelerations(subset=sample)
    else:
        fx, fy = _production_walk(eng)  # paired force blocks
        ax, ay, vis = eng.compute_accelerations(visits=True)
        rax, ray, rvis = ref.accelerations(subset=sample, visits=True)
        assert np.array_equal(vis[sample], rvis), "node-visit counts differ"
        assert bits_equal(fx[sample], rax) and bits_equal(fy[sample], ray), "production walk"
    bad = np.flatnonzero(ax[sample].view(np.int64) != rax.view(np.int64))
    assert bad.size == 0, f"ax: {bad.size} of {len(sample)} sampled bodies differ"
    assert bits_equal(ay[sample], ray)
    eng.close()
    ref.close()


def test_c4_1e7_full_size_sampled():
    """C4 at its full size (uniform cloud, N = 1e7, theta 0.5): 4097 sampled bodies."""
    _assert_sampled_evaluation(scenes.config_scene("c4"), 0.5, 2441)


def test_c3x8_8e6_weak_scaling_scene_sampled():
    """The 8-GPU weak-scaling scene (two disks, 8e6 bodies) on one GPU: 4000 sampled bodies."""
    _assert_sampled_evaluation(scenes.config_scene("c3x8"), 0.5, 2000)


def test_c5_full_size_theta0_sampled():
    """C5 at its full size (N = 262 144, theta = 0, all-pairs kernel): 1024 sampled bodies,
    each the exact direct sum over every leaf in pre-order."""
    _assert_sampled_evaluation(scenes.config_scene("c5"), 0.0, 256)


def test_deep_pairs_chunks_beyond_lds_capacity():
    """Close pairs (1e-2 apart: ~17 nested cells each) and jitter pairs (4e-4 apart) make the
    1024-body chunks need far more node slots than the LDS holds, so the fused emit/COM kernel
    (tree_build.hip k_emit_com) takes its global-memory path; 3 steps bit-identical."""
    rng = np.random.default_rng(31)
    npair = 3000
    cx = rng.uniform(100.0, 2300.0, npair)
    cy = rng.uniform(50.0, 750.0, npair)
    sep = np.where(rng.random(npair) < 0.1, 4e-4, 1e-2)
    ang = rng.uniform(0.0, 2 * np.pi, npair)
    x = np.concatenate([cx, cx + sep * np.cos(ang)])
    y = np.concatenate([cy, cy + sep * np.sin(ang)])
    m = rng.uniform(0.5, 2.0, 2 * npair)
    perm = rng.permutation(2 * npair)
    arrs = (x[perm], y[perm], np.zeros(2 * npair), np.zeros(2 * npair), m[perm])
    eng, ref = _pair(arrs, theta=0.5, merge_min_dist=0.0)
    _assert_acc_equal(eng, ref)
    eng.step(3)
    ref.step(3)
    _assert_state_equal(eng, ref)


def test_bucket_sort_collapse_oversized_buckets():
    """A cloud whose velocities aim every body at the centre: the first drift shrinks it 50x,
    the next one flings it out again, so the previous build's splitters (the adaptive bucket
    sort, tree_build.hip) put thousands of bodies into one bucket -- the global-memory bitonic
    fallback -- and many buckets stay empty.  Three steps, bit-identical to the oracle."""
    x, y, _, _, m = scenes.uniform(30_000, 0.5, seed=12)
    dt = 0.005
    vx = (1200.0 - x) / dt * 0.98
    vy = (400.0 - y) / dt * 0.98
    eng, ref = _pair((x, y, vx, vy, m), theta=0.5, merge_min_dist=0.0)
    for _ in range(3):
        eng.step(1)
        ref.step(1)
        _assert_state_equal(eng, ref)


def test_bucket_sort_steady_evolution_vs_fresh_sort():
    """The bucket sort (splitters from the previous build) and a fresh rocprim sort (a new
    engine on the same state) give identical trees: accelerations and visit counts agree."""
    arrs = scenes.config_scene("c1_code")
    a = bh_amd.Engine(bh_amd.default_params(theta=0.5))
    a.reset_bodies(*arrs)
    a.step(5)
    state = a.get_bodies()
    b = bh_amd.Engine(bh_amd.default_params(theta=0.5))
    b.reset_bodies(*state)
    ra = a.compute_accelerations(visits=True)
    rb = b.compute_accelerations(visits=True)
    for u, v in zip(ra, rb):
        assert bits_equal(np.asarray(u, dtype=np.float64), np.asarray(v, dtype=np.float64))


def test_c3x2_2e6_global_span_path():
    """2e6 bodies: more chunk boundaries than the LDS span pass holds, so the chunk-spanning
    nodes go through the global-memory variant (tree_build.hip k_com_span_global)."""
    arrs = scenes.config_scene("c3x2")
    assert len(arrs[0]) > (1024 << 10)
    eng, ref = _pair(arrs, theta=0.5)
    _assert_acc_equal(eng, ref)
    eng.step(1)
    ref.step(1)
    _assert_state_equal(eng, ref)


def test_physics_engine_mirror_preserves_body_identity():
    """The Kotlin-surface mirror (bh_amd.PhysicsEngine) driven like NBodyPanel: step() updates
    the caller's own Body objects in place and removes merged-away bodies from the caller's
    list (BHA:414-432, 519); survivors are the same objects the reference keeps."""
    from oracle import py_oracle
    bx = [1000.0, 1007.9, 1008.1, 1000.0, 1003.0, 1500.0, 1504.0, 1200.0]
    by = [400.0, 400.0, 400.0, 406.0, 403.0, 300.0, 300.0, 200.0]
    bm = [5000.0, 1.0, 1.0, 2.0, 4500.0, 10.0, 9000.0, 3.0]
    f = scenes.uniform(200, 0.5, seed=9)
    arrs = (np.concatenate([bx, f[0]]), np.concatenate([by, f[1]]), np.concatenate([np.zeros(8), f[2]]),
            np.concatenate([np.zeros(8), f[3]]), np.concatenate([bm, f[4]]))
    saved = bh_amd.Config.theta
    bh_amd.Config.theta = 0.5
    try:
        bodies = [bh_amd.Body(*(float(a[i]) for a in arrs)) for i in range(len(arrs[0]))]
        origin = {id(b): i for i, b in enumerate(bodies)}
        eng = bh_amd.PhysicsEngine(bodies)
        cfg = dict(G=80.0, dt=0.005, theta=0.5, soft2=1.0, width_px=2400, height_px=800,
                   merge_max_mass=4000.0, merge_min_dist=8.0)
        ref = py_oracle.make_engine(*arrs, cfg)
        ref_origin = {id(b): i for i, b in enumerate(ref.bodies)}
        for _ in range(15):
            eng.step()
            ref.step()
        assert eng.get_bodies() is bodies
        assert [origin[id(b)] for b in bodies] == [ref_origin[id(b)] for b in ref.bodies]
        assert len(bodies) < len(arrs[0])
        for b, r in zip(bodies, ref.bodies):
            assert (b.x, b.y, b.vx, b.vy, b.m) == (r.x, r.y, r.vx, r.vy, r.m)
        quads = []
        eng.get_tree_for_debug().visit_quads(lambda q: quads.append(q))
        assert quads[0] == bh_amd.Quad(1200.0, 400.0, 1202.0)
    finally:
        bh_amd.Config.theta = saved


def test_fast_math_sequences_exact():
    """The traversal's reduced sqrt / seeded-reciprocal sequences (traverse.hip) equal IEEE
    sqrt, 1.0/sqrt and 1.0/x bit-for-bit on 2^30 operands across the fast-path range."""
    assert bh_amd.selftest_fast_math(1 << 30, seed=20261015) == 0


def _theta0_mixed_scene():
    """Two disks plus coincident pairs (jitter), out-of-root, zero- and negative-mass bodies."""
    x, y, vx, vy, m = (a.copy() for a in scenes.two_disks(2500, 600))
    rng = np.random.default_rng(21)
    dup = rng.choice(len(x), 30, replace=False)
    ex = np.concatenate([x[dup], x[dup[:10]] + 3e-4, [-5.0, 2403.0, 700.0]])
    ey = np.concatenate([y[dup], y[dup[:10]] - 2e-4, [300.0, 100.0, 900.0]])
    em = np.concatenate([np.full(40, 1.0), [2.0, 2.0, 2.0]])
    x, y, m = np.concatenate([x, ex]), np.concatenate([y, ey]), np.concatenate([m, em])
    vx = np.concatenate([vx, np.zeros(len(ex))])
    vy = np.concatenate([vy, np.zeros(len(ex))])
    m[[7, 99]] = 0.0   # never visited as leaves; their own a = 0/0
    m[[13]] = -1.5     # visited, negative contribution
    perm = rng.permutation(len(x))
    return tuple(a[perm] for a in (x, y, vx, vy, m))


def test_theta0_direct_all_pairs():
    """theta = 0 runs the all-pairs kernel over the tree's leaf list (direct.hip): bit-identical
    to the oracle's tree walk (every leaf, pre-order), incl. jitter, out-of-root, zero and
    negative masses; then full steps through the same path."""
    arrs = _theta0_mixed_scene()
    eng, ref = _pair(arrs, theta=0.0, merge_min_dist=0.0)
    ax, ay = eng.compute_accelerations()        # no visit counts -> the direct kernel
    rax, ray = ref.accelerations()
    assert np.array_equal(ax, rax, equal_nan=True) and np.array_equal(ay, ray, equal_nan=True)
    fin = np.isfinite(rax)
    assert fin.sum() == len(rax) - 2
    assert bits_equal(ax[fin], rax[fin]) and bits_equal(ay[fin], ray[fin])
    _assert_state_equal(eng, ref, nan_ok=True)  # the jitter mutation
    eng2, ref2 = _pair(scenes.two_disks(3000, 700), theta=0.0)
    eng2.step(3)
    ref2.step(3)
    _assert_state_equal(eng2, ref2)


def test_theta0_direct_c5_sampled():
    """C5 geometry at 1/8 scale (uniform cloud, 32768 bodies): one theta = 0 evaluation, every
    body bit-identical to the oracle."""
    arrs = scenes.uniform(32_768, 0.5, seed=5)
    eng, ref = _pair(arrs, theta=0.0)
    ax, ay = eng.compute_accelerations()
    rax, ray = ref.accelerations()
    assert bits_equal(ax, rax) and bits_equal(ay, ray)


@pytest.mark.parametrize("let", ["0", "1"])
def test_rccl_path_single_rank(let, monkeypatch):
    """The multi-GPU evaluation path (shard range, in-place ncclAllGather of (ax, ay) over an
    RCCL communicator; with BH_LET=1 also the LET builds and the ncclAllGather of the cell
    tables) on one rank: bit-identical to the oracle, tree walk and theta = 0."""
    monkeypatch.setenv("BH_LET", let)
    uid = bh_amd.comm_unique_id()
    arrs = scenes.config_scene("c1_code")
    for theta in (0.5, 0.0):
        eng = bh_amd.Engine(bh_amd.default_params(theta=theta), device=0, rank=0, world=1,
                            unique_id=uid)
        eng.reset_bodies(*arrs)
        ref = oracle.Oracle(*arrs, theta=theta)
        eng.step(3)
        ref.step(3)
        _assert_state_equal(eng, ref)
        eng.close()
        ref.close()
        uid = bh_amd.comm_unique_id()


def _rel_err(got, want):
    g = np.stack([np.asarray(a, dtype=np.float64) for a in got])
    w = np.stack([np.asarray(a, dtype=np.float64) for a in want])
    return np.linalg.norm(g - w, axis=0) / np.maximum(np.linalg.norm(w, axis=0), 1e-30)


def test_nbody3d_fp32_accelerations_vs_fp64():
    """GPU.kt physics (fp32 3-D all-pairs, hardware rsqrt) against the float64 restatement of
    the shader (oracle/py_gpu3d.py): tolerance 1e-4 relative per body (median < 1e-6)."""
    from oracle import py_gpu3d
    arrs = py_gpu3d.sphere(4095)
    eng = bh_amd.NBody3D(device=0)
    eng.set(*arrs)
    got = eng.accelerations(G=80.0, softening=1.0)
    # the reference consumes float32 inputs: compare against fp64 math on the rounded inputs
    x, y, z = (np.float32(a).astype(np.float64) for a in arrs[:3])
    m = np.float32(arrs[6]).astype(np.float64)
    want = py_gpu3d.accelerations(x, y, z, m, G=80.0, softening=1.0)
    err = _rel_err(got, want)
    assert np.median(err) < 1e-6 and err.max() < 1e-4, (np.median(err), err.max())
    eng.close()


def test_nbody3d_fp32_steps_vs_fp64():
    """10 semi-implicit Euler steps (GPU.kt:145-146), double-buffered; positions within 1e-4
    relative of the float64 restatement."""
    from oracle import py_gpu3d
    arrs = [np.float32(a).astype(np.float64) for a in py_gpu3d.sphere(2047, seed=3)]
    eng = bh_amd.NBody3D(device=0)
    eng.set(*arrs)
    eng.step(10, dt=0.005, G=80.0, softening=1.0)
    got = eng.get()
    want = py_gpu3d.step(*arrs, k=10, dt=0.005, G=80.0, softening=1.0)
    perr = _rel_err(got[:3], want[:3])
    assert perr.max() < 1e-4, perr.max()
    assert np.array_equal(got[6], np.float32(want[6]))
    eng.close()


def test_c5_fp32_vs_fp64_tolerance_study():
    """C5 geometry (uniform cloud, z = 0) at 1/8 scale: fp32 all-pairs accelerations against the
    exact fp64 theta = 0 engine.  Bound: 1e-3 relative per body at the 99.9th percentile."""
    arrs = scenes.uniform(32_768, 0.5, seed=5)
    exact = bh_amd.Engine(bh_amd.default_params(theta=0.0), device=0)
    exact.reset_bodies(*arrs)
    ax, ay = exact.compute_accelerations()
    x, y, vx, vy, m = exact.get_bodies()  # after the build's jitter, the state the forces used
    eng = bh_amd.NBody3D(device=0)
    eng.set(x, y, np.zeros_like(x), vx, vy, np.zeros_like(x), m)
    fx, fy, fz = eng.accelerations(G=80.0, softening=1.0)
    err = _rel_err((fx, fy), (ax, ay))
    assert np.all(fz == 0.0)
    assert np.percentile(err, 99.9) < 1e-3, np.percentile(err, [50, 99, 99.9, 100])
    eng.close()


@pytest.mark.parametrize("let", ["default", "0"])
@pytest.mark.parametrize("world", [2, 3])
def test_multi_rank_decomposition_in_process(world, let, monkeypatch):
    """The multi-GPU step with `world` ranks on one GPU (bh_create_local: one host thread per
    rank, the in-place all-gather of every round emulated with device-to-device copies, RCCL
    being unable to host several ranks per device): every rank's state after 3 steps of a
    merge-active scene, and one theta = 0 evaluation, bit-identical to the oracle -- with the
    default builds (locally essential trees on every multi-rank engine) and with BH_LET=0
    (every build full and replicated, the accelerations all-gathered)."""
    import threading
    if let == "0":
        monkeypatch.setenv("BH_LET", "0")
    else:
        monkeypatch.delenv("BH_LET", raising=False)
    for theta in (0.5, 0.0):
        arrs = scenes.config_scene("c1_code")
        group = bh_amd.LocalGroup(world)
        engines = [bh_amd.Engine(bh_amd.default_params(theta=theta), device=0, rank=r,
                                 local_group=group) for r in range(world)]
        results, errors = [None] * world, []

        def run(r):
            try:
                engines[r].reset_bodies(*arrs)
                engines[r].step(3)
                results[r] = engines[r].get_bodies()
            except Exception as exc:  # surfaced below
                errors.append(exc)

        threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=120)
        assert not errors, errors
        assert not any(t.is_alive() for t in threads), "rank thread hung"
        ref = oracle.Oracle(*arrs, theta=theta)
        ref.step(3)
        want = ref.get_bodies()
        for r in range(world):
            for k, name in enumerate(FIELDS):
                assert bits_equal(results[r][k], want[k]), f"rank {r} theta {theta}: {name}"
        for e in engines:
            e.close()
        group.close()
        ref.close()


def _run_group(world, params, arrs, calls, quads=None):
    """Every rank of an in-process group: reset, then bh_step(k) for k in calls; states (and,
    with a list `quads`, every rank's getTreeForDebug quads appended to it)."""
    import threading
    group = bh_amd.LocalGroup(world)
    engines = [bh_amd.Engine(params, device=0, rank=r, local_group=group) for r in range(world)]
    results, stats, errors = [None] * world, [None] * world, []
    rank_quads = [None] * world

    def run(r):
        try:
            engines[r].reset_bodies(*arrs)
            for k in calls:
                engines[r].step(k)
            results[r] = engines[r].get_bodies()
            stats[r] = engines[r].let_stats()
            if quads is not None:
                rank_quads[r] = engines[r].get_quads()
                # the lazy lastTree leaves the state alone: still the same bodies after it
                again = engines[r].get_bodies()
                for a, b in zip(again, results[r]):
                    assert np.array_equal(a.view(np.int64), b.view(np.int64))
        except Exception as exc:  # surfaced below
            errors.append(exc)

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    assert not any(t.is_alive() for t in threads), "rank thread hung"
    for e in engines:
        e.close()
    group.close()
    if quads is not None:
        quads.extend(rank_quads)
    return results, stats


def _let_scene(name):
    if name == "c2":
        return scenes.config_scene("c2")
    if name == "disks":
        return scenes.two_disks(60_000, 15_000)
    if name == "cloud":
        return scenes.uniform(150_000, 0.5, seed=9)
    rng = np.random.default_rng(17)
    x, y, vx, vy, m = (a.copy() for a in scenes.uniform(40_000, 0.5, seed=13))
    if name == "jitter":  # coincident and < 1e-3 apart pairs: the build moves positions
        dup = rng.choice(len(x), 300, replace=False)
        near = rng.choice(len(x), 300, replace=False)
        ex = np.concatenate([x[dup], x[near] + 3e-4])
        ey = np.concatenate([y[dup], y[near] - 2e-4])
    else:  # "outside": bodies around and far outside the root cell walk the tree too
        ex = np.concatenate([rng.uniform(-900, -1, 60), rng.uniform(2403, 3500, 60),
                             rng.uniform(0, 2400, 60), [1e7, -1e7]])
        ey = np.concatenate([rng.uniform(-100, 900, 120), rng.uniform(-1500, -803, 60),
                             [5.0, 5.0]])
    k = len(ex)
    arrs = (np.concatenate([x, ex]), np.concatenate([y, ey]), np.concatenate([vx, np.zeros(k)]),
            np.concatenate([vy, np.zeros(k)]), np.concatenate([m, np.full(k, 0.5)]))
    perm = rng.permutation(len(arrs[0]))
    return tuple(a[perm] for a in arrs)


@pytest.mark.parametrize("world,scene,theta", [
    (2, "c2", 0.5), (4, "c2", 0.3), (8, "c2", 1.0), (3, "disks", 0.5), (8, "cloud", 0.5),
    (5, "cloud", 0.7), (4, "jitter", 0.5), (3, "outside", 0.5)])
def test_let_build_multi_rank_vs_single(world, scene, theta, monkeypatch):
    """The sharded build (let.hip): each rank builds only the cells its bodies can open plus the
    top from the exchanged cell values, and its forces -- hence every rank's state -- equal the
    single-GPU engine's bit for bit.  Two bh_step calls (the LET builds run in the middle of a
    call; the last build of a call is the full tree)."""
    monkeypatch.setenv("BH_LET", "1")  # LET builds at every world size (default: from 2 ranks)
    arrs = _let_scene(scene)
    params = bh_amd.default_params(theta=theta, merge_min_dist=0.0 if scene == "jitter" else 8.0)
    single = bh_amd.Engine(params, device=0)
    single.reset_bodies(*arrs)
    for k in (4, 3):
        single.step(k)
    want = single.get_bodies()
    want_quads = single.get_quads()  # lastTree (BHA:435): test_pipelined_call_equals_single_steps
    single.close()                   # ties it to the oracle's
    rank_quads = []
    got, stats = _run_group(world, params, arrs, (4, 3), quads=rank_quads)
    n = len(arrs[0])
    for r in range(world):
        # 8 + 6 builds: the first (caller order after the reset) is full, the other 13 are LET
        # builds (a call's last build too: lastTree is built on demand)
        assert stats[r]["let_builds"] == 13 and stats[r]["full_builds"] == 1, stats[r]
        assert len(rank_quads[r]) == len(want_quads), f"rank {r}: quads"
        for u, v in zip(rank_quads[r], want_quads):
            assert np.array_equal(np.asarray(u).view(np.int64), np.asarray(v).view(np.int64)), \
                f"rank {r}: lastTree quads"
        assert 0 < stats[r]["subset"] <= n and stats[r]["let_nodes"] > 0, stats[r]
        if scene == "cloud" and world == 8:  # the shard: a fraction of the bodies is built
            assert stats[r]["subset"] < n // 2, stats[r]
        for k, name in enumerate(FIELDS):
            assert bits_equal(got[r][k], want[k]), f"rank {r}: {name}"


def test_let_refresh_full_build_inside_a_call():
    """20 steps in one call = 40 builds: a full build sorts the caller's order, 32 LET builds,
    the refresh full build (the replicas' slot order), 6 more LET builds -- every rank's state
    equals the single-GPU engine's bit for bit."""
    arrs = scenes.uniform(120_000, 0.5, seed=41)
    params = bh_amd.default_params(theta=0.5)
    single = bh_amd.Engine(params, device=0)
    single.reset_bodies(*arrs)
    single.step(20)
    want = single.get_bodies()
    single.close()
    got, stats = _run_group(4, params, arrs, (20,))
    for r in range(4):
        assert stats[r]["let_builds"] == 38 and stats[r]["full_builds"] == 2, stats[r]
        for k, name in enumerate(FIELDS):
            assert bits_equal(got[r][k], want[k]), f"rank {r}: {name}"


def test_let_subset_overflow_replays_the_call():
    """The LET subset capacity follows the previous call's subsets (no host round trip per
    build): after a reset to a scene with 4x the bodies every rank's subset outgrows it, every
    rank sees the overflow through the exchange and the call is replayed -- the states still
    equal the single-GPU engine's bit for bit."""
    small = scenes.uniform(50_000, 0.5, seed=21)
    big = scenes.uniform(200_000, 0.5, seed=22)
    params = bh_amd.default_params(theta=0.5)
    single = bh_amd.Engine(params, device=0)
    single.reset_bodies(*small)
    single.step(3)
    single.reset_bodies(*big)
    single.step(3)
    want = single.get_bodies()
    single.close()
    import threading
    world = 4
    group = bh_amd.LocalGroup(world)
    engines = [bh_amd.Engine(params, device=0, rank=r, local_group=group) for r in range(world)]
    got, stats, errors = [None] * world, [None] * world, []

    def run(r):
        try:
            engines[r].reset_bodies(*small)
            engines[r].step(3)
            engines[r].reset_bodies(*big)
            engines[r].step(3)
            got[r] = engines[r].get_bodies()
            stats[r] = engines[r].let_stats()
        except Exception as exc:  # surfaced below
            errors.append(exc)

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    assert not any(t.is_alive() for t in threads), "rank thread hung"
    for e in engines:
        e.close()
    group.close()
    for r in range(world):
        assert stats[r]["overflows"] >= 1, stats[r]
        for k, name in enumerate(FIELDS):
            assert bits_equal(got[r][k], want[k]), f"rank {r}: {name}"


def _nonpositive_scene(kind):
    """A 120 000-body cloud with non-positive masses for the LET halo rule (let.hip
    let_include_gap2): the rule needs every cell's centre of mass inside its cell, which holds
    only because computeMass skips children of mass <= 0 (BHA:189-192) -- a cell of non-positive
    bodies becomes a mass-0 record that no walk visits (BHA:216).  "negative": 40 squares of
    3 .. 40 px whose bodies all have negative mass (both near and far from any rank's range),
    3 % negative singles, out-of-root bodies of both signs, two heavy bodies (merges active).
    "zero": as "negative" plus zero-mass bodies, whose a = 0/0 makes them NaN after the first
    kick (the reference's behaviour), so every later LET build selects every cell."""
    rng = np.random.default_rng(57 if kind == "negative" else 58)
    x, y, vx, vy, m = (a.copy() for a in scenes.uniform(120_000, 0.5, seed=56))
    for _ in range(40):
        cx, cy = rng.uniform(0, 2400), rng.uniform(0, 800)
        half = rng.uniform(1.5, 20.0)
        inside = (np.abs(x - cx) < half) & (np.abs(y - cy) < half)
        m[inside] = -rng.uniform(0.1, 0.9, inside.sum())
    singles = rng.choice(len(x), 3600, replace=False)
    m[singles] = -0.5
    if kind == "zero":
        m[rng.choice(len(x), 200, replace=False)] = 0.0
    ex = np.concatenate([rng.uniform(-600, -1, 40), rng.uniform(2405, 3000, 40), [1200.0, 800.0]])
    ey = np.concatenate([rng.uniform(-300, 1100, 80), [400.0, 200.0]])
    em = np.concatenate([np.where(rng.random(80) < 0.5, -0.7, 0.7), [6000.0, 5000.0]])
    k = len(ex)
    arrs = (np.concatenate([x, ex]), np.concatenate([y, ey]), np.concatenate([vx, np.zeros(k)]),
            np.concatenate([vy, np.zeros(k)]), np.concatenate([m, em]))
    perm = rng.permutation(len(arrs[0]))
    return tuple(a[perm] for a in arrs)


@pytest.mark.parametrize("theta", [0.0, 0.5, 1.0])
def test_massless_cells_of_negative_bodies_are_not_entered(theta):
    """Cells whose bodies all have negative mass get mass 0 (computeMass keeps children of mass
    > 0 only, BHA:189-192), and accumulateForce returns at mass == 0 (BHA:216): the negative
    bodies inside are never reached -- neither by the fast walk (the massless node is a
    skip-leaf) nor by the theta = 0 leaf list (leaves below a massless node are dropped).
    One evaluation and 3 steps, bit-identical to the oracle."""
    rng = np.random.default_rng(71)
    x, y, vx, vy, m = (a.copy() for a in scenes.uniform(30_000, 0.5, seed=70))
    for _ in range(25):
        cx, cy, half = rng.uniform(0, 2400), rng.uniform(0, 800), rng.uniform(2.0, 30.0)
        inside = (np.abs(x - cx) < half) & (np.abs(y - cy) < half)
        m[inside] = -rng.uniform(0.1, 0.9, inside.sum())
    arrs = (x, y, vx, vy, m)
    eng, ref = _pair(arrs, theta=theta)
    _assert_acc_equal(eng, ref)
    eng.step(3)
    ref.step(3)
    _assert_state_equal(eng, ref)


@pytest.mark.parametrize("world,kind", [(4, "negative"), (8, "negative"), (4, "zero")])
def test_let_nonpositive_masses(world, kind, monkeypatch):
    """The LET's halo rule with zero and negative masses: cells whose bodies are all negative
    (mass-0 records) inside and beyond the halo, negative singles and out-of-root bodies, merges
    active -- every rank of the group equals the single-GPU engine bit for bit, and the
    single-GPU engine equals the oracle (NaN payloads of the zero-mass bodies as "both NaN")."""
    monkeypatch.setenv("BH_LET", "1")
    arrs = _nonpositive_scene(kind)
    params = bh_amd.default_params(theta=0.5)
    single = bh_amd.Engine(params, device=0)
    single.reset_bodies(*arrs)
    ref = oracle.Oracle(*arrs, theta=0.5, threads=16)
    for k in (4, 3):
        single.step(k)
        ref.step(k)
    want = single.get_bodies()
    _assert_state_equal(single, ref, nan_ok=(kind == "zero"))
    single.close()
    ref.close()
    got, stats = _run_group(world, params, arrs, (4, 3))
    assert len(want[0]) < len(arrs[0])  # the heavy bodies merged
    for r in range(world):
        assert stats[r]["let_builds"] == 13 and stats[r]["full_builds"] == 1, stats[r]
        if kind == "negative":  # sharded: the halo rule ran, not the select-everything fallback
            assert stats[r]["subset"] < 0.75 * len(want[0]), stats[r]
        for k, name in enumerate(FIELDS):
            assert np.array_equal(got[r][k].view(np.int64), want[k].view(np.int64)), \
                f"rank {r}: {name}"


def test_let_guard_on_one_rank_replays_every_rank(monkeypatch):
    """A rank-local LET fault (k_let_guard tripped on rank 1 only, after the cell tables were
    exchanged: bh_debug_inject) is max-reduced over the ranks at the end of the call, so every
    rank replays it -- none hangs in an unmatched exchange -- and the states still equal the
    single-GPU engine's bit for bit."""
    import threading
    monkeypatch.setenv("BH_LET", "1")
    arrs = scenes.uniform(80_000, 0.5, seed=61)
    params = bh_amd.default_params(theta=0.5)
    single = bh_amd.Engine(params, device=0)
    single.reset_bodies(*arrs)
    single.step(3)
    single.step(2)
    want = single.get_bodies()
    single.close()
    world = 3
    group = bh_amd.LocalGroup(world)
    engines = [bh_amd.Engine(params, device=0, rank=r, local_group=group) for r in range(world)]
    got, stats, errors = [None] * world, [None] * world, []

    def run(r):
        try:
            engines[r].reset_bodies(*arrs)
            if r == 1:
                engines[r].debug_inject(1)
            engines[r].step(3)
            engines[r].step(2)
            got[r] = engines[r].get_bodies()
            stats[r] = engines[r].let_stats()
        except Exception as exc:  # surfaced below
            errors.append(exc)

    threads = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    assert not any(t.is_alive() for t in threads), "rank thread hung"
    for e in engines:
        e.close()
    group.close()
    for r in range(world):
        assert stats[r]["overflows"] == 1, stats[r]  # the same single replay on every rank
        for k, name in enumerate(FIELDS):
            assert bits_equal(got[r][k], want[k]), f"rank {r}: {name}"


def test_let_every_body_in_a_coincident_pair(monkeypatch):
    """Every body a coincident pair: each build moves every body (the h < 1e-3 jitter,
    BHA:146-151) -- on the rank that owns it and on every rank whose halo holds it; the owners'
    positions travel in the exchange and the states still equal the single-GPU engine's bit
    for bit."""
    monkeypatch.setenv("BH_LET", "1")
    base = scenes.uniform(30_000, 0.5, seed=31)
    rng = np.random.default_rng(32)
    perm = rng.permutation(2 * len(base[0]))
    arrs = tuple(np.concatenate([a, a])[perm] for a in base)
    params = bh_amd.default_params(theta=0.5, merge_min_dist=0.0)
    single = bh_amd.Engine(params, device=0)
    single.reset_bodies(*arrs)
    for k in (3, 2):
        single.step(k)
    want = single.get_bodies()
    single.close()
    got, stats = _run_group(2, params, arrs, (3, 2))
    for r in range(2):
        assert stats[r]["let_builds"] > 0, stats[r]
        for k, name in enumerate(FIELDS):
            assert bits_equal(got[r][k], want[k]), f"rank {r}: {name}"


def test_checkpoint_resume_bit_identical(tmp_path):
    """bh_save_state after 6 steps of a merge-active two-disk scene, bh_load_state into a fresh
    engine, 6 more steps: bit-identical to 12 uninterrupted steps and to the oracle; the file
    is readable by the host-side reader and holds the caller-order state and the params."""
    from bh_amd import state_file
    arrs = scenes.two_disks(3000, 800)
    p = bh_amd.default_params(theta=0.6, dt=0.004)
    straight = bh_amd.Engine(p, device=0)
    straight.reset_bodies(*arrs)
    straight.step(12)
    first = bh_amd.Engine(p, device=0)
    first.reset_bodies(*arrs)
    first.step(6)
    path = str(tmp_path / "mid.bhstate")
    first.save_state(path)
    params, saved = state_file.read(path)
    assert params["theta"] == 0.6 and params["dt"] == 0.004 and params["width_px"] == 2400
    for a, b in zip(saved, first.get_bodies()):
        assert bits_equal(a, b)
    first.close()
    resumed = bh_amd.Engine(bh_amd.default_params(), device=0)  # other params until loaded
    resumed.load_state(path)
    assert resumed.params.theta == 0.6
    resumed.step(6)
    for a, b in zip(resumed.get_bodies(), straight.get_bodies()):
        assert bits_equal(a, b)
    ref = oracle.Oracle(*arrs, theta=0.6, dt=0.004)
    ref.step(12)
    _assert_state_equal(resumed, ref)
    assert resumed.num_bodies() < len(arrs[0])  # the merge rule ran on both sides of the save
    with pytest.raises(bh_amd.BhError):
        resumed.load_state(str(tmp_path / "missing.bhstate"))


def test_profiling_timings_do_not_change_results():
    """bench.py's timed region: per-phase HIP events and per-launch traversal samples on, the
    same state as with them off, and every timing positive."""
    arrs = scenes.two_disks(4000, 1000)
    a = bh_amd.Engine(bh_amd.default_params(theta=0.5))
    a.reset_bodies(*arrs)
    a.set_profiling(True)
    a.step(4)
    t = a.last_timings()
    samples = a.traverse_kernel_samples()
    avg, launches = a.traverse_kernel_ms()
    assert t["build"] > 0 and t["traverse"] > 0
    # 8 evaluations; the deep pipeline of small lists (BH_DEEP_PIPE_MAX_N) also evaluates the
    # next call's a(t) beside the last step's second traversal: one more
    assert launches in (8, 9) and len(samples) == launches and np.all(samples > 0)
    assert abs(avg - samples.mean()) < 1e-9
    b = bh_amd.Engine(bh_amd.default_params(theta=0.5))
    b.reset_bodies(*arrs)
    b.step(4)
    for u, v in zip(a.get_bodies(), b.get_bodies()):
        assert bits_equal(u, v)


def test_pipelined_call_equals_single_steps():
    """One GPU, theta > 0: inside a bh_step(k) call every step but the last overlaps its second
    traversal with the merge rule and the next step's first build (engine.cpp, the pipelined
    step).  k = 20 in one call (lane-map re-sorts beside the first traversal, merges mid-call) against 20 calls of one
    step each (never pipelined): the same state bit for bit and the same last tree, both equal
    to the oracle's -- lastTree (BHA:435) is the last step's tree also when earlier steps of the
    call merged bodies (BHA:526 clears it only for the last step's merge)."""
    arrs = scenes.two_disks(30000, 6000)
    bx, by = np.array([900.0, 1500.0]), np.array([400.0, 420.0])
    arrs = (np.concatenate([arrs[0], bx]), np.concatenate([arrs[1], by]),
            np.concatenate([arrs[2], np.zeros(2)]), np.concatenate([arrs[3], np.zeros(2)]),
            np.concatenate([arrs[4], np.array([6000.0, 8000.0])]))
    p = bh_amd.default_params(theta=0.5)
    one = bh_amd.Engine(p)
    one.reset_bodies(*arrs)
    one.step(20)
    many = bh_amd.Engine(p)
    many.reset_bodies(*arrs)
    for _ in range(20):
        many.step(1)
    assert one.num_bodies() < len(arrs[0])  # the heavy bodies merged inside the call
    for u, v in zip(one.get_bodies(), many.get_bodies()):
        assert bits_equal(u, v)
    for u, v in zip(one.get_quads(), many.get_quads()):
        assert bits_equal(u, v)
    ref = oracle.Oracle(*arrs, theta=0.5)
    ref.step(20)
    _assert_state_equal(one, ref)
    for u, v in zip(one.get_quads(), ref.quads()):
        assert bits_equal(u, v)


def _frames_scene():
    """Two disks with two merging heavies, a 6-fold and a 4-fold stack of coincident bodies and
    20 bodies 3.6e-4 from a disk body: the jitter (BHA:146-151) moves bodies in most builds."""
    arrs = scenes.two_disks(30000, 6000)
    ex = np.concatenate([[900.0, 1500.0], np.full(6, 1234.5678), np.full(4, 700.25),
                         arrs[0][:20] + 3e-4])
    ey = np.concatenate([[400.0, 420.0], np.full(6, 321.0123), np.full(4, 500.5),
                         arrs[1][:20] - 2e-4])
    em = np.concatenate([[6000.0, 8000.0], np.ones(30)])
    z = np.zeros(len(ex))
    return tuple(np.concatenate([a, b]) for a, b in zip(arrs, (ex, ey, z, z, em)))


def _assert_arrays_equal(got, want, what):
    assert len(got[0]) == len(want[0]), f"{what}: N {len(got[0])} vs {len(want[0])}"
    for k, name in enumerate(FIELDS):
        bad = np.flatnonzero(np.asarray(got[k]).view(np.int64) != want[k].view(np.int64))
        assert bad.size == 0, f"{what} {name}: {bad.size} words differ, first at {bad[:5]}"


def test_one_step_calls_match_the_oracle_frame_by_frame():
    """The front-end's own pattern: one step() per frame (PNL:290-293), every body read after
    it (PNL:302-306), getTreeForDebug().visitQuads every few frames (PNL:333-340).  Every call's
    last step is pipelined: the call ends with the next step's first tree built (its jitter
    applied to the engine's copy of the state), while the caller sees the bodies as the reference
    holds them after step() -- through bh_get_bodies and through the pinned mirror the step fills
    itself (bh_map_bodies) -- and lastTree is the step's own tree (BHA:435), or, after a merge
    removed a body in the last step, the fresh tree of BHA:329-332.  Frame by frame bit-identical
    to the oracle, with merges and jitter along the way."""
    arrs = _frames_scene()
    p = bh_amd.default_params(theta=0.5)
    eng = bh_amd.Engine(p)
    eng.reset_bodies(*arrs)
    mir = bh_amd.Engine(p)
    mir.reset_bodies(*arrs)
    mir.set_mirror(True)
    ref = oracle.Oracle(*arrs, theta=0.5)
    quad_frames = {1, 2, 5, 9, 10, 14, 19, 23}
    for f in range(24):
        eng.step(1)
        mir.step(1)
        ref.step(1)
        want = ref.get_bodies()
        _assert_arrays_equal(mir.map_bodies(), want, f"frame {f} mirror")
        _assert_arrays_equal(eng.get_bodies(), want, f"frame {f}")
        if f in quad_frames:
            wq = ref.quads()
            for e in (eng, mir):
                for _ in range(2):  # the shim sizes, then fetches: the same tree twice
                    for u, v in zip(e.get_quads(), wq):
                        assert bits_equal(u, v), f"frame {f} quads"
            want = ref.get_bodies()  # a fresh tree jitters the bodies (BHA:146-151)
            _assert_arrays_equal(mir.map_bodies(), want, f"frame {f} mirror after quads")
            _assert_arrays_equal(eng.get_bodies(), want, f"frame {f} after quads")
    assert eng.num_bodies() < len(arrs[0])  # the heavies merged along the way


def test_double_buffered_mirror_views_survive_the_next_step():
    """bh_set_mirror(e, 2), the drop-in's mode: the views bh_map_bodies handed out stay valid
    and unchanged while the next step runs on another thread (ctypes releases the GIL) and
    after it, until the next map -- which holds the oracle's bodies after that step.  A merge
    and a jitter along the way; the caller's upload (reset) between steps too."""
    import threading
    arrs = _frames_scene()
    p = bh_amd.default_params(theta=0.5)
    mir = bh_amd.Engine(p)
    mir.reset_bodies(*arrs)
    mir.set_mirror(True, buffers=2)
    ref = oracle.Oracle(*arrs, theta=0.5)
    held = mir.map_bodies()
    for f in range(16):
        kept = [a.copy() for a in held]
        t = threading.Thread(target=mir.step, args=(1,))
        t.start()
        during = [a.copy() for a in held]  # read while the step runs
        t.join()
        ref.step(1)
        _assert_arrays_equal(during, kept, f"frame {f}: the held views during the step")
        _assert_arrays_equal(held, kept, f"frame {f}: the held views after the step")
        held = mir.map_bodies()
        _assert_arrays_equal(held, ref.get_bodies(), f"frame {f} mirror")
        if f == 7:  # the caller uploads its own list (an edit): the views again from the upload
            b = [a.copy() for a in held]
            b[2][3] += 1.0
            mir.reset_bodies(*b)
            ref = oracle.Oracle(*b, theta=0.5)
            held = mir.map_bodies()
            _assert_arrays_equal(held, ref.get_bodies(), "after the upload")
    assert mir.num_bodies() < len(arrs[0])  # the heavies merged along the way


def _async_call(eng, ref, k, what):
    """One bh_step_begin / bh_step_positions / bh_step_end call against the oracle's k steps:
    the mapped views unchanged during the call; positions and masses at the hand-off final;
    the survivors the complement of bh_last_removed; vx, vy final after the end."""
    held = eng.map_bodies()
    kept = [a.copy() for a in held]
    eng.step_begin(k)
    during = [a.copy() for a in held]
    x, y, m, sv, n0 = eng.step_positions()
    ref.step(k)
    want = ref.get_bodies()
    _assert_arrays_equal(during, kept, f"{what}: the held views during the call")
    assert n0 == len(kept[0]), what
    for got, w, name in ((x, want[0], "x"), (y, want[1], "y"), (m, want[4], "m")):
        assert len(got) == len(w) and bits_equal(got, w), f"{what}: {name} at the hand-off"
    sv = sv.copy()
    eng.step_end()
    removed = eng.last_removed()
    assert np.array_equal(np.setdiff1d(np.arange(n0), removed), sv), f"{what}: survivors"
    full = eng.map_bodies()
    _assert_arrays_equal(full, want, f"{what}: after the end")
    assert full[0].ctypes.data == x.ctypes.data, f"{what}: the hand-off's buffer"
    return len(removed)


def test_async_step_hands_over_positions_before_the_call_ends():
    """bh_step_begin / bh_step_positions / bh_step_end (the drop-in's frame): positions, masses
    and the survivors' list indices of the running call, before its last traversal, equal the
    oracle's after step() (BHA:405-439, 519) -- one-step and three-step calls over merges and
    jitter, a call replayed for a merge mailbox overflow (the hand-off is void, the end's
    mirror is handed over), and a call that fails (an injected tree flag) raising from both."""
    arrs = _frames_scene()
    p = bh_amd.default_params(theta=0.5)
    eng = bh_amd.Engine(p)
    eng.reset_bodies(*arrs)
    eng.set_mirror(True, buffers=2)
    ref = oracle.Oracle(*arrs, theta=0.5)
    merged = 0
    for f in range(12):
        merged += _async_call(eng, ref, 3 if f % 4 == 3 else 1, f"frame {f}")
    assert merged > 0
    eng.step_begin(1)  # the running call owns the engine: other calls are refused meanwhile
    for refused in (lambda: eng.step(1), eng.map_bodies, eng.get_bodies,
                    lambda: eng.step_begin(1)):
        with pytest.raises(bh_amd.BhError) as err:
            refused()
        assert err.value.rc == bh_amd.BH_E_STATE
    eng.step_end()
    ref.step(1)
    _assert_arrays_equal(eng.map_bodies(), ref.get_bodies(), "after the refused calls")
    with pytest.raises(bh_amd.BhError):  # no call begun
        eng.step_positions()
    # the crowd of heavies: the first step's candidate pairs overflow the mailbox (replay)
    rng = np.random.default_rng(77)
    nh = 520
    hx, hy = 1000.0 + 20.0 * rng.random(nh), 400.0 + 20.0 * rng.random(nh)
    field = scenes.uniform(3000, 0.5, seed=17)
    x, y = np.concatenate([hx, field[0]]), np.concatenate([hy, field[1]])
    mm = np.concatenate([rng.uniform(4001.0, 6000.0, nh), field[4]])
    crowd = (x, y, np.zeros(len(x)), np.zeros(len(x)), mm)
    eng.reset_bodies(*crowd)
    ref = oracle.Oracle(*crowd, theta=0.5)
    assert _async_call(eng, ref, 1, "overflowing call") > nh // 2
    _async_call(eng, ref, 1, "after the replay")
    eng.debug_inject(2)  # this call's own second build reports an unsupported geometry
    eng.step_begin(1)
    with pytest.raises(bh_amd.BhError) as err:
        eng.step_positions()
    assert err.value.rc == bh_amd.BH_E_STATE
    with pytest.raises(bh_amd.BhError):
        eng.step_end()
    ref.step(1)
    _assert_arrays_equal(eng.get_bodies(), ref.get_bodies(), "after the failed call")
    _async_call(eng, ref, 1, "after the failure")


def test_one_step_calls_then_reconfigure_checkpoint_and_evaluate(tmp_path):
    """What the caller may do between two pipelined calls, each against the oracle: a root-cell
    change (the prebuilt tree and its jitter belong to the old root and are dropped), a
    checkpoint (the caller-visible state, not the prebuilt one), buildTree + computeAccelerations
    (consumes the prebuilt tree), resetBodies, and a call that must be replayed from its snapshot
    (merge mailbox overflow) right after a pipelined one."""
    arrs = _frames_scene()
    eng, ref = _pair(arrs, theta=0.5)
    for _ in range(3):
        eng.step(1)
        ref.step(1)
    eng.set_params(bh_amd.default_params(theta=0.5, width_px=1920, height_px=1080))
    ref.set_params(oracle.params(theta=0.5, width_px=1920, height_px=1080))
    eng.step(1)
    ref.step(1)
    _assert_state_equal(eng, ref)
    eng.save_state(str(tmp_path / "s.bhs"))
    back = bh_amd.Engine(bh_amd.default_params())
    back.load_state(str(tmp_path / "s.bhs"))
    _assert_state_equal(back, ref)
    back.close()
    eng.step(1)
    ref.step(1)
    ax, ay = eng.compute_accelerations()
    rax, ray = ref.accelerations()
    assert bits_equal(ax, rax) and bits_equal(ay, ray)
    _assert_state_equal(eng, ref)
    eng.step(2)
    ref.step(2)
    _assert_state_equal(eng, ref)
    # a merge-free pipelined call, then the rule switched on: the next call overflows the
    # mailbox and is replayed from the caller-visible state
    rng = np.random.default_rng(77)
    nh = 520
    hx, hy = 1000.0 + 20.0 * rng.random(nh), 400.0 + 20.0 * rng.random(nh)
    field = scenes.uniform(3000, 0.5, seed=17)
    x, y = np.concatenate([hx, field[0]]), np.concatenate([hy, field[1]])
    m = np.concatenate([rng.uniform(4001.0, 6000.0, nh), field[4]])
    crowd = (x, y, np.zeros(len(x)), np.zeros(len(x)), m)
    off = dict(theta=0.5, merge_min_dist=0.0)
    eng.set_params(bh_amd.default_params(**off))
    ref.set_params(oracle.params(**off))
    eng.reset_bodies(*crowd)
    ref.reset_bodies(*crowd)
    eng.step(1)
    ref.step(1)
    eng.set_params(bh_amd.default_params(theta=0.5))
    ref.set_params(oracle.params(theta=0.5))
    eng.step(1)
    ref.step(1)
    _assert_state_equal(eng, ref)
    assert eng.num_bodies() < len(x) - nh // 2


def test_carried_tree_error_is_reported_by_the_call_that_uses_it():
    """A call's last step builds the next call's first tree beside its second traversal
    (BH_PIPE_LAST).  That build belongs to the next step() (BHA:407): an error flag it raises
    (injected here: bh_debug_inject(2 + k) flags the k-th next full build as the jitter replay's
    unsupported-geometry guard would) must fail the NEXT call, not the one that queued it -- and
    the call after that must check its own tree again.  The states stay the oracle's throughout
    (the injected flag does not change the tree)."""
    arrs = _frames_scene()
    eng, ref = _pair(arrs, theta=0.5)
    for _ in range(2):
        eng.step(1)
        ref.step(1)
    eng.debug_inject(3)  # build #0: this call's second build; #1: its last (carried) build
    eng.step(1)          # the carried tree's flag is not this call's
    ref.step(1)
    _assert_state_equal(eng, ref)
    with pytest.raises(bh_amd.BhError) as err:
        eng.step(1)      # this call's first step uses the flagged tree
    assert err.value.rc == bh_amd.BH_E_STATE
    ref.step(1)
    _assert_state_equal(eng, ref)
    eng.step(1)          # a clean tree again
    ref.step(1)
    _assert_state_equal(eng, ref)
    eng.debug_inject(2)  # the next build: this call's own second build
    with pytest.raises(bh_amd.BhError) as err:
        eng.step(1)
    assert err.value.rc == bh_amd.BH_E_STATE
    ref.step(1)
    _assert_state_equal(eng, ref)
    for _ in range(3):
        eng.step(1)
        ref.step(1)
    _assert_state_equal(eng, ref)
