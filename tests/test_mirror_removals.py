"""The PhysicsEngine mirrors' removal bookkeeping (BHA:519) on CPU: the list a step leaves."""


def test_python_mirror_removals_match_removeat():
    """bh_amd.PhysicsEngine applies a step's removals (BHA:519) to the caller's own list: one
    `del` per index for up to two, else one pass -- the same survivors, in the same order, the
    same objects and the same list object as the reference's descending removeAt calls."""
    import numpy as np
    import bh_amd

    class FakeEngine:  # the two calls _pull makes after a step (no GPU)
        def __init__(self, bodies, removed):
            keep = [b for i, b in enumerate(bodies) if i not in set(removed)]
            self.arrays = tuple(np.array([getattr(b, f) for b in keep], dtype=np.float64)
                                for f in ("x", "y", "vx", "vy", "m"))
            self.removed = np.array(removed, dtype=np.int64)

        def get_bodies(self):
            return self.arrays

        def last_removed(self):
            return self.removed

    for removed in ([], [3], [0, 9], [1, 4, 5, 9], list(range(0, 10, 2))):
        bodies = [bh_amd.Body(float(i), 2.0 * i, 0.0, 0.0, 1.0 + i) for i in range(10)]
        want = [b for i, b in enumerate(bodies) if i not in set(removed)]
        pe = bh_amd.PhysicsEngine.__new__(bh_amd.PhysicsEngine)
        pe._bodies = bodies
        pe._eng = FakeEngine(bodies, removed)
        pe._pull(after_step=True)
        assert pe._bodies is bodies and len(bodies) == len(want)
        assert all(a is b for a, b in zip(bodies, want)), removed
