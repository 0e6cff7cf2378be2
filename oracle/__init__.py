"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper of liboracle_bh.so, the C restatement of the reference's CPU hot path
(bh_oracle.c), plus the independent pure-Python restatement (py_oracle.py).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package, and only
as the checker / timed CPU baseline — never as part of the product path.

PARITY UNPINNED: the reference (Kotlin/JVM) has no tests or golden vectors and cannot run
in this image; see bh_oracle.c's header and DESIGN.md.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_bh.so")

_D = ctypes.POINTER(ctypes.c_double)
_I64P = ctypes.POINTER(ctypes.c_int64)


class OracleParams(ctypes.Structure):
    _fields_ = [
        ("G", ctypes.c_double),
        ("dt", ctypes.c_double),
        ("theta", ctypes.c_double),
        ("soft2", ctypes.c_double),
        ("width_px", ctypes.c_int32),
        ("height_px", ctypes.c_int32),
        ("merge_max_mass", ctypes.c_double),
        ("merge_min_dist", ctypes.c_double),
        ("threads", ctypes.c_int32),
        ("_pad", ctypes.c_int32),
    ]


_lib = None


def build():
    subprocess.run(["make", "-C", HERE, "-s"], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    lib.oracle_create.argtypes = [ctypes.POINTER(OracleParams), ctypes.c_int64] + [_D] * 5
    lib.oracle_create.restype = ctypes.c_void_p
    lib.oracle_set_params.argtypes = [ctypes.c_void_p, ctypes.POINTER(OracleParams)]
    lib.oracle_reset_bodies.argtypes = [ctypes.c_void_p, ctypes.c_int64] + [_D] * 5
    lib.oracle_num_bodies.argtypes = [ctypes.c_void_p]
    lib.oracle_num_bodies.restype = ctypes.c_int64
    lib.oracle_get_bodies.argtypes = [ctypes.c_void_p] + [_D] * 5
    lib.oracle_step.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.oracle_accel.argtypes = [ctypes.c_void_p, ctypes.c_int64, _I64P, _D, _D, _I64P]
    lib.oracle_quads.argtypes = [ctypes.c_void_p, _D, _D, _D, ctypes.c_int64]
    lib.oracle_quads.restype = ctypes.c_int64
    lib.oracle_tree_stats.argtypes = [ctypes.c_void_p, _I64P, _I64P]
    lib.oracle_last_timing.argtypes = [ctypes.c_void_p, _D, _D]
    lib.oracle_last_timing.restype = None
    lib.oracle_group_union.argtypes = [ctypes.c_void_p, _I64P, ctypes.c_int64, ctypes.c_int, _I64P,
                                       _I64P]
    lib.oracle_group_union.restype = ctypes.c_int64
    lib.oracle_union_force_stats.argtypes = [_I64P, _I64P]
    lib.oracle_union_force_stats.restype = None
    lib.oracle_deferred_model.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.oracle_deferred_model.restype = None
    lib.oracle_deferred_flushes.argtypes = []
    lib.oracle_deferred_flushes.restype = ctypes.c_int64
    lib.oracle_destroy.argtypes = [ctypes.c_void_p]
    _lib = lib
    return lib


def params(G=80.0, dt=0.005, theta=0.30, soft2=1.0, width_px=2400, height_px=800,
           merge_max_mass=4000.0, merge_min_dist=8.0, threads=0) -> OracleParams:
    return OracleParams(G, dt, theta, soft2, width_px, height_px, merge_max_mass, merge_min_dist,
                        threads, 0)


def _dp(a):
    return a.ctypes.data_as(_D)


class Oracle:
    """The reference PhysicsEngine, restated (BHA:287-532)."""

    def __init__(self, x, y, vx, vy, m, p: OracleParams | None = None, **kw):
        self._lib = load()
        self.p = p if p is not None else params(**kw)
        arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (x, y, vx, vy, m)]
        self._h = ctypes.c_void_p(self._lib.oracle_create(ctypes.byref(self.p), len(arrs[0]),
                                                          *[_dp(a) for a in arrs]))

    def close(self):
        if self._h:
            self._lib.oracle_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, p: OracleParams):
        self.p = p
        self._lib.oracle_set_params(self._h, ctypes.byref(p))

    def reset_bodies(self, x, y, vx, vy, m):
        arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (x, y, vx, vy, m)]
        self._lib.oracle_reset_bodies(self._h, len(arrs[0]), *[_dp(a) for a in arrs])

    def step(self, k=1):
        self._lib.oracle_step(self._h, int(k))

    def num_bodies(self):
        return int(self._lib.oracle_num_bodies(self._h))

    def get_bodies(self):
        n = self.num_bodies()
        out = [np.empty(n, dtype=np.float64) for _ in range(5)]
        self._lib.oracle_get_bodies(self._h, *[_dp(a) for a in out])
        return tuple(out)

    def accelerations(self, subset=None, visits=False):
        """buildTree + computeAccelerations on the current state (mutates via jitter)."""
        if subset is None:
            cnt = self.num_bodies()
            sp = None
        else:
            subset = np.ascontiguousarray(subset, dtype=np.int64)
            cnt = len(subset)
            sp = subset.ctypes.data_as(_I64P)
        ax = np.empty(cnt, dtype=np.float64)
        ay = np.empty(cnt, dtype=np.float64)
        vis = np.empty(cnt, dtype=np.int64)
        self._lib.oracle_accel(self._h, cnt, sp, _dp(ax), _dp(ay), vis.ctypes.data_as(_I64P))
        return (ax, ay, vis) if visits else (ax, ay)

    def last_timing(self):
        """(build seconds, walk seconds) of the last accelerations() call."""
        b, w = ctypes.c_double(0.0), ctypes.c_double(0.0)
        self._lib.oracle_last_timing(self._h, ctypes.byref(b), ctypes.byref(w))
        return b.value, w.value

    def quads(self):
        n = self._lib.oracle_quads(self._h, None, None, None, 0)
        cx, cy, h = (np.empty(n, dtype=np.float64) for _ in range(3))
        self._lib.oracle_quads(self._h, _dp(cx), _dp(cy), _dp(h), n)
        return cx, cy, h

    def group_union(self, order, group=64, per_group=False):
        """(wave iterations, lane visits[, per-group iterations]) of groups of `group`
        consecutive bodies of `order` (analysis helper, see bh_oracle.h)."""
        order = np.ascontiguousarray(order, dtype=np.int64)
        lv = ctypes.c_int64(0)
        pg = np.zeros((len(order) + group - 1) // group, dtype=np.int64)
        it = self._lib.oracle_group_union(self._h, order.ctypes.data_as(_I64P), len(order),
                                          int(group), ctypes.byref(lv), pg.ctypes.data_as(_I64P))
        return (it, lv.value, pg) if per_group else (it, lv.value)

    def union_force_stats(self):
        """(wave iterations with >= 1 contributing lane, contributions) of the last
        group_union (analysis helper)."""
        a, b = ctypes.c_int64(0), ctypes.c_int64(0)
        self._lib.oracle_union_force_stats(ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def deferred_flushes(self, order, q, t, group=64):
        """Force-block executions of the deferred-force model (per-lane FIFO of depth q,
        flushed when one is full or >= t lanes have work) for waves of `order`."""
        self._lib.oracle_deferred_model(int(q), int(t))
        try:
            self.group_union(order, group)
            return int(self._lib.oracle_deferred_flushes())
        finally:
            self._lib.oracle_deferred_model(0, 0)

    def tree_stats(self):
        a = ctypes.c_int64(0)
        b = ctypes.c_int64(0)
        self._lib.oracle_tree_stats(self._h, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value
