"""bh_amd — Python host binding of the MI355X Barnes–Hut engine (libbh_engine.so).

Everything here is plumbing over the C-ABI in include/bh_engine.h; the physics runs in the
HIP kernels of barnes-hut-n-body_amd/csrc.  There is no CPU fallback: if the shared
library is missing or no GPU is visible, the calls fail loudly.

Two layers:
  * `Engine` — 1:1 with the C-ABI, numpy SoA arrays in/out (used by bench.py and tests).
  * `PhysicsEngine`, `Body`, `Quad`, `Config` — a mirror of the reference's Kotlin surface
    (/root/reference/src/main/kotlin/BarnesHutAlg.kt = BHA, Config.kt = CFG) with the same
    names and call pattern NBodyPanel uses, so parity tests read like the reference's use.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from . import scenes  # noqa: F401  (re-export)

_HERE = os.path.dirname(os.path.abspath(__file__))
# BH_ENGINE_LIB selects another in-tree build of the library (A/B timing, tools/ab.sh)
LIB_PATH = os.environ.get("BH_ENGINE_LIB") or os.path.normpath(
    os.path.join(_HERE, "..", "lib", "libbh_engine.so"))

BH_OK = 0
BH_E_INVALID = -1
BH_E_DEVICE = -2
BH_E_COMM = -3
BH_E_CAPACITY = -4
BH_E_STATE = -5

EXPORTED_SYMBOLS = (
    "bh_default_params", "bh_create", "bh_create_dist", "bh_comm_unique_id", "bh_destroy",
    "bh_last_error", "bh_set_params", "bh_get_params", "bh_reset_bodies", "bh_step",
    "bh_num_bodies", "bh_get_bodies", "bh_compute_accelerations", "bh_get_quads",
    "bh_last_timings", "bh_last_tree_nodes", "bh_traverse_kernel_ms",
    "bh_traverse_kernel_samples", "bh_set_profiling",
    "bh_synchronize", "bh_shard_range", "bh_gather_slot", "bh_traversal_stats", "bh_traversal_counters", "bh_last_removed",
    "bh_selftest_fast_math", "bh_scene_galaxy_disk", "bh_scene_kepler_disk", "bh_scene_uniform",
    "bh_nbody3d_create", "bh_nbody3d_destroy", "bh_nbody3d_last_error", "bh_nbody3d_set",
    "bh_nbody3d_step", "bh_nbody3d_accelerations", "bh_nbody3d_get", "bh_nbody3d_last_ms",
    "bh_local_group_create", "bh_local_group_destroy", "bh_create_local",
    "bh_save_state", "bh_load_state", "bh_let_stats", "bh_create_solo", "bh_comm_ranks",
    "bh_debug_inject", "bh_set_mirror", "bh_map_bodies", "bh_create_multi",
    "bh_create_multi_list", "bh_multi_world", "bh_multi_member", "bh_collective_log",
    "bh_collective_log_clear", "bh_step_begin", "bh_step_positions", "bh_step_end",
    "bh_progress",
)


class BhParams(ctypes.Structure):
    """struct bh_params (include/bh_engine.h) — Config fields read by step()."""
    _fields_ = [
        ("G", ctypes.c_double),
        ("dt", ctypes.c_double),
        ("theta", ctypes.c_double),
        ("soft2", ctypes.c_double),
        ("width_px", ctypes.c_int32),
        ("height_px", ctypes.c_int32),
        ("merge_max_mass", ctypes.c_double),
        ("merge_min_dist", ctypes.c_double),
    ]


class BhError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__(f"bh_engine error {rc}: {msg}")
        self.rc = rc


_lib = None
_D = ctypes.POINTER(ctypes.c_double)
_I64P = ctypes.POINTER(ctypes.c_int64)
_VP = ctypes.c_void_p


def load_library(path: str | None = None):
    """Load libbh_engine.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise FileNotFoundError(
            f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    lib.bh_default_params.argtypes = [ctypes.POINTER(BhParams)]
    lib.bh_default_params.restype = None
    lib.bh_create.argtypes = [ctypes.POINTER(BhParams), ctypes.c_int, ctypes.POINTER(_VP)]
    lib.bh_create_dist.argtypes = [ctypes.POINTER(BhParams), ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(_VP)]
    lib.bh_comm_unique_id.argtypes = [ctypes.c_char_p]
    lib.bh_local_group_create.argtypes = [ctypes.c_int, ctypes.POINTER(_VP)]
    lib.bh_local_group_destroy.argtypes = [_VP]
    lib.bh_local_group_destroy.restype = None
    lib.bh_create_local.argtypes = [ctypes.POINTER(BhParams), ctypes.c_int, ctypes.c_int, _VP,
                                    ctypes.POINTER(_VP)]
    lib.bh_create_solo.argtypes = [ctypes.POINTER(BhParams), ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.POINTER(_VP)]
    lib.bh_create_multi.argtypes = [ctypes.POINTER(BhParams), ctypes.c_uint32, ctypes.POINTER(_VP)]
    lib.bh_create_multi_list.argtypes = [ctypes.POINTER(BhParams), ctypes.POINTER(ctypes.c_int32),
                                         ctypes.c_int32, ctypes.POINTER(_VP)]
    lib.bh_multi_world.argtypes = [_VP]
    lib.bh_multi_member.argtypes = [_VP, ctypes.c_int]
    lib.bh_multi_member.restype = _VP
    lib.bh_collective_log.argtypes = [_VP, _I64P, ctypes.c_int64, _I64P]
    lib.bh_collective_log_clear.argtypes = [_VP]
    lib.bh_destroy.argtypes = [_VP]
    lib.bh_destroy.restype = None
    lib.bh_last_error.argtypes = [_VP]
    lib.bh_last_error.restype = ctypes.c_char_p
    lib.bh_set_params.argtypes = [_VP, ctypes.POINTER(BhParams)]
    lib.bh_get_params.argtypes = [_VP, ctypes.POINTER(BhParams)]
    lib.bh_reset_bodies.argtypes = [_VP, ctypes.c_int64, _D, _D, _D, _D, _D]
    lib.bh_step.argtypes = [_VP, ctypes.c_int32]
    lib.bh_save_state.argtypes = [_VP, ctypes.c_char_p]
    lib.bh_load_state.argtypes = [_VP, ctypes.c_char_p]
    lib.bh_num_bodies.argtypes = [_VP]
    lib.bh_num_bodies.restype = ctypes.c_int64
    lib.bh_get_bodies.argtypes = [_VP, _D, _D, _D, _D, _D, ctypes.c_int64, _I64P]
    lib.bh_set_mirror.argtypes = [_VP, ctypes.c_int]
    _DPP = ctypes.POINTER(_D)
    lib.bh_map_bodies.argtypes = [_VP, _DPP, _DPP, _DPP, _DPP, _DPP, _I64P]
    lib.bh_step_begin.argtypes = [_VP, ctypes.c_int32]
    lib.bh_step_positions.argtypes = [_VP, _DPP, _DPP, _DPP,
                                      ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32)), _I64P, _I64P]
    lib.bh_step_end.argtypes = [_VP]
    lib.bh_compute_accelerations.argtypes = [_VP, _D, _D, _I64P]
    lib.bh_get_quads.argtypes = [_VP, _D, _D, _D, ctypes.c_int64, _I64P]
    lib.bh_last_timings.argtypes = [_VP, _D]
    lib.bh_last_tree_nodes.argtypes = [_VP]
    lib.bh_last_tree_nodes.restype = ctypes.c_int64
    lib.bh_traverse_kernel_ms.argtypes = [_VP, _D, _I64P]
    lib.bh_traverse_kernel_samples.argtypes = [_VP, _D, ctypes.c_int64, _I64P]
    lib.bh_set_profiling.argtypes = [_VP, ctypes.c_int]
    lib.bh_synchronize.argtypes = [_VP]
    lib.bh_traversal_stats.argtypes = [_VP, _I64P, _I64P, _I64P]
    lib.bh_traversal_counters.argtypes = [_VP, _I64P]
    lib.bh_let_stats.argtypes = [_VP, _I64P]
    lib.bh_comm_ranks.argtypes = [_VP, ctypes.POINTER(ctypes.c_int32),
                                  ctypes.POINTER(ctypes.c_int32)]
    lib.bh_debug_inject.argtypes = [_VP, ctypes.c_int]
    lib.bh_progress.argtypes = [_VP, _I64P]
    lib.bh_last_removed.argtypes = [_VP, _I64P, ctypes.c_int64, _I64P]
    lib.bh_shard_range.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   _I64P, _I64P]
    lib.bh_gather_slot.argtypes = [ctypes.c_int64, ctypes.c_int, ctypes.c_int64]
    lib.bh_gather_slot.restype = ctypes.c_int64
    lib.bh_selftest_fast_math.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, _I64P]
    _F = ctypes.POINTER(ctypes.c_float)
    lib.bh_nbody3d_create.argtypes = [ctypes.c_int, ctypes.POINTER(_VP)]
    lib.bh_nbody3d_destroy.argtypes = [_VP]
    lib.bh_nbody3d_destroy.restype = None
    lib.bh_nbody3d_last_error.argtypes = [_VP]
    lib.bh_nbody3d_last_error.restype = ctypes.c_char_p
    lib.bh_nbody3d_set.argtypes = [_VP, ctypes.c_int64] + [_F] * 7
    lib.bh_nbody3d_step.argtypes = [_VP, ctypes.c_int32, ctypes.c_float, ctypes.c_float,
                                    ctypes.c_float]
    lib.bh_nbody3d_accelerations.argtypes = [_VP, ctypes.c_float, ctypes.c_float, _F, _F, _F]
    lib.bh_nbody3d_get.argtypes = [_VP] + [_F] * 7 + [ctypes.c_int64, _I64P]
    lib.bh_nbody3d_last_ms.argtypes = [_VP]
    lib.bh_nbody3d_last_ms.restype = ctypes.c_double
    lib.bh_scene_galaxy_disk.argtypes = (
        [ctypes.c_int32] + [ctypes.c_double] * 6 + [ctypes.c_int32, ctypes.c_int64]
        + [ctypes.c_double] * 9 + [_D] * 5)
    lib.bh_scene_kepler_disk.argtypes = (
        [ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_double, ctypes.c_int64]
        + [ctypes.c_double] * 6 + [_D] * 5)
    lib.bh_scene_uniform.argtypes = [ctypes.c_int32, ctypes.c_double, ctypes.c_int64,
                                     ctypes.c_int32, ctypes.c_int32] + [_D] * 5
    if path is None:
        _lib = lib
    return lib


def _dp(a):
    return a.ctypes.data_as(_D) if a is not None else None


def default_params(**over) -> BhParams:
    p = BhParams()
    load_library().bh_default_params(ctypes.byref(p))
    for k, v in over.items():
        setattr(p, k, v)
    return p


SHARD_ROUNDS = 4  # BH_SHARD_ROUNDS (include/bh_engine.h)


def shard_range(n: int, rank: int, world: int, round: int = 0):
    """Lanes [lo, hi) (Hilbert wave order) whose forces `rank` evaluates in round `round` of a
    multi-GPU evaluation (bh_shard_range): rank r owns [(r * rounds) * sub, + rounds * sub), one
    contiguous region; the accelerations of lane q sit at gather_slot(n, world, q), where round
    k's pieces are adjacent, so round k's all-gather is in place."""
    lo = ctypes.c_int64(0)
    hi = ctypes.c_int64(0)
    rc = load_library().bh_shard_range(int(n), int(rank), int(world), int(round),
                                       ctypes.byref(lo), ctypes.byref(hi))
    if rc != BH_OK:
        raise BhError(rc, "bh_shard_range: invalid arguments")
    return lo.value, hi.value


def gather_slot(n: int, world: int, lane: int) -> int:
    """Slot of lane `lane` in the exchange buffer of a multi-GPU evaluation (bh_gather_slot)."""
    g = load_library().bh_gather_slot(int(n), int(world), int(lane))
    if g < 0:
        raise BhError(BH_E_INVALID, "bh_gather_slot: invalid arguments")
    return g


class NBody3D:
    """fp32 3-D all-pairs engine with the physics of the reference's OpenGL compute shader
    (gpu/GPU.kt:101-152: GpuNBody.simulate); see include/bh_engine.h bh_nbody3d_*."""

    def __init__(self, device: int = 0):
        self._lib = load_library()
        self._h = _VP()
        rc = self._lib.bh_nbody3d_create(int(device), ctypes.byref(self._h))
        if rc != BH_OK:
            raise BhError(rc, "bh_nbody3d_create failed")

    def _check(self, rc, what):
        if rc != BH_OK:
            raise BhError(rc, f"{what}: {self._lib.bh_nbody3d_last_error(self._h).decode()}")

    @staticmethod
    def _f(a):
        return np.ascontiguousarray(a, dtype=np.float32)

    def set(self, x, y, z, vx, vy, vz, m):
        arrs = [self._f(a) for a in (x, y, z, vx, vy, vz, m)]
        self._keep = arrs
        ptrs = [a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) for a in arrs]
        self._check(self._lib.bh_nbody3d_set(self._h, len(arrs[0]), *ptrs), "bh_nbody3d_set")
        self.n = len(arrs[0])

    def step(self, k: int = 1, dt: float = 0.005, G: float = 80.0, softening: float = 1.0):
        self._check(self._lib.bh_nbody3d_step(self._h, int(k), dt, G, softening),
                    "bh_nbody3d_step")

    def accelerations(self, G: float = 80.0, softening: float = 1.0):
        out = [np.empty(self.n, dtype=np.float32) for _ in range(3)]
        ptrs = [a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) for a in out]
        self._check(self._lib.bh_nbody3d_accelerations(self._h, G, softening, *ptrs),
                    "bh_nbody3d_accelerations")
        return tuple(out)

    def get(self):
        out = [np.empty(self.n, dtype=np.float32) for _ in range(7)]
        ptrs = [a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) for a in out]
        got = ctypes.c_int64(0)
        self._check(self._lib.bh_nbody3d_get(self._h, *ptrs, self.n, ctypes.byref(got)),
                    "bh_nbody3d_get")
        return tuple(out)

    def last_ms(self) -> float:
        return float(self._lib.bh_nbody3d_last_ms(self._h))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            self._lib.bh_nbody3d_destroy(self._h)
            self._h = _VP()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def selftest_fast_math(n: int, seed: int = 1, device: int = 0) -> int:
    """Mismatches of the traversal's exact in-range sqrt/reciprocal sequences against IEEE
    sqrt, 1/sqrt, 1/x over n generated operands (bh_selftest_fast_math); 0 expected."""
    bad = ctypes.c_int64(-1)
    rc = load_library().bh_selftest_fast_math(int(device), int(n), int(seed), ctypes.byref(bad))
    if rc != BH_OK:
        raise BhError(rc, "bh_selftest_fast_math failed")
    return bad.value


def comm_unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    rc = load_library().bh_comm_unique_id(buf)
    if rc != BH_OK:
        raise BhError(rc, "bh_comm_unique_id failed")
    return buf.raw


class LocalGroup:
    """In-process rank group (bh_local_group_*): the multi-GPU decomposition with device-to-
    device copies in place of RCCL, for `world` engines driven by one thread each."""

    def __init__(self, world: int):
        self._lib = load_library()
        self._h = _VP()
        rc = self._lib.bh_local_group_create(int(world), ctypes.byref(self._h))
        if rc != BH_OK:
            raise BhError(rc, "bh_local_group_create failed")
        self.world = world

    def close(self):  # after every member engine is closed
        if self._h:
            self._lib.bh_local_group_destroy(self._h)
            self._h = _VP()


class Engine:
    """The C-ABI, one call per method.  State lives in HBM; arrays are copied in/out."""

    def __init__(self, params: BhParams | None = None, device: int = 0, rank: int = 0,
                 world: int = 1, unique_id: bytes | None = None,
                 local_group: "LocalGroup | None" = None, solo: bool = False,
                 devices=None, device_mask: int | None = None):
        self._lib = load_library()
        self._h = _VP()
        self._owned = True
        self.params = params if params is not None else default_params()
        if devices is not None:  # one handle over these devices, repeats allowed (multi.cpp)
            arr = (ctypes.c_int32 * len(devices))(*[int(d) for d in devices])
            rc = self._lib.bh_create_multi_list(ctypes.byref(self.params), arr, len(devices),
                                                ctypes.byref(self._h))
            world = len(devices)
        elif device_mask is not None:  # one handle over every GPU of the mask (0: all)
            rc = self._lib.bh_create_multi(ctypes.byref(self.params), int(device_mask),
                                           ctypes.byref(self._h))
            world = None
        elif solo:  # measurement: one rank's share of a `world`-rank step, alone (bh_create_solo)
            rc = self._lib.bh_create_solo(ctypes.byref(self.params), device, rank, world,
                                          ctypes.byref(self._h))
        elif local_group is not None:
            world = local_group.world
            rc = self._lib.bh_create_local(ctypes.byref(self.params), device, rank,
                                           local_group._h, ctypes.byref(self._h))
        elif world > 1 or unique_id is not None:
            rc = self._lib.bh_create_dist(ctypes.byref(self.params), device, rank, world,
                                          unique_id, ctypes.byref(self._h))
        else:
            rc = self._lib.bh_create(ctypes.byref(self.params), device, ctypes.byref(self._h))
        if rc != BH_OK:
            raise BhError(rc, "engine creation failed (is a GPU visible?)")
        if world is None:
            world = int(self._lib.bh_multi_world(self._h))
        self.rank, self.world = rank, world

    def _check(self, rc):
        if rc != BH_OK:
            raise BhError(rc, self._lib.bh_last_error(self._h).decode())

    def close(self):
        if self._h and self._owned:
            self._lib.bh_destroy(self._h)
        self._h = _VP()

    # ---- multi-device handle ------------------------------------------------------------
    def multi_world(self) -> int:
        """Members of a bh_create_multi handle (1 for any other engine)."""
        return int(self._lib.bh_multi_world(self._h))

    def member(self, rank: int) -> "Engine":
        """Member `rank` of a multi-device handle, for diagnostics (a non-owning view: never
        step it alone -- its peers would wait for it)."""
        h = self._lib.bh_multi_member(self._h, int(rank))
        if not h:
            raise BhError(BH_E_INVALID, f"no member {rank}")
        m = Engine.__new__(Engine)
        m._lib, m._h, m._owned = self._lib, _VP(h), False
        m.params, m.rank, m.world = self.params, rank, self.world
        m._parent = self  # keeps the handle alive
        return m

    def collective_log(self):
        """(api call, site, bytes, stream) rows of every collective this engine issued
        (bh_collective_log)."""
        need = ctypes.c_int64(0)
        rc = self._lib.bh_collective_log(self._h, None, 0, ctypes.byref(need))
        if rc not in (BH_OK, BH_E_CAPACITY):
            self._check(rc)
        out = np.zeros((need.value, 4), dtype=np.int64)
        self._check(self._lib.bh_collective_log(self._h, out.ctypes.data_as(_I64P), need.value,
                                                ctypes.byref(need)))
        return out

    def collective_log_clear(self):
        self._check(self._lib.bh_collective_log_clear(self._h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_params(self, params: BhParams):
        self.params = params
        self._check(self._lib.bh_set_params(self._h, ctypes.byref(params)))

    def reset_bodies(self, x, y, vx, vy, m):
        arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (x, y, vx, vy, m)]
        n = len(arrs[0])
        if any(len(a) != n for a in arrs):
            raise ValueError("x, y, vx, vy, m must have equal lengths")
        self._check(self._lib.bh_reset_bodies(self._h, n, *[_dp(a) for a in arrs]))

    def step(self, k: int = 1):
        self._check(self._lib.bh_step(self._h, int(k)))

    def save_state(self, path: str):
        """Checkpoint: Config fields + bodies in caller order (bh_save_state)."""
        self._check(self._lib.bh_save_state(self._h, os.fsencode(path)))

    def load_state(self, path: str):
        """Resume from a bh_save_state file (params and bodies replaced)."""
        self._check(self._lib.bh_load_state(self._h, os.fsencode(path)))
        self.params = BhParams()
        self._check(self._lib.bh_get_params(self._h, ctypes.byref(self.params)))

    def num_bodies(self) -> int:
        return int(self._lib.bh_num_bodies(self._h))

    def get_bodies(self, out=None):
        """bh_get_bodies: (x, y, vx, vy, m) in caller order; `out` = five float64 arrays of at
        least N entries to fill (a caller that reuses its buffers), else new arrays."""
        n = max(self.num_bodies(), 0)  # (-1 while a call begun by step_begin runs: refused below)
        if out is None or any(len(a) < n or a.dtype != np.float64 for a in out):
            out = [np.empty(n, dtype=np.float64) for _ in range(5)]
        got = ctypes.c_int64(0)
        self._check(self._lib.bh_get_bodies(self._h, *[_dp(a) for a in out], n, ctypes.byref(got)))
        return tuple(a[: got.value] for a in out)

    def set_mirror(self, on: bool, buffers: int = 1):
        """bh_set_mirror: every step() call writes the pinned caller-order mirror itself;
        buffers=2: two of them, so map_bodies' views stay valid until the next map_bodies."""
        if buffers not in (1, 2):
            raise ValueError("buffers is 1 or 2")
        self._check(self._lib.bh_set_mirror(self._h, buffers if on else 0))

    def map_bodies(self):
        """bh_map_bodies: read-only numpy views of the pinned mirror (x, y, vx, vy, m), valid
        until the next call that changes the bodies -- copy them to keep them."""
        ptrs = [_D() for _ in range(5)]
        n = ctypes.c_int64(0)
        self._check(self._lib.bh_map_bodies(self._h, *[ctypes.byref(p) for p in ptrs],
                                            ctypes.byref(n)))
        out = []
        for p in ptrs:
            a = np.ctypeslib.as_array(p, shape=(n.value,)) if n.value else np.empty(0)
            a.flags.writeable = False
            out.append(a)
        return tuple(out)

    def step_begin(self, k: int = 1):
        """bh_step_begin: the call runs on the engine's own thread (set_mirror(True, buffers=2))."""
        self._check(self._lib.bh_step_begin(self._h, int(k)))

    def step_positions(self):
        """bh_step_positions: (x, y, m, survivors, n_before) of the running call -- read-only
        views of the mirror buffer it writes (x, y, m final) and survivor j's index in the
        list before the call."""
        ptrs = [_D() for _ in range(3)]
        sv = ctypes.POINTER(ctypes.c_uint32)()
        n, n0 = ctypes.c_int64(0), ctypes.c_int64(0)
        self._check(self._lib.bh_step_positions(self._h, *[ctypes.byref(p) for p in ptrs],
                                                ctypes.byref(sv), ctypes.byref(n), ctypes.byref(n0)))
        out = [np.ctypeslib.as_array(p, shape=(n.value,)) if n.value else np.empty(0)
               for p in ptrs]
        out.append(np.ctypeslib.as_array(sv, shape=(n.value,)) if n.value
                   else np.empty(0, dtype=np.uint32))
        for a in out:
            a.flags.writeable = False
        return (*out, n0.value)

    def step_end(self):
        """bh_step_end: joins the call begun by step_begin; raises its error."""
        self._check(self._lib.bh_step_end(self._h))

    def compute_accelerations(self, visits: bool = False):
        n = self.num_bodies()
        ax = np.empty(n, dtype=np.float64)
        ay = np.empty(n, dtype=np.float64)
        vis = np.empty(n, dtype=np.int64) if visits else None
        self._check(self._lib.bh_compute_accelerations(
            self._h, _dp(ax), _dp(ay), vis.ctypes.data_as(_I64P) if visits else None))
        return (ax, ay, vis) if visits else (ax, ay)

    def last_removed(self):
        """Indices (list before the last step() call) removed by the merge rule, ascending."""
        need = ctypes.c_int64(0)
        rc = self._lib.bh_last_removed(self._h, None, 0, ctypes.byref(need))
        if rc not in (BH_OK, BH_E_CAPACITY):
            self._check(rc)
        out = np.empty(need.value, dtype=np.int64)
        self._check(self._lib.bh_last_removed(self._h, out.ctypes.data_as(_I64P), need.value,
                                              ctypes.byref(need)))
        return out

    def get_quads(self):
        need = ctypes.c_int64(0)
        rc = self._lib.bh_get_quads(self._h, None, None, None, 0, ctypes.byref(need))
        if rc not in (BH_OK, BH_E_CAPACITY):
            self._check(rc)
        n = need.value
        cx, cy, h = (np.empty(n, dtype=np.float64) for _ in range(3))
        self._check(self._lib.bh_get_quads(self._h, _dp(cx), _dp(cy), _dp(h), n, ctypes.byref(need)))
        return cx, cy, h

    def let_stats(self):
        """Multi-rank build sharding: LET builds, full builds, last subset size, last LET nodes."""
        out = np.zeros(5, dtype=np.int64)
        self._check(self._lib.bh_let_stats(self._h, out.ctypes.data_as(_I64P)))
        d = dict(zip(("let_builds", "full_builds", "subset", "let_nodes", "overflows"),
                     out.tolist()))
        return d

    def comm_ranks(self):
        """(ncclCommCount, ncclCommUserRank) of the engine's RCCL communicator; (0, rank) for
        an engine without one (bh_comm_ranks)."""
        c, r = ctypes.c_int32(0), ctypes.c_int32(0)
        self._check(self._lib.bh_comm_ranks(self._h, ctypes.byref(c), ctypes.byref(r)))
        return c.value, r.value

    def debug_inject(self, what: int = 1):
        """Test hook (bh_debug_inject): 1 = the next LET build of this rank trips its guard;
        2 + k = the k-th next full build raises its jitter flag; 100 + k / 200 + k = this rank
        fails host-side before its k-th next collective / group barrier."""
        self._check(self._lib.bh_debug_inject(self._h, int(what)))

    def progress(self):
        """bh_progress (any thread, also while a call runs): dict of api_calls, collectives,
        last_site, busy, failed, comm_aborted."""
        out = np.zeros(4, dtype=np.int64)
        self._check(self._lib.bh_progress(self._h, out.ctypes.data_as(_I64P)))
        f = int(out[3])
        return {"api_calls": int(out[0]), "collectives": int(out[1]), "last_site": int(out[2]),
                "busy": bool(f & 1), "failed": bool(f & 2), "comm_aborted": bool(f & 4)}

    def set_profiling(self, on: bool):
        self._check(self._lib.bh_set_profiling(self._h, 1 if on else 0))

    def last_timings(self):
        out = np.zeros(5, dtype=np.float64)
        self._check(self._lib.bh_last_timings(self._h, _dp(out)))
        return dict(zip(("build", "traverse", "integrate", "merge", "allgather"), out.tolist()))

    def traverse_kernel_ms(self):
        avg = ctypes.c_double(0.0)
        cnt = ctypes.c_int64(0)
        self._check(self._lib.bh_traverse_kernel_ms(self._h, ctypes.byref(avg), ctypes.byref(cnt)))
        return avg.value, cnt.value

    def traverse_kernel_samples(self):
        """Per-launch traversal kernel times (ms) of the last step() call, in launch order."""
        need = ctypes.c_int64(0)
        rc = self._lib.bh_traverse_kernel_samples(self._h, None, 0, ctypes.byref(need))
        if rc not in (BH_OK, BH_E_CAPACITY):
            self._check(rc)
        out = np.empty(need.value, dtype=np.float64)
        self._check(self._lib.bh_traverse_kernel_samples(self._h, _dp(out), need.value,
                                                         ctypes.byref(need)))
        return out

    def traversal_stats(self):
        """(lane visits, wave iterations, waves) of the last compute_accelerations(visits=True);
        lane efficiency = lane_visits / (64 * wave_iters)."""
        a, b, c = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
        self._check(self._lib.bh_traversal_stats(self._h, ctypes.byref(a), ctypes.byref(b),
                                                 ctypes.byref(c)))
        return a.value, b.value, c.value

    def traversal_counters(self):
        """Counters of the last compute_accelerations(visits=True) (bh_traversal_counters):
        dict of lane_visits, lane_contrib, wave_iters, wave_blocks, waves."""
        out = np.zeros(5, dtype=np.int64)
        self._check(self._lib.bh_traversal_counters(self._h, out.ctypes.data_as(_I64P)))
        return dict(zip(("lane_visits", "lane_contrib", "wave_iters", "wave_blocks", "waves"),
                        (int(v) for v in out)))

    def last_tree_nodes(self) -> int:
        return int(self._lib.bh_last_tree_nodes(self._h))

    def synchronize(self):
        self._check(self._lib.bh_synchronize(self._h))


# ---- mirror of the reference's Kotlin surface ----------------------------------------------

@dataclass
class Body:  # BHA:21-25
    x: float
    y: float
    vx: float
    vy: float
    m: float


@dataclass(frozen=True)
class Quad:  # BHA:53-82
    cx: float
    cy: float
    h: float

    def contains(self, b: Body) -> bool:  # BHA:61-62
        return (b.x >= self.cx - self.h and b.x < self.cx + self.h
                and b.y >= self.cy - self.h and b.y < self.cy + self.h)

    def child(self, which: int) -> "Quad":  # BHA:73-81
        hh = self.h / 2.0
        return Quad(self.cx + (hh if which & 1 else -hh), self.cy + (hh if which & 2 else -hh), hh)


class Config:  # CFG:2-39 — mutable globals read live by step()
    WIDTH_PX = 2400
    HEIGHT_PX = 800
    G = 80.0
    DT = 0.005
    SOFTENING = 1.0
    SOFT2 = 1.0 * 1.0
    theta = 0.30
    R = 100.0
    N = 5000
    CENTRAL_MASS = 50_000.0
    MIN_R = 8.0
    TOTAL_SATELLITE_MASS = 5_000.0


class BHTree:
    """getTreeForDebug() result: visitQuads (BHA:265-274) over a pre-order quad list."""

    def __init__(self, cx, cy, h):
        self._q = (cx, cy, h)

    def visit_quads(self, visit):
        cx, cy, h = self._q
        for i in range(len(cx)):
            visit(Quad(float(cx[i]), float(cy[i]), float(h[i])))

    visitQuads = visit_quads


class PhysicsEngine:
    """PhysicsEngine(initialBodies) (BHA:287) — writes results back into the same Body
    objects (BHA:414-432) and shrinks the caller's list on a merge (BHA:519)."""

    def __init__(self, initial_bodies: list, device: int = 0, devices=None):
        self._bodies = initial_bodies
        self.merge_max_mass = 4_000.0          # BHA:315
        self.merge_min_dist = Config.MIN_R     # BHA:321
        # devices: one handle over several GPUs (bh_create_multi_list), else one GPU
        self._eng = Engine(self._params(), device=device, devices=devices)
        self._push()

    def _params(self) -> BhParams:
        return default_params(G=Config.G, dt=Config.DT, theta=Config.theta, soft2=Config.SOFT2,
                              width_px=int(Config.WIDTH_PX), height_px=int(Config.HEIGHT_PX),
                              merge_max_mass=self.merge_max_mass,
                              merge_min_dist=self.merge_min_dist)

    def _soa(self):
        bs = self._bodies
        return np.array([[b.x, b.y, b.vx, b.vy, b.m] for b in bs], dtype=np.float64).reshape(-1, 5)

    def _push(self):
        soa = self._soa()
        self._eng.reset_bodies(*soa.T)
        self._shadow = soa

    def _changed(self) -> bool:
        """Whether the caller's bodies differ (bitwise) from what the engine holds; step()
        re-uploads only then, so the engine keeps its Morton-ordered state across frames."""
        soa = self._soa()
        return soa.shape != self._shadow.shape or not np.array_equal(
            soa.view(np.int64), self._shadow.view(np.int64))

    def _pull(self, after_step=False):
        x, y, vx, vy, m = self._eng.get_bodies()
        n = len(x)
        bs = self._bodies
        if after_step:
            rem = self._eng.last_removed()  # BHA:519 removeAt on the caller's list ...
            if len(rem) <= 2:
                for j in rem[::-1]:
                    del bs[int(j)]
            elif len(rem):  # ... as one pass: the same survivors, objects and list kept
                gone = set(int(j) for j in rem)
                bs[:] = [b for i, b in enumerate(bs) if i not in gone]
        if len(bs) != n:
            raise RuntimeError("engine and caller body lists diverged")
        for i in range(n):
            b = bs[i]
            b.x, b.y, b.vx, b.vy, b.m = float(x[i]), float(y[i]), float(vx[i]), float(vy[i]), float(m[i])
        self._shadow = np.stack([x, y, vx, vy, m], axis=1) if n else np.zeros((0, 5))

    def step(self):  # BHA:405-439
        self._eng.set_params(self._params())
        if self._changed():  # the caller edited bodies between frames
            self._push()
        self._eng.step(1)
        self._pull(after_step=True)

    def get_bodies(self):  # BHA:335
        return self._bodies

    def reset_bodies(self, new_bodies: list):  # BHA:342-349
        self._bodies = new_bodies
        self._push()

    def get_tree_for_debug(self) -> BHTree:  # BHA:329-332
        self._eng.set_params(self._params())
        cx, cy, h = self._eng.get_quads()
        self._pull()
        return BHTree(cx, cy, h)

    getBodies = get_bodies
    resetBodies = reset_bodies
    getTreeForDebug = get_tree_for_debug

    @property
    def engine(self) -> Engine:
        return self._eng
