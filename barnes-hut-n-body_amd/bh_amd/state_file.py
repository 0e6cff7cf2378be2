"""Reader / writer of the engine's on-disk state format (bh_save_state / bh_load_state, layout in
csrc/state_io.cpp): 80-byte little-endian header (magic "BHSTATE1", the uint32 size 64 of the
block from byte 16 to the body arrays, flags, bh_params, N) followed by x, y, vx, vy, m as fp64 arrays in the caller's list order.  Host-only
(numpy); used to inspect checkpoints and to build fixtures without a GPU."""
from __future__ import annotations

import struct

import numpy as np

MAGIC = b"BHSTATE1"
_HDR = struct.Struct("<8sII4dii2dq")  # 80 bytes
PARAM_FIELDS = ("G", "dt", "theta", "soft2", "width_px", "height_px", "merge_max_mass",
                "merge_min_dist")


def write(path, params: dict, x, y, vx, vy, m):
    arrs = [np.ascontiguousarray(a, dtype="<f8") for a in (x, y, vx, vy, m)]
    n = len(arrs[0])
    if any(len(a) != n for a in arrs):
        raise ValueError("x, y, vx, vy, m must have equal lengths")
    hdr = _HDR.pack(MAGIC, 64, 0, float(params["G"]), float(params["dt"]),
                    float(params["theta"]), float(params["soft2"]), int(params["width_px"]),
                    int(params["height_px"]), float(params["merge_max_mass"]),
                    float(params["merge_min_dist"]), n)
    with open(path, "wb") as fh:
        fh.write(hdr)
        for a in arrs:
            fh.write(a.tobytes())


def read(path):
    """(params dict, (x, y, vx, vy, m))"""
    with open(path, "rb") as fh:
        raw = fh.read()
    if len(raw) < _HDR.size:
        raise ValueError("truncated header")
    magic, hb, _flags, G, dt, theta, soft2, w, h, mm, md, n = _HDR.unpack_from(raw)
    if magic != MAGIC or hb != 64:
        raise ValueError("not a BHSTATE1 file")
    if n < 0 or len(raw) != _HDR.size + 40 * n:
        raise ValueError("body arrays do not match N")
    body = np.frombuffer(raw, dtype="<f8", offset=_HDR.size).reshape(5, n)
    params = dict(zip(PARAM_FIELDS, (G, dt, theta, soft2, w, h, mm, md)))
    return params, tuple(body[k].astype(np.float64) for k in range(5))
