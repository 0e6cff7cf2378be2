"""Morton (Z-order) body order over the 2400x800 root, the order of the GPU's slots before the
Hilbert wave grouping.  Analysis helper for the oracle's union-walk models (tools/)."""
import numpy as np


def morton_order(x, y, bits=21, width=2400.0, height=800.0):
    h = max(width, height) / 2.0 + 2.0          # root half-size (BHA:359-366)
    x0, y0 = width / 2.0 - h, height / 2.0 - h
    s = (1 << bits) / (2.0 * h)
    qx = np.clip(((np.asarray(x) - x0) * s).astype(np.int64), 0, (1 << bits) - 1)
    qy = np.clip(((np.asarray(y) - y0) * s).astype(np.int64), 0, (1 << bits) - 1)

    def spread(v):
        v = v.astype(np.uint64)
        out = np.zeros_like(v)
        for b in range(bits):
            out |= ((v >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b)
        return out

    key = spread(qx) | (spread(qy) << np.uint64(1))
    return np.argsort(key, kind="stable").astype(np.int64)
