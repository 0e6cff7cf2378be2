"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's OpenGL compute shader
(/root/reference/src/main/kotlin/gpu/GPU.kt) used as the checker of the fp32 3-D all-pairs
engine (bh_nbody3d_*).  Never imported by the product path.

PARITY UNPINNED: the reference shader needs an OpenGL 4.6 context (LWJGL, GPU.kt:1-60) that
does not exist here, and the reference ships no outputs of it; this restatement follows the
shader text line by line.  It computes in float64 (the truth the fp32 kernel is measured
against with a tolerance); the shader's inversesqrt is implementation-defined, so fp32 results
are not bit-reproducible across GPUs anyway.

  GPU.kt:127-143  acc = sum_{j != i} (G * m_j) * d * invR^3,  d = x_j - x_i,
                  dist2 = d.d + softening^2 (uSoftening = softening^2, GPU.kt:420)
  GPU.kt:145-146  v += acc * dt;  x += v * dt       (semi-implicit Euler)
The shader updates its buffer in place while other invocations read it (a race with no
defined result); the restatement is double-buffered, as SURVEY §8f specifies.
"""
import numpy as np


def accelerations(x, y, z, m, G=80.0, softening=1.0, block=2048):
    x, y, z, m = (np.asarray(a, dtype=np.float64) for a in (x, y, z, m))
    n = len(x)
    soft2 = float(softening) * float(softening)
    ax, ay, az = np.zeros(n), np.zeros(n), np.zeros(n)
    for i0 in range(0, n, block):
        i1 = min(n, i0 + block)
        dx = x[None, :] - x[i0:i1, None]  # other - position (GPU.kt:137)
        dy = y[None, :] - y[i0:i1, None]
        dz = z[None, :] - z[i0:i1, None]
        r2 = dx * dx + dy * dy + dz * dz + soft2  # GPU.kt:138
        inv = 1.0 / np.sqrt(r2)
        w = (G * m[None, :]) * inv * inv * inv  # (uG * other.w) * invR3 (GPU.kt:141)
        idx = np.arange(i0, i1)
        w[idx - i0, idx] = 0.0  # otherIndex == id -> continue (GPU.kt:134)
        ax[i0:i1] = (w * dx).sum(axis=1)
        ay[i0:i1] = (w * dy).sum(axis=1)
        az[i0:i1] = (w * dz).sum(axis=1)
    return ax, ay, az


def step(x, y, z, vx, vy, vz, m, k=1, dt=0.005, G=80.0, softening=1.0):
    x, y, z, vx, vy, vz, m = (np.array(a, dtype=np.float64) for a in (x, y, z, vx, vy, vz, m))
    for _ in range(k):
        ax, ay, az = accelerations(x, y, z, m, G, softening)
        vx += ax * dt  # GPU.kt:145
        vy += ay * dt
        vz += az * dt
        x += vx * dt  # GPU.kt:146
        y += vy * dt
        z += vz * dt
    return x, y, z, vx, vy, vz, m


def sphere(n, w=3440, h=1440, seed=1):
    """A spherical cloud of the shape of GPU.kt:generateSphere (GPU.kt:509-548), drawn with
    numpy's generator (Kotlin's Random(1) stream is not reproduced here) plus the central
    5e6 mass; velocities tangential with speed 300000 / max(10, r)."""
    rng = np.random.default_rng(seed)
    cx, cy, cz = w * 0.5, h * 0.5, min(w, h) * 0.5
    r_max = min(w, h) * 0.45
    r = r_max * np.cbrt(rng.random(n))
    zz = rng.random(n) * 2.0 - 1.0
    phi = rng.random(n) * 2.0 * np.pi
    s = np.sqrt(np.maximum(0.0, 1.0 - zz * zz))
    rx, ry, rz = s * np.cos(phi), s * np.sin(phi), zz
    speed = 300_000.0 / np.maximum(10.0, r)
    polar = np.abs(rz) > 0.99
    ax_, ay_ = np.where(polar, 1.0, 0.0), np.where(polar, 0.0, 1.0)
    tx, ty, tz = ry * 0.0 - rz * ay_, rz * ax_ - rx * 0.0, rx * ay_ - ry * ax_
    ln = np.maximum(np.sqrt(tx * tx + ty * ty + tz * tz), 1e-8)
    x = np.append(cx + r * rx, cx)
    y = np.append(cy + r * ry, cy)
    z = np.append(cz + r * rz, cz)
    vx = np.append(tx / ln * speed, 0.0)
    vy = np.append(ty / ln * speed, 0.0)
    vz = np.append(tz / ln * speed, 0.0)
    m = np.append(np.ones(n), 5_000_000.0)
    return x, y, z, vx, vy, vz, m
