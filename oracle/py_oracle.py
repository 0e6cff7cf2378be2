"""ORACLE (second, independent restatement) — TEST INFRASTRUCTURE ONLY.

Pure-Python, object-per-node restatement of the reference hot path
(/root/reference/src/main/kotlin/BarnesHutAlg.kt = BHA), written from the Kotlin
source independently of oracle/bh_oracle.c so the two can cross-check each other
bit for bit.  Python floats are IEEE binary64 with correctly rounded + - * / and
math.sqrt, and CPython never fuses multiply-add: the JVM's strict semantics.

Only for small N (it is pure-Python loops).  PARITY UNPINNED: no reference output
exists to pin against (no JVM, no reference tests).
"""
from __future__ import annotations

import math
import struct


class Body:  # BHA:21-25
    __slots__ = ("x", "y", "vx", "vy", "m")

    def __init__(self, x, y, vx, vy, m):
        self.x, self.y, self.vx, self.vy, self.m = x, y, vx, vy, m


class Quad:  # BHA:53-82
    __slots__ = ("cx", "cy", "h")

    def __init__(self, cx, cy, h):
        self.cx, self.cy, self.h = cx, cy, h

    def contains(self, b):  # BHA:61-62
        return (b.x >= self.cx - self.h and b.x < self.cx + self.h
                and b.y >= self.cy - self.h and b.y < self.cy + self.h)

    def child(self, which):  # BHA:73-81
        hh = self.h / 2.0
        if which == 0:
            return Quad(self.cx - hh, self.cy - hh, hh)
        if which == 1:
            return Quad(self.cx + hh, self.cy - hh, hh)
        if which == 2:
            return Quad(self.cx - hh, self.cy + hh, hh)
        return Quad(self.cx + hh, self.cy + hh, hh)


def _lsb(v: float) -> int:
    return struct.unpack("<q", struct.pack("<d", v))[0] & 1


class BHTree:  # BHA:95-275
    __slots__ = ("quad", "body", "children", "mass", "comX", "comY")

    def __init__(self, quad):
        self.quad = quad
        self.body = None
        self.children = None
        self.mass = 0.0
        self.comX = 0.0
        self.comY = 0.0

    def is_leaf(self):
        return self.children is None

    def insert(self, b):  # BHA:125-137
        if not self.quad.contains(b):
            return
        if self.body is None and self.is_leaf():
            self.body = b
            return
        if self.is_leaf():
            self.children = [BHTree(self.quad.child(i)) for i in range(4)]  # BHA:159-166
        existing = self.body
        if existing is not None:
            self.body = None
            self._insert_into_child(existing)
        self._insert_into_child(b)

    def _insert_into_child(self, b):  # BHA:145-156
        if self.quad.h < 1e-3:
            eps = 1e-3
            b.x += (+eps) if _lsb(b.x) == 0 else (-eps)
            b.y += (-eps) if _lsb(b.y) == 0 else (+eps)
        ix = 0 if b.x < self.quad.cx else 1
        iy = 0 if b.y < self.quad.cy else 2
        self.children[ix + iy].insert(b)

    def compute_mass(self):  # BHA:173-202
        if self.is_leaf():
            if self.body is not None:
                self.mass, self.comX, self.comY = self.body.m, self.body.x, self.body.y
            else:
                self.mass, self.comX, self.comY = 0.0, self.quad.cx, self.quad.cy
            return
        m_sum = 0.0
        cx = 0.0
        cy = 0.0
        for c in self.children:
            c.compute_mass()
            if c.mass > 0.0:
                m_sum += c.mass
                cx += c.comX * c.mass
                cy += c.comY * c.mass
        self.mass = m_sum
        if m_sum > 0.0:
            self.comX = cx / m_sum
            self.comY = cy / m_sum
        else:
            self.comX = self.quad.cx
            self.comY = self.quad.cy

    def accumulate_force(self, b, theta2, acc, cfg):  # BHA:215-239
        if self.mass == 0.0:
            return
        acc[2] += 1
        if self.is_leaf():
            if self.body is None or self.body is b:
                return
            _point_force_acc(b, self.comX, self.comY, self.mass, acc, cfg)
            return
        dx = self.comX - b.x
        dy = self.comY - b.y
        dist2 = dx * dx + dy * dy + cfg["soft2"]
        s = self.quad.h * 2.0
        s2 = s * s
        if s2 < theta2 * dist2:
            _point_force_acc(b, self.comX, self.comY, self.mass, acc, cfg)
        else:
            for c in self.children:
                c.accumulate_force(b, theta2, acc, cfg)

    def visit_quads(self, visit):  # BHA:265-274
        visit(self.quad)
        if self.children is not None:
            for c in self.children:
                c.visit_quads(visit)


def _point_force_acc(b, px, py, m, acc, cfg):  # BHA:250-259
    dx = px - b.x
    dy = py - b.y
    r2 = dx * dx + dy * dy + cfg["soft2"]
    inv_r = 1.0 / math.sqrt(r2)
    inv_r2 = 1.0 / r2
    f = cfg["G"] * b.m * m * inv_r2
    acc[0] += f * dx * inv_r
    acc[1] += f * dy * inv_r


class PhysicsEngine:  # BHA:287-533
    def __init__(self, bodies, cfg):
        self.bodies = bodies
        self.cfg = dict(cfg)
        self.merge_max_mass = cfg.get("merge_max_mass", 4000.0)
        self.merge_min_dist = cfg.get("merge_min_dist", 8.0)
        self.last_tree = None
        self.visits = []

    def build_tree(self):  # BHA:359-366
        W, H = self.cfg["width_px"], self.cfg["height_px"]
        half = max(W, H) / 2.0 + 2.0
        root = BHTree(Quad(W / 2.0, H / 2.0, half))
        for b in self.bodies:
            root.insert(b)
        root.compute_mass()
        return root

    def compute_accelerations(self, root):  # BHA:374-395 (serial: results are order-free)
        theta2 = self.cfg["theta"] * self.cfg["theta"]
        ax, ay, vis = [], [], []
        for b in self.bodies:
            acc = [0.0, 0.0, 0]
            root.accumulate_force(b, theta2, acc, self.cfg)
            ax.append(acc[0] / b.m)
            ay.append(acc[1] / b.m)
            vis.append(acc[2])
        self.visits = vis
        return ax, ay

    def step(self):  # BHA:405-439
        root = self.build_tree()
        ax, ay = self.compute_accelerations(root)
        dt_half = self.cfg["dt"] * 0.5
        for i, b in enumerate(self.bodies):
            b.vx += ax[i] * dt_half
            b.vy += ay[i] * dt_half
        for b in self.bodies:
            b.x += b.vx * self.cfg["dt"]
            b.y += b.vy * self.cfg["dt"]
        root = self.build_tree()
        ax, ay = self.compute_accelerations(root)
        for i, b in enumerate(self.bodies):
            b.vx += ax[i] * dt_half
            b.vy += ay[i] * dt_half
        self.last_tree = root
        self.merge_close_bodies_if_needed()

    def merge_close_bodies_if_needed(self):  # BHA:463-532
        if self.merge_min_dist <= 0.0 or len(self.bodies) <= 1:
            return
        min_d2 = self.merge_min_dist * self.merge_min_dist
        i = 0
        while i < len(self.bodies):
            bi = self.bodies[i]
            if bi.m > self.merge_max_mass and len(self.bodies) > 1:
                victims = []
                for j, bj in enumerate(self.bodies):
                    if j != i:
                        dx = bj.x - bi.x
                        dy = bj.y - bi.y
                        if dx * dx + dy * dy < min_d2:
                            victims.append(j)
                if victims:
                    for j in sorted(victims, reverse=True):
                        bj = self.bodies[j]
                        if bj is bi:
                            continue
                        bi.m += bj.m
                        del self.bodies[j]
                    i = next(k for k, b in enumerate(self.bodies) if b is bi)
                    self.last_tree = None
            i += 1

    def get_tree_for_debug(self):  # BHA:329-332
        if self.last_tree is None:
            self.last_tree = self.build_tree()
        return self.last_tree


def make_engine(x, y, vx, vy, m, cfg):
    bodies = [Body(float(x[i]), float(y[i]), float(vx[i]), float(vy[i]), float(m[i]))
              for i in range(len(x))]
    return PhysicsEngine(bodies, cfg)


def state(engine):
    bs = engine.bodies
    return ([b.x for b in bs], [b.y for b in bs], [b.vx for b in bs], [b.vy for b in bs],
            [b.m for b in bs])
