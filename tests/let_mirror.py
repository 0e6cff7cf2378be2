"""TEST INFRASTRUCTURE: a CPU, multi-process mirror of the engine's multi-GPU exchange protocol.

One `MirrorRank` per process (torch.distributed / gloo in place of RCCL) runs PhysicsEngine.step()
(/root/reference/src/main/kotlin/BarnesHutAlg.kt = BHA, 405-439) the way `bh_create_dist`
engines do (engine.cpp evaluate / evaluate_let / sync_velocities, let.hip), with the pure-Python
tree of oracle/py_oracle.py in place of the HIP kernels:

  * state replicated on every rank, in the slot order of the last full build (Morton order);
    rank r owns the lanes [r R sub, (r + 1) R sub) (bh_shard_range, R = BH_SHARD_ROUNDS rounds);
  * a full evaluation (after a reset, every 32 LET builds, the last build of a call): every rank
    builds the whole tree (the jitter, BHA:146-151, moves every replica alike), evaluates its
    lanes, and the accelerations are all-gathered round by round in the bh_gather_slot layout;
    every rank then kicks (and drifts) every body;
  * a LET evaluation (every other one): the rank marks the depth-8 cells of its own bodies, adds
    the halo of cells its bodies may open (let_include_gap2), builds the tree of that subset only
    (insertion in caller order), all-gathers its own cells' (comX, comY, mass, count) tables,
    computes the top levels from all tables (computeMass, BHA:184-200), walks own bodies through
    top + local subtrees + remote cell records, kicks its OWN bodies (velocities stay with their
    owners) and all-gathers the new positions, 16 B per body, in the bh_gather_slot layout;
  * velocities are all-gathered (same rounds and slots) before the next full build and at the
    end of a call whose last evaluation was a LET one (every evaluation may be: the call's last
    build's full tree is built on demand by getTreeForDebug, engine.cpp lazy lastTree);
  * the merge rule (BHA:463-532) is replicated: removed bodies are tombstones until the end of
    the call, then every replica compacts;
  * at the end of every call with LET builds the ranks agree on the LET status (an all-reduce:
    engine.cpp agree_let_flags), and after every drifting LET evaluation they exchange their
    drift speed bound (the LET selection's displacement bound, engine.cpp gather_vmax) while the
    full build's slot-block boxes are valid.

Every collective is logged as the engine logs it (bh_collective_log: API call count, site,
bytes every rank receives), so the CPU protocol and the engine's recorded sequence compare
entry by entry (tests/test_dist_gloo.py, tests/test_gpu_multi.py).

The exchanged data is exactly what the engine exchanges, so a bit-identical final state on every
rank (tests/test_dist_gloo.py) shows that the protocol carries everything the reference's
serial step needs.  Only tests/ import this module.
"""
from __future__ import annotations

import math

import numpy as np

from oracle import py_oracle

LET_P = 8                    # depth of the exchanged cells (bh_device.hpp)
LET_CELLS = 1 << (2 * LET_P)
LET_REFRESH = 32             # LET builds between full builds (engine.cpp BH_LET_REFRESH)
LET_TSTRIDE = LET_CELLS + 1  # cell records + status record per exchanged table (bh_device.hpp)
LETCELL_BYTES = 32
# collective sites (engine.cpp CollSite)
COLL_ACC, COLL_POS, COLL_VEL, COLL_TABLE, COLL_FLAGS, COLL_VMAX = 1, 2, 3, 4, 5, 7


class Geometry:
    """Root cell (BHA:360-361) and the exact per-depth half sizes (BHA:74)."""

    def __init__(self, W, H):
        self.cx, self.cy = W / 2.0, H / 2.0
        self.h = [max(W, H) / 2.0 + 2.0]
        while not self.h[-1] < 1e-3:
            self.h.append(self.h[-1] / 2.0)
        self.J = len(self.h) - 1
        self.h += [self.h[-1] / 2.0, self.h[-1] / 4.0]

    def in_root(self, x, y):
        h = self.h[0]
        return (x >= self.cx - h) & (x < self.cx + h) & (y >= self.cy - h) & (y < self.cy + h)

    def keys(self, x, y, dead):
        """Morton keys by exact descent (the same x < cx compares as BHA:153-154); out of the
        root, non-finite or dead: the sentinel (after every real key)."""
        key = np.zeros(len(x), dtype=np.uint64)
        cx = np.full(len(x), self.cx)
        cy = np.full(len(x), self.cy)
        with np.errstate(invalid="ignore"):
            for d in range(self.J):
                ix = ~(x < cx)
                iy = ~(y < cy)
                hh = self.h[d + 1]
                cx = np.where(ix, cx + hh, cx - hh)
                cy = np.where(iy, cy + hh, cy - hh)
                key = (key << np.uint64(2)) | (ix.astype(np.uint64)
                                               | (iy.astype(np.uint64) << np.uint64(1)))
            ok = self.in_root(x, y) & ~dead
        return np.where(ok, key, np.uint64(1) << np.uint64(2 * self.J))

    def cell_of(self, x, y):
        """Depth-8 cell (interleaved column / row bits), of the projection onto the root for an
        outside point (let.hip cell_of / grid_col)."""
        w = 2.0 * self.h[LET_P]
        top = (1 << LET_P) - 1

        def col(p, o):
            q = min(max((p - o) * (1.0 / w), 0.0), float(top))
            c = int(q)
            if c > 0 and p < o + c * w:
                c -= 1
            elif c < top and p >= o + (c + 1) * w:
                c += 1
            return c

        c = col(x, self.cx - self.h[0])
        r = col(y, self.cy - self.h[0])
        out = 0
        for b in range(LET_P):
            out |= ((c >> b) & 1) << (2 * b) | ((r >> b) & 1) << (2 * b + 1)
        return out

    def cell_centre(self, i, d):
        cx, cy = self.cx, self.cy
        for lvl in range(d):
            digit = (i >> (2 * (d - 1 - lvl))) & 3
            hh = self.h[lvl + 1]
            cx = cx + hh if digit & 1 else cx - hh
            cy = cy + hh if digit & 2 else cy - hh
        return cx, cy

    def gap2(self, theta2, soft2):
        """let_include_gap2 (let.hip): the largest whole-cell gap at which a body of an own cell
        might still open a depth-8 cell; < 0 = no LET (replicated builds)."""
        if not theta2 > 0.0 or self.J <= LET_P + 1:
            return -1.0
        s = self.h[LET_P] * 2.0
        w, m = 2.0 * self.h[LET_P], 0.01
        q = s * s * (1.0 + 1e-6) / theta2 - soft2
        r = (m + math.sqrt(q if q > 0.0 else 0.0)) / w
        return -1.0 if r * r > 256.0 else r * r


def shard_layout(lib, n, world):
    """(sub, rounds) and the gather slot of every lane, from the engine library itself
    (bh_shard_range / bh_gather_slot -- host-only functions)."""
    import bh_amd
    sub = bh_amd.shard_range(n, 0, world, 0)[1]
    slots = np.array([bh_amd.gather_slot(n, world, q) for q in range(n)], dtype=np.int64)
    return sub, slots


class MirrorRank:
    def __init__(self, params: dict, rank: int, world: int, comm):
        self.p = dict(params)
        self.rank, self.world, self.comm = rank, world, comm
        self.geo = Geometry(params["width_px"], params["height_px"])
        self.stats = {"let": 0, "full": 0, "vel_syncs": 0, "max_subset": 0, "merged": 0}
        self.log = []        # (api call, site, bytes) per collective, as bh_collective_log
        self.api_calls = 0
        self.boxes_valid = False

    # ---- caller-facing API (bh_reset_bodies / bh_step / bh_get_bodies) --------------------
    def reset_bodies(self, x, y, vx, vy, m):
        self.x, self.y, self.vx, self.vy, self.m = (np.array(a, dtype=np.float64)
                                                     for a in (x, y, vx, vy, m))
        self.cidx = np.arange(len(self.x), dtype=np.int64)
        self.dead = np.zeros(len(self.x), dtype=bool)
        self.st_morton = False
        self.vel_stale = False
        self.let_age = 0
        self.boxes_valid = False
        self.api_calls += 1

    def step(self, k):
        self.api_calls += 1
        n0 = len(self.x)
        may_let = k > 0 and n0 > 0 and self.world >= 2 and self.p["theta"] != 0.0
        for s in range(k):
            self._evaluate("drift", allow_let=True)
            self._evaluate("kick", allow_let=True)  # (the last build's full tree: on demand)
            self._merge()
        if may_let:  # the end-of-call agreement on the LET status (max all-reduce)
            import torch
            flag = torch.zeros(2, dtype=torch.int64)
            self.comm.all_reduce(flag, op=torch.distributed.ReduceOp.MAX)
            self._log(COLL_FLAGS, 8)
        if k > 0:
            self._sync_velocities()  # every replica complete at the API boundary
        if bool(np.any(self.dead)):  # the compaction moves the slots: the engine recomputes
            # the selection's boxes from the positions at the call's end (finish_merges)
            self.boxes_valid = (self.world >= 2 and self.p["theta"] != 0.0
                                and int(np.count_nonzero(~self.dead)) > 0)
        keep = ~self.dead  # one compaction per call; caller indices renumbered in order
        order = np.argsort(self.cidx[keep], kind="stable")
        rank_of = np.empty(len(order), dtype=np.int64)
        rank_of[order] = np.arange(len(order))
        for f in ("x", "y", "vx", "vy", "m"):
            setattr(self, f, getattr(self, f)[keep])
        self.cidx = rank_of
        self.dead = np.zeros(len(self.x), dtype=bool)

    def get_bodies(self):
        order = np.argsort(self.cidx, kind="stable")
        return tuple(getattr(self, f)[order].copy() for f in ("x", "y", "vx", "vy", "m"))

    # ---- exchange helpers -------------------------------------------------------------------
    def _own_lanes(self, n, sub):
        R = _rounds()
        return range(min(n, self.rank * R * sub), min(n, (self.rank + 1) * R * sub))

    def _log(self, site, nbytes):
        self.log.append((self.api_calls, site, int(nbytes)))

    def _exchange(self, n, per_lane, site):
        """per_lane: {own lane q: (a, b)} -> (a, b) of every lane, through the engine's in-place
        round-by-round all-gather layout (gather slot of lane q)."""
        import torch
        sub, slots = shard_layout(None, n, self.world)
        R = _rounds()
        if sub > 0:
            for _ in range(R):
                self._log(site, 8 * 2 * sub * self.world)
        buf = np.zeros(2 * sub * self.world * R)
        for q, (a, b) in per_lane.items():
            buf[2 * slots[q]] = a
            buf[2 * slots[q] + 1] = b
        for k in range(R):  # round k: the pieces of all ranks are adjacent, rank r's at r * sub
            base = 2 * k * self.world * sub
            send = torch.from_numpy(buf[base + 2 * self.rank * sub:
                                        base + 2 * (self.rank + 1) * sub].copy())
            parts = [torch.zeros(2 * sub, dtype=torch.float64) for _ in range(self.world)]
            self.comm.all_gather(parts, send)
            buf[base:base + 2 * self.world * sub] = torch.cat(parts).numpy()
        return buf[2 * slots], buf[2 * slots + 1]

    # ---- one evaluation (engine.cpp evaluate) ----------------------------------------------
    def _evaluate(self, kick, allow_let):
        n = len(self.x)
        theta2 = self.p["theta"] * self.p["theta"]
        gap2 = self.geo.gap2(theta2, self.p["soft2"])
        if allow_let and self.st_morton and self.let_age < LET_REFRESH and gap2 >= 0.0:
            self._evaluate_let(kick, gap2)
            self.let_age += 1
            return
        self.let_age = 0
        self._sync_velocities()
        # full build, replicated: slots take the Morton order, then the reference's serial
        # insertion in list (caller) order moves jittered bodies in every replica alike
        order = np.argsort(self.geo.keys(self.x, self.y, self.dead), kind="stable")
        for f in ("x", "y", "vx", "vy", "m", "cidx", "dead"):
            setattr(self, f, getattr(self, f)[order])
        self.st_morton = True
        self.stats["full"] += 1
        bodies = [py_oracle.Body(float(self.x[i]), float(self.y[i]), 0.0, 0.0, float(self.m[i]))
                  for i in range(n)]
        root = self._tree([i for i in np.argsort(self.cidx, kind="stable") if not self.dead[i]],
                          bodies)
        for i, b in enumerate(bodies):
            self.x[i], self.y[i] = b.x, b.y
        sub, _ = shard_layout(None, n, self.world)
        acc = {}
        for q in self._own_lanes(n, sub):
            acc[q] = (0.0, 0.0) if self.dead[q] else self._force(root, bodies[q])
        ax, ay = self._exchange(n, acc, COLL_ACC)
        if theta2 != 0.0 and self.world >= 2 and n > 0:  # the selection's boxes (engine.cpp)
            self.boxes_valid = True
        dt_half = self.p["dt"] * 0.5  # BHA:412
        live = ~self.dead
        self.vx[live] += ax[live] * dt_half
        self.vy[live] += ay[live] * dt_half
        if kick == "drift":  # BHA:419-422
            self.x[live] += self.vx[live] * self.p["dt"]
            self.y[live] += self.vy[live] * self.p["dt"]

    def _tree(self, insert_order, bodies):
        g = self.geo
        root = py_oracle.BHTree(py_oracle.Quad(g.cx, g.cy, g.h[0]))
        for i in insert_order:  # BHA:363: list order
            root.insert(bodies[i])
        root.compute_mass()
        return root

    def _force(self, root, b):
        acc = [0.0, 0.0, 0]
        root.accumulate_force(b, self.p["theta"] * self.p["theta"], acc, self.p)
        return acc[0] / b.m, acc[1] / b.m  # BHA:390-391

    def _sync_velocities(self):
        """Owner velocities after LET evaluations, all-gathered before a full build permutes the
        replicas (engine.cpp sync_velocities)."""
        if not self.vel_stale:
            return
        self.vel_stale = False
        n = len(self.x)
        sub, _ = shard_layout(None, n, self.world)
        vx, vy = self._exchange(n, {q: (self.vx[q], self.vy[q]) for q in self._own_lanes(n, sub)},
                                COLL_VEL)
        self.vx[:], self.vy[:] = vx, vy
        self.stats["vel_syncs"] += 1

    # ---- the locally essential tree (let.hip) ------------------------------------------------
    def _evaluate_let(self, kick, gap2):
        import torch
        g = self.geo
        n = len(self.x)
        sub, _ = shard_layout(None, n, self.world)
        own = list(self._own_lanes(n, sub))
        own_set = set(own)
        ecell = np.zeros(LET_CELLS, dtype=bool)
        flag_all = False
        for q in own:  # k_let_mark
            if self.dead[q]:
                continue
            if not (math.isfinite(self.x[q]) and math.isfinite(self.y[q])):
                flag_all = True
            else:
                ecell[g.cell_of(self.x[q], self.y[q])] = True
        K = int(math.floor(math.sqrt(gap2))) + 1
        hcell = np.ones(LET_CELLS, dtype=bool) if flag_all else ecell.copy()
        if not flag_all:  # k_let_halo
            for c in np.flatnonzero(ecell):
                ix, iy = _compact(int(c)), _compact(int(c) >> 1)
                for dy in range(-K, K + 1):
                    for dx in range(-K, K + 1):
                        nx, ny = ix + dx, iy + dy
                        if not (0 <= nx < 256 and 0 <= ny < 256):
                            continue
                        gx, gy = max(abs(dx) - 1, 0), max(abs(dy) - 1, 0)
                        if gx * gx + gy * gy <= gap2:
                            hcell[_spread(nx) | (_spread(ny) << 1)] = True
        # k_let_flags: in-root live bodies of built cells, and own bodies that are not
        inside = g.in_root(self.x, self.y) & ~self.dead
        cells = [g.cell_of(self.x[i], self.y[i]) if inside[i] else -1 for i in range(n)]
        subset = [i for i in range(n) if (inside[i] and hcell[cells[i]])
                  or (not inside[i] and i in own_set)]
        self.stats["max_subset"] = max(self.stats["max_subset"], len(subset))
        pos = {i: (float(self.x[i]), float(self.y[i])) for i in subset}
        self.stats["let"] += 1
        # the subset's tree: insertion in caller order; jitter moves the subset's copies only
        bodies = {i: py_oracle.Body(pos[i][0], pos[i][1], 0.0, 0.0, float(self.m[i]))
                  for i in subset}
        inside = {i: bool(g.in_root(bodies[i].x, bodies[i].y)) and not self.dead[i]
                  for i in subset}
        cells = {i: g.cell_of(bodies[i].x, bodies[i].y) if inside[i] else -1 for i in subset}
        ins = sorted((i for i in subset if inside[i]), key=lambda i: self.cidx[i])
        root = self._tree(ins, bodies)
        members = {}
        for i in ins:
            members.setdefault(cells[i], []).append(i)
        # own cells' values (k_let_table): one body -> the body; two or more -> the depth-8 node
        table = np.zeros((LET_CELLS, 6))
        for c in np.flatnonzero(ecell):
            mem = members.get(int(c), [])
            if len(mem) == 1:
                b = bodies[mem[0]]
                table[c] = (b.x, b.y, b.m, 1, 1, self.cidx[mem[0]])
            elif len(mem) >= 2:
                nd = _depth8_node(root, int(c))
                table[c] = (nd.comX, nd.comY, nd.mass, 2, 1, -1)
            else:
                table[c] = (0.0, 0.0, 0.0, 0, 1, -1)
        parts = [torch.zeros(LET_CELLS * 6, dtype=torch.float64) for _ in range(self.world)]
        self.comm.all_gather(parts, torch.from_numpy(table.ravel().copy()))
        self._log(COLL_TABLE, LETCELL_BYTES * LET_TSTRIDE * self.world)
        tables = [t.numpy().reshape(LET_CELLS, 6) for t in parts]
        levels = self._top(tables)
        dt_half, dt = self.p["dt"] * 0.5, self.p["dt"]
        new_pos = {}
        for q in own:  # walk, then the owner's kick (traverse.hip KICK_OWN_DRIFT / KICK_OWN_ONLY)
            if self.dead[q]:
                new_pos[q] = (self.x[q], self.y[q])
                continue
            b = bodies[q]
            fx, fy = self._walk_let(levels, hcell, members, bodies, root, b, self.cidx[q])
            ax, ay = fx / b.m, fy / b.m
            self.vx[q] += ax * dt_half
            self.vy[q] += ay * dt_half
            if kick == "drift":
                new_pos[q] = (b.x + self.vx[q] * dt, b.y + self.vy[q] * dt)
            else:
                new_pos[q] = (b.x, b.y)  # as the build left it (jitter)
        x, y = self._exchange(n, new_pos, COLL_POS)  # 16 B per body: every replica's positions
        if kick == "drift" and self.boxes_valid:  # the drift's speed bound, every rank's
            vmax = torch.zeros(1, dtype=torch.float64)
            got = [torch.zeros(1, dtype=torch.float64) for _ in range(self.world)]
            self.comm.all_gather(got, vmax)
            self._log(COLL_VMAX, 8 * self.world)
        self.x[:], self.y[:] = x, y
        self.vel_stale = True

    def _top(self, tables):
        """Depth 8 from the first rank that provided each cell, then computeMass upwards in
        child order with the mass > 0 filter (let.hip k_let_top_hi / k_let_top_lo)."""
        lv = [None] * (LET_P + 1)
        t8 = np.zeros((LET_CELLS, 6))
        done = np.zeros(LET_CELLS, dtype=bool)
        for t in tables:
            take = (t[:, 4] == 1) & ~done
            t8[take] = t[take]
            done |= take
        lv[LET_P] = [(t8[c, 0], t8[c, 1], t8[c, 2], int(t8[c, 3]), int(t8[c, 5]))
                     for c in range(LET_CELLS)]
        for d in range(LET_P - 1, -1, -1):
            ch = lv[d + 1]
            cur = []
            for i in range(1 << (2 * d)):
                kids = ch[4 * i:4 * i + 4]
                total = sum(k[3] for k in kids)
                if total == 1:
                    cur.append(next(k for k in kids if k[3]))
                elif total >= 2:
                    ms = cx = cy = 0.0
                    for k in kids:
                        if k[2] > 0.0:  # BHA:189-192
                            ms += k[2]
                            cx += k[0] * k[2]
                            cy += k[1] * k[2]
                    if ms > 0.0:
                        cur.append((cx / ms, cy / ms, ms, 2, -1))
                    else:
                        ccx, ccy = self.geo.cell_centre(i, d)
                        cur.append((ccx, ccy, 0.0, 2, -1))
                else:
                    cur.append((0.0, 0.0, 0.0, 0, -1))
            lv[d] = cur
        return lv

    def _walk_let(self, lv, hcell, members, bodies, root, b, b_cidx):
        """accumulateForce (BHA:215-239) over the LET: top nodes, local depth-8 subtrees (the
        subset tree's own nodes), remote cells as childless records."""
        p = self.p
        theta2 = p["theta"] * p["theta"]
        acc = [0.0, 0.0, 0]

        def visit(d, i):
            comX, comY, mass, cnt, who = lv[d][i]
            if cnt == 0 or mass == 0.0:  # empty, or BHA:216
                return
            if cnt == 1:  # a leaf holding one body (BHA:217-221): identity by caller index
                if who != b_cidx:
                    py_oracle._point_force_acc(b, comX, comY, mass, acc, p)
                return
            if d == LET_P and hcell[i]:  # built here: the subtree of the reference's tree
                _depth8_node(root, i).accumulate_force(b, theta2, acc, p)
                return
            dx, dy = comX - b.x, comY - b.y
            dist2 = dx * dx + dy * dy + p["soft2"]
            s = self.geo.h[d] * 2.0
            if s * s < theta2 * dist2:  # BHA:226-228
                py_oracle._point_force_acc(b, comX, comY, mass, acc, p)
            elif d == LET_P:
                raise AssertionError(f"halo rule violated: a body opens remote cell {i}")
            else:
                for q in range(4):
                    visit(d + 1, 4 * i + q)

        visit(0, 0)
        return acc[0], acc[1]

    # ---- merge (BHA:463-532), replicated -----------------------------------------------------
    def _merge(self):
        md = self.p["merge_min_dist"]
        if md <= 0.0 or (~self.dead).sum() <= 1:
            return
        min_d2 = md * md
        order = np.argsort(self.cidx, kind="stable")  # list order
        for i in order:
            if self.dead[i] or not self.m[i] > self.p["merge_max_mass"]:
                continue
            live = np.flatnonzero(~self.dead)
            live = live[live != i]
            dx = self.x[live] - self.x[i]
            dy = self.y[live] - self.y[i]
            victims = live[dx * dx + dy * dy < min_d2]
            for j in sorted(victims, key=lambda j: -self.cidx[j]):  # descending list index
                self.m[i] += self.m[j]
                self.dead[j] = True
                self.stats["merged"] += 1


def _rounds():
    import bh_amd
    return bh_amd.SHARD_ROUNDS


def _spread(v):
    out = 0
    for b in range(LET_P):
        out |= ((v >> b) & 1) << (2 * b)
    return out


def _compact(v):
    out = 0
    for b in range(LET_P):
        out |= ((v >> (2 * b)) & 1) << b
    return out


def _depth8_node(root, c):
    nd = root
    for lvl in range(LET_P):
        nd = nd.children[(c >> (2 * (LET_P - 1 - lvl))) & 3]
    return nd
