"""Multi-rank decomposition on CPU (torch.distributed / gloo, world_size 2).

The engine's multi-GPU step (engine.cpp `evaluate`, bh_create_dist) keeps the state replicated,
builds the same tree on every rank and evaluates forces in BH_SHARD_ROUNDS rounds: in round k
a rank evaluates its Morton-sorted piece bh_shard_range(n, rank, world, k) (each rank owns one
contiguous range; the piece's slots in the buffer are bh_gather_slot), and the round's
interleaved (ax, ay) pieces are all-gathered in place (RCCL on the GPU box, overlapping the
next round) into the slot-indexed buffer, which is scattered back through the sort
permutation.  This test runs exactly that decomposition with gloo in place of RCCL and the
oracle in place of the HIP traversal, and requires the gathered result to be bit-identical to
a single-process evaluation.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def morton_order(x, y, W=2400, H=800):
    """Stable sort permutation by the engine's keys (exact descent, BHA:153-154, 360-361)."""
    cx0, cy0, h0 = W / 2.0, H / 2.0, max(W, H) / 2.0 + 2.0
    hs = [h0]
    while not hs[-1] < 1e-3:
        hs.append(hs[-1] / 2.0)
    J = len(hs) - 1
    hs.append(hs[-1] / 2.0)
    inside = (x >= cx0 - h0) & (x < cx0 + h0) & (y >= cy0 - h0) & (y < cy0 + h0)
    key = np.zeros(len(x), dtype=np.uint64)
    cx = np.full(len(x), cx0)
    cy = np.full(len(x), cy0)
    for d in range(J):
        ix = ~(x < cx)
        iy = ~(y < cy)
        hh = hs[d + 1]
        cx = np.where(ix, cx + hh, cx - hh)
        cy = np.where(iy, cy + hh, cy - hh)
        key = (key << np.uint64(2)) | (ix.astype(np.uint64) | (iy.astype(np.uint64) << np.uint64(1)))
    key = np.where(inside, key, np.uint64(1) << np.uint64(2 * J))
    return np.argsort(key, kind="stable")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "barnes-hut-n-body_amd")]
    import bh_amd
    import oracle
    from bh_amd import scenes

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    arrs = scenes.two_disks(700, 250)
    ref = oracle.Oracle(*arrs, theta=0.5, threads=1)
    x, y = arrs[0], arrs[1]
    perm = morton_order(x, y)
    n = len(x)
    sub = bh_amd.shard_range(n, 0, world, 0)[1]  # whole wavefronts per piece (engine.cpp)
    a2 = np.zeros(2 * sub * world * bh_amd.SHARD_ROUNDS)  # slot-indexed, interleaved
    for k in range(bh_amd.SHARD_ROUNDS):
        lo, hi = bh_amd.shard_range(n, rank, world, k)
        if hi > lo:
            ax, ay = ref.accelerations(subset=perm[lo:hi])  # this rank's piece of round k
            g = bh_amd.gather_slot(n, world, lo)  # the piece's slots in the exchange buffer
            a2[2 * g:2 * (g + hi - lo):2] = ax
            a2[2 * g + 1:2 * (g + hi - lo):2] = ay
        base = 2 * k * world * sub  # in place: rank r's piece sits at base + 2 * r * sub
        send = torch.from_numpy(a2[base + 2 * rank * sub:base + 2 * (rank + 1) * sub].copy())
        gathered = [torch.zeros(2 * sub, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(gathered, send)
        a2[base:base + 2 * world * sub] = torch.cat(gathered).numpy()
    slots = np.array([bh_amd.gather_slot(n, world, q) for q in range(n)])
    full_ax = np.empty(n)
    full_ay = np.empty(n)
    full_ax[perm] = a2[2 * slots]
    full_ay[perm] = a2[2 * slots + 1]
    np.save(os.path.join(out_dir, f"ax{rank}.npy"), full_ax)
    np.save(os.path.join(out_dir, f"ay{rank}.npy"), full_ay)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_evaluation_matches_single_process(tmp_path, world):
    import bh_amd  # noqa: F401  (library must load before spawning)
    import oracle
    from bh_amd import scenes

    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    arrs = scenes.two_disks(700, 250)
    ax, ay = oracle.Oracle(*arrs, theta=0.5, threads=1).accelerations()
    for r in range(world):
        gx = np.load(tmp_path / f"ax{r}.npy")
        gy = np.load(tmp_path / f"ay{r}.npy")
        assert np.array_equal(gx.view(np.int64), ax.view(np.int64)), f"rank {r} ax"
        assert np.array_equal(gy.view(np.int64), ay.view(np.int64)), f"rank {r} ay"


def test_morton_order_matches_tree_preorder():
    """The sort order used to shard is the tree's leaf pre-order (child 0..3 = ascending
    Morton digit, BHA:73-81): leaves appear in sorted order in visitQuads' walk."""
    from bh_amd import scenes
    x, y, *_ = scenes.uniform(64, 1.0, seed=2)
    perm = morton_order(x, y)
    # consecutive sorted bodies must never be "out of order" w.r.t. the first differing level
    cx0, cy0 = 1200.0, 400.0
    q = [(x[i] >= cx0) + 2 * (y[i] >= cy0) for i in perm]
    assert q == sorted(q)
