"""Host-side check of the work-queue traversal's task mapping (traverse.hip k_traverse_q).

Each XCD x hands out tickets k = 0, 1, 2, ... from its own counter and maps them to the wave task
v = ((k // C) * 8 + x) * C + k % C (C = BH_TRAV_XCD_RUN): the runs of C waves that xcd_block gives
XCD x in the plain launch.  A wave stops at its XCD's first ticket past the last task, so the
mapping must be increasing in k for every x and, over all XCDs, hit every task exactly once.
"""
import pytest

C = 64  # BH_TRAV_XCD_RUN


def task(k, x):
    return ((k // C) * 8 + x) * C + k % C


@pytest.mark.parametrize("waves", [1, 7, 8, 63, 64, 65, 511, 512, 513, 4096, 15625, 15626])
def test_every_task_once(waves):
    seen = []
    for x in range(8):
        k, prev = 0, -1
        while True:
            v = task(k, x)
            assert v > prev  # increasing: the first ticket past the end ends the XCD's sequence
            prev = v
            if v >= waves:
                break
            seen.append(v)
            k += 1
    assert sorted(seen) == list(range(waves))


def test_runs_match_the_plain_launch_xcd():
    # the plain launch's xcd_block puts logical wave v on XCD (v // C) % 8 within full groups
    for x in range(8):
        for k in range(5 * C):
            assert (task(k, x) // C) % 8 == x
