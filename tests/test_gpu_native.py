"""The boundary exercised from native code (tests/c/, built by __graft_entry__.build()):

* abi_harness (C) performs the Kotlin drop-in's JNI call sequence (INTEGRATION.md §1:
  bh_set_params -> upload only when the caller's list changed -> bh_step(1) ->
  bh_last_removed applied once -> bh_get_bodies; bh_get_quads for getTreeForDebug) over
  NBodyPanel's frame sequence (PNL:103,247-262,282-291,333-340);
* mirror_harness (C++) drives bh::PhysicsEngine (csrc/physics_engine.hpp) the same way.

Both check every frame against the C restatement of the reference bit for bit, plus body
identity after merges and the quads of visitQuads (BHA:265-274, 329-332, 519)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(__file__), "c", "bin")


@pytest.mark.parametrize("exe", ["abi_harness", "mirror_harness"])
def test_native_harness(exe):
    path = os.path.join(BIN, exe)
    assert os.path.exists(path), f"{path} missing: run __graft_entry__.build()"
    r = subprocess.run([path], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bit-identical to the oracle" in r.stdout
    print(r.stdout.strip())
