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


@pytest.mark.parametrize("exe,devices", [("abi_harness", None), ("mirror_harness", None),
                                         ("abi_harness", "0,0,0"), ("mirror_harness", "0,0"),
                                         ("abi_harness", "chunked")])
def test_native_harness(exe, devices):
    """devices: the same frames through ONE engine handle over that device list (repeats: the
    members exchange by device-to-device copies) -- the Kotlin drop-in's Native.create with
    BH_DEVICES set, the C++ mirror's multi-device constructor.  "chunked": one device, the
    shim's compare/removal/unpack passes split over worker threads even for these short lists
    (at C3 they always are)."""
    path = os.path.join(BIN, exe)
    assert os.path.exists(path), f"{path} missing: run __graft_entry__.build()"
    env = dict(os.environ)
    args = [path]
    if devices == "chunked":
        env["BH_SHIM_PAR_MIN"], env["BH_SHIM_THREADS"] = "256", "7"
        devices = None
    if devices:
        env["BH_MULTI_MIN_BODIES"] = "0"  # the decomposition even for these small scenes
        if exe == "abi_harness":
            env["BH_DEVICES"] = devices
        else:
            args.append(devices)
    r = subprocess.run(args, capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bit-identical to the oracle" in r.stdout
    if devices:
        assert f"on {len(devices.split(','))} device(s)" in r.stdout, r.stdout
    if exe == "abi_harness":
        assert "0 shadow allocations after the constructor" in r.stdout, r.stdout
    print(r.stdout.strip())


def test_drop_in_frame_cost_at_c3():
    """The Kotlin drop-in's per-frame host work at C3 (1e6 bodies) beside the GPU step, through
    the real JNI glue: no allocation per frame, and the host side (in-place compare, getInto
    from the pinned mirror, unpack into the Body objects) reported in ms per frame."""
    import json
    path = os.path.join(BIN, "abi_harness")
    r = subprocess.run([path, "--c3-frames", "20"], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["bodies"] > 990_000 and line["allocations_per_frame"] == 0.0, line
    assert line["uploads"] == 0, line  # the caller never edited the bodies
    print(json.dumps(line))
