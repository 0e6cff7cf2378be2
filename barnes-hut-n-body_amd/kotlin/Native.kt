// Native.kt -- the JNI natives of the drop-in PhysicsEngine (PhysicsEngine.kt), implemented by
// barnes-hut-n-body_amd/jni/bh_jni.c (Java_Native_*) over the C-ABI include/bh_engine.h.
// Build the library where a JDK exists:
//     make -C barnes-hut-n-body_amd jni JAVA_HOME=/path/to/jdk      -> lib/libbh_jni.so
// and run with -Djava.library.path=barnes-hut-n-body_amd/lib.
// tests/test_kotlin_dropin.py checks these declarations against bh_jni.c's exports.

import java.nio.ByteBuffer

object Native {
    init {
        System.loadLibrary("bh_jni")
    }

    /** One GPU, HIP device `device` (the default); the engine fills its pinned body mirror every
     *  step. */
    external fun create(device: Int): Long

    /** bh_create_multi over the HIP devices of `deviceMask` (bit d = device d, 0 = every visible
     *  GPU): opt-in -- the distinct-device RCCL path has not run on more than one GPU yet. */
    external fun createMask(deviceMask: Int): Long

    /** bh_set_params: Config.G/DT/theta/SOFT2/WIDTH_PX/HEIGHT_PX (CFG:5-23) + merge knobs. */
    external fun setParams(
        h: Long, G: Double, dt: Double, theta: Double, soft2: Double,
        w: Int, hgt: Int, mergeMaxMass: Double, mergeMinDist: Double
    )

    /** bh_reset_bodies from SoA [x..., y..., vx..., vy..., m...] of n bodies. */
    external fun reset(h: Long, n: Int, soa: DoubleArray)

    /** bh_step(k). */
    external fun step(h: Long, k: Int)

    /** bh_step_begin(k): the step runs on the engine's own thread (two-buffer mirror). */
    external fun stepBegin(h: Long, k: Int)

    /** The running step's hand-off (bh_step_positions): the mirror buffer it writes as a direct
     *  buffer (x, y, m final; vx, vy after stepEnd + map), info = [n, stride, n before]. */
    external fun positions(h: Long, info: LongArray): ByteBuffer

    /** The running step's survivors: int32 list indices before it, ascending (BHA:519). */
    external fun survivors(h: Long): ByteBuffer

    /** bh_step_end: joins the step begun by stepBegin; its error as an exception. */
    external fun stepEnd(h: Long)

    /** The bodies into the caller's SoA array [x[0..n) y[n..2n) vx vy m] from the engine's pinned
     *  mirror (bh_map_bodies), no allocation; returns n, or -n if soa holds fewer than 5 n. */
    external fun getInto(h: Long, soa: DoubleArray): Int

    /** The engine's pinned caller-order mirror itself as a direct buffer (five fp64 planes x, y,
     *  vx, vy, m at multiples of info[1] doubles; info[0] = n): nothing copied.  Valid and
     *  unchanged until the next map (two mirror buffers: a running step writes the other). */
    external fun map(h: Long, info: LongArray): ByteBuffer

    /** bh_get_quads as interleaved (cx, cy, h) triples in visitQuads order. */
    external fun quads(h: Long): DoubleArray

    /** bh_last_removed: list indices the last step() removed (BHA:519). */
    external fun lastRemoved(h: Long): IntArray
}
