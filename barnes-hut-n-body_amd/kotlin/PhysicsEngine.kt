// PhysicsEngine.kt -- drop-in replacement of the reference's `class PhysicsEngine`
// (src/main/kotlin/BarnesHutAlg.kt:287-532, "BHA"), backed by the MI355X engine
// libbh_engine.so through the JNI natives of Native.kt (barnes-hut-n-body_amd/jni/bh_jni.c).
//
// Install (INTEGRATION.md §1): delete `class PhysicsEngine` (BHA:287-532) from BarnesHutAlg.kt
// -- Body, Acc, Quad and BHTree stay as they are -- and add this file and Native.kt to
// src/main/kotlin (default package).  NBodyPanel.kt compiles unchanged: it calls
// PhysicsEngine(list), step(), getBodies(), resetBodies(list) and
// getTreeForDebug().visitQuads { q -> ... } (NBodyPanel.kt:103,144,224-233,262,284-291,302,333).
//
// Same semantics as the reference: step() is one leapfrog KDK step with the merge rule
// (BHA:405-439), updating the caller's Body objects in place and removing merged bodies from the
// caller's list with the same removeAt calls (BHA:519), so every surviving Body keeps its
// identity; the quadtree jitter (BHA:146-151) moves bodies exactly as the reference does.

import java.nio.ByteOrder
import java.nio.DoubleBuffer
import java.nio.IntBuffer
import java.util.concurrent.atomic.AtomicBoolean
import kotlinx.coroutines.Dispatchers
import kotlinx.coroutines.launch
import kotlinx.coroutines.runBlocking

/** getTreeForDebug()'s result: the engine's quad list in visitQuads order (BHA:265-274). */
class QuadList(private val q: DoubleArray) {
    /** Pre-order over every cell (root, then children 0..3 recursively), as BHTree.visitQuads. */
    fun visitQuads(visit: (Quad) -> Unit) {
        var i = 0
        while (i + 2 < q.size) {
            visit(Quad(q[i], q[i + 1], q[i + 2]))
            i += 3
        }
    }
}

class PhysicsEngine(initialBodies: MutableList<Body>) {
    private var bodies: MutableList<Body> = initialBodies
    // One GPU (-Dbh.device, default 0); opt-in: -Dbh.deviceMask (bit d = HIP device d, 0 = every
    // visible GPU) -- bh_create_multi, one handle, every step fanned out over the GPUs and joined
    // (BHA:374-395).  (BH_DEVICES in the environment overrides either with a device list.)
    private val handle: Long = System.getProperty("bh.deviceMask")?.let { Native.createMask(Integer.decode(it)) }
        ?: Native.create(Integer.decode(System.getProperty("bh.device", "0")))
    // What the engine holds, read in place: its pinned caller-order mirror (Native.map, five
    // planes of `stride` doubles), mapped again after every native call that changes it; the
    // upload array is reused (grown only) -- no per-frame allocation that grows with N
    private val info = LongArray(2)
    private val info3 = LongArray(3)                        // Native.positions' [n, stride, n before]
    private var mirror: DoubleBuffer = DoubleBuffer.allocate(0)
    private var stride = 0
    private var mirrorN = -1
    private var upload = DoubleArray(0)
    private var spare = arrayOfNulls<Body>(0)                // the removal pass's (grown only)

    /** BHA:315 -- bodies heavier than this absorb neighbours closer than mergeMinDist. */
    var mergeMaxMass: Double = 4_000.0

    /** BHA:321 -- merge distance in pixels; <= 0 switches the merge rule off. */
    var mergeMinDist: Double = Config.MIN_R

    init {
        params()
        push()
    }

    /** BHA:335 */
    fun getBodies(): List<Body> = bodies

    /** BHA:342-349 */
    fun resetBodies(newBodies: MutableList<Body>) {
        bodies = newBodies
        push()
    }

    /** BHA:405-439: one step; Config is read live, as the reference reads it. */
    fun step() {
        params()
        if (bodies.size != mirrorN) {                        // the caller added or removed bodies
            push()
            Native.step(handle, 1)
            pull(afterStep = true)
            return
        }
        // The step runs on the engine's own thread (Native.stepBegin) while the caller's list is
        // compared against the mapped mirror -- the step writes the engine's other buffer
        // (Native.create's bh_set_mirror(e, 2)); an edited list is uploaded and stepped again,
        // the upload replacing that step's result
        Native.stepBegin(handle, 1)
        val edited = try {
            changed()
        } catch (t: Throwable) {
            runCatching { Native.stepEnd(handle) }
            throw t
        }
        if (edited) {
            // that step ran on the state before the edit: its result -- and an error it met, e.g.
            // on the tree the previous call left (whose flags it took over) -- is replaced
            runCatching { Native.stepEnd(handle) }
            push()
            Native.step(handle, 1)
            pull(afterStep = true)
            return
        }
        // The step's hand-off, once its merge rule is done and before its last traversal: the
        // survivors first, then positions and masses -- the removals (BHA:519) and the x, y, m
        // unpack run beside the traversal; after it only vx, vy are left
        var failed: Throwable? = null
        try {
            val ids = Native.survivors(handle).order(ByteOrder.nativeOrder()).asIntBuffer()
            val n = ids.capacity()
            if (n != bodies.size) keepSurvivors(ids, n)
            val a = Native.positions(handle, info3).order(ByteOrder.nativeOrder()).asDoubleBuffer()
            val s = info3[1].toInt()
            chunks(n) { lo, hi ->
                for (i in lo until hi) {
                    val b = bodies[i]
                    b.x = a.get(i); b.y = a.get(s + i); b.m = a.get(4 * s + i)
                }
            }
        } catch (t: Throwable) {
            failed = t
        }
        try {
            Native.stepEnd(handle)
        } catch (t: Throwable) {
            throw failed ?: t
        }
        failed?.let { throw it }
        val n = map()
        check(n == bodies.size) { "engine and caller body lists diverged" }
        val a = mirror
        val s = stride
        chunks(n) { lo, hi ->
            for (i in lo until hi) {
                val b = bodies[i]
                b.vx = a.get(2 * s + i); b.vy = a.get(3 * s + i)
            }
        }
    }

    /** The step's removals (BHA:519) from its survivors (ids[j] = survivor j's index before the
     *  step, ascending): the list the reference's removeAt calls leave, gathered in chunks into a
     *  reused spare array and set back -- the same list object, the same Body objects. */
    private fun keepSurvivors(ids: IntBuffer, n: Int) {
        if (spare.size < n) spare = arrayOfNulls(n)
        val out = spare
        chunks(n) { lo, hi -> for (j in lo until hi) out[j] = bodies[ids.get(j)] }
        chunks(n) { lo, hi -> for (j in lo until hi) bodies[j] = out[j]!! }
        bodies.subList(n, bodies.size).clear()
    }

    /** BHA:329-332: the last step's tree, or a fresh one (which may jitter bodies). */
    fun getTreeForDebug(): QuadList {
        params()
        val q = Native.quads(handle)                        // [cx0, cy0, h0, cx1, ...]
        pull(afterStep = false)
        return QuadList(q)
    }

    private fun params() = Native.setParams(
        handle, Config.G, Config.DT, Config.theta, Config.SOFT2,
        Config.WIDTH_PX, Config.HEIGHT_PX, mergeMaxMass, mergeMinDist
    )

    // The O(N) passes over the caller's bodies in chunks on Dispatchers.Default, joined -- the
    // reference's own fan-out (BHA:374-395, 408); short lists stay on the caller's thread
    private val workers = Runtime.getRuntime().availableProcessors().coerceIn(1, 16)

    private inline fun chunks(n: Int, crossinline body: (Int, Int) -> Unit) {
        if (n < 65_536 || workers == 1) { body(0, n); return }
        val parts = 4 * workers                             // a worker on a busy core takes fewer
        val per = (n + parts - 1) / parts
        runBlocking {
            for (w in 0 until parts) {
                val lo = w * per
                val hi = minOf(n, lo + per)
                if (lo < hi) launch(Dispatchers.Default) { body(lo, hi) }
            }
        }
    }

    /** Whether the caller's bodies differ (bitwise) from what the engine holds -- in place. */
    private fun changed(): Boolean {
        val n = bodies.size
        if (n != mirrorN) return true
        val a = mirror
        val s = stride
        val diff = AtomicBoolean(false)
        chunks(n) { lo, hi ->
            for (i in lo until hi) {
                val b = bodies[i]
                if (b.x.toRawBits() != a.get(i).toRawBits() ||
                    b.y.toRawBits() != a.get(s + i).toRawBits() ||
                    b.vx.toRawBits() != a.get(2 * s + i).toRawBits() ||
                    b.vy.toRawBits() != a.get(3 * s + i).toRawBits() ||
                    b.m.toRawBits() != a.get(4 * s + i).toRawBits()) { diff.set(true); break }
            }
        }
        return diff.get()
    }

    /** The engine's mirror, mapped after a native call that changed it; returns n. */
    private fun map(): Int {
        mirror = Native.map(handle, info).order(ByteOrder.nativeOrder()).asDoubleBuffer()
        stride = info[1].toInt()
        mirrorN = info[0].toInt()
        return mirrorN
    }

    private fun push() {
        val n = bodies.size
        if (upload.size < 5 * n) upload = DoubleArray(5 * n)
        val a = upload
        for ((i, b) in bodies.withIndex()) {
            a[i] = b.x; a[n + i] = b.y; a[2 * n + i] = b.vx; a[3 * n + i] = b.vy; a[4 * n + i] = b.m
        }
        Native.reset(handle, n, a)
        map()                                               // (the engine's copy, as uploaded)
    }

    /** afterStep: apply the step's removals (BHA:519) once -- the list the reference's removeAt
     *  calls (highest index first) leave, made in one pass: each removeAt shifts the tail, tens of
     *  them per C3 frame cost ~16 ms at 1e6 bodies (tests/c/abi_harness.c --c3-frames).  The
     *  pass runs in chunks: survivors into a reused spare array, then back (set, no structural
     *  change), so the caller keeps the same list object with the same Body objects in it. */
    private fun pull(afterStep: Boolean) {
        if (afterStep) {
            val rem = Native.lastRemoved(handle)            // ascending; usually empty
            if (rem.size <= 2) {
                for (k in rem.indices.reversed()) bodies.removeAt(rem[k])
            } else {
                val n0 = bodies.size
                val base = rem[0]                           // survivors slide down, in order:
                if (spare.size < n0 - base) spare = arrayOfNulls(n0 - base)
                val out = spare
                chunks(n0 - base) { lo, hi ->               // into the spare array, chunk by chunk
                    val k = rem.binarySearch(base + lo)
                    var r = if (k >= 0) k else -k - 1       // removals below this chunk
                    var w = lo - r
                    for (i in base + lo until base + hi) {
                        if (r < rem.size && rem[r] == i) { r++; continue }
                        out[w++] = bodies[i]
                    }
                }
                val m = n0 - base - rem.size
                chunks(m) { lo, hi -> for (i in lo until hi) bodies[base + i] = out[i]!! }
                bodies.subList(base + m, n0).clear()        // the tail, one range removal
            }
        }
        val n = map()                                       // the engine's pinned mirror, in place
        check(n == bodies.size) { "engine and caller body lists diverged" }
        val a = mirror
        val s = stride
        chunks(n) { lo, hi ->
            for (i in lo until hi) {
                val b = bodies[i]
                b.x = a.get(i); b.y = a.get(s + i); b.vx = a.get(2 * s + i); b.vy = a.get(3 * s + i)
                b.m = a.get(4 * s + i)
            }
        }
    }
}
