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
    // bh_create_multi over the GPUs of -Dbh.deviceMask (bit d = HIP device d; default 0 = every
    // visible GPU): one handle, every step fanned out over the GPUs and joined (BHA:374-395)
    private val handle: Long = Native.create(Integer.decode(System.getProperty("bh.deviceMask", "0")))
    // SoA of what the engine holds (x[0..n) y[n..2n) vx vy m), reused frame after frame: no
    // per-frame allocation that grows with N
    private var shadow = DoubleArray(0)
    private var shadowN = -1

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
        if (changed()) push()                                // upload only if the caller edited bodies
        Native.step(handle, 1)
        pull(afterStep = true)
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

    /** Whether the caller's bodies differ (bitwise) from what the engine holds -- in place. */
    private fun changed(): Boolean {
        val n = bodies.size
        if (n != shadowN) return true
        val a = shadow
        for (i in 0 until n) {
            val b = bodies[i]
            if (b.x.toRawBits() != a[i].toRawBits() || b.y.toRawBits() != a[n + i].toRawBits() ||
                b.vx.toRawBits() != a[2 * n + i].toRawBits() ||
                b.vy.toRawBits() != a[3 * n + i].toRawBits() ||
                b.m.toRawBits() != a[4 * n + i].toRawBits()) return true
        }
        return false
    }

    private fun push() {
        val n = bodies.size
        if (shadow.size < 5 * n) shadow = DoubleArray(5 * n)
        val a = shadow
        for ((i, b) in bodies.withIndex()) {
            a[i] = b.x; a[n + i] = b.y; a[2 * n + i] = b.vx; a[3 * n + i] = b.vy; a[4 * n + i] = b.m
        }
        Native.reset(handle, n, a)
        shadowN = n
    }

    /** afterStep: apply the step's removals (BHA:519) once -- the list the reference's removeAt
     *  calls (highest index first) leave, made in one pass: each removeAt shifts the tail, tens of
     *  them per C3 frame cost ~16 ms at 1e6 bodies (tests/c/abi_harness.c --c3-frames). */
    private fun pull(afterStep: Boolean) {
        if (afterStep) {
            val rem = Native.lastRemoved(handle)            // ascending; usually empty
            if (rem.size <= 2) {
                for (k in rem.indices.reversed()) bodies.removeAt(rem[k])
            } else {
                val n0 = bodies.size
                var w = rem[0]                              // survivors slide down, in order
                var r = 0
                for (i in rem[0] until n0) {
                    if (r < rem.size && rem[r] == i) { r++; continue }
                    bodies[w++] = bodies[i]
                }
                bodies.subList(w, n0).clear()               // the tail, one range removal
            }
        }
        var n = Native.getInto(handle, shadow)              // the engine's pinned mirror, SoA
        if (n < 0) {                                        // (only after a reset to more bodies)
            shadow = DoubleArray(-5 * n)
            n = Native.getInto(handle, shadow)
        }
        check(n == bodies.size) { "engine and caller body lists diverged" }
        val a = shadow
        for (i in 0 until n) {
            val b = bodies[i]
            b.x = a[i]; b.y = a[n + i]; b.vx = a[2 * n + i]; b.vy = a[3 * n + i]; b.m = a[4 * n + i]
        }
        shadowN = n
    }
}
