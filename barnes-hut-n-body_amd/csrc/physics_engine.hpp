// C++ host mirror of the reference's Kotlin surface (BarnesHutAlg.kt = BHA, Config.kt = CFG)
// over the C-ABI in include/bh_engine.h.  Same names, same argument meaning, same call
// pattern as NBodyPanel uses (PNL:103,144,224-233,262,285,291,302,333-340): a caller that
// drove the Kotlin PhysicsEngine drives this one unchanged.
//
// Error behaviour: the reference has no error channel (impossible states are NPEs); here a
// device or argument error throws std::runtime_error carrying bh_last_error().
#pragma once
#include <functional>
#include <stdexcept>
#include <vector>

#include "bh_engine.h"

namespace bh {

// BHA:21-25
struct Body {
    double x, y, vx, vy, m;
};

// BHA:53-82
struct Quad {
    double cx, cy, h;
    bool contains(const Body &b) const {  // BHA:61-62
        return b.x >= cx - h && b.x < cx + h && b.y >= cy - h && b.y < cy + h;
    }
    Quad child(int which) const;  // BHA:73-81
};

// CFG:2-39 — the mutable global the engine reads live at every step().
struct Config {
    static inline int WIDTH_PX = 2400;    // CFG:5
    static inline int HEIGHT_PX = 800;    // CFG:8
    static inline double G = 80.0;        // CFG:11
    static inline double DT = 0.005;      // CFG:14
    static inline double SOFTENING = 1.0; // CFG:17
    static inline const double SOFT2 = 1.0 * 1.0;  // CFG:20 (a val: frozen at init)
    static inline double theta = 0.30;    // CFG:23
    static inline double R = 100.0;       // CFG:26
    static inline int N = 5000;           // CFG:29
    static constexpr double CENTRAL_MASS = 50000.0;          // CFG:32
    static constexpr double MIN_R = 8.0;                     // CFG:35
    static constexpr double TOTAL_SATELLITE_MASS = 5000.0;   // CFG:38
};

// The debug view returned by getTreeForDebug() (BHA:329): visitQuads (BHA:265-274).
class BHTree {
public:
    explicit BHTree(std::vector<Quad> quads) : quads_(std::move(quads)) {}
    void visitQuads(const std::function<void(const Quad &)> &visit) const {
        for (const Quad &q : quads_) visit(q);
    }
    size_t size() const { return quads_.size(); }

private:
    std::vector<Quad> quads_;  // pre-order, as the recursive visit produces them
};

// BHA:287-533
class PhysicsEngine {
public:
    // PhysicsEngine(initialBodies) — adopts the caller's list (BHA:295) on HIP device `device`.
    explicit PhysicsEngine(std::vector<Body> &initialBodies, int device = 0);
    // ... over several GPUs behind one handle (bh_create_multi_list; repeats allowed)
    PhysicsEngine(std::vector<Body> &initialBodies, const std::vector<int> &devices);
    ~PhysicsEngine();
    PhysicsEngine(const PhysicsEngine &) = delete;
    PhysicsEngine &operator=(const PhysicsEngine &) = delete;

    void step();                                      // BHA:405-439
    const std::vector<Body> &getBodies() const;       // BHA:335
    void resetBodies(std::vector<Body> &newBodies);   // BHA:342-349
    BHTree getTreeForDebug();                         // BHA:329-332

    double mergeMaxMass = 4000.0;        // BHA:315
    double mergeMinDist = Config::MIN_R; // BHA:321

    bh_engine *handle() { return eng_; }

private:
    void init();
    void pushParams();
    void pushBodies();
    void mapMirror();
    bool bodiesChanged() const;
    void pullBodies(bool afterStep);
    void check(int rc) const;

    std::vector<Body> *bodies_;
    bh_engine *eng_ = nullptr;
    // What the engine holds, in the caller's order: its pinned mirror (two buffers,
    // bh_set_mirror(e, 2)), mapped after every call that changed it.  step() compares the list
    // against it in place while the step already runs (the step writes the other buffer) and
    // re-uploads only when the caller edited a body, so the engine keeps its Morton-ordered state.
    const double *mir_[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    int64_t mirN_ = -1;
};

}  // namespace bh
