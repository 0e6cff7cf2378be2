// C++ PhysicsEngine mirror over the C-ABI (see physics_engine.hpp).
#include "physics_engine.hpp"

#include <cstring>
#include <string>

namespace bh {

Quad Quad::child(int which) const {
    const double hh = h / 2.0;
    switch (which) {
    case 0: return Quad{cx - hh, cy - hh, hh};
    case 1: return Quad{cx + hh, cy - hh, hh};
    case 2: return Quad{cx - hh, cy + hh, hh};
    default: return Quad{cx + hh, cy + hh, hh};
    }
}

void PhysicsEngine::check(int rc) const {
    if (rc != BH_OK)
        throw std::runtime_error(std::string("bh_engine: ") + bh_last_error(eng_) + " (rc=" +
                                 std::to_string(rc) + ")");
}

PhysicsEngine::PhysicsEngine(std::vector<Body> &initialBodies, int device)
    : bodies_(&initialBodies) {
    bh_params p;
    bh_default_params(&p);
    int rc = bh_create(&p, device, &eng_);
    if (rc != BH_OK) throw std::runtime_error("bh_create failed (rc=" + std::to_string(rc) + ")");
    init();
}

PhysicsEngine::PhysicsEngine(std::vector<Body> &initialBodies, const std::vector<int> &devices)
    : bodies_(&initialBodies) {
    bh_params p;
    bh_default_params(&p);
    std::vector<int32_t> d(devices.begin(), devices.end());
    int rc = bh_create_multi_list(&p, d.data(), (int32_t)d.size(), &eng_);
    if (rc != BH_OK)
        throw std::runtime_error("bh_create_multi_list failed (rc=" + std::to_string(rc) + ")");
    init();
}

void PhysicsEngine::init() {
    check(bh_set_mirror(eng_, 2));  // every step writes the caller-order bodies to pinned memory
    pushParams();
    pushBodies();
}

PhysicsEngine::~PhysicsEngine() { bh_destroy(eng_); }

// Config is read live by the reference at every step (BHA:225,256,360-361,378,412,420).
void PhysicsEngine::pushParams() {
    bh_params p;
    p.G = Config::G;
    p.dt = Config::DT;
    p.theta = Config::theta;
    p.soft2 = Config::SOFT2;
    p.width_px = Config::WIDTH_PX;
    p.height_px = Config::HEIGHT_PX;
    p.merge_max_mass = mergeMaxMass;
    p.merge_min_dist = mergeMinDist;
    check(bh_set_params(eng_, &p));
}

void PhysicsEngine::pushBodies() {
    const size_t n = bodies_->size();
    std::vector<double> x(n), y(n), vx(n), vy(n), m(n);
    for (size_t i = 0; i < n; ++i) {
        const Body &b = (*bodies_)[i];
        x[i] = b.x; y[i] = b.y; vx[i] = b.vx; vy[i] = b.vy; m[i] = b.m;
    }
    check(bh_reset_bodies(eng_, (int64_t)n, x.data(), y.data(), vx.data(), vy.data(), m.data()));
    mapMirror();  // (the engine's copy, as uploaded)
}

void PhysicsEngine::mapMirror() {
    check(bh_map_bodies(eng_, &mir_[0], &mir_[1], &mir_[2], &mir_[3], &mir_[4], &mirN_));
}

// Bitwise against the mapped mirror: a caller that wrote the same value back (or a NaN) does
// not force an upload.
bool PhysicsEngine::bodiesChanged() const {
    const size_t n = bodies_->size();
    if ((int64_t)n != mirN_) return true;
    for (size_t i = 0; i < n; ++i) {
        const Body &b = (*bodies_)[i];
        if (std::memcmp(&b.x, mir_[0] + i, 8) || std::memcmp(&b.y, mir_[1] + i, 8) ||
            std::memcmp(&b.vx, mir_[2] + i, 8) || std::memcmp(&b.vy, mir_[3] + i, 8) ||
            std::memcmp(&b.m, mir_[4] + i, 8))
            return true;
    }
    return false;
}

// Write results back into the SAME Body objects (the reference mutates in place,
// BHA:414-432) and shrink the list after a merge (BHA:519).
void PhysicsEngine::pullBodies(bool afterStep) {
    if (afterStep) {  // BHA:519: remove the merged-away bodies from the caller's own list
        int64_t cnt = 0;
        int rc = bh_last_removed(eng_, nullptr, 0, &cnt);
        if (rc != BH_OK && rc != BH_E_CAPACITY) check(rc);
        std::vector<int64_t> rem((size_t)cnt);
        check(bh_last_removed(eng_, rem.data(), cnt, &cnt));
        if (rem.size() <= 2) {
            for (auto it = rem.rbegin(); it != rem.rend(); ++it)
                bodies_->erase(bodies_->begin() + *it);
        } else {  // the list those erase calls leave, in one pass (each erase shifts the tail)
            size_t w = (size_t)rem[0], q = 0;
            for (size_t i = (size_t)rem[0]; i < bodies_->size(); ++i) {
                if (q < rem.size() && (size_t)rem[q] == i) {
                    ++q;
                    continue;
                }
                (*bodies_)[w++] = (*bodies_)[i];
            }
            bodies_->resize(w);
        }
    }
    mapMirror();  // the engine's pinned mirror, filled by the step itself
    const int64_t got = mirN_;
    if ((int64_t)bodies_->size() != got) throw std::runtime_error("engine and caller lists diverged");
    for (int64_t i = 0; i < got; ++i)
        (*bodies_)[(size_t)i] = Body{mir_[0][i], mir_[1][i], mir_[2][i], mir_[3][i], mir_[4][i]};
}

void PhysicsEngine::step() {
    pushParams();
    if ((int64_t)bodies_->size() != mirN_) {  // the caller added or removed bodies
        pushBodies();
        check(bh_step(eng_, 1));
        pullBodies(true);
        return;
    }
    // The step runs on the engine's thread while the list is compared against the mapped mirror
    // (bh_step_begin: the step writes the other buffer); an edited list is uploaded and stepped
    // again, the upload replacing that step's result.
    check(bh_step_begin(eng_, 1));
    bool edited = false;
    try {
        edited = bodiesChanged();
    } catch (...) {
        (void)bh_step_end(eng_);
        throw;
    }
    if (edited) {
        // (that step ran on the state before the edit: its result -- and an error it met, e.g. on
        // the tree the previous call left, whose flags it took over -- is replaced by the upload)
        (void)bh_step_end(eng_);
        pushBodies();
        check(bh_step(eng_, 1));
        pullBodies(true);
        return;
    }
    // The hand-off (bh_step_positions), before the step's last traversal: the survivors first --
    // the removals (BHA:519) as one in-place pass, survivor j at list index sv[j] >= j --, then
    // the final positions and masses; after bh_step_end only vx, vy are left.
    const uint32_t *sv = nullptr;
    const double *x = nullptr, *y = nullptr, *m = nullptr;
    int64_t n = 0, n0 = 0;
    int rc = bh_step_positions(eng_, nullptr, nullptr, nullptr, &sv, &n, &n0);
    if (rc == BH_OK && n != (int64_t)bodies_->size()) {
        for (int64_t j = 0; j < n; ++j) (*bodies_)[(size_t)j] = (*bodies_)[sv[j]];
        bodies_->resize((size_t)n);
    }
    if (rc == BH_OK) rc = bh_step_positions(eng_, &x, &y, &m, nullptr, &n, &n0);
    if (rc == BH_OK)
        for (int64_t i = 0; i < n; ++i) {
            Body &b = (*bodies_)[(size_t)i];
            b.x = x[i];
            b.y = y[i];
            b.m = m[i];
        }
    const int rc_end = bh_step_end(eng_);
    check(rc != BH_OK ? rc : rc_end);
    mapMirror();
    if (mirN_ != (int64_t)bodies_->size()) throw std::runtime_error("engine and caller lists diverged");
    for (int64_t i = 0; i < mirN_; ++i) {
        Body &b = (*bodies_)[(size_t)i];
        b.vx = mir_[2][i];
        b.vy = mir_[3][i];
    }
}

const std::vector<Body> &PhysicsEngine::getBodies() const { return *bodies_; }

void PhysicsEngine::resetBodies(std::vector<Body> &newBodies) {
    bodies_ = &newBodies;
    pushBodies();
}

BHTree PhysicsEngine::getTreeForDebug() {
    pushParams();
    int64_t need = 0;
    int rc = bh_get_quads(eng_, nullptr, nullptr, nullptr, 0, &need);
    if (rc != BH_OK && rc != BH_E_CAPACITY) check(rc);
    std::vector<double> cx(need), cy(need), h(need);
    int64_t got = 0;
    check(bh_get_quads(eng_, cx.data(), cy.data(), h.data(), need, &got));
    std::vector<Quad> quads((size_t)got);
    for (int64_t i = 0; i < got; ++i) quads[(size_t)i] = Quad{cx[i], cy[i], h[i]};
    pullBodies(false);  // building a fresh tree can jitter positions (BHA:146-151)
    return BHTree(std::move(quads));
}

}  // namespace bh
