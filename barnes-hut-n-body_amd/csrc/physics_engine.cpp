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
    check(bh_set_mirror(eng_, 1));  // every step writes the caller-order bodies to pinned memory
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
    shadow_ = *bodies_;
}

// Bitwise: a caller that wrote the same value back (or a NaN) does not force an upload.
bool PhysicsEngine::bodiesChanged() const {
    return bodies_->size() != shadow_.size() ||
           std::memcmp(bodies_->data(), shadow_.data(), sizeof(Body) * shadow_.size()) != 0;
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
    const double *x, *y, *vx, *vy, *m;  // the engine's pinned mirror, filled by the step itself
    int64_t got = 0;
    check(bh_map_bodies(eng_, &x, &y, &vx, &vy, &m, &got));
    if ((int64_t)bodies_->size() != got) throw std::runtime_error("engine and caller lists diverged");
    for (int64_t i = 0; i < got; ++i) (*bodies_)[(size_t)i] = Body{x[i], y[i], vx[i], vy[i], m[i]};
    shadow_ = *bodies_;
}

void PhysicsEngine::step() {
    pushParams();
    if (bodiesChanged()) pushBodies();  // the caller edited bodies between frames
    check(bh_step(eng_, 1));
    pullBodies(true);
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
