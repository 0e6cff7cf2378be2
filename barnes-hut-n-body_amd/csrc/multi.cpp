// The multi-device PhysicsEngine handle (bh_create_multi / bh_create_multi_list, multi.hpp).
//
// Members are the ranks of the multi-GPU decomposition (engine.cpp): with distinct devices they
// exchange over RCCL communicators made in this process (ncclCommInitAll: xGMI between the
// GPUs), one member per communicator, each driven by its own host thread -- the same collectives,
// in the same order, as one process per GPU (bh_create_dist).  A device listed twice cannot host
// two RCCL ranks ("invalid usage"), so a list with repeats -- and BH_MULTI_EXCHANGE=copy -- uses an
// in-process group instead (bh_create_local: device-to-device copies of the same pieces, rounds
// and in-place layout; peer access between distinct devices).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "bh_engine.h"
#include "multi.hpp"

namespace bh {
void set_error(bh_engine *e, const std::string &msg);  // engine.cpp
}

namespace bh {

struct Multi {
    int world = 0;
    std::vector<bh_engine *> members;
    std::vector<int> devices;
    bh_local_group *group = nullptr;  // copy exchange (repeated devices / BH_MULTI_EXCHANGE=copy)
    bool rccl = false;
    // set by a member whose call failed: every member's waits poll it (engine.cpp wait_stream)
    // and every member refuses further calls until the handle's bh_reset_bodies (multi_repair)
    std::atomic<bool> abort{false};
    std::atomic<bool> busy{false};  // run() is not reentrant: a second caller gets kBusy
    static constexpr int kBusy = 1;
    // the worker pool: member r > 0 runs on threads[r - 1]; member 0 on the caller's thread
    std::vector<std::thread> threads;
    std::mutex mu;
    std::condition_variable go, done;
    uint64_t gen = 0;
    int pending = 0;
    bool quit = false;
    const std::function<int(bh_engine *, int)> *task = nullptr;
    std::vector<int> rc;

    void worker(int r) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<int(bh_engine *, int)> *t;
            {
                std::unique_lock<std::mutex> lk(mu);
                go.wait(lk, [&] { return quit || gen != seen; });
                if (quit) return;
                seen = gen;
                t = task;
            }
            const int v = (*t)(members[(size_t)r], r);
            std::lock_guard<std::mutex> lk(mu);
            rc[(size_t)r] = v;
            if (--pending == 0) done.notify_all();
        }
    }

    int run(const std::function<int(bh_engine *, int)> &fn) {
        bool idle = false;
        if (!busy.compare_exchange_strong(idle, true)) return kBusy;
        {
            std::lock_guard<std::mutex> lk(mu);
            task = &fn;
            pending = world - 1;
            for (int &v : rc) v = BH_OK;
            ++gen;
        }
        go.notify_all();
        const int r0 = fn(members[0], 0);
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return pending == 0; });
        rc[0] = r0;
        task = nullptr;
        busy.store(false);
        for (int v : rc)
            if (v != BH_OK) return v;
        return BH_OK;
    }
};

int multi_all(Multi *mu, bh_engine *facade, const std::function<int(bh_engine *, int)> &fn) {
    const int rc = mu->run(fn);
    if (rc == Multi::kBusy) {
        set_error(facade, "another call of this handle is running on another thread");
        return BH_E_STATE;
    }
    if (rc != BH_OK) {
        for (int r = 0; r < mu->world; ++r)
            if (mu->rc[(size_t)r] != BH_OK) {
                set_error(facade, std::string("rank ") + std::to_string(r) + ": " +
                                      bh_last_error(mu->members[(size_t)r]));
                break;
            }
    }
    return rc;
}

bh_engine *multi_member(const Multi *mu, int rank) {
    if (!mu || rank < 0 || rank >= mu->world) return nullptr;
    return mu->members[(size_t)rank];
}

int multi_world(const Multi *mu) { return mu ? mu->world : 1; }

// bh_reset_bodies of the handle after a failed call: the members' RCCL communicators -- one of
// them aborted, the others in an unknown state -- are all aborted and made anew (the members'
// streams are drained by their own resets), and the abort flag is cleared; the in-process group
// is reset by the members' own resets.
int multi_repair(Multi *mu, bh_engine *facade) {
    if (!mu || !mu->abort.load()) return BH_OK;
    if (mu->rccl) {
        for (bh_engine *m : mu->members) member_drop_comm(m);
        std::vector<ncclComm_t> comms((size_t)mu->world, nullptr);
        int cur = 0;
        (void)hipGetDevice(&cur);
        const ncclResult_t nr = ncclCommInitAll(comms.data(), mu->world, mu->devices.data());
        (void)hipSetDevice(cur);
        if (nr != ncclSuccess) {
            set_error(facade, std::string("bh_reset_bodies: ncclCommInitAll: ") +
                                  ncclGetErrorString(nr));
            return BH_E_COMM;
        }
        for (int r = 0; r < mu->world; ++r) member_set_comm(mu->members[(size_t)r], comms[(size_t)r]);
    }
    mu->abort.store(false);
    return BH_OK;
}

void multi_destroy(Multi *mu) {
    if (!mu) return;
    if (!mu->threads.empty() && mu->world > 1) {  // the members' teardown in parallel (RCCL)
        std::function<int(bh_engine *, int)> fn = [](bh_engine *m, int) {
            bh_destroy(m);
            return BH_OK;
        };
        mu->run(fn);
    } else {
        for (bh_engine *m : mu->members) bh_destroy(m);
    }
    {
        std::lock_guard<std::mutex> lk(mu->mu);
        mu->quit = true;
    }
    mu->go.notify_all();
    for (std::thread &t : mu->threads) t.join();
    if (mu->group) bh_local_group_destroy(mu->group);
    delete mu;
}

}  // namespace bh

using namespace bh;

namespace {

// Members made one by one on the caller's thread; the pool afterwards.  On failure everything
// made so far is torn down.
int make_multi(const bh_params *p, const std::vector<int> &dev, bh_engine **out) {
    const int world = (int)dev.size();
    bool repeated = false;
    for (int i = 0; i < world; ++i)
        for (int j = 0; j < i; ++j) repeated = repeated || dev[(size_t)i] == dev[(size_t)j];
    const char *xv = std::getenv("BH_MULTI_EXCHANGE");
    const bool copy = repeated || (xv && std::strcmp(xv, "copy") == 0);
    Multi *mu = new Multi();
    mu->world = world;
    mu->rc.assign((size_t)world, BH_OK);
    mu->members.assign((size_t)world, nullptr);
    auto fail = [&](int rc, const std::string &why) {
        std::fprintf(stderr, "bh_create_multi: %s\n", why.c_str());
        multi_destroy(mu);
        return rc;
    };
    std::vector<ncclComm_t> comms;
    int cur_dev = 0;
    (void)hipGetDevice(&cur_dev);  // (the peer loop sets devices: the caller's is restored)
    struct Restore {
        int d;
        ~Restore() { (void)hipSetDevice(d); }
    } restore{cur_dev};
    mu->devices = dev;
    if (copy) {
        int rc = bh_local_group_create(world, &mu->group);
        if (rc != BH_OK) return fail(rc, "bh_local_group_create failed");
        // distinct devices read each other's exchange buffers directly (xGMI)
        for (int i = 0; i < world; ++i)
            for (int j = 0; j < world; ++j) {
                if (dev[(size_t)i] == dev[(size_t)j]) continue;
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, dev[(size_t)i], dev[(size_t)j]) == hipSuccess &&
                    can && hipSetDevice(dev[(size_t)i]) == hipSuccess) {
                    const hipError_t e = hipDeviceEnablePeerAccess(dev[(size_t)j], 0);
                    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                        return fail(BH_E_DEVICE, std::string("hipDeviceEnablePeerAccess: ") +
                                                     hipGetErrorString(e));
                    (void)hipGetLastError();
                }
            }
    } else {
        comms.assign((size_t)world, nullptr);
        const ncclResult_t nr = ncclCommInitAll(comms.data(), world, dev.data());
        if (nr != ncclSuccess)
            return fail(BH_E_COMM, std::string("ncclCommInitAll: ") + ncclGetErrorString(nr));
        mu->rccl = true;
    }
    for (int r = 0; r < world; ++r) {
        bh_engine *m = nullptr;
        const int rc = member_create(p, dev[(size_t)r], r, world, copy ? nullptr : comms[(size_t)r],
                                     mu->group, &m);
        if (rc != BH_OK) {
            // (the communicators not yet handed to a member are freed here)
            for (int q = r; q < world && !copy; ++q) (void)ncclCommDestroy(comms[(size_t)q]);
            mu->members.resize((size_t)r);
            mu->world = r;
            return fail(rc, "member " + std::to_string(r) + " on device " +
                                std::to_string(dev[(size_t)r]) + " could not be created");
        }
        mu->members[(size_t)r] = m;
        member_set_abort(m, &mu->abort);
    }
    for (int r = 1; r < world; ++r) mu->threads.emplace_back([mu, r] { mu->worker(r); });
    bh_engine *f = nullptr;
    int rc = facade_create(p, mu, &f);
    if (rc != BH_OK) return fail(rc, "facade");
    if (mu->rccl) {  // every member at once: the check is a collective
        rc = multi_all(mu, f, [](bh_engine *m, int) { return member_agree(m); });
        if (rc != BH_OK) {
            std::fprintf(stderr, "bh_create_multi: %s\n", bh_last_error(f));
            bh_destroy(f);  // (destroys the members through the facade)
            return rc;
        }
    }
    *out = f;
    return BH_OK;
}

}  // namespace

extern "C" {

int bh_create_multi_list(const bh_params *p, const int32_t *devices, int32_t count,
                         bh_engine **out) {
    if (!out || !p || count < 1 || !devices) return BH_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) return BH_E_DEVICE;
    std::vector<int> dev((size_t)count);
    for (int32_t i = 0; i < count; ++i) {
        if (devices[i] < 0 || devices[i] >= ndev) return BH_E_INVALID;
        dev[(size_t)i] = devices[i];
    }
    // one GPU: the pipelined engine (BH_MULTI_EXCHANGE=rccl keeps the decomposition: a one-rank
    // RCCL communicator from ncclCommInitAll, which tests the in-process RCCL path on one GPU)
    const char *xv = std::getenv("BH_MULTI_EXCHANGE");
    if (count == 1 && !(xv && std::strcmp(xv, "rccl") == 0)) return bh_create(p, dev[0], out);
    return make_multi(p, dev, out);
}

int bh_create_multi(const bh_params *p, uint32_t device_mask, bh_engine **out) {
    if (!out || !p) return BH_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return BH_E_DEVICE;
    std::vector<int32_t> dev;
    for (int d = 0; d < 32 && d < ndev; ++d)
        if (device_mask == 0u || (device_mask >> d) & 1u) dev.push_back(d);
    if (dev.empty() || (ndev < 32 && (device_mask >> ndev) != 0u)) return BH_E_INVALID;
    return bh_create_multi_list(p, dev.data(), (int32_t)dev.size(), out);
}

}  // extern "C"
