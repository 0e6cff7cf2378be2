// One PhysicsEngine handle over several GPUs (bh_create_multi, include/bh_engine.h).
//
// The reference's engine fans every step out over worker threads and joins them before step()
// returns (computeAccelerations, BHA:374-395: repeat(workers) launch {...} inside runBlocking,
// BHA:408, 426).  The multi-device handle does the same over GPUs: it owns one member engine per
// device -- the ranks of the multi-GPU decomposition (replicated state, locally essential tree
// builds, RCCL all-gathers over xGMI) -- and one host thread per member after the first, which
// runs on the caller's thread.  Every call that changes the state runs on every member at once
// and returns when all are done; calls that only read the state read member 0's replica (every
// replica is complete at the API boundary).
#pragma once

#include <atomic>
#include <functional>

#include "bh_engine.h"

namespace bh {

struct Multi;

// fn(member, rank) on every member in parallel, joined; BH_OK or the first failing member's
// code, its message copied into the facade's bh_last_error
int multi_all(Multi *mu, bh_engine *facade, const std::function<int(bh_engine *, int)> &fn);
bh_engine *multi_member(const Multi *mu, int rank);
int multi_world(const Multi *mu);
void multi_destroy(Multi *mu);  // destroys the members, joins the threads
// bh_reset_bodies after a failed call: fresh RCCL communicators for every member, abort cleared
int multi_repair(Multi *mu, bh_engine *facade);

// engine.cpp: the pieces a multi-device handle is made of
int facade_create(const bh_params *p, Multi *mu, bh_engine **out);
// a rank of an in-process decomposition: RCCL member on an in-process communicator (comm, from
// ncclCommInitAll), or a member of an in-process group (device-to-device copies)
int member_create(const bh_params *p, int device, int rank, int world, void *comm,
                  bh_local_group *group, bh_engine **out);
// the per-process settings check of bh_create_dist (a collective: every member at once)
int member_agree(bh_engine *e);
// the handle's abort flag, which the member's waits poll (a failed peer ends them)
void member_set_abort(bh_engine *e, std::atomic<bool> *flag);
// after a failed call: the member's communicator aborted (if still alive), then a new one
void member_drop_comm(bh_engine *e);
void member_set_comm(bh_engine *e, void *comm);
// getTreeForDebug's tree on a member (the first half of bh_get_quads: every rank builds it, so
// every replica takes the same jitter); the walk is member 0's
int quads_prepare(bh_engine *e);

}  // namespace bh
