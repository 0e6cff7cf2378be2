// Engine host code and the C-ABI (include/bh_engine.h).
//
// Replaces PhysicsEngine (BHA:287-532).  The engine owns the body state in HBM as SoA fp64
// arrays in Morton ("slot") order plus each body's caller-list index (cidx), the tree
// workspace, and one HIP stream.  A step is the reference's step() (BHA:405-439) as a fixed
// kernel sequence on that stream; the only host round trip is the merge rule's (BHA:463-532)
// candidate mailbox, and only while heavy bodies exist.
//
// Multi-GPU (bh_create_dist): every rank holds a replica of the state and owns one contiguous
// range of the Hilbert wave order.  The build is sharded: each rank builds a locally essential
// tree (let.hip) -- the cells its bodies may open, plus the top assembled from every rank's cell
// values (one all-gather of the cell tables) -- evaluates its range, kicks (and drifts) its own
// bodies in the traversal's epilogue, and the new positions (16 B per body) are all-gathered in
// place with RCCL over xGMI; velocities stay with their owners until the next full build, before
// which they are all-gathered.  Every BH_LET_REFRESH builds, after a reset and for the last build
// of every bh_step call (lastTree, BHA:435) the full tree is built by every rank; its
// accelerations are all-gathered and every rank integrates every body.  The merge rule is
// replicated (identical inputs, identical outcome) and needs no exchange.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "bh_device.hpp"
#include "bh_engine.h"
#include "multi.hpp"

using namespace bh;

namespace {
constexpr int kPhases = 5;  // build, traverse, integrate, merge, allgather
}  // namespace

namespace bh {
void set_error(bh_engine *e, const std::string &msg);  // for the C-ABI's other translation units
}

// In-process rank group (bh_local_group_*): `world` engines of one process, one host thread
// each, that exchange the force pieces through device-to-device copies instead of RCCL -- the
// same pieces, rounds and in-place layout as the ncclAllGather path, so the multi-rank
// decomposition runs on one GPU (RCCL refuses several ranks per device).
//
// Every wait has a way out (the reference's join always returns, BHA:408, 426): a member whose
// call fails aborts the group (abort()), which wakes every member waiting in barrier() and makes
// every later barrier return false, until the members' bh_reset_bodies (reset()); a barrier that
// waits longer than BH_COMM_TIMEOUT_S aborts the group itself.
namespace {
// seconds a multi-rank engine waits for its peers (a barrier, a collective on the device) before
// it gives up and aborts (BH_COMM_TIMEOUT_S; 0 = forever)
double comm_timeout_s() {
    static const double t = [] {
        const char *v = std::getenv("BH_COMM_TIMEOUT_S");
        return v ? std::atof(v) : 300.0;
    }();
    return t;
}
}  // namespace

struct bh_local_group {
    int world = 0;
    std::vector<bh_engine *> members;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::atomic<bool> aborted{false};
    bool timed_out = false;  // (under mu) the abort came from a barrier's deadline
    // false: the group was aborted (before or while this member waited)
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted.load()) return false;
        const uint64_t gen = generation;
        if (++arrived == world) {
            arrived = 0;
            ++generation;
            cv.notify_all();
            return true;
        }
        auto pred = [&] { return generation != gen || aborted.load(); };
        const double t = comm_timeout_s();
        if (t > 0.0) {
            if (!cv.wait_for(lk, std::chrono::duration<double>(t), pred)) {
                timed_out = true;
                aborted.store(true);
                cv.notify_all();
                return false;
            }
        } else {
            cv.wait(lk, pred);
        }
        return generation != gen;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted.store(true);
        cv.notify_all();
    }
    // every member's bh_reset_bodies after an abort (no member waits: their calls have returned)
    void reset() {
        std::lock_guard<std::mutex> lk(mu);
        if (!aborted.load()) return;
        arrived = 0;
        ++generation;
        timed_out = false;
        aborted.store(false);
    }
};

struct bh_engine {
    bh::Multi *multi = nullptr;  // a multi-device handle (multi.cpp): the members do the work
    // ... or, for a body list below multi_min bodies, one pipelined single-GPU engine on the first
    // device (like the reference's min(cores, n) workers, BHA:377): a step of a few 1e5 bodies is
    // launch-bound, and splitting it only adds launches and exchanges
    bh_engine *one = nullptr;
    bool use_one = false;
    int64_t multi_min = 0;
    bh_params p{};
    Geometry geo{};
    int device = 0;
    hipStream_t stream = nullptr;
    int rank = 0, world = 1;
    ncclComm_t comm = nullptr;
    bh_local_group *group = nullptr;             // in-process ranks (test path), or RCCL:
    hipStream_t comm_stream = nullptr;            // all-gathers, overlapping the next round
    // odd rounds' traversals: at 8 ranks a round is under one dispatch generation of waves, so
    // consecutive rounds run concurrently on two streams instead of each waiting for the tail
    hipStream_t stream2 = nullptr;
    hipEvent_t built_ev = nullptr;
    hipEvent_t round_ev[BH_SHARD_ROUNDS] = {};   // round k's forces written (compute stream)
    hipEvent_t gathered_ev = nullptr;            // every round gathered (comm stream)

    int64_t n = 0;     // live bodies
    int64_t cap = 0;   // allocated bodies
    int J_alloc = -1;  // J the node array was sized for

    BodyState st{};   // current state, slot (Morton) order
    BodyState alt{};  // second buffer: build / compaction target, copy-out staging
    double *a2 = nullptr;  // interleaved accelerations (slot order), 2 * chunk * world
    double *ax = nullptr, *ay = nullptr;  // caller-order copy-out staging

    uint64_t *keys = nullptr, *keys_s = nullptr;
    uint32_t *keys32 = nullptr, *keys32_s = nullptr;
    uint32_t *idx = nullptr, *perm = nullptr;
    uint32_t *perm2 = nullptr;  // the pipelined step's overlapped build's permutation
    int8_t *cpl = nullptr;
    uint32_t *cnt = nullptr, *base = nullptr;
    uint32_t *cell_start = nullptr;
    Node *nodes = nullptr;
    size_t node_cap = 0;
    uint32_t *span_list = nullptr, *super_list = nullptr;
    bh::SpanSlot *span_children = nullptr;
    uint32_t *scalars = nullptr;  // [1] tree error flags
    uint32_t *visits32 = nullptr;
    uint32_t *contrib32 = nullptr;     // per-body point-force contributions (diagnostics)
    uint32_t *wave_iters = nullptr;  // per-wave union of visited nodes (diagnostics)
    uint32_t *wave_blocks = nullptr; // per-wave point-force blocks executed (diagnostics)
    int64_t stat_lane_visits = 0, stat_wave_iters = 0, stat_waves = 0;
    int64_t stat_lane_contrib = 0, stat_wave_blocks = 0;

    // merge
    uint32_t *heavy = nullptr;
    uint32_t *keep = nullptr, *pos = nullptr;
    MergePair *box = nullptr;  // candidate pairs: header + pairs
    uint32_t box_cap = 0;
    uint32_t box_need = 0;     // pairs a step needed beyond the capacity (grown on retry)
    BodyState snap{};          // state at the start of a bh_step call (exact merge retry)
    int64_t snap_cap = 0, snap_n = 0;
    uint32_t *dlog = nullptr;        // removal log of the running bh_step call (caller indices)
    uint32_t *dead_sorted = nullptr; // the log sorted, for the compaction's renumbering
    uint64_t *rkeys = nullptr;       // replay sort scratch (long candidate lists)
    uint32_t *ridx = nullptr;
    uint32_t *mbits = nullptr;       // victim bitmap over caller indices (long lists)
    uint32_t *mslot = nullptr;       // caller index -> slot of the victims
    int64_t dlog_cap = 0;
    bool heavy_possible = true;  // false once a step saw no heavy body (heavies never appear)
    // the last build listed the heavy bodies in its order (heavy, count in scalars[14]): the merge
    // rule that follows it needs no k_heavy pass (the pipelined step's second build)
    bool heavy_ready = false;
    bool heavy_dirty = false;  // scalars[14] may be nonzero (a list no merge rule consumed)
    bool merge_ran = false;      // the running bh_step call launched the merge rule
    std::vector<int64_t> removed;  // removals of the last bh_step call, ascending (BHA:519)
    void *pin = nullptr;  // pinned staging for small read-backs (coherent: kernels write it too)
    void *pin_dev = nullptr;
    size_t pin_bytes = 0;

    void *scratch = nullptr;
    size_t scratch_bytes = 0;

    // adaptive bucket sort (tree_build.hip): splitters written by every build
    uint64_t *spl = nullptr;
    uint32_t *bcount = nullptr, *bstart = nullptr;
    uint32_t spl_nb = 0;  // splitters of the last build; 0 = none (next build sorts with rocprim)

    // theta = 0 all-pairs path (direct.hip), allocated on first use
    uint8_t *leaf_flags = nullptr;
    uint32_t *leaf_sel = nullptr, *leaf_count = nullptr;
    int32_t *leaf_cover = nullptr;  // 2 (node_cap + 1): subtrees of massless nodes
    LeafList leaves{nullptr};
    void *leaf_tmp = nullptr;
    size_t leaf_tmp_bytes = 0;
    size_t leaf_node_cap = 0;  // node capacity the flags were sized for
    int64_t leaf_cap = 0;

    bool tree_valid = false;  // lastTree (BHA:304): keys_s / cpl / base / nodes are current
    // Multi-rank engines end a call with a LET build too; lastTree is then built on demand by
    // bh_get_quads from the positions that build saw (lt_x, lt_y), without touching the state
    bool lazy_tree = false;
    double *lt_x = nullptr, *lt_y = nullptr;
    int64_t lt_cap = 0;

    // Hilbert lane map of the single-GPU traversal (tree_build.hip lane_order): lane -> slot
    uint32_t *lanes = nullptr;
    bool lanes_valid = false;  // the map is a permutation of the current slots
    int lanes_age = 0;         // builds since the last Hilbert sort
    // a due re-sort of the pipelined step's lane map, run beside the next first traversal on its
    // own buffers (lane_refresh_beside) and swapped in before the second build
    bool lane_defer = false;   // this overlapped build may leave a due re-sort to that
    bool lane_hold = false;    // this second build leaves a due re-sort to the next overlapped one
    bool lr_pending = false;   // a re-sort is due from the prebuilt tree's keys
    bool lr_ready = false;     // lanes_next holds it once lr_ev completes
    uint32_t *lanes_next = nullptr, *lr_hkey = nullptr, *lr_hkey_s = nullptr, *lr_slot = nullptr;
    void *lr_scratch = nullptr;
    size_t lr_scratch_bytes = 0;
    int64_t lr_cap = 0;
    hipEvent_t lr_ev = nullptr;
    const uint32_t *a2_lanes = nullptr;  // the last evaluation wrote a2 by lane of this map
    GatherLayout a2_layout{};            // ... at the lane's gather slot (multi-rank rounds)

    // multi-rank locally essential tree (let.hip): subset state and tree workspace
    // BH_LET unset: LET builds from BH_LET_MIN_WORLD ranks up (round 3, solo C4 rank 0, ms per
    // step LET / replicated: 2 ranks 9.80 / 10.21, 3 ranks 7.00 / 7.98, 4 ranks 5.53 / 6.80,
    // 8 ranks 3.43 / 5.19; round 2 had 10.45 / 10.15 at 2 ranks, hence 4 then);
    // BH_LET=1 at any world size, BH_LET=0 never
    bool let_on = true;
    bool let_forced = false;
    int let_age = 0;            // LET builds since the last full build
    int64_t let_builds = 0, full_builds = 0, let_last_sub = 0;
    int64_t let_known = 0;       // largest subset of the last bh_step call (0: unknown)
    int64_t let_overflows = 0;   // calls replayed for a subset overflow
    uint32_t s_spl_nb = 0;       // splitters of the last LET build (subset bucket sort)
    bool st_morton = false;     // slots are in the Morton order of a full build (not caller order)
    bool vel_stale = false;     // LET evaluations integrated only own bodies: velocities of the
                                // others are exchanged before the next full build
    LetBufs L{};
    int64_t let_cap = 0;        // n capacity of the per-body LET arrays
    // the selection's candidate blocks (let.hip LetSweep): the boxes of the state's 256-slot
    // blocks at the last full build, and the displacement bound since (disp[0]; the speed words
    // after it: own, then every rank's, exchanged at the end of every drifting LET evaluation)
    uint32_t *let_box = nullptr;
    double *disp = nullptr;
    bool boxes_valid = false;
    // the selection's marks were cleared by the last LET build's lane map (for n bodies)
    bool let_clean = false;
    int64_t let_clean_n = -1;
    int builds_since_box = 0;   // builds since then that may have jittered positions
    int64_t let_sub_cap = 0;    // subset capacity of the subset tree workspace
    int let_J = -1;
    size_t let_node_cap = 0;
    BodyState sub_src{}, sub_dst{};
    uint64_t *s_keys = nullptr, *s_keys_s = nullptr, *s_spl = nullptr;
    uint32_t *s_keys32 = nullptr, *s_keys32_s = nullptr, *s_idx = nullptr, *s_perm = nullptr;
    int8_t *s_cpl = nullptr;
    uint32_t *s_cnt = nullptr, *s_base = nullptr, *s_cell_start = nullptr;
    uint32_t *s_span_list = nullptr, *s_super_list = nullptr, *s_bcount = nullptr,
             *s_bstart = nullptr;
    bh::SpanSlot *s_span_children = nullptr;
    Node *s_nodes = nullptr;
    hipEvent_t table_ev = nullptr;
    int64_t set_cap = 0;        // n capacity of the per-body arrays L.lanes, L.subpos
    hipEvent_t sub_cnt_ev = nullptr;
    uint32_t *sub_cnt_h = nullptr;    // pinned: the last selection's subset size (sub_cnt_ev)
    bool sub_cnt_pending = false;

    LetCell *pub_table = nullptr;     // in-process group: the table this member exchanges now
    hipEvent_t pub_table_ev = nullptr;
    bool inject_guard = false;  // bh_debug_inject(1): the next LET build trips k_let_guard
    int inject_build = -1;      // bh_debug_inject(2 + k): the k-th next full build raises its
                                // jitter flag (as the unsupported-geometry guard would)
    bool agree_failed = false;  // in-process group: this member could not read a peer's flags
    // pipelined step (one GPU): the next step's first build runs on pipe_stream while this step's
    // second traversal runs; it builds into nodes_alt / alt, and the traversal reads copies of
    // what that build and the merge rule overwrite (masses, flags, lane map, node count)
    Node *nodes_alt = nullptr;
    size_t nodes_alt_cap = 0;
    double *m_trav = nullptr;
    uint32_t *cidx_trav = nullptr, *lanes_trav = nullptr, *T_trav = nullptr;
    bool tc_want = false, tc_done = false;  // build_into: the copies above made by k_emit_com
    uint32_t *tc_box = nullptr;             // (and the merge rule's mailbox header cleared)
    int64_t trav_cap = 0;
    bool prebuilt = false;  // the current step's first build was made by the previous step
    // ... by the previous call's last step: that build's error flags are in scalars[10] (they
    // belong to the step that uses the tree, the next call's first, which takes them over)
    bool carried_flags = false;
    // deep pipeline: the previous step also evaluated a(t) on that tree (beside its own second
    // traversal), by lane of the current map, with these force parameters
    bool forces_ready = false;
    // the velocities are still in the previous slot order, in alt (the overlapped build's
    // permutation, read by the next step's first kick); null: st holds them
    const uint32_t *vel_perm = nullptr;
    ForceParams fp_ready{0.0, 0.0, 0.0};
    double *a2_alt = nullptr;  // a2's compaction target (the carried forces over removals)
    int64_t a2_alt_cap = 0;
    bool fuse_keys = false;   // the next KICK_DRIFT traversal writes the next build's keys / buckets
    bool keys_ready = false;  // ... and it did: the next full build skips k_morton, k_bucket_count
    hipEvent_t pipe_ev[3] = {nullptr, nullptr, nullptr};
    hipStream_t pipe_stream = nullptr;  // the overlapped work's stream (BH_PIPE_PRIORITY)
    // A call's last step is pipelined too (the front-end calls bh_step(1) once per frame): the
    // call then ends with the next step's first tree already built (prebuilt: st in its order,
    // jitter applied, nodes).  What the caller sees -- the reference's bodies after step(), before
    // the next buildTree's jitter (BHA:146-151) -- is `view` (the previous slot order); lastTree
    // (BHA:435) is nodes_alt with its walk structures copied aside (lt_keys, lt_cpl, lt_base).
    // The next bh_step consumes the prebuilt tree; bh_set_params (geometry), bh_reset_bodies and
    // a replay drop it.
    BodyState view{};
    int64_t view_cap = 0;
    bool view_pending = false;
    uint64_t *lt_keys = nullptr;
    int8_t *lt_cpl = nullptr;
    uint32_t *lt_base = nullptr;
    int64_t lt_walk_cap = 0;
    bool lt_aside = false;  // lastTree is (nodes_alt, lt_keys, lt_cpl, lt_base)
    // Pinned caller-order mirror of the bodies (bh_set_mirror / bh_map_bodies): x, y, vx, vy, m
    // at stride mir_cap, filled by the step itself on mir_stream
    bool mirror_on = false;
    double *mir = nullptr;        // pinned host, 5 * mir_cap: the buffer the copies write
    // bh_set_mirror(e, 2): two buffers; the copies write the one bh_map_bodies did not hand out
    // last (mir_front), so a caller reads the mapped bodies while the next bh_step runs
    double *mir_buf[2] = {nullptr, nullptr};
    int mir_nbuf = 1;
    int mir_front = -1;
    double *mir_stage = nullptr;  // device, 5 * mir_cap (caller order, compacted)
    uint32_t *mir_keep = nullptr, *mir_pos = nullptr;  // device, caller order
    int64_t mir_cap = 0;
    void *mir_tmp = nullptr;      // the mirror's scan scratch (the overlapped build uses `scratch`)
    size_t mir_tmp_bytes = 0;
    bool mir_fresh = false;       // the mirror (after mir_ev) holds the current caller state
    bool mir_launched = false;    // ... launched by the running call's last step
    int64_t mir_n = 0;
    hipStream_t mir_stream = nullptr;
    hipEvent_t mir_ev = nullptr;   // copy-out complete
    hipEvent_t mir_ev2 = nullptr;  // the mirror's kernels are done reading the state
    hipEvent_t mir_in[2] = {nullptr, nullptr};
    // bh_step_begin / bh_step_positions / bh_step_end (two mirror buffers only): the call runs
    // on step_thr of the handle the caller holds; the engine that fills the mirror (this one, or
    // a multi handle's member 0) hands over positions, masses and the survivors' list indices of
    // the running call once its last merge rule is done (mid_*), before the last traversal
    std::thread step_thr;
    std::atomic<bool> async_running{false};
    int async_rc = 0;
    int64_t mid_n0 = 0;              // bodies before the running call
    bool mid_surv_done = false;      // the survivors were derived from the call's removals
    bh_engine *mid_eng = nullptr;    // the running call's mirror engine
    std::mutex mid_mu;
    std::condition_variable mid_cv;
    bool mid_armed = false, mid_ready = false, mid_done = false, mid_void = false;
    double *mid_buf = nullptr;       // the mirror buffer of the hand-off
    int64_t mid_stride = 0;
    hipEvent_t mid_ev = nullptr;     // the hand-off's copies are done
    hipEvent_t mid_sv_ev = nullptr;  // ... its survivors' (copied first)
    // pinned, MIRROR_HDR + mir_cap (mirror_survivors): scalars[0..4) at the hand-off (tree
    // flags, removals, mailbox overflow), then survivor j's index in the list before the call
    uint32_t *mir_idx = nullptr;
    uint32_t *mir_idx_stage = nullptr;  // device, the same
    hipEvent_t mir_ev3 = nullptr;
    // one GPU: the previous evaluation's wave durations and the longest-first run order
    // (slot 0: the one-GPU launch over all lanes; 1 + k: LET round k's piece)
    uint32_t *wave_cost = nullptr, *run_order = nullptr;
    int64_t cost_stride = 0, order_stride = 0;
    int64_t order_n[1 + BH_SHARD_ROUNDS] = {};  // run_order slot j: a permutation of the runs
                                               // of a launch over order_n[j] lanes (0: none)
    // Between LET evaluations the new positions stay in the exchange buffer (a2, by lane of
    // pos_lanes at pos_layout's gather slots): the next selection reads them there, and the
    // replica's x, y are written only when something else needs them (materialize_positions)
    bool pos_pending = false;
    const uint32_t *pos_lanes = nullptr;
    GatherLayout pos_layout{};
    uint32_t *inv_lanes = nullptr;  // slot -> gather slot of its lane (the selection's reads)
    bool inv_valid = false;         // ... for the current lane map, n and layout
    // bh_create_solo (measurement): no peers; their cells' values from the last full build
    bool solo = false;
    LetCell *solo_table = nullptr;
    uint8_t *solo_all = nullptr;    // every cell marked
    double *solo_xchg = nullptr;    // BH_SOLO_XCHG: receive buffer of the emulated exchange
    int64_t solo_xchg_cap = 0;
    uint32_t *solo_cstart = nullptr;

    // profiling
    bool profiling = false;
    std::vector<hipEvent_t> ev;
    std::vector<int> ev_phase;
    std::vector<int> ev_weight;  // traversal intervals: evaluations they contain
    size_t ev_used = 0;
    double phase_ms[kPhases] = {0, 0, 0, 0, 0};
    double trav_ms_sum = 0.0;
    int64_t trav_launches = 0;
    std::vector<double> trav_samples;  // per-launch traversal times of the last call (ms)
    bool timings_pending = false;

    // the collectives this rank issued, in host issue order (bh_collective_log): every rank of a
    // decomposition must issue the same sequence, or RCCL pairs mismatched calls and hangs
    std::vector<int64_t> coll_log;  // (api call, site, bytes, stream) per collective
    int64_t api_calls = 0;          // state-changing API calls made on this engine

    // Failure of a multi-rank call (the reference's join always returns, BHA:408, 426): a rank
    // whose call fails -- or that finds a peer failed, or waits past BH_COMM_TIMEOUT_S -- marks
    // itself failed, aborts its in-process group / RCCL communicator (ncclCommAbort) so that no
    // peer waits for it, and every state-changing call returns BH_E_COMM until bh_reset_bodies
    std::atomic<bool> *abort_flag = nullptr;  // a multi-device handle's members: shared, set by
                                              // any member that failed (multi.cpp)
    bool comm_failed = false;
    bool comm_lost = false;      // the RCCL communicator was aborted (a new one is needed)
    std::string fail_msg;
    int inject_coll = -1;        // bh_debug_inject(100 + k): fail before the k-th next collective
    int inject_barrier = -1;     // bh_debug_inject(200 + k): ... before the k-th next group barrier
    // progress, readable from any thread while a call runs (bh_progress: heartbeats)
    std::atomic<int64_t> prog_api{0}, prog_coll{0};
    std::atomic<int> prog_site{0}, prog_busy{0};

    std::string err;
};

namespace {

#define HIPCHK(e, expr)                                                                  \
    do {                                                                                 \
        hipError_t _st = (expr);                                                         \
        if (_st != hipSuccess) {                                                         \
            (e)->err = std::string(#expr) + ": " + hipGetErrorString(_st);              \
            return BH_E_DEVICE;                                                          \
        }                                                                                \
    } while (0)

#define NCCLCHK(e, expr)                                                                 \
    do {                                                                                 \
        ncclResult_t _st = (expr);                                                       \
        if (_st != ncclSuccess) {                                                        \
            (e)->err = std::string(#expr) + ": " + ncclGetErrorString(_st);              \
            return BH_E_COMM;                                                            \
        }                                                                                \
    } while (0)

#define TRY(expr)                      \
    do {                               \
        int _rc = (expr);              \
        if (_rc != BH_OK) return _rc;  \
    } while (0)

// One collective of a multi-rank engine (RCCL call, or its in-process copies): logged so that
// tests can check that every rank issues the same sequence (bh_collective_log).
enum CollSite {
    COLL_ACC = 1,       // a round of accelerations (full evaluation), in-place all-gather
    COLL_POS = 2,       // a round of new positions (LET evaluation)
    COLL_VEL = 3,       // a round of owners' velocities (before a full build, at a call's end)
    COLL_TABLE = 4,     // the LET cell tables
    COLL_FLAGS = 5,     // the end-of-call LET status words, max all-reduce
    COLL_SETTINGS = 6,  // the per-process settings check at creation (min and max all-reduce)
    COLL_VMAX = 7,      // every rank's drift speed bound (LET selection), after a drifting round
};
enum CollStream { CS_MAIN = 0, CS_COMM = 1 };
// Called before every collective: logs it, counts it for the heartbeat, and trips an injected
// host-side failure (bh_debug_inject(100 + k)) -- the rank then returns before the collective its
// peers have issued, exactly as a rank-local error would.
int coll_log(bh_engine *e, int site, int64_t bytes, int stream) {
    if (e->world <= 1 && !e->comm) return BH_OK;
    if (e->inject_coll >= 0 && e->inject_coll-- == 0) {
        e->err = "injected host-side failure before a collective (bh_debug_inject)";
        return BH_E_COMM;
    }
    e->prog_coll.fetch_add(1);
    e->prog_site.store(site);
    if (e->coll_log.size() >= ((size_t)1 << 22)) return BH_OK;  // (bounded: 1 M entries)
    e->coll_log.insert(e->coll_log.end(), {e->api_calls, (int64_t)site, bytes, (int64_t)stream});
    return BH_OK;
}

bool multi_rank(const bh_engine *e) { return (e->comm || e->group || e->comm_lost) && !e->solo; }

bool peers_aborted(const bh_engine *e) {
    return (e->group && e->group->aborted.load()) || (e->abort_flag && e->abort_flag->load());
}

// An in-process group's barrier, with its way out: false from an aborted group -> BH_E_COMM.
int group_barrier(bh_engine *e) {
    if (e->inject_barrier >= 0 && e->inject_barrier-- == 0) {
        e->err = "injected host-side failure before a group barrier (bh_debug_inject)";
        return BH_E_COMM;
    }
    if (!e->group->barrier()) {
        std::lock_guard<std::mutex> lk(e->group->mu);
        e->err = e->group->timed_out
                     ? "group barrier: a peer did not arrive within BH_COMM_TIMEOUT_S"
                     : "group barrier: aborted (a peer rank's call failed)";
        return BH_E_COMM;
    }
    return BH_OK;
}

// Poll stream s until it is idle, at most `secs` seconds (0: forever).  hipErrorNotReady on expiry.
hipError_t drain_stream(hipStream_t s, double secs) {
    if (!s) return hipSuccess;
    const auto t0 = std::chrono::steady_clock::now();
    for (int spins = 0;; ++spins) {
        const hipError_t q = hipStreamQuery(s);
        if (q != hipErrorNotReady) return q;
        if (secs > 0.0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > secs)
            return hipErrorNotReady;
        if (spins < 2000) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// Abort this rank's RCCL communicator (its kernels waiting for peers exit) and let every stream
// of the engine drain, bounded.  The engine keeps no communicator afterwards (comm_lost).
void abort_comm(bh_engine *e) {
    if (e->comm) {
        (void)ncclCommAbort(e->comm);
        e->comm = nullptr;
        e->comm_lost = true;
    }
    for (hipStream_t s : {e->stream, e->stream2, e->comm_stream, e->pipe_stream, e->mir_stream})
        (void)drain_stream(s, 30.0);
}

// A multi-rank call failed on this rank (rc != BH_OK): mark the engine failed and make sure no
// peer waits for it -- abort the in-process group or the multi-device handle's members (the
// flag every member's waits poll), and this rank's communicator.
int fail_multi_rank(bh_engine *e, int rc) {
    if (rc == BH_OK || !multi_rank(e)) return rc;
    if (!e->comm_failed) e->fail_msg = e->err;
    e->comm_failed = true;
    if (e->group) e->group->abort();
    if (e->abort_flag) e->abort_flag->store(true);
    abort_comm(e);
    return rc;
}

// Wait until stream s is idle.  Multi-rank engines poll: a collective whose peers never arrive
// would block a plain hipStreamSynchronize forever.  With RCCL the wait ends -- the communicator
// aborted, BH_E_COMM -- on an asynchronous RCCL error, when another member of the handle failed,
// or after BH_COMM_TIMEOUT_S; an in-process group's device waits are on recorded events and
// always end (its barriers carry the abort), so it only gets the deadline.
int wait_stream(bh_engine *e, hipStream_t s) {
    if (!multi_rank(e)) {
        HIPCHK(e, hipStreamSynchronize(s));
        return BH_OK;
    }
    const double limit = comm_timeout_s();
    const auto t0 = std::chrono::steady_clock::now();
    const char *why = nullptr;
    for (int spins = 0;; ++spins) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) return BH_OK;
        if (q != hipErrorNotReady) {
            e->err = std::string("hipStreamQuery: ") + hipGetErrorString(q);
            return BH_E_DEVICE;
        }
        if (e->comm) {
            ncclResult_t ar = ncclSuccess;
            if (ncclCommGetAsyncError(e->comm, &ar) == ncclSuccess && ar != ncclSuccess &&
                ar != ncclInProgress)
                why = "RCCL reported an asynchronous error";
            else if (e->abort_flag && e->abort_flag->load())
                why = "another member of the handle failed";
        }
        if (!why && limit > 0.0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit)
            why = "timed out (BH_COMM_TIMEOUT_S) waiting for the device: a collective whose peers "
                  "never arrived?";
        if (why) break;
        if (spins < 2000) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    e->err = std::string("wait for the device: ") + why;
    abort_comm(e);
    return BH_E_COMM;
}

#define SYNC(e, s) TRY(wait_stream((e), (s)))

// Root cell (BHA:360-361) and the exact per-depth half-sizes (BHA:74).
int make_geometry(const bh_params &p, Geometry &g, std::string &err) {
    if (p.width_px <= 0 || p.height_px <= 0) {
        err = "width_px and height_px must be positive";
        return BH_E_INVALID;
    }
    std::memset(&g, 0, sizeof(g));
    const int W = p.width_px, H = p.height_px;
    g.root_cx = (double)W / 2.0;
    g.root_cy = (double)H / 2.0;
    g.root_h = (double)std::max(W, H) / 2.0 + 2.0;
    g.h[0] = g.root_h;
    for (int d = 1; d < MAX_DEPTH_TAB; ++d) g.h[d] = g.h[d - 1] / 2.0;
    int J = -1;
    for (int d = 0; d < MAX_DEPTH_TAB; ++d)
        if (g.h[d] < 1e-3) {
            J = d;
            break;
        }
    if (J < 1 || J > 30 || J + 3 > MAX_DEPTH_TAB) {
        err = "root cell too large for 64-bit Morton keys (jitter depth > 30)";
        return BH_E_INVALID;
    }
    g.J = J;
    for (int d = 0; d < MAX_DEPTH_TAB; ++d) {
        double s = g.h[d] * 2.0;  // BHA:226
        g.s2[d] = s * s;
    }
    return BH_OK;
}

template <typename T>
int dev_alloc(bh_engine *e, T *&ptr, size_t count) {
    if (ptr) {
        (void)hipFree(ptr);
        ptr = nullptr;
    }
    if (count == 0) count = 1;
    HIPCHK(e, hipMalloc((void **)&ptr, count * sizeof(T)));
    return BH_OK;
}

int alloc_state(bh_engine *e, BodyState &s, size_t cap) {
    TRY(dev_alloc(e, s.x, cap));
    TRY(dev_alloc(e, s.y, cap));
    TRY(dev_alloc(e, s.vx, cap));
    TRY(dev_alloc(e, s.vy, cap));
    TRY(dev_alloc(e, s.m, cap));
    TRY(dev_alloc(e, s.cidx, cap));
    return BH_OK;
}

size_t node_capacity(int64_t n, int J) {
    // T = sum_a (1 + max(0, c(a) - c(a-1))) <= n + (J+1) * (n/2 + 2)
    return (size_t)n + (size_t)(J + 1) * ((size_t)n / 2 + 2) + 16;
}

// Capacity for n bodies.  Growing drops the live state (callers reset it); a change of the
// jitter depth J only re-sizes the tree workspace.
int ensure_capacity(bh_engine *e, int64_t n) {
    const int J = e->geo.J;
    if (n <= e->cap && J == e->J_alloc) return BH_OK;
    const int64_t cap = std::max<int64_t>(n, std::max<int64_t>(e->cap, 1));
    if (n > e->cap || !e->st.x) {
        TRY(alloc_state(e, e->st, cap));
        TRY(alloc_state(e, e->alt, cap));
        // multi-GPU: rounds x world pieces of whole wavefronts (bh_shard_range)
        const int64_t padded = (e->comm || e->group || e->solo) ? shard_sub(cap, e->world, BH_SHARD_ROUNDS) *
                                             e->world * BH_SHARD_ROUNDS
                                       : cap;
        TRY(dev_alloc(e, e->a2, 2 * padded));
        TRY(dev_alloc(e, e->ax, cap));
        TRY(dev_alloc(e, e->ay, cap));
        TRY(dev_alloc(e, e->keys, cap));
        TRY(dev_alloc(e, e->keys_s, cap));
        TRY(dev_alloc(e, e->keys32, cap));
        TRY(dev_alloc(e, e->keys32_s, cap));
        TRY(dev_alloc(e, e->idx, cap));
        TRY(dev_alloc(e, e->perm, cap));
        TRY(dev_alloc(e, e->perm2, cap));
        TRY(dev_alloc(e, e->cpl, cap + 32));  // slack for word-wise scans
        TRY(dev_alloc(e, e->cnt, cap + 1));
        TRY(dev_alloc(e, e->base, cap + 1));
        TRY(dev_alloc(e, e->visits32, cap));
        TRY(dev_alloc(e, e->contrib32, cap));
        TRY(dev_alloc(e, e->lanes, cap));
        e->lanes_valid = e->lr_pending = e->lr_ready = false;
        e->inv_valid = false;
        TRY(dev_alloc(e, e->wave_iters, cap / 64 + 2));
        TRY(dev_alloc(e, e->wave_blocks, cap / 64 + 2));
        e->cost_stride = cap / 64 + 2;
        e->order_stride = (int64_t)wave_order_runs(cap) + 1;
        TRY(dev_alloc(e, e->wave_cost, (size_t)(e->cost_stride * (1 + BH_SHARD_ROUNDS))));
        HIPCHK(e, hipMemsetAsync(e->wave_cost, 0,
                                 sizeof(uint32_t) * (size_t)(e->cost_stride * (1 + BH_SHARD_ROUNDS)),
                                 e->stream));
        TRY(dev_alloc(e, e->run_order, (size_t)(e->order_stride * (1 + BH_SHARD_ROUNDS))));
        for (int64_t &o : e->order_n) o = 0;
        TRY(dev_alloc(e, e->heavy, cap));
        TRY(dev_alloc(e, e->keep, cap));
        TRY(dev_alloc(e, e->pos, cap));
        TRY(dev_alloc(e, e->spl, (size_t)sort_buckets(cap) + 2));
        TRY(dev_alloc(e, e->bcount, (size_t)sort_buckets(cap) + 2));
        TRY(dev_alloc(e, e->bstart, (size_t)sort_buckets(cap) + 2));
        HIPCHK(e, hipMemsetAsync(e->bcount, 0, sizeof(uint32_t) * ((size_t)sort_buckets(cap) + 2),
                                 e->stream));
        e->spl_nb = 0;
        e->keys_ready = false;
        e->cap = cap;
    }
    size_t ncap = node_capacity(e->cap, J);
    if (ncap > e->node_cap || J != e->J_alloc) {
        TRY(dev_alloc(e, e->nodes, ncap));
        TRY(dev_alloc(e, e->span_list, (size_t)(J + 2) * span_stride_for(e->cap)));
        TRY(dev_alloc(e, e->span_children, (size_t)(J + 2) * span_stride_for(e->cap)));
        TRY(dev_alloc(e, e->super_list,
                      (size_t)(J + 2) * span_groups(span_stride_for(e->cap))));
        TRY(dev_alloc(e, e->cell_start,
                      ((size_t)1 << (2 * std::min(J, CELL_TABLE_MAX_DEPTH))) + 2));
        e->node_cap = ncap;
        e->J_alloc = J;
    }
    size_t cb = std::max(tree_scratch_bytes(e->cap, J), compact_scratch_bytes(e->cap));
    cb = std::max(cb, let_scratch_bytes(e->cap));
    if (cb > e->scratch_bytes) {
        if (e->scratch) (void)hipFree(e->scratch);
        e->scratch = nullptr;
        HIPCHK(e, hipMalloc(&e->scratch, cb));
        e->scratch_bytes = cb;
    }
    return BH_OK;
}

TreeBuffers tree_buffers(bh_engine *e) {
    TreeBuffers b;
    b.src = e->st;
    b.dst = e->alt;
    b.keys = e->keys;
    b.keys_s = e->keys_s;
    b.keys32 = e->keys32;
    b.keys32_s = e->keys32_s;
    b.idx = e->idx;
    b.perm = e->perm;
    b.cpl = e->cpl;
    b.cnt = e->cnt;
    b.base = e->base;
    b.cell_start = e->cell_start;
    b.nodes = e->nodes;
    b.scalars = e->scalars;
    b.span_list = e->span_list;
    b.span_stride = span_stride_for(e->cap);
    b.span_children = e->span_children;
    b.super_list = e->super_list;
    b.scratch = e->scratch;
    b.scratch_bytes = e->scratch_bytes;
    b.spl = e->spl;
    b.spl_nb = e->spl_nb;
    b.bcount = e->bcount;
    b.bstart = e->bstart;
    return b;
}

// ---- profiling events ----------------------------------------------------------------
// weight: force evaluations inside a traversal interval (the deep pipeline's holds two)
int mark(bh_engine *e, int phase, int weight = 1) {  // close the interval of `phase` begun at the last mark
    if (!e->profiling) return BH_OK;
    // phases are contiguous on the stream: the previous phase's end mark starts the next one
    if (phase < 0 && e->ev_used > 0) return BH_OK;
    if (e->ev_used + 1 > e->ev.size()) {
        // timing-only events: a device-scope release, no system-scope fence (the default one
        // writes back and invalidates the caches: ~10 us of idle GPU per event in the step)
        hipEvent_t ev;
        if (hipEventCreateWithFlags(&ev, hipEventDisableSystemFence) != hipSuccess) {
            (void)hipGetLastError();
            HIPCHK(e, hipEventCreate(&ev));
        }
        e->ev.push_back(ev);
        e->ev_phase.push_back(-1);
        e->ev_weight.push_back(1);
    }
    HIPCHK(e, hipEventRecord(e->ev[e->ev_used], e->stream));
    e->ev_phase[e->ev_used] = phase;  // phase of the interval ending here (-1: start marker)
    e->ev_weight[e->ev_used] = weight;
    ++e->ev_used;
    e->timings_pending = true;
    return BH_OK;
}

int collect_timings(bh_engine *e) {
    if (!e->timings_pending) return BH_OK;
    SYNC(e, e->stream);
    for (int k = 0; k < kPhases; ++k) e->phase_ms[k] = 0.0;
    e->trav_ms_sum = 0.0;
    e->trav_launches = 0;
    e->trav_samples.clear();
    for (size_t i = 1; i < e->ev_used; ++i) {
        int ph = e->ev_phase[i];
        if (ph < 0) continue;
        float ms = 0.f;
        HIPCHK(e, hipEventElapsedTime(&ms, e->ev[i - 1], e->ev[i]));
        e->phase_ms[ph] += ms;
        if (ph == 1) {  // per evaluation: an interval holding w evaluations counts w times
            const int w = e->ev_weight[i];
            e->trav_ms_sum += ms;
            e->trav_launches += w;
            for (int j = 0; j < w; ++j) e->trav_samples.push_back(ms / w);
        }
    }
    e->timings_pending = false;
    return BH_OK;
}

// The pipelined step's first traversal also computes the second build's Morton keys and
// bucket counts (KICK_DRIFT epilogue, bh_device.hpp MortonFuse).
#ifndef BH_FUSE_KEYS
#define BH_FUSE_KEYS 1
#endif

// ---- buildTree() (BHA:359-366): sort + build; the state moves to the new Morton order ----
#ifndef BH_LANE_REFRESH
// builds between Hilbert re-sorts of the lane map (0: Morton lanes).  With the re-sort beside the
// first traversal (BH_LANE_DEFER) a fresher map pays: C3 1.84-1.85 ms per step at 16, 1.82-1.83 at
// 8, 1.814-1.820 at 6, 1.82-1.83 at 4 (round 4, profiles/r04L2_lane_refresh_ab.txt)
#define BH_LANE_REFRESH 6
#endif
#ifndef BH_LANE_REFRESH_SHARDED
#define BH_LANE_REFRESH_SHARDED 16  // multi-rank engines (no pipelined step: the re-sort is in line)
#endif
#ifndef BH_LANE_DEFER
#define BH_LANE_DEFER 1  // pipelined steps re-sort beside the first traversal (lane_refresh_beside)
#endif
// overlap: the pipelined step's build on stream `s` -- into nodes_alt and alt without the
// velocities (permute_velocities follows) and without the final swap (the caller swaps)
// overlap: the pipelined step's next tree, built beside the second traversal into nodes_alt /
// alt with its own permutation (perm2; the traversal reads perm), velocities left to
// permute_velocities.  keep_v: the velocities stay in the previous slot order (in alt after the
// swap) for a traversal that permutes them as it kicks (KickArgs::perm).
// carry: a call's last overlapped build, whose tree the next call uses -- its error flags go to
// scalars[10] instead of the running call's scalars[1] (evaluate / bh_get_quads take them over)
#ifndef BH_HEAVY_CARRY
#define BH_HEAVY_CARRY 1  // the pipelined step's second build lists the heavy bodies (k_prep)
#endif
// heavy_list: k_prep lists the merge rule's heavy bodies in this build's order (the rule follows
// the build before any other build: masses change only in the rule, BHA:518)
int build_into(bh_engine *e, hipStream_t s, bool overlap, bool keep_v = false, bool carry = false,
               bool heavy_list = false) {
    const int64_t n = e->n;
    TreeBuffers tb = tree_buffers(e);
    if (heavy_list && e->heavy_dirty)  // (a list no rule consumed: a call that failed between)
        HIPCHK(e, hipMemsetAsync(e->scalars + 14, 0, sizeof(uint32_t), s));
    e->heavy_ready = heavy_list && n > 0;
    if (e->heavy_ready) {
        e->heavy_dirty = true;
        tb.heavy = e->heavy;
        tb.heavy_count = e->scalars + 14;
        tb.heavy_thr = e->p.merge_max_mass;
    }
    if (overlap) {
        tb.src.vx = tb.src.vy = nullptr;
        tb.nodes = e->nodes_alt;
        tb.perm = e->perm2;
    }
    if (carry) tb.scalars = e->scalars + 9;  // (the build writes scalars[1] of its buffers)
    if (keep_v) tb.src.vx = tb.src.vy = nullptr;
    // Hilbert waves (every rank alike): re-sorted every BH_LANE_REFRESH builds, carried through
    // the build's permutation by k_emit_com in between
    const bool use_lanes = BH_LANE_REFRESH > 0 && n > 0 && e->p.theta != 0.0;
    const int every = (e->comm || e->group || e->solo) ? BH_LANE_REFRESH_SHARDED : BH_LANE_REFRESH;
    const bool due = use_lanes && e->lanes_valid && e->lanes_age >= every;
    // (pipelined steps: the re-sort is left to the next first traversal's side, see
    // lane_refresh_beside; the map is carried through this build meanwhile)
    const bool defer = due && BH_LANE_DEFER && ((overlap && e->lane_defer) || e->lane_hold);
    const bool refresh = use_lanes && (!e->lanes_valid || (due && !defer));
    tb.lanes_remap = use_lanes && !refresh ? e->lanes : nullptr;
    // the second traversal's copies made by the build (k_emit_com) instead of k_trav_inputs --
    // not when the map is re-sorted after the build (lane_order rewrites it)
    e->tc_done = e->tc_want && n > 0 && !refresh;
    if (e->tc_done) {
        tb.tc.m = e->m_trav;
        tb.tc.cidx = e->cidx_trav;
        tb.tc.lanes = tb.lanes_remap ? e->lanes_trav : nullptr;
        tb.tc.T = e->T_trav;
        tb.tc.box_header = e->tc_box;
    }
    tb.keys_ready = e->keys_ready && !overlap;
    e->keys_ready = false;
    if (!overlap) e->mir_fresh = false;  // the jitter may move bodies
    HIPCHK(e, tree_build(tb, n, e->geo, s));
    if (e->inject_build >= 0 && e->inject_build-- == 0) {  // bh_debug_inject(2 + k)
        take_u32(tb.scalars + 1, e->scalars + 11, s, 1u);
        HIPCHK(e, hipGetLastError());
    }
    ++e->full_builds;
    e->inv_valid = false;  // the map follows this build's permutation
    if (use_lanes) {
        if (refresh) HIPCHK(e, lane_order(tb, n, e->geo.J, true, e->lanes, s));
        e->lanes_valid = true;
        e->lanes_age = refresh ? 1 : e->lanes_age + 1;
        if (defer && overlap) e->lr_pending = true;
    } else {
        e->lanes_valid = e->lr_pending = e->lr_ready = false;  // this build's permutation was not applied to the map
    }
    e->spl_nb = sort_buckets(n);  // k_prep wrote this build's splitters
    e->st_morton = true;
    if (overlap) return BH_OK;
    if (n > 0) std::swap(e->st, e->alt);
    if (e->solo && n > 0 && e->p.theta != 0.0) {  // the peers' cell values for later LET builds
        if (!e->solo_table) {
            TRY(dev_alloc(e, e->solo_table, LET_TSTRIDE));
            HIPCHK(e, hipMemsetAsync(e->solo_table, 0, sizeof(LetCell) * LET_TSTRIDE, e->stream));
            TRY(dev_alloc(e, e->solo_all, LET_CELLS));
            TRY(dev_alloc(e, e->solo_cstart, LET_CELLS + 1));
            HIPCHK(e, hipMemsetAsync(e->solo_all, 1, LET_CELLS, e->stream));
        }
        LetBufs Ls{};
        Ls.ecell = e->solo_all;
        Ls.cstart = e->solo_cstart;
        Ls.table = e->solo_table;
        TreeBuffers tm = tree_buffers(e);
        tm.dst = e->st;  // the sorted state
        HIPCHK(e, let_table(n, e->geo, Ls, tm, e->stream));
    }
    e->tree_valid = true;
    return BH_OK;
}

// The velocities left in the previous slot order by a pipelined step (vel_perm) -> st, for any
// reader other than the next step's first kick (materialize_positions calls it: every reader of
// the replica outside the step does that first).
#ifndef BH_FOLD_VEL_PERM
#define BH_FOLD_VEL_PERM 1
#endif
int materialize_velocities(bh_engine *e) {
    if (!e->vel_perm) return BH_OK;
    permute_velocities(e->n, e->vel_perm, e->alt.vx, e->alt.vy, e->st.vx, e->st.vy, e->stream);
    e->vel_perm = nullptr;
    HIPCHK(e, hipGetLastError());
    return BH_OK;
}

int build(bh_engine *e) {
    TRY(materialize_velocities(e));
    return build_into(e, e->stream, false);
}

// theta = 0 workspace: flags per node slot, selected indices and the leaf list per body.
int ensure_direct(bh_engine *e) {
    if (e->leaf_node_cap == e->node_cap && e->leaf_cap == e->cap) return BH_OK;
    TRY(dev_alloc(e, e->leaf_flags, e->node_cap));
    TRY(dev_alloc(e, e->leaf_sel, (size_t)e->node_cap));
    TRY(dev_alloc(e, e->leaf_count, 1));
    TRY(dev_alloc(e, e->leaf_cover, 2 * ((size_t)e->node_cap + 1)));
    TRY(dev_alloc(e, e->leaves.rec, 4 * (size_t)e->cap));  // (x, y, m, slot) per leaf
    const size_t tb = leaf_select_bytes((int64_t)e->node_cap);
    if (e->leaf_tmp) (void)hipFree(e->leaf_tmp);
    e->leaf_tmp = nullptr;
    HIPCHK(e, hipMalloc(&e->leaf_tmp, tb));
    e->leaf_tmp_bytes = tb;
    e->leaf_node_cap = e->node_cap;
    e->leaf_cap = e->cap;
    return BH_OK;
}

// The previous call's carried tree is used now: its build's error flags become this call's.
int take_carried_flags(bh_engine *e) {
    if (!e->carried_flags) return BH_OK;
    e->carried_flags = false;
    take_u32(e->scalars + 1, e->scalars + 10, e->stream);
    HIPCHK(e, hipGetLastError());
    return BH_OK;
}

// ... or it is dropped unused (resetBodies, a root-cell change, a replay).
int drop_carried_flags(bh_engine *e) {
    if (!e->carried_flags) return BH_OK;
    e->carried_flags = false;
    HIPCHK(e, hipMemsetAsync(e->scalars + 10, 0, sizeof(uint32_t), e->stream));
    return BH_OK;
}

// ---- one force evaluation: buildTree() + computeAccelerations() (BHA:359-395) -------------
// theta == 0 (config C5): the criterion never accepts (BHA:226-228), so the force is the
// direct sum over the tree's non-empty leaves in pre-order -- run by the all-pairs kernel
// (direct.hip) on the leaf list instead of the tree walk; bit-identical either way.  The
// visit-counting diagnostic keeps the walk (it counts internal nodes too).
//
// Multi-GPU (e->comm): BH_SHARD_ROUNDS rounds; round k evaluates this rank's piece of the
// Morton order (bh_shard_range) on the compute stream, then the pieces of round k are
// all-gathered in place on the comm stream while round k + 1 is evaluated; the compute
// stream waits for the last gather before the kick.  Pieces of different rounds and ranks
// are disjoint, so the concurrent writes never overlap.
// kick (one GPU, tree walk): the following KDK update is fused into the traversal's epilogue
// and *fused is set; otherwise the caller runs the integration kernel on a2.
#ifndef BH_FUSE_KICK
#define BH_FUSE_KICK 1
#endif
#ifndef BH_ROUND_WEIGHTS
#define BH_ROUND_WEIGHTS 1, 1, 1, 1  // relative sizes of a rank's rounds (BH_ROUND_FRACS)
#endif

// ---- multi-rank: the build as a locally essential tree (let.hip) ----------------------
int pinned_reserve(bh_engine *e, size_t bytes);
#ifndef BH_LET_FUSE_KEYS
#define BH_LET_FUSE_KEYS 1  // the subset gather writes the LET build's keys and buckets
#endif
#ifndef BH_LET_REFRESH
#define BH_LET_REFRESH 32  // LET builds between full builds (the replicated Morton order)
#endif
// s: the stream the set is built on next (the fills of fresh buffers are ordered before it: a
// plain hipMemset is not ordered with the engine's non-blocking streams)
int let_alloc(bh_engine *e, int64_t n_sub, hipStream_t s = nullptr) {
    if (!s) s = e->stream;
    const int J = e->geo.J;
    if (e->let_cap < e->cap || !e->L.ecell) {  // the selection's per-body and per-cell arrays
        const int64_t cap = e->cap;
        LetBufs &L = e->L;
        TRY(dev_alloc(e, L.ecell, LET_CELLS));
        TRY(dev_alloc(e, L.hcell, LET_CELLS));
        TRY(dev_alloc(e, L.flag_all, 1));
        TRY(dev_alloc(e, L.flag8, cap));
        TRY(dev_alloc(e, L.sel, let_sel_blocks(cap) + 2));
        TRY(dev_alloc(e, L.selpos, let_sel_blocks(cap) + 2));
        TRY(dev_alloc(e, e->inv_lanes, cap));
        e->inv_valid = false;
        TRY(dev_alloc(e, L.own, cap));
        TRY(dev_alloc(e, L.own_blk, let_sel_blocks(cap) + 2));
        TRY(dev_alloc(e, L.rowmask, 256 * 8));
        TRY(dev_alloc(e, e->let_box, let_sel_blocks(cap) + 2));
        TRY(dev_alloc(e, e->disp, 2 + (size_t)e->world));
        HIPCHK(e, hipMemsetAsync(e->disp, 0, sizeof(double) * (2 + (size_t)e->world), s));
        L.vmax = reinterpret_cast<unsigned long long *>(e->disp + 1);
        L.nvmax = 1 + e->world;
        e->boxes_valid = false;
        e->let_clean = false;  // (new buffers)
        TRY(alloc_state(e, e->sub_src, cap));
        e->let_cap = cap;
    }
    if (e->set_cap < e->cap || !e->L.cstart) {  // this set's per-cell and per-body arrays
        const int64_t cap = e->cap;
        LetBufs &L = e->L;
        TRY(dev_alloc(e, L.cstart, LET_CELLS + 1));
        TRY(dev_alloc(e, L.table, LET_TSTRIDE));
        TRY(dev_alloc(e, L.tables, (size_t)e->world * LET_TSTRIDE));
        // (solo: the tables of ranks 2 .. world-1 stay zero -- nothing tagged -- for good)
        HIPCHK(e, hipMemsetAsync(L.tables, 0, sizeof(LetCell) * (size_t)e->world * LET_TSTRIDE, s));
        TRY(dev_alloc(e, L.levels, ((size_t)1 << (2 * LET_P + 2)) / 3 + 1));
        TRY(dev_alloc(e, L.w, LET_CELLS + 1));
        TRY(dev_alloc(e, L.posc, LET_CELLS + 1));
        TRY(dev_alloc(e, L.bsz, LET_CELLS + 1));
        TRY(dev_alloc(e, L.csrc, LET_CELLS + 1));
        TRY(dev_alloc(e, L.ccnt, LET_CELLS + 1));
        TRY(dev_alloc(e, L.cpos, LET_CELLS + 1));
        TRY(dev_alloc(e, L.lanes, cap));
        TRY(dev_alloc(e, L.subpos, cap));
        if (!e->table_ev) HIPCHK(e, hipEventCreateWithFlags(&e->table_ev, hipEventDisableTiming));
        e->set_cap = cap;
    }
    e->L.scratch = e->scratch;
    e->L.scratch_bytes = e->scratch_bytes;
    if (n_sub <= e->let_sub_cap && J == e->let_J) return BH_OK;
    // the subset's tree workspace, grown with headroom (the subset drifts between builds)
    const int64_t sc = std::min<int64_t>(e->cap, std::max<int64_t>(n_sub + n_sub / 4, 1024));
    TRY(alloc_state(e, e->sub_dst, sc));
    TRY(dev_alloc(e, e->s_keys, sc));
    TRY(dev_alloc(e, e->s_keys_s, sc));
    TRY(dev_alloc(e, e->s_keys32, sc));
    TRY(dev_alloc(e, e->s_keys32_s, sc));
    TRY(dev_alloc(e, e->s_idx, sc));
    TRY(dev_alloc(e, e->s_perm, sc));
    TRY(dev_alloc(e, e->s_cpl, sc + 32));
    TRY(dev_alloc(e, e->s_cnt, sc + 1));
    TRY(dev_alloc(e, e->s_base, sc + 1));
    TRY(dev_alloc(e, e->s_cell_start, ((size_t)1 << (2 * std::min(J, CELL_TABLE_MAX_DEPTH))) + 2));
    const size_t ncap = node_capacity(sc, J);
    TRY(dev_alloc(e, e->s_nodes, ncap));
    e->let_node_cap = ncap + 2 * (size_t)LET_CELLS + 64;
    TRY(dev_alloc(e, e->L.nodes, e->let_node_cap));
    e->L.node_cap = (uint32_t)std::min<size_t>(e->let_node_cap, 0xFFFFFFF0u);
    TRY(dev_alloc(e, e->s_span_list, (size_t)(J + 2) * span_stride_for(sc)));
    TRY(dev_alloc(e, e->s_span_children, (size_t)(J + 2) * span_stride_for(sc)));
    TRY(dev_alloc(e, e->s_super_list, (size_t)(J + 2) * span_groups(span_stride_for(sc))));
    TRY(dev_alloc(e, e->s_spl, (size_t)sort_buckets(sc) + 2));
    TRY(dev_alloc(e, e->s_bcount, (size_t)sort_buckets(sc) + 2));
    TRY(dev_alloc(e, e->s_bstart, (size_t)sort_buckets(sc) + 2));
    HIPCHK(e, hipMemsetAsync(e->s_bcount, 0, sizeof(uint32_t) * ((size_t)sort_buckets(sc) + 2), s));
    e->s_spl_nb = 0;
    e->let_sub_cap = sc;
    e->let_J = J;
    return BH_OK;
}

TreeBuffers let_tree_buffers(bh_engine *e) {
    TreeBuffers b;
    b.src = e->sub_src;
    b.src.vy = nullptr;  // (a subset's vx carries the replicated slot; its vy is never read)
    b.dst = e->sub_dst;
    b.keys = e->s_keys;
    b.keys_s = e->s_keys_s;
    b.keys32 = e->s_keys32;
    b.keys32_s = e->s_keys32_s;
    b.idx = e->s_idx;
    b.perm = e->s_perm;
    b.cpl = e->s_cpl;
    b.cnt = e->s_cnt;
    b.base = e->s_base;
    b.cell_start = e->s_cell_start;
    b.nodes = e->s_nodes;
    b.scalars = e->scalars;
    b.span_list = e->s_span_list;
    b.span_stride = span_stride_for(e->let_sub_cap);
    b.span_children = e->s_span_children;
    b.super_list = e->s_super_list;
    b.scratch = e->scratch;
    b.scratch_bytes = e->scratch_bytes;
    b.spl = e->s_spl;
    // the subset is compacted from the Morton-ordered state, nearly sorted: the adaptive bucket
    // sort with the previous LET build's splitters (any splitters partition correctly)
    b.spl_nb = e->s_spl_nb;
    b.bcount = e->s_bcount;
    b.bstart = e->s_bstart;
    return b;
}

// LET subset capacity: the largest subset seen + headroom (a subset beyond it replays the call)
#ifndef BH_LET_HEADROOM_SHIFT
#define BH_LET_HEADROOM_SHIFT 3
#endif
inline int64_t let_capacity(int64_t known) {
    return known + (known >> BH_LET_HEADROOM_SHIFT) + 4096;
}
#ifndef BH_SPL_EXTEND
#define BH_SPL_EXTEND 1
#endif
#ifndef BH_LET_MIN_WORLD
#define BH_LET_MIN_WORLD 2
#endif
bool let_active(const bh_engine *e) {
    return e->let_on && (e->let_forced || e->world >= BH_LET_MIN_WORLD);
}

// Stream of round k (even: the engine's stream; odd: stream2, started after the build).
int round_streams(bh_engine *e) {
    if (!e->stream2) {
        HIPCHK(e, hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking));
        HIPCHK(e, hipEventCreateWithFlags(&e->built_ev, hipEventDisableTiming));
    }
    HIPCHK(e, hipEventRecord(e->built_ev, e->stream));
    HIPCHK(e, hipStreamWaitEvent(e->stream2, e->built_ev, 0));
    return BH_OK;
}

// Round k's in-place all-gather of W doubles per lane on the comm stream (RCCL), or the peers'
// pieces copied in (in-process group: the caller has passed a barrier after every member
// recorded round_ev[ev_round]; ev_round < 0: the peers' events were waited for already).
bool solo_xchg_on() {
    static const bool on = [] {
        const char *v = std::getenv("BH_SOLO_XCHG");
        return v && std::strcmp(v, "0") != 0;
    }();
    return on;
}

int gather_round(bh_engine *e, const GatherLayout &gl, int k, int W, int ev_round, int site) {
    const int64_t size = gl.off[k + 1] - gl.off[k];
    double *piece = e->a2 + W * (int64_t)e->world * gl.off[k];  // round k, rank 0
    if (size <= 0) return BH_OK;
    TRY(coll_log(e, site, (int64_t)sizeof(double) * W * size * e->world, CS_COMM));
    if (e->comm) {
        NCCLCHK(e, ncclAllGather(piece + W * e->rank * size, piece, (size_t)(W * size),
                                 ncclDouble, e->comm, e->comm_stream));
    } else if (e->solo && e->world > 1 && solo_xchg_on()) {
        // measurement only (tools/solo_rank.py): the bytes a rank receives per round, as one
        // device copy of the own piece on the comm stream -- the copy kernel competes for wave
        // slots with the traversal rounds the way the all-gather's kernel would; peers' positions
        // stay where they are (the copy goes to a scratch buffer)
        const int64_t need = (int64_t)W * size * (e->world - 1);
        if (e->solo_xchg_cap < need) {
            TRY(dev_alloc(e, e->solo_xchg, (size_t)need));
            e->solo_xchg_cap = need;
        }
        for (int q = 1; q < e->world; ++q)
            HIPCHK(e, hipMemcpyAsync(e->solo_xchg + (int64_t)W * size * (q - 1),
                                     piece + W * e->rank * size, sizeof(double) * W * size,
                                     hipMemcpyDeviceToDevice, e->comm_stream));
    } else if (e->group) {
        for (int q = 0; q < e->world; ++q) {
            if (q == e->rank) continue;
            bh_engine *peer = e->group->members[q];
            if (ev_round >= 0)
                HIPCHK(e, hipStreamWaitEvent(e->comm_stream, peer->round_ev[ev_round], 0));
            const int64_t off = W * ((int64_t)e->world * gl.off[k] + q * size);
            HIPCHK(e, hipMemcpyAsync(e->a2 + off, peer->a2 + off, sizeof(double) * W * size,
                                     hipMemcpyDeviceToDevice, e->comm_stream));
        }
    }
    return BH_OK;
}

// The positions a sequence of LET evaluations left in the exchange buffer -> the replica (every
// body's slot), before anything but the next selection reads x, y (a full build, the merge rule,
// the copy-out) or reuses a2 (accelerations, the velocity exchange).  A subset overflow (scalars[4],
// the call is replayed) leaves the replica as it was.
int materialize_positions(bh_engine *e) {
    TRY(materialize_velocities(e));
    if (!e->pos_pending) return BH_OK;
    e->pos_pending = false;
    if (e->n <= 0) return BH_OK;
    let_set_pos(e->n, e->pos_lanes, e->a2, e->pos_layout, e->st.x, e->st.y, e->scalars + 4,
                e->stream);
    HIPCHK(e, hipGetLastError());
    return BH_OK;
}

// Velocities after owner-integrated LET evaluations: every rank holds current velocities of its
// own bodies only; before a full build (which permutes and re-assigns the bodies) the owners'
// (vx, vy) are all-gathered once, in the same rounds and slots as the forces.
int sync_velocities(bh_engine *e) {
    if (!e->vel_stale) return BH_OK;
    e->vel_stale = false;
    const int64_t n = e->n;
    if (n <= 0 || e->solo) return BH_OK;  // solo: no peers (their bodies keep their velocities)
    const int R = BH_SHARD_ROUNDS;
    const int64_t sub = shard_sub(n, e->world, R);
    const uint32_t *lanes = e->lanes_valid ? e->lanes : nullptr;
    const LetPieces pc{n, sub, e->world, e->rank, R, lanes};
    const GatherLayout gl = shard_layout(n, e->world);
    if (e->group) {  // peers are done reading our previous pieces
        TRY(group_barrier(e));
        for (bh_engine *peer : e->group->members)
            if (peer != e) HIPCHK(e, hipStreamWaitEvent(e->stream, peer->gathered_ev, 0));
    }
    let_pack_vel(pc, e->st.vx, e->st.vy, e->a2, gl, e->stream);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->round_ev[0], e->stream));
    HIPCHK(e, hipStreamWaitEvent(e->comm_stream, e->round_ev[0], 0));
    if (e->group) TRY(group_barrier(e));
    for (int k = 0; k < R; ++k) TRY(gather_round(e, gl, k, 2, k == 0 ? 0 : -1, COLL_VEL));
    HIPCHK(e, hipEventRecord(e->gathered_ev, e->comm_stream));
    HIPCHK(e, hipStreamWaitEvent(e->stream, e->gathered_ev, 0));
    let_unpack_vel(n, lanes, e->a2, gl, e->st.vx, e->st.vy, e->stream);
    HIPCHK(e, hipGetLastError());
    return BH_OK;
}

// One LET evaluation with its integration (kick: KICK_DRIFT after a(t), KICK_ONLY after
// a(t+dt)); *done = false when it does not apply (the caller builds the full tree).  Each lane
// kicks its own body (velocity in the replicated state, owner only) and sends the body's new
// position -- drifted, or as the build left it (jitter, BHA:146-151) -- so every replica takes
// all positions from the exchange.
int wave_order_for(bh_engine *e, int slot, int64_t lanes, hipStream_t s, WaveOrder &wo);
int wave_order_next(bh_engine *e, int slot, int64_t lanes, hipStream_t s);

// Every rank's LET cell table into L.tables, on stream s.  RCCL: one all-gather on the engine's
// stream.  In-process group: each member publishes its table and event, then copies every
// member's.
int exchange_tables(bh_engine *e, hipStream_t s) {
    const size_t tbytes = sizeof(LetCell) * (size_t)LET_TSTRIDE;
    TRY(coll_log(e, COLL_TABLE, (int64_t)(tbytes * (size_t)e->world), CS_MAIN));
    if (e->comm) {
        NCCLCHK(e, ncclAllGather(e->L.table, e->L.tables, tbytes, ncclUint8, e->comm, s));
    } else if (e->solo) {  // own values first, the rest from the last full build
        HIPCHK(e, hipMemcpyAsync(e->L.tables, e->L.table, tbytes, hipMemcpyDeviceToDevice, s));
        if (e->world > 1 && e->solo_table)
            HIPCHK(e, hipMemcpyAsync(e->L.tables + LET_TSTRIDE, e->solo_table, tbytes,
                                     hipMemcpyDeviceToDevice, s));
    } else {
        // (a member reads the published pointers after the barrier; it publishes again only
        // after the round barriers that follow, which every member passes first)
        e->pub_table = e->L.table;
        e->pub_table_ev = e->table_ev;
        HIPCHK(e, hipEventRecord(e->table_ev, s));
        TRY(group_barrier(e));
        for (int q = 0; q < e->world; ++q) {
            bh_engine *peer = e->group->members[q];
            if (peer != e) HIPCHK(e, hipStreamWaitEvent(s, peer->pub_table_ev, 0));
            HIPCHK(e, hipMemcpyAsync(e->L.tables + (size_t)q * LET_TSTRIDE, peer->pub_table, tbytes,
                                     hipMemcpyDeviceToDevice, s));
        }
    }
    return BH_OK;
}

// Every rank's drift speed bound (its own bodies' max |v| after the kick, L.vmax[0]) into
// L.vmax[1 + rank], on the exchange stream behind the rounds (which it waited for): RCCL, or the
// peers' words copied (in-process group).  A solo rank has no peers: its own word is the bound.
int gather_vmax(bh_engine *e) {
    TRY(coll_log(e, COLL_VMAX, (int64_t)sizeof(unsigned long long) * e->world, CS_COMM));
    if (e->comm) {
        NCCLCHK(e, ncclAllGather(e->L.vmax, e->L.vmax + 1, 1, ncclUint64, e->comm,
                                 e->comm_stream));
    } else if (e->group) {
        for (bh_engine *peer : e->group->members)
            if (peer != e)
                HIPCHK(e, hipMemcpyAsync(e->L.vmax + 1 + peer->rank, peer->L.vmax,
                                         sizeof(unsigned long long), hipMemcpyDeviceToDevice,
                                         e->comm_stream));
    }
    return BH_OK;
}

int evaluate_let(bh_engine *e, KickMode kick, bool *done) {
    *done = false;
    if (kick != KICK_DRIFT && kick != KICK_ONLY) return BH_OK;
    const int64_t n = e->n;
    const double gap2 = let_include_gap2(e->geo, e->p.theta * e->p.theta, e->p.soft2);
    if (gap2 < 0.0 || n <= 0) return BH_OK;
    const int R = BH_SHARD_ROUNDS;
    const int64_t sub = shard_sub(n, e->world, R);
    // the pieces are lane ranges of the Hilbert wave map when it is current (as in the full
    // path), else slot ranges; a2 is written by lane either way
    const uint32_t *lanes = e->lanes_valid ? e->lanes : nullptr;
    const LetPieces pc{n, sub, e->world, e->rank, R, lanes};
    TRY(mark(e, -1));
    if (e->group) {  // peers are done reading our previous table and pieces
        TRY(group_barrier(e));
        for (bh_engine *peer : e->group->members)
            if (peer != e) HIPCHK(e, hipStreamWaitEvent(e->stream, peer->gathered_ev, 0));
    }
    int64_t n_sub = 0;
    {
        TRY(let_alloc(e, 0));
        // subset capacity: the largest subset of the previous call + headroom, no host round trip;
        // a subset beyond it is an overflow every rank sees after the exchange, and bh_step replays
        // the call with the observed size (the first LET build of an engine reads its size once)
        // (the selection writes sub_src, sized for the whole state; padding up to S = n is harmless).
        // Within a call the size follows the previous selection's when its read-back has landed
        // (a contracting cloud's subsets grow by more than the headroom over a 100-step call:
        // round 4 saw one replay of the C4 / 8 call).  Never waited for: a blocking wait here cost
        // 0.2 ms per solo C4 / 8 step (3.67 against 3.43-3.53 ms).
        if (e->let_known > 0 && e->sub_cnt_pending && hipEventQuery(e->sub_cnt_ev) == hipSuccess) {
            e->sub_cnt_pending = false;
            e->let_known = std::max<int64_t>(e->let_known, *e->sub_cnt_h);
        }
        int64_t S = e->let_known > 0 ? std::min<int64_t>(n, let_capacity(e->let_known)) : n;
        PosSrc ps{nullptr, GatherLayout{}, nullptr};
        if (e->pos_pending && lanes != e->pos_lanes) TRY(materialize_positions(e));  // map changed
        if (e->pos_pending) {  // the previous LET evaluation's positions, straight from a2
            if (!e->inv_valid) {  // per lane map: each slot's position in the exchange buffer
                let_gather_slots(n, lanes, e->pos_layout, e->inv_lanes, e->stream);
                HIPCHK(e, hipGetLastError());
                e->inv_valid = true;
            }
            ps = PosSrc{e->a2, e->pos_layout, e->inv_lanes};
        }
        // the subset build's keys and buckets from the gather when its buffers and splitters are
        // those of the previous LET build (same S capacity and J; not the first build, which sorts
        // with rocprim and sizes the subset afterwards)
        // a grown capacity S: splitters for its new padding tail (else one bucket takes it all
        // and sorts it alone: up to 1 ms per build while the call's largest subset still grows)
        if (BH_SPL_EXTEND && e->s_spl_nb > 0 && S <= e->let_sub_cap && e->geo.J == e->let_J &&
            sort_buckets(S) > e->s_spl_nb) {
            extend_splitters(e->s_spl, e->s_spl_nb, sort_buckets(S), e->geo.J, e->stream);
            HIPCHK(e, hipGetLastError());
            e->s_spl_nb = sort_buckets(S);
        }
        MortonFuse mf{};
        const bool fuse = BH_LET_FUSE_KEYS && e->let_known > 0 && e->s_spl_nb > 0 &&
                          S <= e->let_sub_cap && e->geo.J == e->let_J && e->s_keys;
        if (fuse)
            mf = MortonFuse{e->s_keys, e->s_keys32, e->s_spl, e->s_spl_nb, e->s_cnt, e->s_base,
                            e->s_bcount};
        // only the slot blocks that may hold a body of a built cell (LetSweep): the jitter of
        // every build since the boxes moved a body by at most 2 x 2e-3 per axis (BHA:146-151)
        const LetSweep sw{e->let_box, e->disp, 4.0e-3 * (double)(e->builds_since_box + 1),
                          e->boxes_valid};
        HIPCHK(e, let_select(e->st, ps, e->geo, pc, gap2, e->L, e->sub_src, S, e->scalars,
                             e->stream, mf, sw, e->let_clean && e->let_clean_n == n));
        e->let_clean = false;
        ++e->builds_since_box;
        if (e->let_known > 0) {
            if (!e->sub_cnt_h) {
                HIPCHK(e, hipHostMalloc((void **)&e->sub_cnt_h, 64, hipHostMallocDefault));
                HIPCHK(e, hipEventCreateWithFlags(&e->sub_cnt_ev, hipEventDisableTiming));
            }
            HIPCHK(e, hipMemcpyAsync(e->sub_cnt_h, e->L.selpos + let_sel_blocks(n),
                                     sizeof(uint32_t), hipMemcpyDeviceToHost, e->stream));
            HIPCHK(e, hipEventRecord(e->sub_cnt_ev, e->stream));
            e->sub_cnt_pending = true;
        }
        if (e->let_known <= 0) {
            TRY(pinned_reserve(e, 64));
            uint32_t *h = static_cast<uint32_t *>(e->pin);
            HIPCHK(e, hipMemcpyAsync(h, e->L.selpos + let_sel_blocks(n), sizeof(uint32_t), hipMemcpyDeviceToHost,
                                     e->stream));
            SYNC(e, e->stream);
            e->let_known = std::max<int64_t>(h[0], 1);
            S = std::min<int64_t>(n, let_capacity(e->let_known));  // padded above
        }
        TRY(let_alloc(e, S));
        n_sub = S;  // padded: bodies past the real subset are dead
        ++e->let_builds;
        TreeBuffers sb = let_tree_buffers(e);
        sb.keys_ready = fuse && e->s_spl_nb > 0;  // (let_alloc above kept the buffers: S fitted)
        HIPCHK(e, tree_build(sb, n_sub, e->geo, e->stream));
        e->s_spl_nb = sort_buckets(n_sub);  // k_prep wrote this build's splitters
        HIPCHK(e, let_table(n_sub, e->geo, e->L, sb, e->stream));
        TRY(exchange_tables(e, e->stream));
        {
            // bh_debug_inject: a node array of one record makes k_let_guard fire on this rank only,
            // exactly as a broken invariant would (empty tree, idle lanes, replay flag set)
            const uint32_t node_cap = e->L.node_cap;
            if (e->inject_guard) e->L.node_cap = 1u;
            e->inject_guard = false;
            const hipError_t rc = let_assemble(n_sub, e->geo, pc, e->L, sb, e->scalars, e->stream,
                                               &e->let_clean);
            e->let_clean_n = n;
            e->L.node_cap = node_cap;
            HIPCHK(e, rc);
        }
    }
    TRY(mark(e, 0));
    const ForceParams fp{e->p.G, e->p.soft2, e->p.theta * e->p.theta};
    const int W = 2;  // (x, y) per lane
    KickArgs ka{kick == KICK_DRIFT ? KICK_OWN_DRIFT : KICK_OWN_ONLY, e->st.vx, e->st.vy,
                e->p.dt * 0.5, e->p.dt, lanes};  // BHA:412
    const bool bound = kick == KICK_DRIFT && e->boxes_valid;  // the drift's speed bound
    if (bound) ka.vmax = e->L.vmax;
    const GatherLayout gl = shard_layout(n, e->world);
    // measurement: the peers' bodies keep their positions (already in a2 after a LET evaluation)
    if (e->solo && !e->pos_pending) let_fill_pos(n, lanes, e->st.x, e->st.y, e->a2, gl, e->stream);
    TRY(round_streams(e));
    for (int k = 0; k < R; ++k) {
        int64_t lo = 0, hi = 0;
        bh_shard_range(n, e->rank, e->world, k, &lo, &hi);
        hipStream_t rs = (k & 1) ? e->stream2 : e->stream;
        // lane q of the piece writes slot gather_slot(q) = q - lo + gather_slot(lo)
        double *a2r = e->a2 + W * (gather_slot(gl, lo) - lo);
        WaveOrder wo;
        TRY(wave_order_for(e, 1 + k, hi - lo, rs, wo));
        traverse(e->L.nodes, e->let_node_cap, e->L.posc + LET_CELLS, e->sub_dst.x, e->sub_dst.y,
                 e->sub_dst.m, e->sub_dst.cidx, lo, hi, e->geo, fp, a2r, nullptr, rs,
                 &ka, e->L.lanes, &wo);
        HIPCHK(e, hipGetLastError());
        TRY(wave_order_next(e, 1 + k, hi - lo, rs));
        HIPCHK(e, hipEventRecord(e->round_ev[k], rs));
        HIPCHK(e, hipStreamWaitEvent(e->comm_stream, e->round_ev[k], 0));
        if (e->group) TRY(group_barrier(e));
        TRY(gather_round(e, gl, k, W, k, COLL_POS));
    }
    if (bound) TRY(gather_vmax(e));  // behind the last round, on the exchange stream
    TRY(mark(e, 1));
    HIPCHK(e, hipEventRecord(e->gathered_ev, e->comm_stream));
    HIPCHK(e, hipStreamWaitEvent(e->stream, e->gathered_ev, 0));
    if (bound) {  // the bound now covers every rank's drift
        let_disp_add(e->disp, e->L.vmax, e->L.nvmax, e->p.dt, e->stream);
        HIPCHK(e, hipGetLastError());
    }
    TRY(mark(e, 4));
    e->pos_pending = true;  // every body's new position is in a2 (by lane, gather slots)
    e->pos_lanes = lanes;
    e->pos_layout = gl;
    e->vel_stale = true;
    e->a2_lanes = lanes;
    e->a2_layout = gl;
    e->tree_valid = false;  // the full tree was not built
    *done = true;
    return BH_OK;
}

// Longest-first wave dispatch for a one-GPU traversal over all n lanes (traverse.hip).
#ifndef BH_TRAV_LPT
#define BH_TRAV_LPT 0  // measured without gain; the wave durations stay recordable
#endif
// The order for the next launch is made right after each launch (wave_order_next), off the
// traversal's timed interval; a launch over another lane count first makes its own.
// slot: 0 for the one-GPU launch, 1 + k for LET round k; lanes: the launch's lane count.
// Below BH_LPT_MIN_LANES every wave starts at once anyway (8192 wave slots per GPU).
#ifndef BH_LPT_MIN_LANES
#define BH_LPT_MIN_LANES 131072
#endif
int wave_order_for(bh_engine *e, int slot, int64_t lanes, hipStream_t s, WaveOrder &wo) {
    wo = WaveOrder{};
    if (!BH_TRAV_LPT || lanes < BH_LPT_MIN_LANES || wave_order_runs(lanes) == 0) return BH_OK;
    uint32_t *cost = e->wave_cost + slot * e->cost_stride;
    uint32_t *order = e->run_order + slot * e->order_stride;
    if (e->order_n[slot] != lanes) {  // the order must be a permutation of this launch's runs
        HIPCHK(e, wave_order(cost, lanes, order, s));
        e->order_n[slot] = lanes;
    }
    wo.order = order;
    wo.cost = cost;
    return BH_OK;
}

int wave_order_next(bh_engine *e, int slot, int64_t lanes, hipStream_t s) {
    if (!BH_TRAV_LPT || lanes <= 0 || e->order_n[slot] != lanes) return BH_OK;
    HIPCHK(e, wave_order(e->wave_cost + slot * e->cost_stride, lanes,
                         e->run_order + slot * e->order_stride, s));
    return BH_OK;
}

int evaluate(bh_engine *e, uint32_t *visits, KickMode kick = KICK_NONE, bool *fused = nullptr,
             bool allow_let = false, bool *let_used = nullptr) {
    if (fused) *fused = false;
    if (let_used) *let_used = false;
    // (the pieces are ranges of the slot order: spatially compact only once a full build has
    // put the state into Morton order -- after a reset it is the caller's order)
    if (allow_let && !visits && (e->comm || e->group || e->solo) && let_active(e) &&
        e->p.theta != 0.0 &&
        e->st_morton && e->let_age < BH_LET_REFRESH) {
        bool done = false;
        TRY(evaluate_let(e, kick, &done));
        if (done) {
            ++e->let_age;
            if (let_used) *let_used = true;
            if (fused) *fused = true;  // integrated in the evaluation
            return BH_OK;
        }
    }
    e->let_age = 0;
    const int64_t n = e->n;
    bool have_forces = false;  // a(t) on this tree, evaluated ahead by the previous step
    if (e->prebuilt) {  // the pipelined step built this tree (single GPU: nothing deferred)
        e->prebuilt = false;
        TRY(take_carried_flags(e));
        e->view_pending = false;  // its jitter is now part of the state (BHA:146-151)
        e->mir_fresh = false;
        have_forces = e->forces_ready;
    } else {
        TRY(materialize_positions(e));  // the replica's x, y; a2 is free again
        TRY(sync_velocities(e));        // before the full build permutes the state
        TRY(mark(e, -1));
        TRY(build(e));
        if ((e->comm || e->group || e->solo) && let_active(e) && e->p.theta != 0.0 && n > 0) {
            // the LET selections until the next full build scan only the slot blocks whose box
            // (the cells of their bodies now, in this build's slot order) may reach a built cell
            TRY(let_alloc(e, 0));
            let_boxes(n, e->st, e->geo, e->let_box, e->stream);
            HIPCHK(e, hipGetLastError());
            HIPCHK(e, hipMemsetAsync(e->disp, 0, sizeof(double), e->stream));
            e->boxes_valid = true;
            e->builds_since_box = 0;
        }
        TRY(mark(e, 0));
    }
    e->forces_ready = false;
    ForceParams fp{e->p.G, e->p.soft2, e->p.theta * e->p.theta};  // BHA:378
    have_forces = have_forces && fp.G == e->fp_ready.G && fp.soft2 == e->fp_ready.soft2 &&
                  fp.theta2 == e->fp_ready.theta2;
    const uint32_t *d_T = e->base + n;
    const bool direct = fp.theta2 == 0.0 && !visits;
    if (direct) {
        TRY(ensure_direct(e));
        HIPCHK(e, leaf_list_build(e->nodes, d_T, (int64_t)e->node_cap, e->leaf_flags, e->leaf_sel,
                                  e->leaf_count, e->leaves, n, e->leaf_cover, e->leaf_tmp,
                                  e->leaf_tmp_bytes, e->stream));
    }
    const TraverseCounters counters{visits, e->contrib32, e->wave_iters, e->wave_blocks};
    const uint32_t *lanes = e->lanes_valid ? e->lanes : nullptr;  // [lo, hi): lane ranges
    e->a2_lanes = direct ? nullptr : lanes;
    e->a2_layout = GatherLayout{};
    auto forces = [&](int64_t lo, int64_t hi, uint32_t *vis, hipStream_t fs, double *a2) {
        if (direct)
            direct_forces(e->leaves, e->leaf_count, e->st.x, e->st.y, e->st.m, lo, hi, fp.G,
                          fp.soft2, a2, fs);
        else
            traverse(e->nodes, e->node_cap, d_T, e->st.x, e->st.y, e->st.m, e->st.cidx, lo, hi, e->geo, fp,
                     a2, vis ? &counters : nullptr, fs, nullptr, lanes);
    };
    if ((!e->comm && !e->group && !e->solo) || visits) {
        if (BH_FUSE_KICK && kick != KICK_NONE && !direct && !visits && fused) {
            KickArgs ka{kick, e->st.vx, e->st.vy, e->p.dt * 0.5, e->p.dt};
            if (e->vel_perm && kick == KICK_DRIFT && !have_forces) {  // v[p] = old v[perm[p]]
                ka.svx = e->alt.vx;
                ka.svy = e->alt.vy;
                ka.perm = e->vel_perm;
                e->vel_perm = nullptr;
            }
            TRY(materialize_velocities(e));  // (any other path: permuted first)
            // (not into a breadth-first walk: one body per wave would make one bucket-count
            // atomic per body -- C1 'R' 37.6 against 21.2 us for the kick-only walk --, the build's
            // k_morton_count aggregates them per wave)
            if (BH_FUSE_KEYS && e->fuse_keys && kick == KICK_DRIFT && e->spl_nb > 0 && n > 0 &&
                !traverse_is_bfs(e->node_cap, 0, n, KICK_DRIFT, false)) {
                ka.mf = MortonFuse{e->keys, e->keys32, e->spl, e->spl_nb, e->cnt, e->base,
                                   e->bcount};
                e->keys_ready = true;
            }
            e->fuse_keys = false;
            if (have_forces && kick == KICK_DRIFT) {
                // a(t) is in a2 by lane (the previous step's deep pipeline): the epilogue alone
                TRY(mark(e, -1));
                kick_drift_keys(n, e->a2, e->st.x, e->st.y, e->st.vx, e->st.vy, e->st.cidx,
                                ka.dtHalf, ka.dt, lanes, e->geo, ka.mf, e->stream);
                HIPCHK(e, hipGetLastError());
                *fused = true;
                TRY(mark(e, 2));
                return BH_OK;
            }
            WaveOrder wo;
            TRY(wave_order_for(e, 0, n, e->stream, wo));
            traverse(e->nodes, e->node_cap, d_T, e->st.x, e->st.y, e->st.m, e->st.cidx, 0, n, e->geo, fp,
                     e->a2, nullptr, e->stream, &ka, lanes, &wo);
            *fused = true;
            HIPCHK(e, hipGetLastError());
            TRY(mark(e, 1));
            return wave_order_next(e, 0, n, e->stream);
        } else {
            forces(0, n, visits, e->stream, e->a2);
        }
        HIPCHK(e, hipGetLastError());
        TRY(mark(e, 1));
        return BH_OK;
    }
    const int64_t sub = shard_sub(n, e->world, BH_SHARD_ROUNDS);
    if (e->solo)  // measurement: the peers' bodies get no force
        HIPCHK(e, hipMemsetAsync(e->a2, 0, sizeof(double) * 2 * (size_t)(sub * e->world *
                                                                         BH_SHARD_ROUNDS),
                                 e->stream));
    if (e->group) {  // a collective's implicit ordering: peers' copies of our last pieces done
        TRY(group_barrier(e));
        for (bh_engine *peer : e->group->members)
            if (peer != e) HIPCHK(e, hipStreamWaitEvent(e->stream, peer->gathered_ev, 0));
    }
    TRY(round_streams(e));
    const GatherLayout gl = shard_layout(n, e->world);
    e->a2_layout = gl;
    for (int k = 0; k < BH_SHARD_ROUNDS; ++k) {
        int64_t lo = 0, hi = 0;
        bh_shard_range(n, e->rank, e->world, k, &lo, &hi);
        hipStream_t rs = (k & 1) ? e->stream2 : e->stream;
        forces(lo, hi, nullptr, rs, e->a2 + 2 * (gather_slot(gl, lo) - lo));
        HIPCHK(e, hipGetLastError());
        HIPCHK(e, hipEventRecord(e->round_ev[k], rs));
        HIPCHK(e, hipStreamWaitEvent(e->comm_stream, e->round_ev[k], 0));
        if (e->group) TRY(group_barrier(e));  // every member recorded round k
        TRY(gather_round(e, gl, k, 2, k, COLL_ACC));
    }
    TRY(mark(e, 1));
    HIPCHK(e, hipEventRecord(e->gathered_ev, e->comm_stream));
    HIPCHK(e, hipStreamWaitEvent(e->stream, e->gathered_ev, 0));
    TRY(mark(e, 4));
    return BH_OK;
}

int check_tree_flags(bh_engine *e) {
    uint32_t flags = 0;
    HIPCHK(e, hipMemcpyAsync(&flags, e->scalars + 1, sizeof(uint32_t), hipMemcpyDeviceToHost,
                             e->stream));
    SYNC(e, e->stream);
    if (flags) {
        e->err = "jitter replay reached an unsupported geometry (body stayed inside a depth J+1 cell)";
        return BH_E_STATE;
    }
    return BH_OK;
}

// ---- merge rule (BHA:463-532) ---------------------------------------------------------
// Entirely on the device, no host round trip: heavy bodies (m > mergeMaxMass) and every
// (heavy, body) pair closer than mergeMinDist are collected in parallel, then one workgroup
// replays the reference's sequential rule over the pairs sorted by caller index
// (integrate.hip k_merge_replay).  Removed bodies become tombstones that leave the tree, the
// candidate search and the output at once; the state is compacted once per bh_step call
// (finish_merges).  Heavy bodies only gain mass and never appear, so once a call ends with
// none the rule is skipped until the bodies or mergeMaxMass change.
int pinned_reserve(bh_engine *e, size_t bytes) {
    if (bytes <= e->pin_bytes) return BH_OK;
    if (e->pin) (void)hipHostFree(e->pin);
    e->pin = nullptr;
    size_t nb = std::max<size_t>(bytes, 1 << 16);
    // coherent: kernels write their small results here directly (finish_merges' read-back)
    HIPCHK(e, hipHostMalloc(&e->pin, nb, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(e, hipHostGetDevicePointer(&e->pin_dev, e->pin, 0));
    e->pin_bytes = nb;
    return BH_OK;
}

int merge_bufs(bh_engine *e) {
    // two candidate pairs per body, or what an overflowing step needed (bh_step's retry)
    const uint32_t cap = (uint32_t)std::min<int64_t>(
        0xFFFFFFF0ll, std::max<int64_t>({1 << 16, 2 * e->cap, (int64_t)e->box_need}));
    if (!e->box || e->box_cap < cap) {
        e->box_cap = cap;
        TRY(dev_alloc(e, e->box, (size_t)cap + 1));
        TRY(dev_alloc(e, e->rkeys, 2 * (size_t)cap));
        TRY(dev_alloc(e, e->ridx, 2 * (size_t)cap));
    }
    if (e->dlog_cap < e->cap) {  // at most every body is removed within one call
        TRY(dev_alloc(e, e->dlog, (size_t)e->cap + 1));
        TRY(dev_alloc(e, e->dead_sorted, (size_t)e->cap + 1));
        TRY(dev_alloc(e, e->mbits, ((size_t)e->cap >> 5) + 2));
        TRY(dev_alloc(e, e->mslot, (size_t)e->cap + 1));
        e->dlog_cap = e->cap;
    }
    return BH_OK;
}

// s: the engine's stream, or pipe_stream in the pipelined step (no phase marks there)
// header_zeroed: the caller cleared the mailbox header on an earlier stream position (the
// pipelined step does it before the second traversal, where a fill kernel is not starved)
int merge(bh_engine *e, hipStream_t s = nullptr, bool header_zeroed = false) {
    if (e->p.merge_min_dist <= 0.0 || e->n <= 1 || !e->heavy_possible) return BH_OK;  // BHA:465
    const bool marks = !s;
    if (!s) s = e->stream;
    TRY(materialize_positions(e));
    if (marks) TRY(mark(e, -1));
    TRY(merge_bufs(e));
    const double minD2 = e->p.merge_min_dist * e->p.merge_min_dist;  // BHA:468
    uint32_t *hc = e->heavy_ready ? e->scalars + 14 : nullptr;  // listed by the last build
    e->heavy_ready = false;
    if (hc) e->heavy_dirty = false;  // (k_merge_replay clears the count)
    merge_candidates(e->n, e->st.x, e->st.y, e->st.m, e->st.cidx, e->p.merge_max_mass, minD2,
                     e->heavy, e->box, e->box_cap, s, header_zeroed, hc);
    merge_replay(e->box, e->box_cap, e->st.m, e->st.cidx, e->scalars, e->dlog, e->rkeys, e->ridx,
                 e->mbits, e->mslot, e->n, s, hc);
    HIPCHK(e, hipGetLastError());
    e->merge_ran = true;
    if (marks) TRY(mark(e, 3));
    return BH_OK;
}

// End of a bh_step call (the stream is idle): read the removal count, compact the state and
// renumber caller indices; record the removals for bh_last_removed.  *overflow receives the
// candidate count of a step whose pairs did not fit the mailbox (nothing is compacted then:
// the call is replayed from its snapshot with a larger mailbox, see bh_step).
// *tree_flags receives scalars[1] (the builds' error flags) when the merge rule ran (the same
// read-back), else *have_flags stays false.
int finish_merges(bh_engine *e, uint32_t *overflow, uint32_t *tree_flags = nullptr,
                  bool *have_flags = nullptr) {
    *overflow = 0;
    e->removed.clear();
    if (!e->merge_ran) return BH_OK;
    e->merge_ran = false;
    TRY(materialize_positions(e));
    // one round trip: the counts, the mailbox header and the first DLOG_AHEAD removals (a step
    // removes tens of bodies at C3) come back together
    constexpr uint32_t DLOG_AHEAD = 4096;
    TRY(pinned_reserve(e, 64 + 2 * sizeof(uint32_t) * DLOG_AHEAD));
    uint32_t *h = static_cast<uint32_t *>(e->pin);
    uint32_t *hlog = h + 16, *hsorted = h + 16 + DLOG_AHEAD;
    // (one kernel writes it all into the pinned buffer: no copies -- four were four blit kernels,
    // and a DMA copy queued behind the mirror's 40 MB on the same engine, round 4 trace)
    const uint32_t ahead = (uint32_t)std::min<int64_t>(DLOG_AHEAD, e->dlog_cap);
    pack_readback(e->scalars, e->box, e->dlog, ahead, static_cast<uint32_t *>(e->pin_dev),
                  e->stream);
    HIPCHK(e, hipGetLastError());
    SYNC(e, e->stream);
    if (tree_flags) *tree_flags = h[1];
    if (have_flags) *have_flags = true;
    const uint32_t nd = h[2];
    const uint32_t nd_before_last = h[12];  // removals before the call's last merge rule
    const MergeHeader hdr = *reinterpret_cast<const MergeHeader *>(h + 4);
    if (h[3]) {
        *overflow = h[3];
        return BH_OK;
    }
    if (hdr.heavies == 0) e->heavy_possible = false;
    if (nd == 0) return BH_OK;
    std::vector<uint32_t> dead(nd);
    if (nd <= ahead) {
        std::memcpy(dead.data(), hlog, 4 * (size_t)nd);
    } else {
        HIPCHK(e, hipMemcpy(dead.data(), e->dlog, 4 * (size_t)nd, hipMemcpyDeviceToHost));
    }
    std::sort(dead.begin(), dead.end());
    if (nd <= DLOG_AHEAD) {  // from pinned memory, in stream order: no wait
        std::memcpy(hsorted, dead.data(), 4 * (size_t)nd);
        HIPCHK(e, hipMemcpyAsync(e->dead_sorted, hsorted, 4 * (size_t)nd, hipMemcpyHostToDevice,
                                 e->stream));
    } else {
        HIPCHK(e, hipMemcpy(e->dead_sorted, dead.data(), 4 * (size_t)nd, hipMemcpyHostToDevice));
    }
    const int64_t n = e->n;
    if (e->view_pending) {  // the caller-visible state (the previous order) loses the same bodies
        HIPCHK(e, compact_state(n, e->keep, e->view, e->alt, e->dead_sorted, nd, e->pos,
                                e->scratch, e->scratch_bytes, e->stream));
        std::swap(e->view, e->alt);
    }
    // (a prebuilt tree stays valid: the removed bodies were tombstones in its build, sentinel keys
    // at the tail of its order, so the compaction moves no slot the tree refers to, and its node
    // count base[n'] is the same for every n' at or past the last body in the tree)
    HIPCHK(e, compact_state(n, e->keep, e->st, e->alt, e->dead_sorted, nd, e->pos, e->scratch,
                            e->scratch_bytes, e->stream));
    std::swap(e->st, e->alt);
    e->boxes_valid = false;  // the slots moved
    if (e->lanes_valid) {  // carry the wave grouping over the removals (no re-sort)
        HIPCHK(e, compact_lanes(n, e->lanes, e->keep, e->pos, e->idx, e->keys32, e->keys32_s,
                                e->scratch, e->scratch_bytes, e->stream));
        std::swap(e->lanes, e->keys32_s);
        e->inv_valid = false;
        if (e->prebuilt && e->forces_ready) {
            // the next step's a(t), already evaluated by lane, follows its lanes (flag, qpos)
            if (e->a2_alt_cap < e->cap) {
                TRY(dev_alloc(e, e->a2_alt, 2 * (size_t)e->cap));
                e->a2_alt_cap = e->cap;
            }
            compact_lane_pairs(n, e->idx, e->keys32, e->a2, e->a2_alt, e->stream);
            HIPCHK(e, hipGetLastError());
            std::swap(e->a2, e->a2_alt);  // (one GPU: both hold 2 cap doubles)
        }
    } else {
        e->forces_ready = false;
    }
    e->n = n - (int64_t)nd;
    e->inv_valid = false;  // another n: another exchange layout
    if ((e->comm || e->group || e->solo) && let_active(e) && e->p.theta != 0.0 && e->n > 0 &&
        e->st_morton && !e->pos_pending) {
        // the LET selections until the next full build: boxes of the compacted slots from the
        // positions now (materialized at the call's end), the displacement bound restarting here
        TRY(let_alloc(e, 0));
        let_boxes(e->n, e->st, e->geo, e->let_box, e->stream);
        HIPCHK(e, hipGetLastError());
        HIPCHK(e, hipMemsetAsync(e->disp, 0, sizeof(double), e->stream));
        e->boxes_valid = true;
        e->builds_since_box = 0;
    }
    e->removed.assign(dead.begin(), dead.end());
    // BHA:526: lastTree = null only when the last step's merge rule removed a body.  Bodies
    // removed by earlier steps were tombstones in the last build (sentinel keys: the tail of its
    // order), so its first n - nd sorted keys still describe the whole tree.
    if (nd != nd_before_last) {
        e->tree_valid = false;
        e->lazy_tree = false;
        e->lt_aside = false;
    } else if (e->lazy_tree) {  // the snapshot follows the compaction (its tombstones were not built)
        compact_pair(n, e->keep, e->pos, e->lt_x, e->lt_y, e->alt.x, e->alt.y, e->stream);
        HIPCHK(e, hipGetLastError());
        std::swap(e->lt_x, e->alt.x);
        std::swap(e->lt_y, e->alt.y);
    }
    SYNC(e, e->stream);
    return BH_OK;
}

// Copy of the state at the start of a bh_step call that may merge: if a step's candidate
// pairs overflow the mailbox, the call is replayed from here with a larger one, so the rule
// (BHA:478-520) holds for any number of pairs.
int copy_state(bh_engine *e, const BodyState &src, const BodyState &dst, int64_t n) {
    if (n <= 0) return BH_OK;
    const size_t d = sizeof(double) * (size_t)n;
    HIPCHK(e, hipMemcpyAsync(dst.x, src.x, d, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(dst.y, src.y, d, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(dst.vx, src.vx, d, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(dst.vy, src.vy, d, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(dst.m, src.m, d, hipMemcpyDeviceToDevice, e->stream));
    HIPCHK(e, hipMemcpyAsync(dst.cidx, src.cidx, sizeof(uint32_t) * (size_t)n,
                             hipMemcpyDeviceToDevice, e->stream));
    return BH_OK;
}

int snapshot(bh_engine *e) {
    TRY(materialize_positions(e));
    if (e->snap_cap < e->cap) {
        TRY(alloc_state(e, e->snap, (size_t)e->cap));
        e->snap_cap = e->cap;
    }
    e->snap_n = e->n;
    // after a pipelined call the caller's state is the view (the prebuilt tree's jitter is not
    // applied yet): a replay starts from it and builds its own first tree.  The call never writes
    // the view's buffers (its own last step makes a new view from `alt`), so the snapshot takes
    // them over instead of copying 44 B per body
    if (e->view_pending && e->view_cap == e->snap_cap) {
        std::swap(e->snap, e->view);
        return BH_OK;
    }
    return copy_state(e, e->view_pending ? e->view : e->st, e->snap, e->n);
}

int restore(bh_engine *e) {
    e->vel_perm = nullptr;  // (the snapshot is complete)
    TRY(copy_state(e, e->snap, e->st, e->snap_n));
    e->n = e->snap_n;
    TRY(drop_carried_flags(e));
    e->prebuilt = false;
    e->view_pending = false;
    e->lt_aside = false;
    e->mir_fresh = false;
    e->spl_nb = 0;  // the splitters describe the discarded builds' order
    e->keys_ready = false;
    e->lanes_valid = e->lr_pending = e->lr_ready = false;
    e->inv_valid = false;
    e->pos_pending = false;  // the snapshot holds every position
    e->boxes_valid = false;
    e->heavy_possible = true;
    e->tree_valid = false;
    e->st_morton = false;
    e->vel_stale = false;  // the snapshot is a consistent replica
    return BH_OK;
}

// End of a bh_step call with LET builds (every rank's stream is idle): the call's LET status words
// scalars[4] (some subset overflowed, or a rank-local guard fired) and scalars[5] (largest subset),
// max-reduced over the ranks, so that every rank replays the call or none does.
int agree_let_flags(bh_engine *e, uint32_t ls[2], uint32_t *own_sub) {
    HIPCHK(e, hipMemcpy(ls, e->scalars + 4, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    *own_sub = ls[1];
    if (!e->solo) TRY(coll_log(e, COLL_FLAGS, 2 * sizeof(uint32_t), CS_MAIN));
    if (e->comm) {
        NCCLCHK(e, ncclAllReduce(e->scalars + 4, e->scalars + 4, 2, ncclUint32, ncclMax, e->comm,
                                 e->stream));
        HIPCHK(e, hipMemcpyAsync(ls, e->scalars + 4, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                 e->stream));
        SYNC(e, e->stream);
        return BH_OK;
    }
    if (!e->group) return BH_OK;  // solo: no peers
    // a member that cannot read a peer's flags must not decide alone: every member sees its
    // failure after the second barrier and all return an error together (none replays)
    e->agree_failed = false;  // (its previous value was read before this call's LET barriers)
    TRY(group_barrier(e));      // every member's call is complete on the device
    for (bh_engine *peer : e->group->members) {
        if (peer == e) continue;
        uint32_t q[2] = {0, 0};
        const hipError_t rc = hipMemcpy(q, peer->scalars + 4, sizeof(q), hipMemcpyDeviceToHost);
        if (rc != hipSuccess) {
            e->agree_failed = true;
            e->err = std::string("agree_let_flags: ") + hipGetErrorString(rc);
            break;
        }
        ls[0] = std::max(ls[0], q[0]);
        ls[1] = std::max(ls[1], q[1]);
    }
    TRY(group_barrier(e));  // nobody clears its flags (a replay) before every member has read them
    bool failed = false;
    for (bh_engine *peer : e->group->members) failed = failed || peer->agree_failed;
    if (failed) {
        if (!e->agree_failed) e->err = "agree_let_flags: a peer could not read the LET flags";
        return BH_E_DEVICE;
    }
    return BH_OK;
}

// ---- the pipelined step (one GPU) -----------------------------------------------------
// Step s's second traversal (a(t+dt), BHA:421-433) and step s+1's first build (BHA:359, over the
// same positions after the merge rule, BHA:438) are independent: the kick writes only
// velocities, the merge rule only masses and flags, and the build reads neither velocities nor
// the traversal's output.  So the merge rule and the next build run on a second stream while the
// traversal runs -- the build kernels (single-workgroup span passes, scans, sorts: ~260 us of
// mostly under-filled launches per build at C3) fill the chip next to the traversal's tail.
// The traversal reads copies of what they overwrite (masses, flags, lane map, node count) and
// the build writes the other node array; the velocities follow the build's permutation once
// the kick is done.  Every kernel sees the inputs of the sequential order: bit-identical.
#ifndef BH_PIPELINE
#define BH_PIPELINE 1
#endif
#ifndef BH_PIPE_PRIORITY
#define BH_PIPE_PRIORITY 1  // the overlapped work's stream at the highest priority
#endif
// The deep pipeline: the next step's a(t) evaluated beside this step's second traversal (kick +
// drift + keys as their own pass) -- for body lists up to BH_DEEP_PIPE_MAX_N.  Measured slower at
// C3 (1.925 against 1.884 ms per step, round 4): the next tree is ready only after the
// traversal's last waves are placed, so the two evaluations barely overlap and share the caches
// when they do.  A small list leaves most of the GPU idle in each traversal (a few hundred waves
// on 1 024 SIMDs), so there the two evaluations run side by side (round 6).
#ifndef BH_DEEP_PIPE_MAX_N
#define BH_DEEP_PIPE_MAX_N 0
#endif
int64_t deep_pipe_max_n() {
    static const int64_t v = [] {
        const char *t = std::getenv("BH_DEEP_PIPE_MAX_N");
        return t ? (int64_t)std::atoll(t) : (int64_t)BH_DEEP_PIPE_MAX_N;
    }();
    return v;
}
#ifndef BH_PIPE_LAST
#define BH_PIPE_LAST 1  // pipeline a call's last step too (the next call starts on its tree)
#endif
bool pipelined(const bh_engine *e, bool last) {
    return BH_PIPELINE && BH_FUSE_KICK && (!last || BH_PIPE_LAST) && e->n > 0 && !e->comm &&
           !e->group && !e->solo && e->p.theta != 0.0;
}

// The overlap and mirror streams of a one-GPU engine.  HIP hands a process's streams its few
// hardware queues (GPU_MAX_HW_QUEUES = 4) in creation order, so bh_create makes the overlap
// stream right after the engine's own, and a caller that reads the mirror enables it right after
// bh_create: made later, after another engine's streams (bench.py's counter probe), the mirror's
// copies shared a queue with the step's kernels (C3 one-step calls with the mirror: 3.25 -> 2.3
// ms).  An engine that never enables the mirror holds two queues, not three.
// The exchange stream (RCCL all-gathers, or the in-process copies) at the high priority: its
// few workgroups are dispatched ahead of the traversal rounds' queued ones as soon as a slot
// frees, instead of in the last round's tail (BH_COMM_PRIORITY=0: the default priority)
#ifndef BH_COMM_PRIORITY
#define BH_COMM_PRIORITY 1
#endif
hipError_t comm_stream_create(hipStream_t *s) {
    int lo = 0, hi = 0;
    hipError_t rc = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (rc != hipSuccess) return rc;
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, BH_COMM_PRIORITY ? hi : lo);
}

// The pipelined step's cross-stream events order work on this device only: no system-scope fence
// when they are recorded (the default one writes back and invalidates the caches for the host)
#ifndef BH_PIPE_EV_NOFENCE
#define BH_PIPE_EV_NOFENCE 1
#endif
constexpr unsigned kPipeEvFlags =
    hipEventDisableTiming | (BH_PIPE_EV_NOFENCE ? hipEventDisableSystemFence : 0u);
int pipe_streams(bh_engine *e) {
    for (hipEvent_t &ev : e->pipe_ev)
        if (!ev) HIPCHK(e, hipEventCreateWithFlags(&ev, kPipeEvFlags));
    if (!e->pipe_stream) {
        // the traversal fills every wave slot with a queue of waiting workgroups: at the default
        // priority the overlapped kernels would be dispatched only in its tail
        int lo = 0, hi = 0;
        HIPCHK(e, hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(e, hipStreamCreateWithPriority(&e->pipe_stream, hipStreamNonBlocking,
                                              BH_PIPE_PRIORITY ? hi : lo));
    }
    return BH_OK;
}

int mirror_streams(bh_engine *e) {
    if (!e->mir_stream) {
        int lo = 0, hi = 0;
        HIPCHK(e, hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(e, hipStreamCreateWithPriority(&e->mir_stream, hipStreamNonBlocking, hi));
        for (hipEvent_t *ev : {&e->mir_ev, &e->mir_ev2, &e->mir_ev3, &e->mir_in[0], &e->mir_in[1],
                               &e->mid_ev, &e->mid_sv_ev})
            HIPCHK(e, hipEventCreateWithFlags(ev, hipEventDisableTiming));
    }
    return BH_OK;
}

int pipe_alloc(bh_engine *e, bool last) {
    if (e->nodes_alt_cap < e->node_cap) {
        TRY(dev_alloc(e, e->nodes_alt, e->node_cap));
        e->nodes_alt_cap = e->node_cap;
    }
    if (last && e->view_cap < e->cap) {
        TRY(alloc_state(e, e->view, (size_t)e->cap));
        e->view_cap = e->cap;
    }
    if (last && e->lt_walk_cap < e->cap) {
        TRY(dev_alloc(e, e->lt_keys, (size_t)e->cap));
        TRY(dev_alloc(e, e->lt_cpl, (size_t)e->cap + 32));  // (as cpl: they trade places)
        TRY(dev_alloc(e, e->lt_base, (size_t)e->cap + 1));
        e->lt_walk_cap = e->cap;
    }
    if (e->trav_cap < e->cap) {
        TRY(dev_alloc(e, e->m_trav, (size_t)e->cap));
        TRY(dev_alloc(e, e->cidx_trav, (size_t)e->cap));
        TRY(dev_alloc(e, e->lanes_trav, (size_t)e->cap));
        if (!e->T_trav) TRY(dev_alloc(e, e->T_trav, 1));
        e->trav_cap = e->cap;
    }
    return pipe_streams(e);
}

// ---- the pinned caller-order mirror (bh_set_mirror / bh_map_bodies) -------------------
// The front-end reads every body after every step (PNL:302-306).  With the mirror on, a call's
// last step writes the bodies in the caller's order (after the call's removals, BHA:519) into
// pinned host memory itself: positions and masses as soon as the merge rule is done, velocities
// when the last traversal's kick is -- the device-to-host copies run on the DMA engines while the
// overlapped next build (and the traversal's tail) still run.
int mirror_alloc(bh_engine *e) {
    if (e->mir_cap < e->cap || (e->mir_nbuf == 2 && !e->mir_buf[1])) {
        for (double *&b : e->mir_buf) {
            if (b) (void)hipHostFree(b);
            b = nullptr;
        }
        e->mir = nullptr;
        e->mir_cap = 0;
        e->mir_front = -1;
        for (int i = 0; i < e->mir_nbuf; ++i)
            HIPCHK(e, hipHostMalloc((void **)&e->mir_buf[i], sizeof(double) * 5 * (size_t)e->cap,
                                    hipHostMallocDefault));
        e->mir = e->mir_buf[0];
        if (e->mir_idx) (void)hipHostFree(e->mir_idx);
        e->mir_idx = nullptr;
        if (e->mir_nbuf == 2) {  // the survivors' list indices for bh_step_positions
            const size_t w = MIRROR_HDR + (size_t)e->cap;
            HIPCHK(e, hipHostMalloc((void **)&e->mir_idx, sizeof(uint32_t) * w, hipHostMallocDefault));
            TRY(dev_alloc(e, e->mir_idx_stage, w));
        }
        TRY(dev_alloc(e, e->mir_stage, 5 * (size_t)e->cap));
        TRY(dev_alloc(e, e->mir_keep, (size_t)e->cap));
        TRY(dev_alloc(e, e->mir_pos, (size_t)e->cap));
        const size_t tb = compact_scratch_bytes(e->cap);
        if (e->mir_tmp) (void)hipFree(e->mir_tmp);
        e->mir_tmp = nullptr;
        HIPCHK(e, hipMalloc(&e->mir_tmp, tb));
        e->mir_tmp_bytes = tb;
        e->mir_cap = e->cap;
        e->mir_fresh = false;
    }
    return mirror_streams(e);
}

// src: the state the caller sees (tombstones of the running call still in it); its positions,
// masses and caller indices are final once after_pos's queued work is, its velocities once
// after_vel's is.  e->n bodies (before the call's compaction).
// The velocities are gathered on after_vel itself, right behind their producer: queued on the
// mirror stream they waited for the positions' host copies (~0.35 ms in the one-step call,
// which waits for them before its compaction -- round 4 drop-in trace).  (Kernels storing
// straight into coherent pinned memory instead of the staging copies measured slower: one-step
// calls with the mirror 3.33 against 3.20 ms.)
// (in two parts, so that the positions can be queued before the work after_vel still gets)
// in_line: the index and the gather run on after_pos itself, only the copies on the mirror
// stream (before a traversal: queued beside it they wait for its first waves to retire)
int mirror_pos(bh_engine *e, const BodyState &src, hipStream_t after_pos, bool in_line = false) {
    TRY(mirror_alloc(e));
    if (e->mir_nbuf == 2 && e->mir_buf[1])  // never the buffer the caller holds
        e->mir = e->mir_buf[e->mir_front == 0 ? 1 : 0];
    const int64_t n = e->n;
    const int64_t c = e->mir_cap;
    hipStream_t ms = e->mir_stream;
    hipStream_t ws = in_line ? after_pos : ms;
    if (!in_line) {
        HIPCHK(e, hipEventRecord(e->mir_in[0], after_pos));
        HIPCHK(e, hipStreamWaitEvent(ms, e->mir_in[0], 0));
    }
    if (n > 0) {
        double *st = e->mir_stage;
        HIPCHK(e, mirror_index(n, src.cidx, e->mir_keep, e->mir_pos, e->mir_tmp, e->mir_tmp_bytes,
                               ws));
        HIPCHK(e, hipEventRecord(e->mir_in[1], ws));  // the caller positions are known
        const double *s3[3] = {src.x, src.y, src.m};
        double *d3[3] = {st, st + c, st + 4 * c};
        mirror_scatter(n, src.cidx, e->mir_pos, 3, s3, d3, ws);
        HIPCHK(e, hipGetLastError());
        if (e->mir_idx) {  // two buffers: the survivors' indices in the list before the call
            mirror_survivors(n, e->mir_keep, e->mir_pos, e->scalars, e->mir_idx_stage, ws);
            HIPCHK(e, hipGetLastError());
        }
        HIPCHK(e, hipEventRecord(e->mir_ev3, ws));  // the positions' gather is done
        if (in_line) HIPCHK(e, hipStreamWaitEvent(ms, e->mir_ev3, 0));
        if (e->mir_idx) {  // first: the caller's removal pass needs only them (bh_step_positions)
            HIPCHK(e, hipMemcpyAsync(e->mir_idx, e->mir_idx_stage,
                                     sizeof(uint32_t) * (MIRROR_HDR + (size_t)n),
                                     hipMemcpyDeviceToHost, ms));
            HIPCHK(e, hipEventRecord(e->mid_sv_ev, ms));
        }
        for (int j : {0, 1, 4})  // (the survivors are a prefix of each array)
            HIPCHK(e, hipMemcpyAsync(e->mir + j * c, st + j * c, sizeof(double) * n,
                                     hipMemcpyDeviceToHost, ms));
    }
    return BH_OK;
}

int mirror_vel(bh_engine *e, const BodyState &src, hipStream_t after_vel) {
    const int64_t n = e->n;
    const int64_t c = e->mir_cap;
    hipStream_t ms = e->mir_stream;
    if (n > 0) {
        double *st = e->mir_stage;
        HIPCHK(e, hipStreamWaitEvent(after_vel, e->mir_in[1], 0));
        const double *s2[2] = {src.vx, src.vy};
        double *d2[2] = {st + 2 * c, st + 3 * c};
        mirror_scatter(n, src.cidx, e->mir_pos, 2, s2, d2, after_vel);
        HIPCHK(e, hipGetLastError());
        HIPCHK(e, hipStreamWaitEvent(after_vel, e->mir_ev3, 0));
        HIPCHK(e, hipEventRecord(e->mir_ev2, after_vel));  // no mirror kernel reads the state
        HIPCHK(e, hipStreamWaitEvent(ms, e->mir_ev2, 0));
        for (int j : {2, 3})
            HIPCHK(e, hipMemcpyAsync(e->mir + j * c, st + j * c, sizeof(double) * n,
                                     hipMemcpyDeviceToHost, ms));
    } else {
        HIPCHK(e, hipEventRecord(e->mir_ev2, after_vel));
        HIPCHK(e, hipStreamWaitEvent(ms, e->mir_ev2, 0));
    }
    HIPCHK(e, hipEventRecord(e->mir_ev, ms));
    e->mir_launched = true;
    return BH_OK;
}

int mirror_launch(bh_engine *e, const BodyState &src, hipStream_t after_pos, hipStream_t after_vel) {
    TRY(mirror_pos(e, src, after_pos));
    return mirror_vel(e, src, after_vel);
}

// The second evaluation of a pipelined step: build, second traversal with the fused kick, and
// next step's first build; e->prebuilt tells the next evaluation its tree is there.
// last: the call's last step -- this step's tree is lastTree (BHA:435): its walk structures are
// copied aside before the overlapped build reuses them, and the state before that build's jitter
// (the previous slot order) becomes the caller-visible `view`.

// The second traversal's input copies (masses, flags, lane map, node count) written by the
// second build's k_emit_com instead of a k_trav_inputs launch between the build and the traversal.
#ifndef BH_TRAV_COPY_IN_BUILD
#define BH_TRAV_COPY_IN_BUILD 1
#endif
#ifndef BH_PIPE_REUSE_MARK
#define BH_PIPE_REUSE_MARK 1
#endif
int evaluate_pipelined(bh_engine *e, bool last) {
    const int64_t n = e->n;
    hipStream_t s = e->stream;
    // the merge rule's mailbox header is cleared by k_trav_inputs below (after the previous merge
    // rule, which the engine's stream waited for, and before the overlapped one): a fill of its
    // own sat on the engine's hardware queue between the build and the traversal
    const bool merging = e->p.merge_min_dist > 0.0 && e->n > 1 && e->heavy_possible;
    if (merging) TRY(merge_bufs(e));
    TRY(mark(e, -1));
    if (e->lr_ready) {  // the re-sorted lane map (prebuilt order), carried on by this build
        HIPCHK(e, hipStreamWaitEvent(s, e->lr_ev, 0));
        std::swap(e->lanes, e->lanes_next);
        e->lr_ready = false;
        e->lanes_age = 0;
    }
    e->lane_hold = true;
    e->tc_want = BH_TRAV_COPY_IN_BUILD != 0;
    e->tc_box = merging ? reinterpret_cast<uint32_t *>(e->box) : nullptr;
    // velocities: permuted by the kick below; the heavy list for the merge rule that follows
    const int rc_b2 = build_into(e, s, false, true, false, merging && BH_HEAVY_CARRY);
    e->lane_hold = false;
    e->tc_want = false;
    TRY(rc_b2);
    TRY(mark(e, 0));
    // with profiling on, the overlapped chain waits for the timing event just recorded after the
    // build (when nothing else follows the build on this stream): each event recorded on the
    // stream holds the next kernel back by a few microseconds
    const hipEvent_t built_mark = e->profiling && e->ev_used > 0 && e->tc_done && BH_PIPE_REUSE_MARK
                                      ? e->ev[e->ev_used - 1]
                                      : nullptr;
    const bool lanes = e->lanes_valid;
    if (!e->tc_done) {  // (the build made them otherwise)
        copy_trav_inputs(n, e->st.m, e->m_trav, e->st.cidx, e->cidx_trav,
                         lanes ? e->lanes : nullptr, e->lanes_trav, e->base + n, e->T_trav, s,
                         merging ? e->box : nullptr);
        HIPCHK(e, hipGetLastError());
    }
    e->tc_done = false;
    // With the mirror on, a call's last step runs the merge rule and the mirror's caller-order
    // gather of positions and masses before the traversal (~0.15 ms in line): the mirror's 40 MB
    // cross PCIe from then on instead of from when the overlapped merge rule and gather find wave
    // slots beside the traversal, ~0.45 ms later (round 4 drop-in trace)
    const bool early = last && e->mirror_on;
    if (early) {
        copy_u32(e->scalars + 8, e->scalars + 2, s);  // the removals before the last merge rule
        HIPCHK(e, hipGetLastError());
        TRY(merge(e, s, merging));  // BHA:438 (the traversal reads its own copies of m, cidx)
        TRY(mirror_pos(e, e->st, s, true));
        if (e->mid_armed && e->mir_idx && n > 0) {  // bh_step_positions: the hand-off
            HIPCHK(e, hipEventRecord(e->mid_ev, e->mir_stream));
            {
                std::lock_guard<std::mutex> lk(e->mid_mu);
                e->mid_buf = e->mir;
                e->mid_stride = e->mir_cap;
                e->mid_ready = true;
            }
            e->mid_cv.notify_all();
        }
    }
    if (built_mark && !early) {
        HIPCHK(e, hipStreamWaitEvent(e->pipe_stream, built_mark, 0));
    } else {
        HIPCHK(e, hipEventRecord(e->pipe_ev[0], s));
        HIPCHK(e, hipStreamWaitEvent(e->pipe_stream, e->pipe_ev[0], 0));
    }
    const ForceParams fp{e->p.G, e->p.soft2, e->p.theta * e->p.theta};  // BHA:378
    KickArgs ka{KICK_ONLY, e->st.vx, e->st.vy, e->p.dt * 0.5, e->p.dt};
    if (n > 0) {  // (the build swapped: the previous order's velocities are in alt)
        ka.svx = e->alt.vx;
        ka.svy = e->alt.vy;
        ka.perm = e->perm;
    }
    WaveOrder wo;
    TRY(wave_order_for(e, 0, n, s, wo));
    traverse(e->nodes, e->node_cap, e->T_trav, e->st.x, e->st.y, e->m_trav, e->cidx_trav, 0, n,
             e->geo, fp, e->a2, nullptr, s, &ka, lanes ? e->lanes_trav : nullptr, &wo);
    HIPCHK(e, hipGetLastError());
    const bool deep = deep_pipe_max_n() > 0 && e->n <= deep_pipe_max_n();
    if (!deep) TRY(mark(e, 1));
    TRY(wave_order_next(e, 0, n, s));
    if (last) {
        hipStream_t ps = e->pipe_stream;
        // lastTree's walk (bh_get_quads): this build's sorted keys, prefix lengths and node
        // offsets stay where they are, the overlapped build below writes the other set (a copy
        // aside ran as a blit beside the traversal: ~0.5 ms, with the merge rule queued behind it)
        std::swap(e->keys_s, e->lt_keys);
        std::swap(e->cpl, e->lt_cpl);
        std::swap(e->base, e->lt_base);
        if (!early) {  // the call's removal count before its last merge rule (BHA:526)
            copy_u32(e->scalars + 8, e->scalars + 2, ps);
            HIPCHK(e, hipGetLastError());
        }
    }
    if (!early) TRY(merge(e, e->pipe_stream, merging));  // BHA:438
    if (early) TRY(mirror_vel(e, e->st, s));  // the velocities once the kick is done
    e->lane_defer = !last;  // (a call ends with a compaction: its last build re-sorts in place)
    const int rc_b1 = build_into(e, e->pipe_stream, true, false, last);  // step s+1's first tree (BHA:359)
    e->lane_defer = false;
    TRY(rc_b1);
    if (deep) {
        // ... and a(t) of step s+1 on it (BHA:407-408): a force evaluation reads positions and
        // masses only, so it runs beside this traversal, whose tail it fills; the next step's
        // kick and drift need this traversal's velocities and run after both (kick_drift_keys)
        traverse(e->nodes_alt, e->nodes_alt_cap, e->base + n, e->alt.x, e->alt.y, e->alt.m,
                 e->alt.cidx, 0, n, e->geo, fp, e->a2, nullptr, e->pipe_stream, nullptr,
                 e->lanes_valid ? e->lanes : nullptr, nullptr);
        HIPCHK(e, hipGetLastError());
    }
    HIPCHK(e, hipEventRecord(e->pipe_ev[1], e->pipe_stream));
    HIPCHK(e, hipStreamWaitEvent(s, e->pipe_ev[1], 0));
    if (deep) TRY(mark(e, 1, 2));  // this traversal, the overlapped chain, the next a(t)
    if (!last && !deep && BH_FOLD_VEL_PERM) {
        e->vel_perm = e->perm2;  // the next step's first kick reads them through the permutation
    } else {
        permute_velocities(n, e->perm2, e->st.vx, e->st.vy, e->alt.vx, e->alt.vy, s);
        HIPCHK(e, hipGetLastError());
    }
    TRY(mark(e, 0));  // the wait for the overlapped build and the velocity permutation
    std::swap(e->st, e->alt);
    std::swap(e->nodes, e->nodes_alt);
    std::swap(e->node_cap, e->nodes_alt_cap);
    e->prebuilt = true;
    e->carried_flags = last;
    e->forces_ready = deep;
    e->fp_ready = fp;
    if (last) {  // the previous order's state (kicked, merged, not yet jittered) is what the caller sees
        std::swap(e->view, e->alt);
        e->view_pending = true;
        e->lt_aside = true;
    }
    return BH_OK;
}

#ifndef BH_LAZY_LASTTREE
#define BH_LAZY_LASTTREE 1
#endif
// The positions the call's last build starts from (its jitter moves some of them): kept for the
// lazy lastTree of bh_get_quads (16 B per body, device copies).
int snapshot_positions(bh_engine *e) {
    const int64_t n = e->n;
    TRY(materialize_positions(e));
    if (e->lt_cap < e->cap) {
        TRY(dev_alloc(e, e->lt_x, (size_t)e->cap));
        TRY(dev_alloc(e, e->lt_y, (size_t)e->cap));
        e->lt_cap = e->cap;
    }
    if (n > 0) {
        HIPCHK(e, hipMemcpyAsync(e->lt_x, e->st.x, sizeof(double) * n, hipMemcpyDeviceToDevice,
                                 e->stream));
        HIPCHK(e, hipMemcpyAsync(e->lt_y, e->st.y, sizeof(double) * n, hipMemcpyDeviceToDevice,
                                 e->stream));
    }
    return BH_OK;
}

// The lane map's due Hilbert re-sort (build_into), from the prebuilt tree's sorted keys, on the
// overlap stream beside the first traversal -- which walks the map carried through that build --
// into lanes_next, swapped in before the second build carries it on (evaluate_pipelined).  The
// traversal writes none of these buffers (its fused epilogue writes keys / keys32, not keys_s).
// Made in the overlapped build, the re-sort ran after the chain and outlasted the second
// traversal by ~0.12 ms once every 8 steps (round 4 timeline).
int lane_refresh_beside(bh_engine *e) {
    e->lr_pending = false;
    const int64_t n = e->n;
    if (n <= 0 || !e->lanes_valid) return BH_OK;
    if (e->lr_cap < e->cap) {
        for (uint32_t **q : {&e->lanes_next, &e->lr_hkey, &e->lr_hkey_s, &e->lr_slot}) {
            if (*q) (void)hipFree(*q);
            *q = nullptr;
        }
        if (e->lr_scratch) (void)hipFree(e->lr_scratch);
        e->lr_scratch = nullptr;
        e->lr_cap = 0;
        for (uint32_t **q : {&e->lanes_next, &e->lr_hkey, &e->lr_hkey_s, &e->lr_slot})
            TRY(dev_alloc(e, *q, (size_t)e->cap));
        e->lr_scratch_bytes = lane_sort_bytes(e->cap);
        HIPCHK(e, hipMalloc(&e->lr_scratch, e->lr_scratch_bytes));
        e->lr_cap = e->cap;
    }
    if (!e->lr_ev) HIPCHK(e, hipEventCreateWithFlags(&e->lr_ev, kPipeEvFlags));
    HIPCHK(e, lane_order_into(e->keys_s, n, e->geo.J, e->lr_hkey, e->lr_hkey_s, e->lr_slot,
                              e->lr_scratch, e->lr_scratch_bytes, e->lanes_next, e->pipe_stream));
    HIPCHK(e, hipEventRecord(e->lr_ev, e->pipe_stream));
    e->lr_ready = true;
    return BH_OK;
}

// ---- one PhysicsEngine.step() (BHA:405-439) ------------------------------------------
// last: the final step of a bh_step call -- its second build is the full tree (lastTree,
// BHA:435, for getTreeForDebug) also on a multi-rank engine that shards its builds.
int step_once(bh_engine *e, bool last) {
    const int64_t n = e->n;
    const double dtHalf = e->p.dt * 0.5;  // BHA:412
    if (pipelined(e, last)) {
        TRY(pipe_alloc(e, last));
        if (e->lr_pending && e->prebuilt) TRY(lane_refresh_beside(e));
        e->lr_pending = false;
        bool fused = false;
        e->fuse_keys = true;  // and the second build's keys and bucket counts
        TRY(evaluate(e, nullptr, KICK_DRIFT, &fused, true));  // a(t), kick + drift fused
        if (!fused) {
            e->err = "pipelined step: the first evaluation did not fuse its kick";
            return BH_E_STATE;
        }
        TRY(evaluate_pipelined(e, last));  // a(t+dt), the kick, the merge rule and the next tree
        e->tree_valid = true;
        return BH_OK;
    }
    if (n > 0) {
        bool fused = false;  // one GPU: the kicks ride in the traversal's epilogue
        // (multi-rank LET evaluations integrate their own bodies too: fused)
        TRY(evaluate(e, nullptr, KICK_DRIFT, &fused, true));  // a(t)
        if (!fused) {
            TRY(mark(e, -1));
            kick_drift(n, e->a2, e->st.x, e->st.y, e->st.vx, e->st.vy, dtHalf, e->p.dt,
                       e->stream, e->a2_lanes, e->a2_layout, e->boxes_valid ? e->L.vmax : nullptr);
            HIPCHK(e, hipGetLastError());
            if (e->boxes_valid) {  // every rank drifted every body: its own bound is everyone's
                let_disp_add(e->disp, e->L.vmax, e->L.nvmax, e->p.dt, e->stream);
                HIPCHK(e, hipGetLastError());
            }
            TRY(mark(e, 2));
        }
        // the call's last build: a full tree for getTreeForDebug (lastTree, BHA:435) -- or, on a
        // multi-rank engine, a LET build like the others, its input positions kept for a lazy
        // full build in bh_get_quads
        const bool lazy = last && BH_LAZY_LASTTREE && (e->comm || e->group || e->solo);
        if (lazy) TRY(snapshot_positions(e));
        bool let2 = false;
        TRY(evaluate(e, nullptr, KICK_ONLY, &fused, !last || lazy, &let2));  // a(t+dt)
        if (!fused) {
            TRY(mark(e, -1));
            kick(n, e->a2, e->st.vx, e->st.vy, dtHalf, e->stream, e->a2_lanes, e->a2_layout);
            HIPCHK(e, hipGetLastError());
            TRY(mark(e, 2));
        }
        e->tree_valid = !let2;  // lastTree = root (BHA:435)
        e->lazy_tree = lazy && let2;
    }
    if (last)  // the call's removal count before its last merge rule (finish_merges, BHA:526)
        HIPCHK(e, hipMemcpyAsync(e->scalars + 8, e->scalars + 2, sizeof(uint32_t),
                                 hipMemcpyDeviceToDevice, e->stream));
    return merge(e);  // BHA:438
}

// ---- getTreeForDebug().visitQuads (BHA:265-274) from the Morton structure ------------
struct QuadWalker {
    const Geometry &g;
    const std::vector<uint64_t> &keys;
    const std::vector<int8_t> &cpl;
    const std::vector<uint32_t> &base;
    const Node *nodes;  // device
    double *cx, *cy, *h;
    int64_t cap, k = 0;
    int rc = BH_OK;

    void emit(double qx, double qy, double qh) {
        if (k < cap) {
            cx[k] = qx;
            cy[k] = qy;
            h[k] = qh;
        }
        ++k;
    }
    static void child(double qx, double qy, double qh, int which, double &ox, double &oy,
                      double &oh) {  // BHA:73-81
        double hh = qh / 2.0;
        ox = (which & 1) ? qx + hh : qx - hh;
        oy = (which & 2) ? qy + hh : qy - hh;
        oh = hh;
    }
    void leaf_children(double qx, double qy, double qh) {
        for (int q = 0; q < 4; ++q) {
            double ox, oy, oh;
            child(qx, qy, qh, q, ox, oy, oh);
            emit(ox, oy, oh);
        }
    }
    void rec(int L, int64_t lo, int64_t hi, double qx, double qy, double qh) {
        emit(qx, qy, qh);
        if (hi - lo < 2) return;  // empty or single-body leaf
        if (L == g.J) {           // jitter cell: children from the replay
            int cp = lo > 0 ? (int)cpl[lo - 1] : -1;
            uint32_t ni = base[lo] + (uint32_t)(L - cp - 1);
            Node nd;
            if (hipMemcpy(&nd, nodes + ni, sizeof(Node), hipMemcpyDeviceToHost) != hipSuccess) {
                rc = BH_E_DEVICE;
                return;
            }
            uint32_t jmask = (nd.meta >> NODE_JMASK_SHIFT) & 0xFu;
            for (int q = 0; q < 4; ++q) {
                double ox, oy, oh;
                child(qx, qy, qh, q, ox, oy, oh);
                emit(ox, oy, oh);
                if (jmask & (1u << q)) leaf_children(ox, oy, oh);
            }
            return;
        }
        const int shift = 2 * (g.J - 1 - L);
        int64_t s = lo;
        for (int q = 0; q < 4; ++q) {
            int64_t e2 = s;
            while (e2 < hi && (int)((keys[e2] >> shift) & 3u) == q) ++e2;
            double ox, oy, oh;
            child(qx, qy, qh, q, ox, oy, oh);
            rec(L + 1, s, e2, ox, oy, oh);
            s = e2;
        }
    }
};

void set_defaults(bh_params *p) {
    p->G = 80.0;                 // CFG:11
    p->dt = 0.005;               // CFG:14
    p->theta = 0.30;             // CFG:23
    p->soft2 = 1.0 * 1.0;        // CFG:17,20
    p->width_px = 2400;          // CFG:5
    p->height_px = 800;          // CFG:8
    p->merge_max_mass = 4000.0;  // BHA:315
    p->merge_min_dist = 8.0;     // BHA:321 = Config.MIN_R (CFG:35)
}

int engine_init(bh_engine *e, const bh_params *p, int device) {
    if (!p) {
        e->err = "params is NULL";
        return BH_E_INVALID;
    }
    e->p = *p;
    TRY(make_geometry(e->p, e->geo, e->err));
    e->device = device;
    if (const char *v = std::getenv("BH_LET")) {
        e->let_on = std::strcmp(v, "0") != 0;
        e->let_forced = std::strcmp(v, "1") == 0;
    }
    HIPCHK(e, hipSetDevice(device));
    HIPCHK(e, hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
    TRY(dev_alloc(e, e->scalars, 16));
    HIPCHK(e, hipMemsetAsync(e->scalars, 0, 16 * sizeof(uint32_t), e->stream));
    TRY(ensure_capacity(e, 1));
    return BH_OK;
}

void free_state(BodyState &s) {
    void *p[] = {s.x, s.y, s.vx, s.vy, s.m, s.cidx};
    for (void *q : p)
        if (q) (void)hipFree(q);
}

}  // namespace

// Round sizes of a rank's lane range (BH_ROUND_FRACS="a,b,c,d": relative weights; default
// below): whole wavefronts, the same on every rank (bh_shard_range, bh_gather_slot).
static const double *round_cum() {
    struct Cum {
        double c[BH_SHARD_ROUNDS + 1];
        Cum() {
            double w[BH_SHARD_ROUNDS] = {BH_ROUND_WEIGHTS};
            if (const char *v = std::getenv("BH_ROUND_FRACS")) {
                double t[BH_SHARD_ROUNDS];
                int k = 0;
                const char *p = v;
                while (k < BH_SHARD_ROUNDS && *p) {
                    char *end = nullptr;
                    t[k] = std::strtod(p, &end);
                    if (end == p || !(t[k] > 0.0)) break;
                    ++k;
                    p = *end == ',' ? end + 1 : end;
                }
                if (k == BH_SHARD_ROUNDS)
                    for (int j = 0; j < k; ++j) w[j] = t[j];
            }
            double tot = 0.0;
            for (double x : w) tot += x;
            c[0] = 0.0;
            for (int j = 0; j < BH_SHARD_ROUNDS; ++j) c[j + 1] = c[j] + w[j] / tot;
        }
    };
    static const Cum cum;  // thread-safe initialisation (the in-process ranks are threads)
    return cum.c;
}

GatherLayout bh::shard_layout(int64_t n, int world) {
    GatherLayout L{};
    const int64_t sub = shard_sub(n, world, BH_SHARD_ROUNDS);
    L.span = sub * BH_SHARD_ROUNDS;
    L.world = world;
    const double *cum = round_cum();
    L.off[0] = 0;
    for (int k = 1; k < BH_SHARD_ROUNDS; ++k)
        L.off[k] = std::max<int64_t>(L.off[k - 1],
                                     std::min<int64_t>(L.span, (int64_t)(cum[k] * (double)L.span) / 64 * 64));
    L.off[BH_SHARD_ROUNDS] = L.span;
    return L;
}

void bh::set_error(bh_engine *e, const std::string &msg) {
    if (e) e->err = msg;
}

// The per-process settings that decide which collectives a step issues and how large each piece
// is -- BH_LET (LET builds: the cell-table all-gather) and BH_ROUND_FRACS (the round sizes of
// bh_shard_range / bh_gather_slot) -- must be equal on every rank, or the collectives stop
// matching and the run hangs.  Min- and max-reduced over the ranks at creation: every rank sees
// the same comparison, so all of them fail together on a mismatch.
static int agree_settings(bh_engine *e) {
    constexpr int K = 2 + BH_SHARD_ROUNDS + 1;
    double v[K];
    v[0] = e->let_on ? 1.0 : 0.0;
    v[1] = e->let_forced ? 1.0 : 0.0;
    const double *cum = round_cum();
    for (int j = 0; j <= BH_SHARD_ROUNDS; ++j) v[2 + j] = cum[j];
    // device scratch from the engine's own buffers (allocated by ensure_capacity: no allocation
    // that could fail on one rank only), and every rank takes part in both all-reduces whatever
    // happened locally, so a local failure cannot leave the peers waiting in a collective
    double *d = static_cast<double *>(e->scratch);
    double lo[K], hi[K];
    TRY(coll_log(e, COLL_SETTINGS, (int64_t)sizeof(double) * 2 * K, CS_MAIN));
    ncclResult_t nr = ncclSuccess;
    if (!d || e->scratch_bytes < sizeof(double) * 3 * K) {
        e->err = "agree_settings: no device scratch";
        return BH_E_STATE;  // (every rank: the buffers are sized alike)
    }
    hipError_t hr = hipMemcpyAsync(d, v, sizeof(v), hipMemcpyHostToDevice, e->stream);
    if (hr != hipSuccess)  // NaN bit patterns (if the device still takes a fill): no match
        (void)hipMemsetAsync(d, 0xFF, sizeof(v), e->stream);
    ncclResult_t n1 = ncclAllReduce(d, d + K, K, ncclFloat64, ncclMin, e->comm, e->stream);
    ncclResult_t n2 = ncclAllReduce(d, d + 2 * K, K, ncclFloat64, ncclMax, e->comm, e->stream);
    nr = n1 != ncclSuccess ? n1 : n2;
    hipError_t h2 = hipMemcpyAsync(lo, d + K, sizeof(lo), hipMemcpyDeviceToHost, e->stream);
    if (h2 == hipSuccess) h2 = hipMemcpyAsync(hi, d + 2 * K, sizeof(hi), hipMemcpyDeviceToHost, e->stream);
    if (h2 == hipSuccess && wait_stream(e, e->stream) != BH_OK) return BH_E_COMM;  // (bounded)
    if (hr == hipSuccess) hr = h2;
    if (nr != ncclSuccess) {
        e->err = std::string("agree_settings: ") + ncclGetErrorString(nr);
        return BH_E_COMM;
    }
    if (hr != hipSuccess) {
        e->err = std::string("agree_settings: ") + hipGetErrorString(hr);
        return BH_E_DEVICE;
    }
    for (int j = 0; j < K; ++j)
        if (lo[j] != hi[j]) {
            e->err = "BH_LET / BH_ROUND_FRACS differ between ranks: every rank must run with the "
                     "same settings";
            return BH_E_INVALID;
        }
    return BH_OK;
}

// ---- the multi-device handle's pieces (multi.hpp) -----------------------------------------
#ifndef BH_MULTI_MIN_BODIES
// body lists below this run on one GPU behind a multi-device handle.  A LET evaluation costs ~40
// launches of >= 4.5 us per build (two per step) plus 8 round launches and the exchanges
// whatever the size, ~0.6 ms per step; one GPU steps 1e5 bodies in 0.55 ms and 1e6 in 1.8 ms,
// so the split pays from a few 1e5 bodies on (an estimate: no multi-GPU box was available).
#define BH_MULTI_MIN_BODIES 400000
#endif
int bh::facade_create(const bh_params *p, bh::Multi *mu, bh_engine **out) {
    bh_engine *f = new bh_engine();
    f->p = *p;
    if (make_geometry(f->p, f->geo, f->err) != BH_OK) {
        delete f;
        return BH_E_INVALID;
    }
    f->multi = mu;
    f->world = multi_world(mu);
    f->multi_min = 0;
    if (const char *v = std::getenv("BH_MULTI_MIN_BODIES")) f->multi_min = std::atoll(v);
    else f->multi_min = BH_MULTI_MIN_BODIES;
    *out = f;
    return BH_OK;
}

int bh::member_agree(bh_engine *e) {
    if (!e->comm) return BH_OK;
    HIPCHK(e, hipSetDevice(e->device));  // (a pool thread: RCCL calls on the member's device)
    return agree_settings(e);
}

void bh::member_set_abort(bh_engine *e, std::atomic<bool> *flag) { e->abort_flag = flag; }

void bh::member_drop_comm(bh_engine *e) {
    if (e->comm) {
        (void)hipSetDevice(e->device);
        (void)ncclCommAbort(e->comm);
        e->comm = nullptr;
        e->comm_lost = true;
    }
}

void bh::member_set_comm(bh_engine *e, void *comm) {
    e->comm = static_cast<ncclComm_t>(comm);
    e->comm_lost = false;
}

// (comm: an RCCL communicator made in this process; on failure it stays the caller's)
int bh::member_create(const bh_params *p, int device, int rank, int world, void *comm,
                      bh_local_group *group, bh_engine **out) {
    if (group) return bh_create_local(p, device, rank, group, out);
    if (!out || !comm || world < 1 || rank < 0 || rank >= world) return BH_E_INVALID;
    *out = nullptr;
    bh_engine *e = new bh_engine();
    e->rank = rank;
    e->world = world;
    int rc = engine_init(e, p, device);
    if (rc == BH_OK) {
        e->comm = static_cast<ncclComm_t>(comm);
        hipError_t hr = comm_stream_create(&e->comm_stream);
        for (int k = 0; k < BH_SHARD_ROUNDS && hr == hipSuccess; ++k)
            hr = hipEventCreateWithFlags(&e->round_ev[k], hipEventDisableTiming);
        if (hr == hipSuccess) hr = hipEventCreateWithFlags(&e->gathered_ev, hipEventDisableTiming);
        if (hr != hipSuccess) {
            e->err = std::string("comm stream/events: ") + hipGetErrorString(hr);
            rc = BH_E_DEVICE;
        }
    }
    if (rc == BH_OK) {  // the accelerations buffer in rounds x world pieces
        const int64_t cap = e->cap;
        e->cap = 0;
        rc = ensure_capacity(e, cap);
    }
    if (rc != BH_OK) {
        std::fprintf(stderr, "bh_create_multi (rank %d): %s\n", rank, e->err.c_str());
        e->comm = nullptr;
        bh_destroy(e);
        return rc;
    }
    *out = e;
    return BH_OK;
}

// getTreeForDebug (BHA:329-332): lastTree if the last step kept it, else a fresh tree -- built
// here, its jitter applied to the state as the reference's buildTree applies it.
int bh::quads_prepare(bh_engine *e) {
    HIPCHK(e, hipSetDevice(e->device));
    const int64_t n = e->n;
    TRY(materialize_positions(e));
    if (!e->tree_valid && (e->comm || e->group || e->solo)) {
        // multi-rank: the tree is built into the workspace from the positions of the call's last
        // build (the lazy lastTree) or the current ones (getTreeForDebug's fresh tree), and the
        // state stays as it is -- a rank's slot order and lane map must not change on its own
        HIPCHK(e, hipMemsetAsync(e->scalars + 1, 0, sizeof(uint32_t), e->stream));
        if (n > 0) {
            TreeBuffers tb = tree_buffers(e);
            if (e->lazy_tree) {
                tb.src.x = e->lt_x;
                tb.src.y = e->lt_y;
            }
            tb.src.vx = tb.src.vy = nullptr;  // positions, masses and flags are all it reads
            tb.spl_nb = 0;                    // the caller's splitters describe another order
            tb.lanes_remap = nullptr;
            HIPCHK(e, tree_build(tb, n, e->geo, e->stream));
            if (!e->lazy_tree) {
                // getTreeForDebug's fresh buildTree moves the bodies it jitters (BHA:146-151,
                // 329-331): the moved positions go back into the replica in its own slot order
                // (every rank makes the same calls, so the replicas stay equal)
                unpermute_positions(n, e->perm, tb.dst.x, tb.dst.y, e->st.x, e->st.y, e->stream);
                HIPCHK(e, hipGetLastError());
                e->mir_fresh = false;
                ++e->builds_since_box;  // (its jitter, for the LET selection's bound)
            }
            e->spl_nb = 0;  // k_prep wrote splitters of this order
            e->keys_ready = false;
            TRY(check_tree_flags(e));
        } else {
            HIPCHK(e, hipMemsetAsync(e->base, 0, sizeof(uint32_t), e->stream));
        }
        e->tree_valid = true;  // until the next step (a second call walks the same tree)
    } else if (!e->tree_valid && e->view_pending) {
        // getTreeForDebug's fresh tree (BHA:329-332) is the one the pipelined call already built
        // from the caller's bodies after its merge rule: its jitter becomes part of the state, and
        // the next step builds its own first tree from these positions (BHA:407)
        e->view_pending = false;
        e->prebuilt = false;
        e->mir_fresh = false;
        e->tree_valid = true;
        HIPCHK(e, hipMemsetAsync(e->scalars + 1, 0, sizeof(uint32_t), e->stream));
        TRY(take_carried_flags(e));
        if (n > 0) TRY(check_tree_flags(e));
    } else if (!e->tree_valid) {  // getTreeForDebug builds a fresh tree (BHA:329-332)
        HIPCHK(e, hipMemsetAsync(e->scalars + 1, 0, sizeof(uint32_t), e->stream));
        TRY(build(e));
        if (n > 0) TRY(check_tree_flags(e));
    }
    return BH_OK;
}

// A multi-device handle's calls: on the engine that holds the bodies -- every member, or the
// single-GPU engine of a small body list -- and, for the settings (params, profiling, mirror),
// on both, so that either is current when a reset switches between them.
namespace {
int multi_fan(bh_engine *e, const std::function<int(bh_engine *, int)> &fn, bool both) {
    int rc = BH_OK;
    if (e->use_one) {
        rc = fn(e->one, 0);
        if (rc != BH_OK) e->err = bh_last_error(e->one);
    }
    if (!e->use_one || both) {
        const int r2 = multi_all(e->multi, e, fn);
        if (rc == BH_OK) rc = r2;
    }
    if (both && !e->use_one && e->one && rc == BH_OK) {
        rc = fn(e->one, 0);
        if (rc != BH_OK) e->err = bh_last_error(e->one);
    }
    return rc;
}
bh_engine *multi_active0(const bh_engine *e) { return e->use_one ? e->one : multi_member(e->multi, 0); }
}  // namespace
#define MULTI_FAN(e, both, call)                                                        \
    do {                                                                                \
        if ((e)->multi)                                                                 \
            return multi_fan((e), [&](bh_engine *m_, int r_) {                          \
                (void)r_;                                                               \
                return call;                                                            \
            }, both);                                                                   \
    } while (0)
#define MULTI_ALL(e, call) MULTI_FAN(e, false, call)
#define MULTI_BOTH(e, call) MULTI_FAN(e, true, call)
// the calls that only read the state: the active engine's member 0 (every replica is complete at
// the API boundary)
#define MULTI_M0(e) ((e)->multi ? multi_active0(e) : (e))

// A call begun by bh_step_begin owns the engine until bh_step_end: the other calls that use
// the engine are refused (BH_E_STATE, without touching the error text the call may be writing)
// from any thread but the call's own.
#define ASYNC_GUARD(e)                                                                         \
    do {                                                                                       \
        if ((e)->async_running && std::this_thread::get_id() != (e)->step_thr.get_id())      \
            return BH_E_STATE;                                                                 \
    } while (0)

// A rank of a decomposition whose last call failed -- here or on a peer (the group / handle was
// aborted) -- refuses the calls that use the replica or issue collectives until bh_reset_bodies:
// every rank refuses alike, so none waits in a collective the others never issue.
namespace {
int comm_refused(bh_engine *e) {
    if (!multi_rank(e) || (!e->comm_failed && !peers_aborted(e))) return BH_OK;
    e->err = "a previous call of this multi-rank engine failed (" +
             (e->comm_failed ? e->fail_msg : std::string("on a peer rank")) +
             "); bh_reset_bodies before the next call";
    return BH_E_COMM;
}
}  // namespace
#define COMM_GUARD(e) TRY(comm_refused(e))

// =========================================================================================
extern "C" {

static int last_removed(const bh_engine *e, int64_t *idx, int64_t cap, int64_t *n_out);

void bh_default_params(bh_params *p) {
    if (p) set_defaults(p);
}

int bh_create(const bh_params *p, int device, bh_engine **out) {
    if (!out) return BH_E_INVALID;
    *out = nullptr;
    bh_engine *e = new bh_engine();
    int rc = engine_init(e, p, device);
    // the overlap stream right after the engine's own (HIP hands a process's few hardware queues
    // out in stream creation order); the mirror's is made by bh_set_mirror, which a caller that
    // reads the mirror calls right after bh_create (the shims do)
    if (rc == BH_OK) rc = pipe_streams(e);
    if (rc != BH_OK) {
        std::fprintf(stderr, "bh_create: %s\n", e->err.c_str());
        bh_destroy(e);
        return rc;
    }
    *out = e;
    return BH_OK;
}

int bh_comm_unique_id(void *out128) {
    if (!out128) return BH_E_INVALID;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return BH_E_COMM;
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id must be 128 bytes");
    std::memcpy(out128, &id, sizeof(id));
    return BH_OK;
}

int bh_create_dist(const bh_params *p, int device, int rank, int world, const void *unique_id,
                   bh_engine **out) {
    if (!out || world < 1 || rank < 0 || rank >= world || (world > 1 && !unique_id))
        return BH_E_INVALID;
    *out = nullptr;
    bh_engine *e = new bh_engine();
    e->rank = rank;
    e->world = world;
    int rc = engine_init(e, p, device);
    if (rc == BH_OK && unique_id) {  // world == 1 with an id: the RCCL path on one rank
        ncclUniqueId id;
        std::memcpy(&id, unique_id, sizeof(id));
        ncclResult_t nr = ncclCommInitRank(&e->comm, world, id, rank);
        if (nr != ncclSuccess) {
            e->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(nr);
            rc = BH_E_COMM;
        }
        hipError_t hr = comm_stream_create(&e->comm_stream);
        for (int k = 0; k < BH_SHARD_ROUNDS && hr == hipSuccess; ++k)
            hr = hipEventCreateWithFlags(&e->round_ev[k], hipEventDisableTiming);
        if (hr == hipSuccess) hr = hipEventCreateWithFlags(&e->gathered_ev, hipEventDisableTiming);
        if (rc == BH_OK && hr != hipSuccess) {
            e->err = std::string("comm stream/events: ") + hipGetErrorString(hr);
            rc = BH_E_DEVICE;
        }
        // the accelerations buffer is laid out in rounds x world pieces from now on
        if (rc == BH_OK) {
            const int64_t cap = e->cap;
            e->cap = 0;
            rc = ensure_capacity(e, cap);
        }
        if (rc == BH_OK) rc = agree_settings(e);
    }
    if (rc != BH_OK) {
        std::fprintf(stderr, "bh_create_dist: %s\n", e->err.c_str());
        bh_destroy(e);
        return rc;
    }
    *out = e;
    return BH_OK;
}

int bh_local_group_create(int world, bh_local_group **out) {
    if (!out || world < 1) return BH_E_INVALID;
    bh_local_group *g = new bh_local_group();
    g->world = world;
    g->members.assign((size_t)world, nullptr);
    *out = g;
    return BH_OK;
}

void bh_local_group_destroy(bh_local_group *g) { delete g; }

int bh_create_local(const bh_params *p, int device, int rank, bh_local_group *group,
                    bh_engine **out) {
    if (!out || !group || rank < 0 || rank >= group->world || group->members[rank])
        return BH_E_INVALID;
    *out = nullptr;
    bh_engine *e = new bh_engine();
    e->rank = rank;
    e->world = group->world;
    int rc = engine_init(e, p, device);
    if (rc == BH_OK) {
        hipError_t hr = comm_stream_create(&e->comm_stream);
        for (int k = 0; k < BH_SHARD_ROUNDS && hr == hipSuccess; ++k)
            hr = hipEventCreateWithFlags(&e->round_ev[k], hipEventDisableTiming);
        if (hr == hipSuccess) hr = hipEventCreateWithFlags(&e->gathered_ev, hipEventDisableTiming);
        if (hr != hipSuccess) {
            e->err = std::string("comm stream/events: ") + hipGetErrorString(hr);
            rc = BH_E_DEVICE;
        }
    }
    if (rc == BH_OK) {
        e->group = group;
        const int64_t cap = e->cap;  // the accelerations buffer in rounds x world pieces
        e->cap = 0;
        rc = ensure_capacity(e, cap);
    }
    if (rc != BH_OK) {
        std::fprintf(stderr, "bh_create_local: %s\n", e->err.c_str());
        e->group = nullptr;
        bh_destroy(e);
        return rc;
    }
    group->members[rank] = e;
    *out = e;
    return BH_OK;
}

int bh_create_solo(const bh_params *p, int device, int rank, int world, bh_engine **out) {
    if (!out || world < 1 || rank < 0 || rank >= world) return BH_E_INVALID;
    *out = nullptr;
    bh_engine *e = new bh_engine();
    e->rank = rank;
    e->world = world;
    int rc = engine_init(e, p, device);
    if (rc == BH_OK) {
        hipError_t hr = comm_stream_create(&e->comm_stream);
        for (int k = 0; k < BH_SHARD_ROUNDS && hr == hipSuccess; ++k)
            hr = hipEventCreateWithFlags(&e->round_ev[k], hipEventDisableTiming);
        if (hr == hipSuccess) hr = hipEventCreateWithFlags(&e->gathered_ev, hipEventDisableTiming);
        if (hr != hipSuccess) {
            e->err = std::string("comm stream/events: ") + hipGetErrorString(hr);
            rc = BH_E_DEVICE;
        }
    }
    if (rc == BH_OK) {
        e->solo = true;
        const int64_t cap = e->cap;  // the pieces buffer in rounds x world pieces
        e->cap = 0;
        rc = ensure_capacity(e, cap);
    }
    if (rc != BH_OK) {
        std::fprintf(stderr, "bh_create_solo: %s\n", e->err.c_str());
        bh_destroy(e);
        return rc;
    }
    *out = e;
    return BH_OK;
}

void bh_destroy(bh_engine *e) {
    if (!e) return;
    if (e->step_thr.joinable()) e->step_thr.join();  // a call begun by bh_step_begin
    if (e->multi) {  // the members, their threads and the exchange; then the handle itself
        bh_destroy(e->one);
        multi_destroy(e->multi);
        delete e;
        return;
    }
    (void)hipSetDevice(e->device);
    // (a rank of a decomposition waits for its streams at most BH_COMM_TIMEOUT_S: a collective
    // whose peers are gone never completes; after a failed call its communicator is aborted --
    // ncclCommDestroy would wait for the peers)
    const double drain_s = multi_rank(e) ? std::max(comm_timeout_s(), 1.0) : 0.0;
    if (e->comm && (e->comm_failed || peers_aborted(e))) abort_comm(e);
    (void)drain_stream(e->stream, drain_s);
    if (e->comm && drain_stream(e->comm_stream, drain_s) != hipSuccess) abort_comm(e);
    if (e->comm) (void)ncclCommDestroy(e->comm);
    if (e->group && e->rank < (int)e->group->members.size() && e->group->members[e->rank] == e)
        e->group->members[e->rank] = nullptr;
    for (hipEvent_t ev : e->round_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (e->gathered_ev) (void)hipEventDestroy(e->gathered_ev);
    if (e->comm_stream) (void)hipStreamDestroy(e->comm_stream);
    if (e->stream2) {
        (void)hipStreamSynchronize(e->stream2);
        (void)hipStreamDestroy(e->stream2);
    }
    if (e->built_ev) (void)hipEventDestroy(e->built_ev);
    for (hipEvent_t ev : e->pipe_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (e->pipe_stream) {
        (void)hipStreamSynchronize(e->pipe_stream);
        (void)hipStreamDestroy(e->pipe_stream);
    }
    if (e->mir_stream) {
        (void)hipStreamSynchronize(e->mir_stream);
        (void)hipStreamDestroy(e->mir_stream);
    }
    for (hipEvent_t ev : {e->mir_ev, e->mir_ev2, e->mir_ev3, e->mir_in[0], e->mir_in[1], e->mid_ev,
                          e->mid_sv_ev})
        if (ev) (void)hipEventDestroy(ev);
    for (double *b : e->mir_buf)
        if (b) (void)hipHostFree(b);
    if (e->mir_idx) (void)hipHostFree(e->mir_idx);
    free_state(e->view);
    free_state(e->st);
    free_state(e->alt);
    free_state(e->snap);
    free_state(e->sub_src);
    free_state(e->sub_dst);
    if (e->sub_cnt_ev) (void)hipEventDestroy(e->sub_cnt_ev);
    if (e->sub_cnt_h) (void)hipHostFree(e->sub_cnt_h);
    if (e->table_ev) (void)hipEventDestroy(e->table_ev);
    void *lets[] = {e->L.own_blk, e->L.rowmask, e->let_box, e->disp, e->inv_lanes, e->L.csrc, e->L.ccnt, e->L.cpos, e->solo_table, e->solo_all, e->solo_cstart, e->L.ecell, e->L.hcell, e->L.own, e->L.subpos, e->L.flag_all, e->L.flag8, e->L.sel, e->L.selpos, e->L.cstart,
                    e->L.table, e->L.tables, e->L.levels, e->L.w, e->L.posc, e->L.bsz,
                    e->L.nodes, e->L.lanes, e->s_keys, e->s_keys_s, e->s_spl, e->s_keys32,
                    e->s_keys32_s, e->s_idx, e->s_perm, e->s_cpl, e->s_cnt, e->s_base,
                    e->s_cell_start, e->s_span_list, e->s_super_list, e->s_bcount, e->s_bstart,
                    e->s_span_children, e->s_nodes};
    for (void *q : lets)
        if (q) (void)hipFree(q);
    void *ptrs[] = {e->a2, e->ax, e->ay, e->keys, e->keys_s, e->keys32, e->keys32_s, e->idx, e->perm, e->perm2, e->cpl, e->cnt,
                    e->base, e->cell_start, e->nodes, e->span_list, e->super_list,
                    e->span_children, e->scalars, e->visits32, e->contrib32, e->lanes, e->wave_iters, e->wave_blocks, e->heavy, e->keep,
                    e->pos, e->box, e->dlog, e->dead_sorted, e->rkeys, e->ridx, e->mbits, e->mslot, e->scratch,
                    e->leaf_flags, e->leaf_sel, e->leaf_count, e->leaf_cover, e->leaves.rec,
                    e->leaf_tmp, e->spl, e->bcount, e->bstart, e->nodes_alt, e->wave_cost, e->run_order,
                    e->m_trav, e->cidx_trav, e->lanes_trav, e->T_trav, e->solo_xchg,
                    e->lt_x, e->lt_y, e->a2_alt, e->lt_keys, e->lt_cpl, e->lt_base, e->mir_stage,
                    e->mir_keep, e->mir_pos, e->mir_tmp, e->mir_idx_stage, e->lanes_next, e->lr_hkey, e->lr_hkey_s,
                    e->lr_slot, e->lr_scratch};
    for (void *q : ptrs)
        if (q) (void)hipFree(q);
    for (hipEvent_t ev : e->ev) (void)hipEventDestroy(ev);
    if (e->lr_ev) (void)hipEventDestroy(e->lr_ev);
    if (e->pin) (void)hipHostFree(e->pin);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

const char *bh_last_error(const bh_engine *e) { return e ? e->err.c_str() : "null engine"; }

int bh_set_params(bh_engine *e, const bh_params *p) {
    if (!e || !p) return BH_E_INVALID;
    ASYNC_GUARD(e);
    Geometry g;
    TRY(make_geometry(*p, g, e->err));
    if (e->multi) {
        e->p = *p;
        e->geo = g;
    }
    MULTI_BOTH(e, bh_set_params(m_, p));
    HIPCHK(e, hipSetDevice(e->device));
    const bool geo_changed = std::memcmp(&g, &e->geo, sizeof(g)) != 0;
    if (p->merge_max_mass != e->p.merge_max_mass || p->merge_min_dist != e->p.merge_min_dist)
        e->heavy_possible = true;
    e->p = *p;
    if (geo_changed) {
        TRY(materialize_positions(e));
        if (e->view_pending) {
            // the prebuilt tree (and its jitter) belong to the old root cell: back to the state the
            // caller sees, in its own slot order (the lane map described the prebuilt order)
            std::swap(e->st, e->view);
            e->view_pending = false;
            e->lanes_valid = e->lr_pending = e->lr_ready = false;
        }
        TRY(drop_carried_flags(e));
        e->prebuilt = false;
        e->lt_aside = false;
        e->boxes_valid = false;  // another grid
        e->geo = g;
        e->tree_valid = false;
        e->lazy_tree = false;
        e->spl_nb = 0;  // keys change meaning
        e->keys_ready = false;
        e->lanes_valid = e->lr_pending = e->lr_ready = false;
        e->inv_valid = false;
        if (g.J != e->J_alloc) {  // tree workspace sized for another depth; the state stays
            SYNC(e, e->stream);
            TRY(ensure_capacity(e, e->n));
        }
    }
    return BH_OK;
}

int bh_get_params(const bh_engine *e, bh_params *p) {
    if (!e || !p) return BH_E_INVALID;
    e = MULTI_M0(e);
    *p = e->p;
    return BH_OK;
}

int bh_reset_bodies(bh_engine *e, int64_t n, const double *x, const double *y, const double *vx,
                    const double *vy, const double *m) {
    if (!e || n < 0 || (n > 0 && (!x || !y || !vx || !vy || !m))) return BH_E_INVALID;
    ASYNC_GUARD(e);
    if (n >= (int64_t)NODE_BODY_MASK) {
        e->err = "too many bodies";
        return BH_E_INVALID;
    }
    if (e->multi) {  // resetBodies picks the engine for this body list (BHA:377's min(cores, n))
        const bool one = n < e->multi_min;
        if (one && !e->one) {
            bh_engine *m0 = multi_member(e->multi, 0);
            bh_engine *o = nullptr;
            const int rc = bh_create(&m0->p, m0->device, &o);
            if (rc != BH_OK) {
                e->err = "the single-GPU engine for a small body list could not be created";
                return rc;
            }
            if (m0->mirror_on) TRY(bh_set_mirror(o, m0->mir_nbuf));
            TRY(bh_set_profiling(o, m0->profiling ? 1 : 0));
            e->one = o;
        }
        e->use_one = one;
    }
    if (e->multi) TRY(multi_repair(e->multi, e));  // after a failed call: fresh communicators
    MULTI_ALL(e, bh_reset_bodies(m_, n, x, y, vx, vy, m));
    e->prog_api.store(++e->api_calls);
    HIPCHK(e, hipSetDevice(e->device));
    if (multi_rank(e) && (e->comm_failed || e->comm_lost || peers_aborted(e))) {
        // the way back from a failed call: every stream idle, the group's barriers usable again
        if (e->comm_lost) {
            e->err = "bh_reset_bodies: the RCCL communicator was aborted after a failed call; "
                     "create the engine anew";
            return BH_E_COMM;
        }
        for (hipStream_t s : {e->stream, e->stream2, e->comm_stream, e->pipe_stream, e->mir_stream})
            if (drain_stream(s, 30.0) != hipSuccess) {
                e->err = "bh_reset_bodies: a stream did not drain after the failed call";
                return BH_E_DEVICE;
            }
        e->comm_failed = false;
        e->fail_msg.clear();
        if (e->group) e->group->reset();
    }
    SYNC(e, e->stream);
    TRY(drop_carried_flags(e));
    e->vel_perm = nullptr;  // (the state is replaced)
    TRY(ensure_capacity(e, n));
    if (n > 0) {  // slot order = caller order until the first build
        HIPCHK(e, hipMemcpyAsync(e->st.x, x, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->st.y, y, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->st.vx, vx, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->st.vy, vy, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
        HIPCHK(e, hipMemcpyAsync(e->st.m, m, sizeof(double) * n, hipMemcpyHostToDevice, e->stream));
        iota_u32(e->st.cidx, n, e->stream);
        HIPCHK(e, hipGetLastError());
    }
    SYNC(e, e->stream);
    e->n = n;
    e->heavy_possible = true;
    e->removed.clear();
    e->tree_valid = false;  // BHA:348
    e->lazy_tree = false;
    e->prebuilt = false;    // other bodies: the pipelined call's next tree is void
    e->view_pending = false;
    e->lt_aside = false;
    e->mir_fresh = false;
    e->spl_nb = 0;          // other bodies: the first build sorts from scratch
    e->keys_ready = false;
    e->lanes_valid = e->lr_pending = e->lr_ready = false;
    e->st_morton = false;
    e->vel_stale = false;
    e->pos_pending = false;
    e->inv_valid = false;
    e->boxes_valid = false;
    return BH_OK;
}

static int step_call(bh_engine *e, int32_t k);
static int step_call_rank(bh_engine *e, int32_t k);

int bh_step(bh_engine *e, int32_t k) {
    if (!e || k < 0) return BH_E_INVALID;
    ASYNC_GUARD(e);
    return step_call(e, k);
}

// bh_step's work (bh_step_begin's thread calls it directly): a multi-device handle's members, or
// this engine's steps -- a rank of a decomposition refuses them after a failed call, and a call
// that fails on it aborts its peers' waits (fail_multi_rank)
static int step_call(bh_engine *e, int32_t k) {
    MULTI_ALL(e, bh_step(m_, k));  // every GPU's share of every step, joined (BHA:374-395, 408)
    COMM_GUARD(e);
    e->prog_busy.store(1);
    const int rc = fail_multi_rank(e, step_call_rank(e, k));
    e->prog_busy.store(0);
    return rc;
}

static int step_call_rank(bh_engine *e, int32_t k) {
    e->prog_api.store(++e->api_calls);
    HIPCHK(e, hipSetDevice(e->device));
    const bool may_merge = k > 0 && e->n > 1 && e->p.merge_min_dist > 0.0 && e->heavy_possible;
    // a multi-rank call with LET builds may have to be replayed with a larger subset capacity
    const bool may_let = k > 0 && e->n > 0 && (e->comm || e->group || e->solo) && let_active(e) &&
                         e->p.theta != 0.0;
    if (may_merge || may_let) TRY(snapshot(e));
    // the previous call's pipelined last step built this call's first tree (a replay does not
    // use it: restore() starts from the caller-visible state)
    const bool carried = k > 0 && e->prebuilt;
    if (k > 0) {
        e->mir_fresh = false;
        e->lt_aside = false;  // lastTree will be this call's (nodes_alt is rebuilt below)
    }
    int let_replays = 0;
    for (bool first = true;; first = false) {
        e->ev_used = 0;
        e->timings_pending = false;
        if (!first && e->mid_armed) {  // a replay: an earlier attempt's hand-off is void
            std::lock_guard<std::mutex> lk(e->mid_mu);
            e->mid_void = true;
        }
        // the subset splitters are trusted only within a call (another scene after a reset
        // would put most of a subset into one bucket): the first LET build sorts with rocprim
        e->s_spl_nb = 0;
        HIPCHK(e, hipMemsetAsync(e->scalars + 1, 0, 5 * sizeof(uint32_t), e->stream));
        e->removed.clear();
        e->merge_ran = false;
        if (k > 0) e->prebuilt = first && carried;
        e->lazy_tree = false;
        e->mir_launched = false;
        for (int32_t s = 0; s < k; ++s) TRY(step_once(e, s + 1 == k));
        // a copy-out launched by the last pipelined step reads the state the compaction (or a
        // replay's restore) below rewrites
        if (e->mir_launched) HIPCHK(e, hipStreamWaitEvent(e->stream, e->mir_ev2, 0));
        // (one GPU: no wait here -- the merge bookkeeping's read-back below, or the tree flags'
        // when nothing merged, is queued behind the steps and waited for once)
        if (may_let) SYNC(e, e->stream);
        if (may_let) {  // LET subset sizes of this call: [4] some rank overflowed, [5] largest
            uint32_t ls[2] = {0, 0};
            // [4] can be set after the cell tables were exchanged (k_let_guard, k_let_w): on one
            // rank only.  Every rank must take the same decision, or one replays alone and issues
            // collectives its peers never match -- so the flags are max-reduced over the ranks.
            uint32_t own_sub = 0;
            TRY(agree_let_flags(e, ls, &own_sub));
            if (ls[1] > 0) {
                e->let_last_sub = own_sub;
                e->let_known = std::max<int64_t>(ls[1], ls[0] ? e->let_known : 1);
            }
            if (ls[0]) {  // every rank saw the overflow (exchanged): all replay the call
                // (the builds after an overflow saw a damaged state, so a replay can meet a
                // larger subset than observed; the third replay builds subsets of any size)
                if (++let_replays >= 3) e->let_known = e->n;
                ++e->let_overflows;
                e->removed.clear();
                e->merge_ran = false;
                TRY(restore(e));
                continue;
            }
        }
        // every replica complete at the API boundary: after a call that ended with a LET
        // evaluation the positions are in the exchange buffer and the peers' velocities with
        // their owners (every rank runs this: the velocity all-gather is collective)
        if (e->vel_stale && k > 0) {
            TRY(materialize_positions(e));
            TRY(sync_velocities(e));
        }
        // the merge bookkeeping first, so that an error below leaves a compacted state
        uint32_t overflow = 0, tflags = 0;
        bool have_flags = false;
        TRY(finish_merges(e, &overflow, &tflags, &have_flags));  // (reads the flags too)
        int tree_rc = BH_OK;
        if (e->n > 0 && k > 0) {
            if (!have_flags) {
                tree_rc = check_tree_flags(e);
            } else if (tflags) {
                e->err = "jitter replay reached an unsupported geometry (body stayed inside a "
                         "depth J+1 cell)";
                tree_rc = BH_E_STATE;
            }
        }
        if (overflow) {  // a step's candidate pairs exceeded the mailbox: replay the call
            if (!may_merge) {
                e->err = "merge rule: candidate mailbox overflow without a snapshot";
                return BH_E_STATE;
            }
            e->box_need = (uint32_t)std::min<uint64_t>(0xFFFFFFF0ull, 2ull * overflow);
            TRY(merge_bufs(e));
            TRY(restore(e));
            continue;
        }
        if (tree_rc != BH_OK) return tree_rc;
        break;
    }
    if (k > 0 && e->mirror_on) {
        if (!e->mir_launched)  // the call's last step was not pipelined: copy out now
            TRY(mirror_launch(e, e->view_pending ? e->view : e->st, e->stream, e->stream));
        // the next call reuses the buffers the mirror's kernels read (not its host copies)
        HIPCHK(e, hipStreamWaitEvent(e->stream, e->mir_ev2, 0));
        e->mir_fresh = true;
        e->mir_n = e->n;
    }
    if (e->profiling) TRY(collect_timings(e));
    return BH_OK;
}

int bh_step_begin(bh_engine *e, int32_t k) {
    if (!e || k < 0) return BH_E_INVALID;
    if (e->async_running) return BH_E_STATE;  // (its call may be writing the error text)
    bh_engine *t = MULTI_M0(e);  // the engine whose mirror the call fills
    if (!t->mirror_on || t->mir_nbuf != 2) {
        e->err = "bh_step_begin: needs the two-buffer mirror (bh_set_mirror(e, 2))";
        return BH_E_STATE;
    }
    if (e->step_thr.joinable()) e->step_thr.join();
    {
        std::lock_guard<std::mutex> lk(t->mid_mu);
        t->mid_armed = k > 0;
        t->mid_ready = t->mid_done = t->mid_void = false;
    }
    e->mid_eng = t;
    e->mid_n0 = t->n;
    e->mid_surv_done = false;
    e->async_rc = BH_OK;
    e->async_running = true;
    e->step_thr = std::thread([e, t, k] {
        const int rc = step_call(e, k);
        {
            std::lock_guard<std::mutex> lk(t->mid_mu);
            e->async_rc = rc;
            t->mid_armed = false;
            t->mid_done = true;
        }
        t->mid_cv.notify_all();
    });
    return BH_OK;
}

int bh_step_positions(bh_engine *e, const double **x, const double **y, const double **m,
                      const uint32_t **survivors, int64_t *n_out, int64_t *n_before) {
    if (!e) return BH_E_INVALID;
    if (!e->async_running || !e->mid_eng) {
        e->err = "bh_step_positions: no call begun (bh_step_begin)";
        return BH_E_STATE;
    }
    bh_engine *t = e->mid_eng;
    const double *buf = nullptr;
    int64_t stride = 0, n = 0;
    std::unique_lock<std::mutex> lk(t->mid_mu);
    t->mid_cv.wait(lk, [t] { return t->mid_ready || t->mid_done; });
    if (!t->mid_done && !t->mid_void) {  // the hand-off: usable unless the call will replay
        buf = t->mid_buf;
        stride = t->mid_stride;
        lk.unlock();
        // x, y, m not asked for: the survivors are enough (their copy runs ahead of the planes')
        HIPCHK(e, hipEventSynchronize(x || y || m ? t->mid_ev : t->mid_sv_ev));
        const uint32_t *h = t->mir_idx;  // scalars[1] tree flags, [2] removals, [3] overflow
        n = e->mid_n0 - (int64_t)h[2];
        lk.lock();
        if (h[1] || h[3] || t->mid_void) buf = nullptr;  // an error or a replay follows: the end
    }
    if (!buf) {  // no hand-off (a call whose last step is not pipelined, or a replay): the end
        t->mid_cv.wait(lk, [t] { return t->mid_done; });
        lk.unlock();
        if (e->async_rc != BH_OK) return e->async_rc;
        HIPCHK(e, hipEventSynchronize(t->mir_ev));
        buf = t->mir;
        stride = t->mir_cap;
        n = t->mir_n;
        if (!e->mid_surv_done) {  // the survivors from the call's removals: a mirror written
            // after the call's compaction numbers its bodies in the list after the call
            int64_t nr = 0;
            int rc = last_removed(e, nullptr, 0, &nr);
            if (rc != BH_OK && rc != BH_E_CAPACITY) return rc;
            std::vector<int64_t> rem((size_t)std::max<int64_t>(nr, 1));
            TRY(last_removed(e, rem.data(), nr, &nr));
            uint32_t *sv = t->mir_idx + MIRROR_HDR;
            int64_t j = 0, r = 0;
            for (int64_t i = 0; i < e->mid_n0; ++i) {
                if (r < nr && rem[(size_t)r] == i) {
                    ++r;
                    continue;
                }
                sv[j++] = (uint32_t)i;
            }
            if (j != n) {
                e->err = "bh_step_positions: the removals do not match the mirror";
                return BH_E_STATE;
            }
            e->mid_surv_done = true;
        }
    }
    if (x) *x = buf;
    if (y) *y = buf + stride;
    if (m) *m = buf + 4 * stride;
    if (survivors) *survivors = t->mir_idx + MIRROR_HDR;
    if (n_out) *n_out = n;
    if (n_before) *n_before = e->mid_n0;
    return BH_OK;
}

int bh_step_end(bh_engine *e) {
    if (!e) return BH_E_INVALID;
    if (!e->async_running) {
        e->err = "bh_step_end: no call begun (bh_step_begin)";
        return BH_E_STATE;
    }
    e->step_thr.join();
    e->async_running = false;
    e->mid_eng = nullptr;
    return e->async_rc;
}

int64_t bh_num_bodies(const bh_engine *e) {
    if (!e) return -1;
    if (e->async_running && std::this_thread::get_id() != e->step_thr.get_id())
        return -1;  // (a call begun by bh_step_begin writes n: ask after bh_step_end)
    return MULTI_M0(e)->n;
}

int bh_get_bodies(bh_engine *e, double *x, double *y, double *vx, double *vy, double *m,
                  int64_t cap, int64_t *n_out) {
    if (!e) return BH_E_INVALID;
    ASYNC_GUARD(e);
    if (e->multi) {  // every replica is complete at the API boundary: member 0's
        const int rc = bh_get_bodies(MULTI_M0(e), x, y, vx, vy, m, cap, n_out);
        if (rc != BH_OK) e->err = bh_last_error(MULTI_M0(e));
        return rc;
    }
    COMM_GUARD(e);  // (a failed call's replica is not the reference's state)
    if (n_out) *n_out = e->n;
    if (cap < e->n) return BH_E_CAPACITY;
    HIPCHK(e, hipSetDevice(e->device));
    TRY(materialize_positions(e));
    const int64_t n = e->n;
    if (n > 0) {  // back to caller (list) order, staged in the second state buffer
        const BodyState &s = e->view_pending ? e->view : e->st;  // (not the prebuilt tree's jitter)
        const double *src[5] = {s.x, s.y, s.vx, s.vy, s.m};
        double *stage[5] = {e->alt.x, e->alt.y, e->alt.vx, e->alt.vy, e->alt.m};
        scatter_to_caller(n, s.cidx, 5, src, stage, e->stream);
        HIPCHK(e, hipGetLastError());
        double *dst[5] = {x, y, vx, vy, m};
        for (int k = 0; k < 5; ++k)
            if (dst[k])
                HIPCHK(e, hipMemcpyAsync(dst[k], stage[k], sizeof(double) * n,
                                         hipMemcpyDeviceToHost, e->stream));
    }
    SYNC(e, e->stream);
    return BH_OK;
}

int bh_set_mirror(bh_engine *e, int enabled) {
    if (!e) return BH_E_INVALID;
    ASYNC_GUARD(e);
    if (enabled < 0 || enabled > 2) {
        e->err = "bh_set_mirror: enabled is 0, 1 or 2";
        return BH_E_INVALID;
    }
    // (member 0's replica fills the mirror; the others' bh_set_mirror only reserves its stream)
    MULTI_BOTH(e, r_ == 0 ? bh_set_mirror(m_, enabled) : BH_OK);
    HIPCHK(e, hipSetDevice(e->device));
    e->mirror_on = enabled != 0;
    if (e->mirror_on && enabled != e->mir_nbuf) {  // another buffer count: made anew
        if (e->mir_stream) SYNC(e, e->mir_stream);
        e->mir_nbuf = enabled;
        e->mir_cap = 0;
        e->mir_fresh = false;
    }
    if (e->mirror_on) TRY(mirror_alloc(e));
    return BH_OK;
}

int bh_map_bodies(bh_engine *e, const double **x, const double **y, const double **vx,
                  const double **vy, const double **m, int64_t *n_out) {
    if (!e) return BH_E_INVALID;
    ASYNC_GUARD(e);
    if (e->multi) {
        const int rc = bh_map_bodies(MULTI_M0(e), x, y, vx, vy, m, n_out);
        if (rc != BH_OK) e->err = bh_last_error(MULTI_M0(e));
        return rc;
    }
    COMM_GUARD(e);
    HIPCHK(e, hipSetDevice(e->device));
    if (!e->mir_fresh || e->mir_cap < e->n) {  // not written by the last call: copy out now
        TRY(materialize_positions(e));
        e->mir_launched = false;
        TRY(mirror_launch(e, e->view_pending ? e->view : e->st, e->stream, e->stream));
        HIPCHK(e, hipStreamWaitEvent(e->stream, e->mir_ev2, 0));
        e->mir_fresh = true;
        e->mir_n = e->n;
    }
    HIPCHK(e, hipEventSynchronize(e->mir_ev));
    const int64_t c = e->mir_cap;
    const double *b = e->mir;
    e->mir_front = b == e->mir_buf[1] ? 1 : 0;
    if (x) *x = b;
    if (y) *y = b + c;
    if (vx) *vx = b + 2 * c;
    if (vy) *vy = b + 3 * c;
    if (m) *m = b + 4 * c;
    if (n_out) *n_out = e->mir_n;
    return BH_OK;
}

static int compute_accelerations_rank(bh_engine *e, double *ax, double *ay, int64_t *visits);

int bh_compute_accelerations(bh_engine *e, double *ax, double *ay, int64_t *visits) {
    if (!e) return BH_E_INVALID;
    ASYNC_GUARD(e);
    // (every member builds and evaluates -- the build may jitter every replica alike; member 0
    // hands the results out)
    if (e->multi) {  // (the visit-counting walk is not sharded: every member counts)
        std::vector<std::vector<int64_t>> vis((size_t)multi_world(e->multi));
        const int64_t nb = bh_num_bodies(e);
        if (visits)
            for (size_t r = 1; r < vis.size(); ++r) vis[r].resize((size_t)std::max<int64_t>(nb, 1));
        MULTI_ALL(e, bh_compute_accelerations(m_, r_ == 0 ? ax : nullptr, r_ == 0 ? ay : nullptr,
                                              !visits ? nullptr
                                                      : r_ == 0 ? visits : vis[(size_t)r_].data()));
    }
    COMM_GUARD(e);
    return fail_multi_rank(e, compute_accelerations_rank(e, ax, ay, visits));
}

static int compute_accelerations_rank(bh_engine *e, double *ax, double *ay, int64_t *visits) {
    e->prog_api.store(++e->api_calls);
    HIPCHK(e, hipSetDevice(e->device));
    const int64_t n = e->n;
    e->ev_used = 0;
    e->timings_pending = false;
    HIPCHK(e, hipMemsetAsync(e->scalars + 1, 0, sizeof(uint32_t), e->stream));
    if (n > 0) {
        TRY(evaluate(e, visits ? e->visits32 : nullptr));
        e->mir_fresh = false;
        scatter_acc_to_caller(n, e->st.cidx, e->a2, e->ax, e->ay, e->stream, e->a2_lanes,
                              e->a2_layout);
        HIPCHK(e, hipGetLastError());
        SYNC(e, e->stream);
        TRY(check_tree_flags(e));
        if (ax) HIPCHK(e, hipMemcpy(ax, e->ax, sizeof(double) * n, hipMemcpyDeviceToHost));
        if (ay) HIPCHK(e, hipMemcpy(ay, e->ay, sizeof(double) * n, hipMemcpyDeviceToHost));
        if (visits) {
            std::vector<uint32_t> v((size_t)n), c((size_t)n);
            HIPCHK(e, hipMemcpy(v.data(), e->visits32, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
            HIPCHK(e, hipMemcpy(c.data(), e->st.cidx, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
            int64_t lane_sum = 0;
            for (int64_t i = 0; i < n; ++i) {
                visits[c[(size_t)i]] = v[(size_t)i];
                lane_sum += v[(size_t)i];
            }
            HIPCHK(e, hipMemcpy(v.data(), e->contrib32, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
            int64_t contrib_sum = 0;
            for (int64_t i = 0; i < n; ++i) contrib_sum += v[(size_t)i];
            const int64_t waves = (n + 63) / 64;
            std::vector<uint32_t> wi((size_t)waves), wb((size_t)waves);
            HIPCHK(e, hipMemcpy(wi.data(), e->wave_iters, sizeof(uint32_t) * waves,
                                hipMemcpyDeviceToHost));
            HIPCHK(e, hipMemcpy(wb.data(), e->wave_blocks, sizeof(uint32_t) * waves,
                                hipMemcpyDeviceToHost));
            int64_t wsum = 0, bsum = 0;
            for (uint32_t w : wi) wsum += w;
            for (uint32_t w : wb) bsum += w;
            e->stat_lane_visits = lane_sum;
            e->stat_lane_contrib = contrib_sum;
            e->stat_wave_iters = wsum;
            e->stat_wave_blocks = bsum;
            e->stat_waves = waves;
        }
    }
    if (e->profiling) TRY(collect_timings(e));
    return BH_OK;
}

int bh_get_quads(bh_engine *e, double *cx, double *cy, double *h, int64_t cap, int64_t *n_out) {
    if (!e || cap < 0 || (cap > 0 && (!cx || !cy || !h))) return BH_E_INVALID;
    ASYNC_GUARD(e);
    if (e->multi) {  // every member builds getTreeForDebug's tree (the same jitter in every
                     // replica); member 0 walks it
        const int rc = multi_fan(e, [](bh_engine *m, int) {
            TRY(comm_refused(m));
            return fail_multi_rank(m, quads_prepare(m));
        }, false);
        if (rc != BH_OK) return rc;
        const int rc0 = bh_get_quads(MULTI_M0(e), cx, cy, h, cap, n_out);
        if (rc0 != BH_OK) e->err = bh_last_error(MULTI_M0(e));
        return rc0;
    }
    COMM_GUARD(e);
    TRY(fail_multi_rank(e, quads_prepare(e)));
    const int64_t n = e->n;
    std::vector<uint64_t> keys((size_t)n);
    std::vector<int8_t> cpl((size_t)n);
    std::vector<uint32_t> base((size_t)n + 1);
    SYNC(e, e->stream);
    // lastTree kept aside by a pipelined last step, or the tree in the build buffers
    const bool aside = e->tree_valid && e->lt_aside;
    if (n > 0) {
        HIPCHK(e, hipMemcpy(keys.data(), aside ? e->lt_keys : e->keys_s, sizeof(uint64_t) * n,
                            hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(cpl.data(), aside ? e->lt_cpl : e->cpl, n, hipMemcpyDeviceToHost));
        HIPCHK(e, hipMemcpy(base.data(), aside ? e->lt_base : e->base, sizeof(uint32_t) * (n + 1),
                            hipMemcpyDeviceToHost));
    }
    int64_t M = 0;
    const uint64_t SENT = sentinel_key(e->geo.J);
    while (M < n && keys[(size_t)M] != SENT) ++M;
    QuadWalker w{e->geo, keys, cpl, base, aside ? e->nodes_alt : e->nodes, cx, cy, h, cap};
    w.rec(0, 0, M, e->geo.root_cx, e->geo.root_cy, e->geo.root_h);
    if (w.rc != BH_OK) return w.rc;
    if (n_out) *n_out = w.k;
    return w.k > cap ? BH_E_CAPACITY : BH_OK;
}

int bh_last_removed(const bh_engine *e, int64_t *idx, int64_t cap, int64_t *n_out) {
    if (!e || cap < 0 || (cap > 0 && !idx)) return BH_E_INVALID;
    // (a call begun by bh_step_begin writes the log: read it after bh_step_end)
    if (e->async_running && std::this_thread::get_id() != e->step_thr.get_id()) return BH_E_STATE;
    return last_removed(e, idx, cap, n_out);
}

static int last_removed(const bh_engine *e, int64_t *idx, int64_t cap, int64_t *n_out) {
    e = MULTI_M0(e);
    // caller indices are not renumbered inside a call, so the log is already relative to the
    // list before the call
    if (n_out) *n_out = (int64_t)e->removed.size();
    if ((int64_t)e->removed.size() > cap) return BH_E_CAPACITY;
    for (size_t i = 0; i < e->removed.size(); ++i) idx[i] = e->removed[i];
    return BH_OK;
}

int bh_last_timings(const bh_engine *e, double *out5) {
    if (!e || !out5) return BH_E_INVALID;
    e = MULTI_M0(e);
    for (int k = 0; k < kPhases; ++k) out5[k] = e->phase_ms[k];
    return BH_OK;
}

int64_t bh_last_tree_nodes(const bh_engine *e) {
    if (e) e = MULTI_M0(e);
    if (!e || e->n <= 0) return 0;
    uint32_t T = 0;
    const uint32_t *base = e->lt_aside ? e->lt_base : e->base;
    if (hipMemcpy(&T, base + e->n, sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return T;
}

int bh_traverse_kernel_ms(const bh_engine *e, double *avg_ms, int64_t *launches) {
    if (!e || !avg_ms) return BH_E_INVALID;
    e = MULTI_M0(e);
    *avg_ms = e->trav_launches ? e->trav_ms_sum / (double)e->trav_launches : 0.0;
    if (launches) *launches = e->trav_launches;
    return BH_OK;
}

int bh_traverse_kernel_samples(const bh_engine *e, double *ms, int64_t cap, int64_t *n_out) {
    if (!e || cap < 0 || (cap > 0 && !ms)) return BH_E_INVALID;
    e = MULTI_M0(e);
    const int64_t n = (int64_t)e->trav_samples.size();
    if (n_out) *n_out = n;
    if (n > cap) return BH_E_CAPACITY;
    for (int64_t i = 0; i < n; ++i) ms[i] = e->trav_samples[(size_t)i];
    return BH_OK;
}

int bh_traversal_stats(const bh_engine *e, int64_t *lane_visits, int64_t *wave_iters,
                       int64_t *waves) {
    if (!e || !lane_visits || !wave_iters || !waves) return BH_E_INVALID;
    e = MULTI_M0(e);
    *lane_visits = e->stat_lane_visits;
    *wave_iters = e->stat_wave_iters;
    *waves = e->stat_waves;
    return BH_OK;
}

int bh_traversal_counters(const bh_engine *e, int64_t *out5) {
    if (!e || !out5) return BH_E_INVALID;
    e = MULTI_M0(e);
    out5[0] = e->stat_lane_visits;
    out5[1] = e->stat_lane_contrib;
    out5[2] = e->stat_wave_iters;
    out5[3] = e->stat_wave_blocks;
    out5[4] = e->stat_waves;
    return BH_OK;
}

int bh_let_stats(const bh_engine *e, int64_t *out4) {
    if (!e || !out4) return BH_E_INVALID;
    e = MULTI_M0(e);
    out4[4] = e->let_overflows;
    out4[0] = e->let_builds;
    out4[1] = e->full_builds;
    out4[2] = e->let_last_sub;
    uint32_t T = 0;
    if (e->L.posc &&
        hipMemcpy(&T, e->L.posc + LET_CELLS, sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return BH_E_DEVICE;
    out4[3] = T;
    return BH_OK;
}

int bh_set_profiling(bh_engine *e, int enabled) {
    if (!e) return BH_E_INVALID;
    ASYNC_GUARD(e);
    MULTI_BOTH(e, bh_set_profiling(m_, enabled));
    e->profiling = enabled != 0;
    return BH_OK;
}

int bh_shard_range(int64_t n, int rank, int world, int round, int64_t *lo, int64_t *hi) {
    if (n < 0 || world < 1 || rank < 0 || rank >= world || round < 0 ||
        round >= BH_SHARD_ROUNDS || !lo || !hi)
        return BH_E_INVALID;
    const GatherLayout L = shard_layout(n, world);  // whole wavefronts
    *lo = std::min<int64_t>(n, (int64_t)rank * L.span + L.off[round]);  // in the own range
    *hi = std::min<int64_t>(n, (int64_t)rank * L.span + L.off[round + 1]);
    return BH_OK;
}

int64_t bh_gather_slot(int64_t n, int world, int64_t lane) {
    if (n < 0 || world < 1 || lane < 0) return -1;
    return gather_slot(shard_layout(n, world), lane);
}

int bh_selftest_fast_math(int device, int64_t n, uint64_t seed, int64_t *mismatches) {
    if (!mismatches || n < 0) return BH_E_INVALID;
    *mismatches = -1;
    unsigned long long *d_bad = nullptr, h_bad = 0;
    if (hipSetDevice(device) != hipSuccess) return BH_E_DEVICE;
    if (hipMalloc((void **)&d_bad, sizeof(*d_bad)) != hipSuccess) return BH_E_DEVICE;
    bool ok = hipMemset(d_bad, 0, sizeof(*d_bad)) == hipSuccess &&
              bh::selftest_fast_math(n, seed, d_bad, nullptr) == hipSuccess &&
              hipMemcpy(&h_bad, d_bad, sizeof(h_bad), hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipFree(d_bad);
    if (!ok) return BH_E_DEVICE;
    *mismatches = (int64_t)h_bad;
    return BH_OK;
}

int bh_synchronize(bh_engine *e) {
    if (!e) return BH_E_INVALID;
    ASYNC_GUARD(e);
    MULTI_ALL(e, bh_synchronize(m_));
    HIPCHK(e, hipSetDevice(e->device));
    SYNC(e, e->stream);
    return BH_OK;
}

int bh_comm_ranks(const bh_engine *e, int32_t *nranks, int32_t *rank) {
    if (!e || !nranks || !rank) return BH_E_INVALID;
    e = MULTI_M0(e);
    *nranks = 0;
    *rank = e->rank;
    if (!e->comm) return BH_OK;
    int c = 0, r = 0;
    if (ncclCommCount(e->comm, &c) != ncclSuccess || ncclCommUserRank(e->comm, &r) != ncclSuccess)
        return BH_E_COMM;
    *nranks = c;
    *rank = r;
    return BH_OK;
}

int bh_debug_inject(bh_engine *e, int what) {
    if (!e) return BH_E_INVALID;
    ASYNC_GUARD(e);
    MULTI_ALL(e, bh_debug_inject(m_, what));  // (one member alone: bh_multi_member)
    if (what < 1 || what >= 300) {
        e->err = "bh_debug_inject: unknown fault";
        return BH_E_INVALID;
    }
    if (what == 99) {  // the carried tree (the next call's first) raises its error flag now
        if (!e->carried_flags || !e->prebuilt) {
            e->err = "bh_debug_inject(99): no tree carried to the next call";
            return BH_E_STATE;
        }
        HIPCHK(e, hipMemsetAsync(e->scalars + 10, 1, sizeof(uint32_t), e->stream));
        return BH_OK;
    }
    if (what == 1) e->inject_guard = true;
    else if (what >= 200) e->inject_barrier = what - 200;
    else if (what >= 100) e->inject_coll = what - 100;
    else e->inject_build = what - 2;
    return BH_OK;
}

int bh_progress(const bh_engine *e, int64_t *out4) {
    if (!e || !out4) return BH_E_INVALID;
    e = MULTI_M0(e);  // (a member's own: bh_multi_member)
    out4[0] = e->prog_api.load();
    out4[1] = e->prog_coll.load();
    out4[2] = e->prog_site.load();
    const bool failed = e->comm_failed || (multi_rank(e) && peers_aborted(e));  // (will refuse)
    out4[3] = (e->prog_busy.load() ? 1 : 0) | (failed ? 2 : 0) | (e->comm_lost ? 4 : 0);
    return BH_OK;
}

int bh_multi_world(const bh_engine *e) {
    if (!e) return 0;
    return e->multi && !e->use_one ? multi_world(e->multi) : 1;
}

bh_engine *bh_multi_member(bh_engine *e, int rank) {
    if (!e) return nullptr;
    if (!e->multi) return rank == 0 ? e : nullptr;
    if (e->use_one) return rank == 0 ? e->one : nullptr;
    return multi_member(e->multi, rank);
}

int bh_collective_log(const bh_engine *e, int64_t *out4, int64_t cap, int64_t *n_out) {
    if (!e || cap < 0 || (cap > 0 && !out4)) return BH_E_INVALID;
    e = MULTI_M0(e);
    const int64_t n = (int64_t)e->coll_log.size() / 4;
    if (n_out) *n_out = n;
    if (n > cap) return BH_E_CAPACITY;
    std::copy(e->coll_log.begin(), e->coll_log.end(), out4);
    return BH_OK;
}

int bh_collective_log_clear(bh_engine *e) {
    if (!e) return BH_E_INVALID;
    ASYNC_GUARD(e);
    MULTI_BOTH(e, bh_collective_log_clear(m_));
    e->coll_log.clear();
    return BH_OK;
}

}  // extern "C"
