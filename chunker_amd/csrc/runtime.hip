// runtime.hip -- host runtime behind the C ABI (include/chunker_gpu.h).
//
// Per device: a pool of workspaces (device scratch grown on demand, a pinned
// staging area, an own stream, timing events), the uploaded GEAR table, and lazy
// once-only initialisation.  Every call takes a workspace from the pool, so the ABI
// is re-entrant for the reference's concurrent callers (HTTP thread per
// connection, BEAM dirty schedulers, rayon).  There is no CPU fallback: without a
// usable gfx950 device every compute entry point returns CG_E_NO_DEVICE.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gear_table.h"
#include "runtime.h"

namespace cgrt {

static_assert(sizeof(cg_desc) == 48, "cg_desc must be 48 bytes");

thread_local std::string t_err;
thread_local uint64_t t_detail[3];  // ChunkingError fields of the last failure (cg_last_error_detail)
thread_local int t_status = CG_OK;
thread_local std::vector<double> t_stage_ms;
std::atomic<int> g_profiling{0};
#ifndef CG_B3_FUSED_PLAN
#define CG_B3_FUSED_PLAN 1
#endif
// BLAKE3 group map built by the walk + assembly (1) or by k_b3_plan (0): test hook
// cg_test_b3_fused_plan
std::atomic<int> g_b3_fused_plan{CG_B3_FUSED_PLAN};
#ifndef CG_B3_PACKED
#define CG_B3_PACKED 1
#endif
// BLAKE3 leaves packed across chunks (k_b3_leaves, with the assembly-built map) or one
// 64-leaf group per wave (k_b3_groups): test hook cg_test_b3_packed
std::atomic<int> g_b3_packed{CG_B3_PACKED};

int fail(int code, const std::string &msg) {
    t_err = msg;
    t_status = code;
    t_detail[0] = t_detail[1] = t_detail[2] = 0;
    return code;
}

void clear_error() {
    t_err.clear();
    t_status = CG_OK;
    t_detail[0] = t_detail[1] = t_detail[2] = 0;
}

// ChunkingError::Bounds { data_len, offset, length } (src/chunking.rs:38-42)
int fail_bounds(uint64_t data_len, uint64_t offset, uint64_t length, const std::string &what) {
    fail(CG_E_BOUNDS, what);
    t_detail[0] = data_len;
    t_detail[1] = offset;
    t_detail[2] = length;
    return CG_E_BOUNDS;
}

// ChunkingError::BufferLimitExceeded { attempted, limit } (src/chunking.rs:49-50): a device
// allocation of `attempted` bytes failed with `limit` bytes of device memory free.
int fail_limit(uint64_t attempted, const std::string &what) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
    fail(CG_E_BUFFER_LIMIT, what);
    t_detail[0] = attempted;
    t_detail[1] = free_b;
    return CG_E_BUFFER_LIMIT;
}

int fail_detail(int code, const std::string &msg, const uint64_t detail[3]) {
    fail(code, msg);
    for (int i = 0; i < 3; ++i) t_detail[i] = detail[i];
    return code;
}

static std::atomic<uint32_t> g_fail_alloc{0};  // countdown: the allocation that takes it to 0 fails

bool test_alloc_fault() {
    uint32_t v = g_fail_alloc.load(std::memory_order_relaxed);
    while (v != 0)
        if (g_fail_alloc.compare_exchange_weak(v, v - 1, std::memory_order_relaxed)) return v == 1;
    return false;
}

int hip_fail(hipError_t e, const char *what, uint64_t attempted) {
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
        (void)hipGetLastError();  // clear the sticky allocation error
        return fail_limit(attempted, std::string("device allocation failed: ") + what);
    }
    if (e == hipErrorNoDevice || e == hipErrorNoBinaryForGpu || e == hipErrorInvalidDevice)
        return fail(CG_E_NO_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
    return fail(CG_E_IO, std::string(what) + ": " + hipGetErrorString(e));
}

// ---------------------------------------------------------------------------
// FastCDC v2020 tables [ext fastcdc 4.0.1]: GEAR[256] and MASKS[26].  The compiled-in
// set comes from tables/*.txt; cg_set_cdc_tables installs another one process-wide.
// Fail closed: a chunking call refuses to run while the placeholder GEAR is installed,
// and any other table set must first reproduce the reference's golden fixture
// (src/chunking.rs:1266-1297) on the GPU (cg_selftest, run lazily on first use), unless
// CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR=1 -- the test / bench opt-in -- is set.
// ---------------------------------------------------------------------------
std::mutex g_tab_mu;
std::shared_ptr<const Tables> g_tab;
std::atomic<uint64_t> g_tab_epoch{1};
std::atomic<uint64_t> g_verified_epoch{0};  // epoch whose tables passed the selftest

std::shared_ptr<const Tables> tables() {
    std::lock_guard<std::mutex> g(g_tab_mu);
    if (!g_tab) {
        auto t = std::make_shared<Tables>();
        memcpy(t->gear, CG_DEFAULT_GEAR, sizeof t->gear);
        memcpy(t->masks, CG_MASKS, sizeof t->masks);
        t->epoch = g_tab_epoch.load();
        t->placeholder = CG_GEAR_IS_PLACEHOLDER != 0;
        g_tab = t;
    }
    return g_tab;
}

bool allow_unverified_tables() {
    const char *v = getenv("CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR");
    return v && v[0] == '1' && v[1] == 0;
}

uint32_t logarithm2(uint32_t v) { return (uint32_t)std::round(std::log2((double)v)); }

struct DevicePool {
    std::mutex mu;
    std::vector<Workspace *> free_list;
};
constexpr int MAX_DEV = 64;
DevicePool g_pools[MAX_DEV];

int current_device(int *dev) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
        return fail(CG_E_NO_DEVICE, "no HIP device visible: the chunker engine has no CPU fallback");
    HIP_TRY(hipGetDevice(dev));
    if (*dev < 0 || *dev >= MAX_DEV) return fail(CG_E_NO_DEVICE, "device index out of range");
    return CG_OK;
}

int acquire(Workspace **out) {
    int dev = 0, st = current_device(&dev);
    if (st) return st;
    DevicePool &pool = g_pools[dev];
    {
        std::lock_guard<std::mutex> g(pool.mu);
        if (!pool.free_list.empty()) {
            *out = pool.free_list.back();
            pool.free_list.pop_back();
            return CG_OK;
        }
    }
    Workspace *ws = new Workspace();
    st = ws->init(dev);
    if (st) {
        delete ws;
        return st;
    }
    *out = ws;
    return CG_OK;
}

void release(Workspace *ws) {
    DevicePool &pool = g_pools[ws->device];
    std::lock_guard<std::mutex> g(pool.mu);
    pool.free_list.push_back(ws);
}

// Upload the snapshot's GEAR table to this workspace (once per table epoch).
int ensure_gear(Workspace *ws, const Tables &t) {
    if (ws->gear_epoch == t.epoch && ws->gear.p) return CG_OK;
    int st = ws->gear.ensure(256 * sizeof(uint64_t), "gear");
    if (st) return st;
    HIP_TRY(hipMemcpy(ws->gear.p, t.gear, sizeof t.gear, hipMemcpyHostToDevice));
    ws->gear_epoch = t.epoch;
    return CG_OK;
}

// The SHA-256 kernel's spin-guard word (launch_sha256 d_err): zeroed before a digest
// launch, copied back with the call's other results, checked after the stream sync.
int sha_err_arm(Workspace *ws, hipStream_t st) {
    int rc;
    if ((rc = ws->sha_err.ensure(64, "sha err"))) return rc;
    if ((rc = ws->err_stage.ensure(64))) return rc;
    ws->err_stage.as<uint32_t>()[0] = 0;
    HIP_TRY(hipMemsetAsync(ws->sha_err.p, 0, 4, st));
    return CG_OK;
}
int sha_err_fetch(Workspace *ws, hipStream_t st) {
    HIP_TRY(hipMemcpyAsync(ws->err_stage.p, ws->sha_err.p, 4, hipMemcpyDeviceToHost, st));
    return CG_OK;
}
int sha_err_check(Workspace *ws) {  // after the stream sync
    if (ws->err_stage.p && ws->err_stage.as<uint32_t>()[0])
        return fail(CG_E_IO, "SHA-256 digest: a producer/consumer hand-off hit the kernel's spin guard; "
                             "the digests of this call are invalid");
    return CG_OK;
}

int resolve(uint64_t mn, uint64_t avg, uint64_t mx, Opts *o, char *msg, size_t cap) {
    o->min = mn ? mn : DEF_MIN;
    o->avg = avg ? avg : DEF_AVG;
    o->max = mx ? mx : DEF_MAX;
    char buf[160];
    buf[0] = 0;
    int st = CG_OK;
    if (o->min < MINIMUM_MIN || o->min > MINIMUM_MAX) {
        snprintf(buf, sizeof buf, "min_size must be in %llu..=%llu, got %llu", (unsigned long long)MINIMUM_MIN,
                 (unsigned long long)MINIMUM_MAX, (unsigned long long)o->min);
        st = CG_E_INVALID_OPTIONS;
    } else if (o->avg < AVERAGE_MIN || o->avg > AVERAGE_MAX) {
        snprintf(buf, sizeof buf, "avg_size must be in %llu..=%llu, got %llu", (unsigned long long)AVERAGE_MIN,
                 (unsigned long long)AVERAGE_MAX, (unsigned long long)o->avg);
        st = CG_E_INVALID_OPTIONS;
    } else if (o->max < MAXIMUM_MIN || o->max > MAXIMUM_MAX) {
        snprintf(buf, sizeof buf, "max_size must be in %llu..=%llu, got %llu", (unsigned long long)MAXIMUM_MIN,
                 (unsigned long long)MAXIMUM_MAX, (unsigned long long)o->max);
        st = CG_E_INVALID_OPTIONS;
    } else if (o->min > o->avg) {
        snprintf(buf, sizeof buf, "min_size must be <= avg_size");
        st = CG_E_INVALID_OPTIONS;
    } else if (o->avg > o->max) {
        snprintf(buf, sizeof buf, "avg_size must be <= max_size");
        st = CG_E_INVALID_OPTIONS;
    }
    if (msg && cap) {
        strncpy(msg, buf, cap - 1);
        msg[cap - 1] = 0;
    }
    if (st) return fail(st, buf);
    return CG_OK;
}

uint64_t capacity_of(uint64_t len, uint64_t mn) {
    if (len == 0) return 0;
    const uint64_t step = std::max<uint64_t>(2 * (mn / 2), 1);
    return len / step + 1;
}

// Per-segment candidate slots: ~2x the expected candidates per segment + 8,
// rounded to a power of two, at most 64 (denser segments become markers).
uint32_t seg_slots(const CdcParams &p) {
    const double lam = CG_SEG * (std::ldexp(1.0, -__builtin_popcountll(p.mask_s)) +
                                 std::ldexp(1.0, -__builtin_popcountll(p.mask_l)));
    uint32_t c = 8;
    while (c < 64 && c < 2 * lam + 8) c <<= 1;
    return c;
}

// ---------------------------------------------------------------------------
// Digest coalescer (round 4).  Concurrent callers of the synchronous device entry (the
// reference's callers are concurrent: thread-per-connection HTTP,
// crates/proto/nix/src/lib.rs:153-162; BEAM dirty schedulers, src/nif.rs:188-234) each
// run their boundary stages on their own stream; their SHA-256 digests are then merged:
// a caller whose boundary stages are queued submits its chunk list and blocks; one waiting
// caller becomes the leader and launches ONE k_sha256 over every pending batch's chunks,
// after each member's boundary stages (events), on a coalescer set (stream + merged
// buffers) no earlier group still uses.
//
// Policy.  A merged launch sizes its tiers for the whole chip and lasts one chain (the
// longest chunk's) whatever its size, so two merged launches do not overlap on the GPU
// and the rate is set by how many batches each chain carries (K = 32 concurrent callers:
// 199 GiB/s with one set, 100 with two sets -- halved groups, same chains --
// profiles/r04_v4_conc_*).  So a device has ONE set by default (CHUNKER_AMD_COAL_SETS, up
// to 8, for A/B) and the leader (1) leases it, waiting for the previous group's end while
// later callers keep joining the pending list, then (2) waits up to kCoalWindow until every
// caller inside the entry has submitted -- those still launching their boundary stages and
// those of the group that just ended -- and every caller that returned within the last
// kCoalRecent has called again (a server thread calls again as soon as its digests are back),
// so two half-groups taking turns (each carrying half the batches per chain: K = 8, 60 vs
// 110 GiB/s) merge into one, and (3) takes every pending caller (at most CG_COAL_MAX).  A
// caller that does not call again stops being expected kCoalRecent after it returned, so
// a lone caller never waits (its own return is taken off when it calls again).  Each member's stream then
// waits for its group's end, so its own tail (NAR index, spin-guard word) and its
// completion event follow the merged digest.  A group of one runs the ordinary per-batch
// launch on the member's own stream, so a lone caller's latency is unchanged.
//
// What a member can wait for, beyond its own digest's chain: callers only merge past
// coal_min() (the hardware queues less 4, at least 4) in the entry, so a lone caller and up
// to that many concurrent ones never enter a group (they go solo and no leader counts them:
// test_lone_and_few_callers_never_wait_for_the_window); a merged member waits at most kCoalWindow (3 ms) for its group to form plus the
// previous group's remaining chain on the one set (lease_set: <= one longest-chunk chain,
// ~55-75 ms at the default 4 MiB max), i.e. its call returns within window + 2 chains + its
// boundary stages.  bench.py's `concurrent` leg reports the measured per-call p50 / p99 of
// merged and per-batch digests side by side, and the leader's mean wait (cg_coalesce_stats).
// ---------------------------------------------------------------------------
struct CoalGroup {
    hipEvent_t done = nullptr;
    ~CoalGroup() {
        if (done) (void)hipEventDestroy(done);
    }
};

struct CoalSet {
    hipStream_t stream = nullptr;
    bool leased = false;               // a leader is launching on it
    std::shared_ptr<CoalGroup> last;   // its latest merged digest
    DevBuf mdesc, mabs, mtotal, morder, merr;
};

struct Coalescer {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<CoalEntry *> pending;
    int active = 0;         // SHA-256 device-entry callers that have not submitted yet
    int inside = 0;         // SHA-256 device-entry callers that have not returned yet
    int solo = 0;           // of those, callers digesting alone (per-batch launch): never submit
    // when callers returned, newest last (at most the last kCoalRecent's; a caller entering
    // again takes one off): callers between two calls, expected back shortly
    std::deque<std::chrono::steady_clock::time_point> returned;
    bool leading = false;   // a leader is collecting the next group
    // counters (cg_coalesce_stats): groups led, their members, leader waits, windows run out
    uint64_t groups = 0, members = 0, wait_us = 0, window_expired = 0;
    std::vector<std::unique_ptr<CoalSet>> sets;
};
Coalescer g_coal[64];
thread_local CoalActive *t_coal_active = nullptr;
std::atomic<uint32_t> g_coalesce{1};  // test hook cg_test_coalesce
// cg_chunk_batch_device_async_after: 2 (the product) = the whole batch runs on the library
// stream, ordered after inputs_ready only, and the caller's stream waits for its end, so
// the digests of consecutive batches overlap as well (config 2 18.1 -> 35.9 GiB/s, config 5
// 225 -> 360, config 4 695 -> 722; BLAKE3 config 3 equal: its digest fills the chip,
// profiles/r05_v3_split_ab.txt); 1 = only the boundary stages do and the digest joins the
// caller's stream (test hook cg_test_split_mode)
std::atomic<int> g_split_mode{2};

#ifndef CG_COAL_WINDOW_US
#define CG_COAL_WINDOW_US 3000
#endif
#ifndef CG_COAL_RECENT_US
#define CG_COAL_RECENT_US 50000
#endif
constexpr auto kCoalWindow = std::chrono::microseconds(CG_COAL_WINDOW_US);  // longest a leader waits
constexpr auto kCoalRecent = std::chrono::microseconds(CG_COAL_RECENT_US);  // how long a returned caller is expected back

// coalescer sets per device (CHUNKER_AMD_COAL_SETS, 1..8; read once)
static size_t coal_sets() {
    static const size_t n = [] {
        const char *e = getenv("CHUNKER_AMD_COAL_SETS");
        char *end = nullptr;
        const unsigned long v = e && *e ? strtoul(e, &end, 10) : 0;
        return (e && *e && end && *end == 0 && v >= 1 && v <= 8) ? (size_t)v : (size_t)1;
    }();
    return n;
}

Coalescer &coalescer(int dev) { return g_coal[(dev >= 0 && dev < 64) ? dev : 0]; }

// the device entry's caller is about to launch a SHA-256 batch (CoalActive) / is done
CoalActive::CoalActive(int dev) : dev(dev) {
    Coalescer &C = coalescer(dev);
    std::lock_guard<std::mutex> g(C.mu);
    ++C.active;
    ++C.inside;
    if (!C.returned.empty()) C.returned.pop_front();
}
CoalActive::~CoalActive() {
    leave();
    Coalescer &C = coalescer(dev);
    {
        std::lock_guard<std::mutex> g(C.mu);
        --C.inside;
        if (solo) --C.solo;
        const auto now = std::chrono::steady_clock::now();
        while (!C.returned.empty() && now - C.returned.front() > kCoalRecent) C.returned.pop_front();
        C.returned.push_back(now);
    }
    C.cv.notify_all();
}
void CoalActive::leave() {
    if (left) return;
    left = true;
    Coalescer &C = coalescer(dev);
    {
        std::lock_guard<std::mutex> g(C.mu);
        --C.active;
    }
    C.cv.notify_all();
}
// the caller digests its batch alone: a leader stops expecting it until it returns
void CoalActive::go_solo() {
    Coalescer &C = coalescer(dev);
    {
        std::lock_guard<std::mutex> g(C.mu);
        if (!left) --C.active;
        left = true;
        if (!solo) ++C.solo;
        solo = true;
    }
    C.cv.notify_all();
}

static bool set_idle(const CoalSet &S) { return !S.last || hipEventQuery(S.last->done) == hipSuccess; }

// Lease a set whose previous merged digest has ended (its buffers may be regrown).
// Called with the lock held; may release it while waiting for a busy set.
static CoalSet *lease_set(Coalescer &C, std::unique_lock<std::mutex> &lk) {
    for (;;) {
        CoalSet *oldest = nullptr;
        for (auto &S : C.sets) {
            if (S->leased) continue;
            if (set_idle(*S)) {
                S->leased = true;
                return S.get();
            }
            if (!oldest) oldest = S.get();
        }
        if (C.sets.size() < coal_sets()) {
            C.sets.push_back(std::make_unique<CoalSet>());
            C.sets.back()->leased = true;
            return C.sets.back().get();
        }
        if (!oldest) {  // every set is leased by another leader
            C.cv.wait(lk);
            continue;
        }
        std::shared_ptr<CoalGroup> g = oldest->last;
        lk.unlock();
        (void)hipEventSynchronize(g->done);
        lk.lock();
    }
}

// Launch one group (called by its leader without the lock).  A group of one runs on its
// member's stream; a larger group on the leased set S.
static int launch_group(CoalSet *S, std::vector<CoalEntry *> &grp, std::shared_ptr<CoalGroup> &G) {
    G = std::make_shared<CoalGroup>();
    HIP_TRY(hipEventCreateWithFlags(&G->done, hipEventDisableTiming));
    if (grp.size() == 1) {
        CoalEntry *e = grp[0];
        Workspace *ws = e->ws;
        cg::launch_sha256(e->d_data, e->d_abs, e->d_out, e->d_total, e->bound, e->expected, e->max_len,
                          ws->order.as<uint32_t>(), reinterpret_cast<uint8_t *>(e->d_out) + offsetof(cg_desc, hash),
                          sizeof(cg_desc), ws->sha_err.as<uint32_t>(), e->st);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(G->done, e->st));
        return CG_OK;
    }
    int rc;
    if (!S->stream) HIP_TRY(hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking));
    cg::CoalTable t{};
    uint64_t bound = 0, expected = 0, max_len = 0;
    t.n = (uint32_t)grp.size();
    for (size_t b = 0; b < grp.size(); ++b) {
        CoalEntry *e = grp[b];
        t.data[b] = e->d_data;
        t.abs[b] = e->d_abs;
        t.out[b] = reinterpret_cast<DescRaw *>(e->d_out);
        t.total[b] = e->d_total;
        t.bound[b] = e->bound;
        t.err[b] = e->ws->sha_err.as<uint32_t>();
        bound += e->bound;
        expected += e->expected;
        max_len = std::max<uint64_t>(max_len, e->max_len);
        HIP_TRY(hipStreamWaitEvent(S->stream, e->ready, 0));
    }
    // (the set's previous digest has ended, so growing a buffer frees nothing in use)
    if ((rc = S->mdesc.ensure((bound + 1) * sizeof(DescRaw), "coalesced descriptors"))) return rc;
    if ((rc = S->mabs.ensure((bound + 1) * 8, "coalesced addresses"))) return rc;
    if ((rc = S->mtotal.ensure(64, "coalesced total"))) return rc;
    if ((rc = S->morder.ensure(cg::sha256_order_tmp_elems(bound) * 4, "coalesced order"))) return rc;
    if ((rc = S->merr.ensure(64, "coalesced spin guard"))) return rc;
    cg::launch_sha256_coalesced(t, bound, expected, max_len, S->mdesc.as<DescRaw>(), S->mabs.as<uint64_t>(),
                                S->mtotal.as<uint64_t>(), S->morder.as<uint32_t>(), S->merr.as<uint32_t>(), S->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(G->done, S->stream));
    return CG_OK;
}

// Merge only when more callers are in flight than per-batch launches run side by side:
// the process's hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4) less the 4 its other
// streams take (at least CG_COAL_MIN = 4).  Up to that each batch's own launch overlaps
// the others' on a queue of its own, and with the SHA-256 latency tiers (sha256.hip) as
// well as one merged launch (16 queues, K = 12: 169 GiB/s per batch, p99 73 ms); past it
// the per-batch launches queue behind one another on shared queues (K = 16 / 24 / 32:
// 127-133 / 134 / 137 per batch with p99 121-127 ms, against 170 / 182 / 227-241 merged;
// profiles/r05_v29_v31_coalesce_threshold.txt).  Round 4, before the tiers, merged from 8
// callers (profiles/r04_v18_*, r04_v19_*).  Leader window 3 ms: 10 ms gave K = 32 220-279.
#ifndef CG_COAL_MIN
#define CG_COAL_MIN 4
#endif
static size_t coal_min() {
    static const size_t n = [] {
        const char *e = getenv("GPU_MAX_HW_QUEUES");
        char *end = nullptr;
        const unsigned long v = e && *e ? strtoul(e, &end, 10) : 0;
        const size_t q = (e && *e && end && *end == 0 && v >= 1 && v <= 64) ? (size_t)v : (size_t)4;
        return std::max<size_t>(q > 4 ? q - 4 : 0, CG_COAL_MIN);
    }();
    return n;
}
bool coalesce_worth(int dev) {
    Coalescer &C = coalescer(dev);
    std::lock_guard<std::mutex> g(C.mu);
    const auto now = std::chrono::steady_clock::now();
    while (!C.returned.empty() && now - C.returned.front() > kCoalRecent) C.returned.pop_front();
    return (size_t)C.inside + C.returned.size() > coal_min();  // (pending callers are inside)
}

int coalesced_sha256(CoalEntry *e) {
    Coalescer &C = coalescer(e->ws->device);
    HIP_TRY(hipEventCreateWithFlags(&e->ready, hipEventDisableTiming));
    struct EvGuard {
        hipEvent_t ev;
        ~EvGuard() { (void)hipEventDestroy(ev); }
    } evg{e->ready};
    HIP_TRY(hipEventRecord(e->ready, e->st));  // the member's boundary stages (and spin-guard arm) are queued
    std::unique_lock<std::mutex> lk(C.mu);
    C.pending.push_back(e);
    if (e->active) {
        e->active->left = true;  // submitted: no longer holds back a leader
        --C.active;
    }
    C.cv.notify_all();
    while (!e->group && !e->rc) {
        if (!C.leading && !C.pending.empty()) {
            C.leading = true;  // this thread leads the next group
            CoalSet *S = lease_set(C, lk);  // (callers arriving meanwhile join the group)
            // wait until every caller in the entry has submitted: those still launching their
            // boundary stages, and those of the group that just ended, which return and call
            // again as soon as their digests are back (a caller that does not call again
            // leaves the count when it returns)
            const auto t0 = std::chrono::steady_clock::now();
            for (;;) {
                const auto now = std::chrono::steady_clock::now();
                while (!C.returned.empty() && now - C.returned.front() > kCoalRecent) C.returned.pop_front();
                // (callers digesting alone are inside but will not submit)
                const bool more =
                    C.active > 0 || C.pending.size() < (size_t)(C.inside - C.solo) + C.returned.size();
                if (!more || C.pending.size() >= CG_COAL_MAX) break;
                if (now - t0 >= kCoalWindow) {
                    ++C.window_expired;
                    break;
                }
                C.cv.wait_for(lk, std::chrono::microseconds(100));
            }
            C.wait_us += (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
                             std::chrono::steady_clock::now() - t0).count();
            std::vector<CoalEntry *> grp;
            while (!C.pending.empty() && grp.size() < CG_COAL_MAX) {
                grp.push_back(C.pending.front());
                C.pending.pop_front();
            }
            ++C.groups;
            C.members += grp.size();
            C.leading = false;  // the next group may form while this one launches
            if (grp.size() == 1) {  // a group of one runs on its member's stream
                S->leased = false;
                S = nullptr;
            }
            lk.unlock();
            std::shared_ptr<CoalGroup> G;
            const int rc = launch_group(S, grp, G);
            // a failed launch may have left merge work queued that reads the members'
            // buffers: drain it before they return and release their workspaces
            if (rc && S && S->stream) (void)hipStreamSynchronize(S->stream);
            lk.lock();
            if (S) {
                S->leased = false;
                if (!rc) S->last = G;
            }
            for (CoalEntry *m : grp) {
                if (rc) m->rc = rc;
                else m->group = G;
            }
            C.cv.notify_all();
            continue;
        }
        C.cv.wait(lk);
    }
    lk.unlock();
    if (e->rc) return e->rc;
    HIP_TRY(hipStreamWaitEvent(e->st, e->group->done, 0));
    return CG_OK;
}

CdcParams cdc_params(const Opts &o, const Tables &t) {
    CdcParams P;
    const uint32_t bits = logarithm2((uint32_t)o.avg);
    P.min = o.min;
    P.avg = o.avg;
    P.max = o.max;
    P.mask_s = t.masks[bits + 1];
    P.mask_l = t.masks[bits - 1];
    return P;
}

// The workspace buffers a pass over n_nars NARs of total_len bytes needs (boundary
// stages, and the BLAKE3 tree's), sized without launching anything.  launch_batch calls
// it; a stream handle calls it (reserve_pass) to size its workspace for a full slot
// before any digest is in flight, since growing a buffer later frees the old one and
// hipFree waits for the whole device.
int ensure_pass_buffers(Workspace *ws, uint64_t total_len, size_t n_nars, uint64_t total_cap, uint64_t chunk_bound,
                        uint32_t slots, int algo) {
    int rc;
    const uint64_t nseg = (total_len + CG_SEG - 1) / CG_SEG;
    if ((rc = ws->seg_count.ensure((nseg + 1) * 4, "seg_count"))) return rc;
    if ((rc = ws->seg_cand.ensure((nseg * slots + 1) * 4, "seg_cand"))) return rc;
    if ((rc = ws->eoff.ensure((nseg + 1) * 8, "eoff"))) return rc;
    const uint64_t scan_n = std::max<uint64_t>({nseg, (uint64_t)n_nars, total_cap, 1});
    if ((rc = ws->scan_tmp.ensure(cg::exclusive_scan_tmp_elems(scan_n) * 8 + 64, "scan_tmp"))) return rc;
    if ((rc = ws->entries.ensure((nseg * slots + 1) * 8, "entries"))) return rc;
    if ((rc = ws->nar_off.ensure(2 * (n_nars + 1) * 8, "nar_off"))) return rc;
    if ((rc = ws->wchunk.ensure((total_cap + 1) * 16, "wchunk"))) return rc;
    if ((rc = ws->nar_nchunks.ensure((n_nars + 1) * 4, "nar_nchunks"))) return rc;
    if ((rc = ws->nar_first.ensure((n_nars + 1) * 8, "nar_first"))) return rc;
    if ((rc = ws->chunk_abs.ensure((total_cap + 1) * 8, "chunk_abs"))) return rc;
    if (algo == CG_BLAKE3) {
        if ((rc = ws->b3_gcount.ensure((chunk_bound + 1) * 4, "b3_gcount"))) return rc;
        if ((rc = ws->b3_gbase.ensure((chunk_bound + 1) * 8, "b3_gbase"))) return rc;
        if ((rc = ws->b3_gcv.ensure(cg::blake3_cv_bytes(total_len, chunk_bound, true), "b3_gcv"))) return rc;
        if ((rc = ws->b3_gmap.ensure((cg::blake3_group_bound(total_len, chunk_bound) + 1) * 4, "b3_gmap"))) return rc;
    }
    return CG_OK;
}

// The persistent scan's queue: allocated and zeroed (on the batch's stream, ahead of its
// first scan) once per workspace; every scan launch leaves it zeroed again.
int ensure_scan_queue(Workspace *ws, hipStream_t st) {
    if (ws->scanq_zeroed) return CG_OK;
    int rc;
    if ((rc = ws->scanq.ensure(sizeof(cg::ScanQueue), "scan queue"))) return rc;
    // (marked zeroed only once the memset is queued: a failed memset leaves it to the next call)
    HIP_TRY(hipMemsetAsync(ws->scanq.p, 0, ws->scanq.cap, st));
    ws->scanq_zeroed = true;
    return CG_OK;
}

// Walk pieces (walk.hip k_walk_pieces): NARs of at least two piece lengths are also
// walked piece by piece in parallel; a piece is long enough (32 max-size chunks, at
// least 8 MiB) for a walk started at its first byte to meet the NAR's own cut
// sequence within a few chunks.
uint64_t walk_piece_bytes(const Opts &o) { return std::max<uint64_t>(32 * o.max, 8ull << 20); }

// One NAR of len bytes, boundaries only, and a digest of its chunks: every buffer
// launch_batch grows for it (staging blocks, walk pieces, the descriptor array, the
// BLAKE3 map, the persistent scan's queue) allocated now, with launch_batch's own sizes.
int reserve_pass(Workspace *ws, uint64_t len, const Opts &o, int algo) {
    int rc;
    const std::shared_ptr<const Tables> tab = tables();
    const CdcParams P = cdc_params(o, *tab);
    const uint64_t cap = capacity_of(len, o.min);
    if ((rc = ensure_gear(ws, *tab))) return rc;
    if ((rc = ws->out.ensure((cap + 1) * sizeof(cg_desc), "descriptors"))) return rc;
    const uint64_t pb = walk_piece_bytes(o), k = cg::walk_is_speculative(P) ? len / pb : 0;
    const uint64_t np = k >= 2 ? k : 0;
    if ((rc = ws->stage.ensure((4 * 2 + np + (np + 1) / 2) * sizeof(uint64_t), /*mapped=*/true))) return rc;
    if (np) {
        uint64_t lb = 0;
        for (uint64_t j = 0; j < np; ++j) lb += capacity_of(j + 1 < np ? pb : len - j * pb, o.min) + 2;
        if ((rc = ws->pc_first.ensure(2 * 8 + np * 12, "walk pieces"))) return rc;
        if ((rc = ws->pc_count.ensure(np * 4, "walk pieces"))) return rc;
        if ((rc = ws->pc_exit.ensure(np * 8, "walk pieces"))) return rc;
        if ((rc = ws->pc_starts.ensure(std::max<uint64_t>(lb, cap + 2 * np) * 8, "walk pieces"))) return rc;
    }
    if ((rc = ws->first_host.ensure(2 * 8, /*mapped=*/true))) return rc;
    if ((rc = ensure_pass_buffers(ws, len, 1, cap, cap, seg_slots(P), algo))) return rc;
    if (algo == CG_BLAKE3) {
        if ((rc = ws->nar_ngroups.ensure(2 * 2 * 4, "nar_ngroups"))) return rc;
        if ((rc = ws->b3_lbase.ensure((cap + 1) * 8, "b3_lbase"))) return rc;
        if ((rc = ws->b3_lmap.ensure(cg::blake3_leaf_wave_bound(len, cap) * 4, "b3_lmap"))) return rc;
    }
    if (algo == CG_SHA256 && (rc = ws->order.ensure(cg::sha256_order_tmp_elems(cap) * 4, "order"))) return rc;
    // the queue's zeroing must be complete before a scan on any stream reads it
    if ((rc = ensure_scan_queue(ws, ws->stream))) return rc;
    HIP_TRY(hipStreamSynchronize(ws->stream));
    return CG_OK;
}

// The whole device pipeline for one batch.  d_out receives descriptors; the
// digest of descriptor g is written in place at d_out[g].hash.
//
// Node::put mode (crates/node/src/lib.rs:114-132) when d_chunk_ids is set: every
// chunk's ContentId(Chunk, payload) -> d_chunk_ids[32 g], and NAR i's manifest id
// ContentId(Level1Manifest, its chunk ids in order) -> h_manifest_ids[32 i].  The CAS
// stage forks onto ws->side_stream after descriptor assembly and joins before return.
// Launch side: everything up to the copies of the NAR index (and manifest ids, and the
// SHA-256 spin-guard word) into host memory, all queued on `st`; nothing waits.
// finish_batch waits for `st` and checks the results.
int launch_batch(Workspace *ws, const uint8_t *d_data, const uint64_t *h_nar_off, size_t n_nars, const Opts &o,
                 int algo, cg_desc *d_out, size_t out_cap, hipStream_t st, uint8_t *d_chunk_ids,
                 uint8_t *h_manifest_ids, bool digest, BatchLaunch *bl, bool coalesce, hipEvent_t inputs_ready) {
    if (algo != CG_BLAKE3 && algo != CG_SHA256) return fail(CG_E_INVALID_OPTIONS, "unknown hash algorithm");
    if (((uintptr_t)d_data & 15u) != 0) return fail(CG_E_IO, "device input must be 16-byte aligned");
    int rc;
    const uint64_t base0 = n_nars ? h_nar_off[0] : 0;
    const uint64_t total_len = n_nars ? h_nar_off[n_nars] : 0;
    for (size_t i = 0; i < n_nars; ++i)  // NAR i = [off[i], off[i+1]) must lie inside the batch
        if (h_nar_off[i + 1] < h_nar_off[i])
            return fail_bounds(h_nar_off[i + 1], h_nar_off[i], 0, "nar offsets must be non-decreasing");
    (void)base0;

    // one table snapshot for the whole call: GEAR on the device and MASKS in P agree
    const std::shared_ptr<const Tables> tab = tables();
    const CdcParams P = cdc_params(o, *tab);

    // walk pieces (walk_piece_bytes)
    const uint64_t pb = walk_piece_bytes(o);
    uint64_t np = 0, pcap = 0;
    if (cg::walk_is_speculative(P))
        for (size_t i = 0; i < n_nars; ++i) {
            const uint64_t k = (h_nar_off[i + 1] - h_nar_off[i]) / pb;
            if (k >= 2) {
                np += k;
                pcap += capacity_of(h_nar_off[i + 1] - h_nar_off[i], o.min) + 2 * k;
            }
        }

    // host staging: nar_off (n+1), cap_base (n+1), nar_first (n+1), then the piece
    // tables: first (n+1), base (np), nar (np, u32)
    const size_t stage_words = 4 * (n_nars + 1) + np + (np + 1) / 2;
    if ((rc = ws->stage.ensure(stage_words * sizeof(uint64_t), /*mapped=*/true))) return rc;
    uint64_t *s_off = ws->stage.as<uint64_t>();
    uint64_t *s_cap = s_off + (n_nars + 1);
    uint64_t *s_first = s_cap + (n_nars + 1);
    uint64_t *s_pfirst = s_first + (n_nars + 1);
    uint64_t *s_pbase = s_pfirst + (n_nars + 1);
    uint32_t *s_pnar = reinterpret_cast<uint32_t *>(s_pbase + np);
    memcpy(s_off, h_nar_off, (n_nars + 1) * sizeof(uint64_t));
    uint64_t total_cap = 0;
    for (size_t i = 0; i < n_nars; ++i) {
        s_cap[i] = total_cap;
        total_cap += capacity_of(h_nar_off[i + 1] - h_nar_off[i], o.min);
    }
    s_cap[n_nars] = total_cap;
    cg::WalkPiecesHost pieces;
    // host tables -> HBM by extra blocks of the compaction's first kernel reading the mapped
    // staging block (a hipMemcpyAsync from pinned memory waited ~40 us behind the previous
    // call's last kernel before its blit ran, profiles/r03_v16_c3_async_kernel_trace.csv)
    cg::StageIn stage_in;
    auto dev_of = [&](const void *host) {
        return static_cast<const uint8_t *>(ws->stage.dev) + (static_cast<const uint8_t *>(host) -
                                                             static_cast<const uint8_t *>(ws->stage.p));
    };
    if (np) {
        uint64_t g = 0, lb = 0;
        for (size_t i = 0; i < n_nars; ++i) {
            s_pfirst[i] = g;
            const uint64_t len = h_nar_off[i + 1] - h_nar_off[i], k = len / pb;
            if (k < 2) continue;
            for (uint64_t j = 0; j < k; ++j, ++g) {
                const uint64_t plen = j + 1 < k ? pb : len - j * pb;
                s_pbase[g] = lb;
                s_pnar[g] = (uint32_t)i;
                lb += capacity_of(plen, o.min) + 2;
            }
        }
        s_pfirst[n_nars] = g;
        // first / base / nar in one device block, filled by one copy from the staging block
        // they are laid out in contiguously
        if ((rc = ws->pc_first.ensure((n_nars + 1) * 8 + np * 12, "walk pieces"))) return rc;
        if ((rc = ws->pc_count.ensure(np * 4, "walk pieces"))) return rc;
        if ((rc = ws->pc_exit.ensure(np * 8, "walk pieces"))) return rc;
        if ((rc = ws->pc_starts.ensure(std::max<uint64_t>(lb, pcap) * 8, "walk pieces"))) return rc;
        stage_in.add(s_pfirst, ws->pc_first.p, (n_nars + 1) * 8 + np * 12);
        pieces.first = ws->pc_first.as<uint64_t>();
        pieces.base = pieces.first + (n_nars + 1);
        pieces.nar = reinterpret_cast<uint32_t *>(ws->pc_first.as<uint64_t>() + (n_nars + 1) + np);
        pieces.count = ws->pc_count.as<uint32_t>();
        pieces.exit = ws->pc_exit.as<uint64_t>();
        pieces.starts = ws->pc_starts.as<uint64_t>();
        pieces.pb = pb;
        pieces.np = np;
    }

    const uint64_t nseg = (total_len + CG_SEG - 1) / CG_SEG;
    const uint32_t slots = seg_slots(P);
    const uint64_t chunk_bound = std::min<uint64_t>(total_cap, out_cap);
    if ((rc = ensure_gear(ws, *tab))) return rc;
    if ((rc = ensure_pass_buffers(ws, total_len, n_nars, total_cap, chunk_bound, slots, algo))) return rc;
    // The boundary stages' stream: `st` itself, or -- with an inputs-ready event -- the
    // workspace's own stream, ordered after that event only, so the stages (and, in split
    // mode 2, the digest: `ds` below) run beside the digest of the batch queued before on
    // `st`, which reads another workspace.  (One stream per workspace: streams beyond the
    // hardware queues share them and serialise; a second, dedicated stream per workspace
    // measured no better, profiles/r05_v40_one_stream_ab.txt.  Without gain either, commit
    // 686ad6b: that stream at the highest priority, restricted to 32 / 64 CUs, the digest
    // on a CU-masked stream; profiles/r05_v3_split_ab.txt, r05_v12_cumask_ab.txt,
    // r05_v16_v17_stagger_ab.txt.)
    // (BLAKE3 batches stay in stream order: their digest fills the chip by itself, and
    // overlapping it with the next batch measured 1.7 % slower on config 3,
    // profiles/r05_v3_split_ab.txt; waiting for more than inputs_ready is always allowed)
    hipStream_t bs = st;
    if (inputs_ready && algo == CG_SHA256) {
        bs = ws->stream;
        HIP_TRY(hipStreamWaitEvent(bs, inputs_ready, 0));
    } else if (inputs_ready) {
        // BLAKE3: stream order AND the event (its input may be written on another stream,
        // e.g. a copy stream, that `st` knows nothing of)
        HIP_TRY(hipStreamWaitEvent(st, inputs_ready, 0));
    }
    if ((rc = ensure_scan_queue(ws, bs))) return rc;
    // nar_off (n+1) then cap_base (n+1): one block, one copy (s_cap follows s_off in staging)
    const uint64_t *d_nar_off = ws->nar_off.as<uint64_t>(), *d_cap_base = d_nar_off + (n_nars + 1);

    // A timing event between two kernels holds the second back by ~6 us (the event's
    // end-of-pipe timestamp), so mode 2 records only the two around the digest stage.
    const int pmode = g_profiling.load();
    const bool prof = pmode != 0;
    const bool prof_all = pmode == 1;
    stage_in.add(s_off, ws->nar_off.p, 2 * (n_nars + 1) * 8);
    for (int k = 0; k < stage_in.n; ++k) stage_in.src[k] = dev_of(stage_in.src[k]);
    if (prof_all) HIP_TRY(hipEventRecord(ws->ev[EV_START], bs));  // scan stage = the scan kernel alone

    cg::launch_scan(d_data, total_len, ws->gear.as<uint64_t>(), P.mask_s, P.mask_l, slots,
                    ws->seg_count.as<uint32_t>(), ws->seg_cand.as<uint32_t>(), nseg, bs, ws->scanq.as<cg::ScanQueue>());
    if (prof_all) HIP_TRY(hipEventRecord(ws->ev[EV_SCAN], bs));
    // (the host tables ride along the compaction's first launch: the scan needs none of them)
    cg::launch_scan_compact(ws->seg_count.as<uint32_t>(), ws->seg_cand.as<uint32_t>(), ws->eoff.as<uint64_t>(), slots,
                            nseg, ws->entries.as<uint64_t>(), ws->scan_tmp.as<uint64_t>(), bs, stage_in);
    if (prof_all) HIP_TRY(hipEventRecord(ws->ev[EV_COMPACT], bs));
    // BLAKE3: the walk counts each NAR's 64-leaf groups and the assembly builds the group
    // map from them, so launch_blake3 needs no planning kernel of its own
    const bool b3_fuse = algo == CG_BLAKE3 && digest && g_b3_fused_plan.load(std::memory_order_relaxed);
    if (b3_fuse && (rc = ws->nar_ngroups.ensure(2 * (n_nars + 1) * 4, "nar_ngroups"))) return rc;
    cg::B3PlanOut b3plan;
    if (b3_fuse) {
        b3plan.nar_ngroups = ws->nar_ngroups.as<uint32_t>();
        b3plan.group_base = ws->b3_gbase.as<uint64_t>();
        b3plan.gmap = ws->b3_gmap.as<uint32_t>();
        b3plan.bound = chunk_bound;
        if (g_b3_packed.load(std::memory_order_relaxed)) {  // packed leaves (k_b3_leaves)
            b3plan.lmap_cap = cg::blake3_leaf_wave_bound(total_len, chunk_bound);
            if ((rc = ws->b3_lbase.ensure((chunk_bound + 1) * 8, "b3_lbase"))) return rc;
            if ((rc = ws->b3_lmap.ensure(b3plan.lmap_cap * 4, "b3_lmap"))) return rc;
            b3plan.leaf_base = ws->b3_lbase.as<uint64_t>();
            b3plan.lmap = ws->b3_lmap.as<uint32_t>();
        }
    }
    cg::launch_walk(d_data, ws->gear.as<uint64_t>(), ws->entries.as<uint64_t>(), ws->eoff.as<uint64_t>(), nseg,
                    d_nar_off, d_cap_base, n_nars, P, ws->wchunk.as<uint64_t>(),
                    ws->nar_nchunks.as<uint32_t>(), pieces, bs, b3_fuse ? ws->nar_ngroups.as<uint32_t>() : nullptr);
    if (prof_all) HIP_TRY(hipEventRecord(ws->ev[EV_WALK], bs));
    // the NAR index goes straight into mapped host memory from the assembly kernel: a D2H
    // copy after the digest cost ~40 us of idle GPU per call (blit + the runtime's gap
    // before the next call's first copy, profiles/r03_v16_c3_async_kernel_trace.csv)
    if ((rc = ws->first_host.ensure((n_nars + 1) * 8, /*mapped=*/true))) return rc;
    bool first_on_host = false;
    const bool b3_planned =
        cg::launch_assemble(d_nar_off, d_cap_base, ws->wchunk.as<uint64_t>(), ws->nar_nchunks.as<uint32_t>(),
                            ws->nar_first.as<uint64_t>(), n_nars, d_out, out_cap, ws->chunk_abs.as<uint64_t>(),
                            ws->scan_tmp.as<uint64_t>(), bs, b3_fuse ? &b3plan : nullptr,
                            static_cast<uint64_t *>(ws->first_host.dev), &first_on_host);
    if (prof) HIP_TRY(hipEventRecord(ws->ev[EV_ASSEMBLE], bs));
    bl->dstart = ws->ev[EV_ASSEMBLE];
    // The digest's stream: `st`, joined after the boundary stages (split mode 1), or -- split
    // mode 2 -- the library stream itself, so the whole batch is ordered after inputs_ready
    // only and `st` waits for its end (below): a batch's digest then runs beside the digest of
    // the batch queued before it.
    hipStream_t ds = st;
    if (bs != st && g_split_mode.load(std::memory_order_relaxed) == 2) {
        ds = bs;
    } else if (bs != st) {  // join: the digest (and everything after it) follows the boundary stages
        HIP_TRY(hipEventRecord(ws->ev_bdone, bs));
        HIP_TRY(hipStreamWaitEvent(st, ws->ev_bdone, 0));
        if (prof) {
            HIP_TRY(hipEventRecord(ws->ev_dstart, st));
            bl->dstart = ws->ev_dstart;
        }
    }
    const uint64_t *d_total = ws->nar_first.as<uint64_t>() + n_nars;
    uint8_t *d_man = nullptr;
    if (d_chunk_ids) {
        if ((rc = ws->cas_order.ensure(cg::sha256_order_tmp_elems(chunk_bound) * 4, "cas_order"))) return rc;
        if ((rc = ws->ids.ensure((n_nars + 1) * 32, "manifest ids"))) return rc;
        if ((rc = ws->man_abs.ensure((n_nars + 1) * 8, "manifest spans"))) return rc;
        if ((rc = ws->man_desc.ensure((n_nars + 2) * sizeof(cg_desc), "manifest spans"))) return rc;
        d_man = ws->ids.as<uint8_t>();
        if ((rc = ws->ensure_side_stream())) return rc;
        hipStream_t side = ws->side_stream;
        HIP_TRY(hipEventRecord(ws->ev_fork, bs));
        HIP_TRY(hipStreamWaitEvent(side, ws->ev_fork, 0));
        const uint32_t *ord = cg::launch_len_order(d_out, d_total, chunk_bound, o.max, ws->cas_order.as<uint32_t>(), side);
        cg::launch_cas_ids(d_data, ws->chunk_abs.as<uint64_t>(), d_out, d_total, chunk_bound, ord, CG_KIND_CHUNK,
                           d_chunk_ids, 32, side);
        uint64_t *d_man_total = reinterpret_cast<uint64_t *>(ws->man_desc.as<cg_desc>() + n_nars);
        cg::launch_manifest_spans(ws->nar_first.as<uint64_t>(), n_nars, ws->man_abs.as<uint64_t>(), ws->man_desc.p,
                                  d_man_total, side);
        cg::launch_cas_ids(d_chunk_ids, ws->man_abs.as<uint64_t>(), ws->man_desc.p, d_man_total, n_nars, nullptr,
                           CG_KIND_LEVEL1_MANIFEST, d_man, 32, side);
        HIP_TRY(hipEventRecord(ws->ev_cas, side));
        HIP_TRY(hipEventRecord(ws->ev_join, side));
    }
    uint8_t *hash_base = reinterpret_cast<uint8_t *>(d_out) + offsetof(cg_desc, hash);
    bool sha_armed = false;
    if (!digest) {
        // boundaries only (push_drain digests the chunks that became final afterwards)
    } else if (algo == CG_SHA256) {
        if ((rc = ws->order.ensure(cg::sha256_order_tmp_elems(chunk_bound) * 4, "order"))) return rc;
        // expected chunk count: FastCDC's mean chunk is about min + avg on random data
        const uint64_t expected = std::min<uint64_t>(chunk_bound, total_len / (o.min + o.avg) + n_nars);
        if ((rc = sha_err_arm(ws, ds))) return rc;
        sha_armed = true;
        if (coalesce && chunk_bound && coalesce_worth(ws->device)) {
            CoalEntry e{ws, d_data, ws->chunk_abs.as<uint64_t>(), d_out, d_total, chunk_bound, expected, o.max, ds};
            e.active = t_coal_active;
            if ((rc = coalesced_sha256(&e))) return rc;
        } else {
            if (t_coal_active) t_coal_active->go_solo();  // nothing to merge: do not hold a leader back
            cg::launch_sha256(d_data, ws->chunk_abs.as<uint64_t>(), d_out, d_total, chunk_bound, expected, o.max,
                              ws->order.as<uint32_t>(), hash_base, sizeof(cg_desc), ws->sha_err.as<uint32_t>(), ds);
        }
    } else {
        cg::launch_blake3(d_data, ws->chunk_abs.as<uint64_t>(), d_out, d_total, chunk_bound, total_len, hash_base,
                          sizeof(cg_desc), ws->b3_gmap.as<uint32_t>(), ws->b3_gbase.as<uint64_t>(),
                          ws->b3_gcount.as<uint32_t>(), ws->scan_tmp.as<uint64_t>(), ws->b3_gcv.as<uint32_t>(), true,
                          ds, b3_planned, b3_planned ? b3plan.leaf_base : nullptr, b3plan.lmap);
    }
    if (prof) HIP_TRY(hipEventRecord(ws->ev[EV_DIGEST], ds));
    if (d_chunk_ids) HIP_TRY(hipStreamWaitEvent(ds, ws->ev_join, 0));
    HIP_TRY(hipGetLastError());
    if (first_on_host) {
        s_first = ws->first_host.as<uint64_t>();
    } else {
        HIP_TRY(hipMemcpyAsync(s_first, ws->nar_first.p, (n_nars + 1) * 8, hipMemcpyDeviceToHost, ds));
    }
    if (d_man && h_manifest_ids)
        HIP_TRY(hipMemcpyAsync(h_manifest_ids, d_man, n_nars * 32, hipMemcpyDeviceToHost, ds));
    if (sha_armed && (rc = sha_err_fetch(ws, ds))) return rc;
    // the batch's end: the digest-stage timing event when nothing was queued after it (each
    // event between two batches' kernels holds the second back by ~6 us), else one more
    const bool tail_ops = d_chunk_ids || !first_on_host || sha_armed || (d_man && h_manifest_ids);
    if (prof && !tail_ops) {
        bl->done = ws->ev[EV_DIGEST];
    } else {
        HIP_TRY(hipEventRecord(ws->ev_done, ds));
        bl->done = ws->ev_done;
    }
    if (ds != st) HIP_TRY(hipStreamWaitEvent(st, bl->done, 0));  // later work on `st` follows the batch
    bl->s_first = s_first;
    bl->n_nars = n_nars;
    bl->out_cap = out_cap;
    bl->sha_armed = sha_armed;
    bl->pmode = pmode;
    bl->node_put = d_chunk_ids != nullptr;
    return CG_OK;
}

// Wait side: the stream sync, the spin-guard check, the stage times, the NAR index.
int finish_batch(Workspace *ws, hipStream_t st, const BatchLaunch &bl, uint64_t *h_nar_first) {
    int rc;
    (void)st;
    HIP_TRY(hipEventSynchronize(bl.done));
    if (bl.sha_armed && (rc = sha_err_check(ws))) return rc;
    if (bl.pmode) {
        const bool prof_all = bl.pmode == 1;
        t_stage_ms.assign(EV_N - 1 + (bl.node_put ? 1 : 0), prof_all ? 0.0 : std::nan(""));
        for (int k = prof_all ? 1 : EV_DIGEST; k < EV_N; ++k) {
            float ms = 0;
            // (the digest stage opens at bl.dstart: the assembly's event, or after a split
            // batch's join on the caller's stream)
            HIP_TRY(hipEventElapsedTime(&ms, k == EV_DIGEST ? bl.dstart : ws->ev[k - 1], ws->ev[k]));
            t_stage_ms[k - 1] = ms;
        }
        if (bl.node_put) {  // CAS stage: from descriptor assembly to the last id
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, ws->ev[EV_ASSEMBLE], ws->ev_cas));
            t_stage_ms[EV_N - 1] = ms;
        }
    }
    const size_t n = bl.n_nars;
    if (h_nar_first) memcpy(h_nar_first, bl.s_first, (n + 1) * 8);
    if (bl.s_first[n] > bl.out_cap) return fail(CG_E_CAPACITY, "descriptor output array too small");
    return CG_OK;
}

// The whole device pipeline for one batch, waited for.  A launch that fails part-way
// may have queued work on `st`: it is drained before the workspace goes back to the pool.
int run_batch(Workspace *ws, const uint8_t *d_data, const uint64_t *h_nar_off, size_t n_nars, const Opts &o,
              int algo, cg_desc *d_out, size_t out_cap, uint64_t *h_nar_first, hipStream_t st,
              uint8_t *d_chunk_ids, uint8_t *h_manifest_ids, bool digest, bool coalesce) {
    BatchLaunch bl;
    const int rc = launch_batch(ws, d_data, h_nar_off, n_nars, o, algo, d_out, out_cap, st, d_chunk_ids,
                                h_manifest_ids, digest, &bl, coalesce);
    if (rc) {
        (void)hipStreamSynchronize(st);
        return rc;
    }
    return finish_batch(ws, st, bl, h_nar_first);
}

// The reference's golden boundary fixture, fastcdc_boundaries_match_v3_golden_fixture
// (src/chunking.rs:1266-1297): b[i] = (i*31 + i/7) % 251 for 65,659 bytes, chunked at
// (1024, 6000, 16384) -- bits = 13, so it exercises MASKS[14] / MASKS[12] and GEAR[0..250].
constexpr uint64_t FIX_LEN = 64 * 1024 + 123;
constexpr uint64_t FIX_CUTS[10][2] = {{0, 6162},     {6162, 7028},  {13190, 7028}, {20218, 7028}, {27246, 7028},
                                      {34274, 7028}, {41302, 7028}, {48330, 7028}, {55358, 7028}, {62386, 3273}};

// Run the fixture through the GPU pipeline (scan, walk, assembly) with the installed
// tables and compare with the reference's ten boundaries.  On a match the table epoch
// the pipeline used is marked verified.
int selftest_gpu() {
    Workspace *ws = nullptr;
    int rc = acquire(&ws);
    if (rc) return rc;
    WsGuard guard{ws};
    Opts o{1024, 6000, 16384};
    std::vector<uint8_t> fx(FIX_LEN);
    for (uint64_t i = 0; i < FIX_LEN; ++i) fx[i] = (uint8_t)((i * 31 + i / 7) % 251);
    const uint64_t cap = capacity_of(FIX_LEN, o.min);
    if ((rc = ws->in.ensure(FIX_LEN + 256, "input"))) return rc;
    if ((rc = ws->out.ensure((cap + 1) * sizeof(cg_desc), "descriptors"))) return rc;
    HIP_TRY(hipMemcpyAsync(ws->in.p, fx.data(), FIX_LEN, hipMemcpyHostToDevice, ws->stream));
    uint64_t offs[2] = {0, FIX_LEN}, first[2] = {0, 0};
    if ((rc = run_batch(ws, ws->in.as<uint8_t>(), offs, 1, o, CG_SHA256, ws->out.as<cg_desc>(), cap, first,
                        ws->stream, nullptr, nullptr, /*digest=*/false)))
        return rc;
    const uint64_t used_epoch = ws->gear_epoch;
    std::vector<cg_desc> got(first[1]);
    if (first[1]) {
        HIP_TRY(hipMemcpyAsync(got.data(), ws->out.p, first[1] * sizeof(cg_desc), hipMemcpyDeviceToHost, ws->stream));
        HIP_TRY(hipStreamSynchronize(ws->stream));
    }
    bool ok = got.size() == 10;
    for (size_t k = 0; ok && k < 10; ++k) ok = got[k].offset == FIX_CUTS[k][0] && got[k].length == FIX_CUTS[k][1];
    if (ok) {
        g_verified_epoch.store(used_epoch);
        return CG_OK;
    }
    std::string msg = "FastCDC selftest failed: the reference fixture (src/chunking.rs:1266-1297) gave " +
                      std::to_string(got.size()) + " chunks [";
    for (size_t k = 0; k < got.size() && k < 4; ++k)
        msg += (k ? ", (" : "(") + std::to_string(got[k].offset) + "," + std::to_string(got[k].length) + ")";
    msg += got.size() > 4 ? ", ...]" : "]";
    msg += " where fastcdc gives 10 [(0,6162), (6162,7028), ...]";
    if (tables()->placeholder) msg += "; the installed GEAR table is the build's placeholder, not fastcdc 4.0.1's";
    return fail(CG_E_TABLES, msg);
}

// Fail-closed gate in front of every chunking entry point (see Tables above).
int check_tables() {
    if (allow_unverified_tables()) return CG_OK;
    const std::shared_ptr<const Tables> t = tables();
    if (t->placeholder)
        return fail(CG_E_TABLES,
                    "FastCDC GEAR table is the build's placeholder (tables/fastcdc_v2020_gear.txt), not fastcdc "
                    "4.0.1's: chunk boundaries would differ from the reference. Install the crate's GEAR/MASKS with "
                    "cg_set_cdc_tables(), or set CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR=1 to run anyway");
    if (g_verified_epoch.load() == t->epoch) return CG_OK;
    return selftest_gpu();
}

// The reference's own checks on the descriptor list before it is handed out:
// ZeroLengthChunk (src/chunking.rs:567-570) and the bounds check of every
// (offset, length) against the input (:346-356); a GPU list that fails them is an
// engine fault and surfaces as the same errors, never as silently bad chunks.
int check_descriptors(const cg_desc *out, const uint64_t *first, const uint64_t *off, size_t n_nars) {
    for (size_t i = 0; i < n_nars; ++i) {
        const uint64_t len = off[i + 1] - off[i];
        for (uint64_t g = first[i]; g < first[i + 1]; ++g) {
            if (out[g].length == 0) return fail(CG_E_ZERO_LENGTH_CHUNK, "FastCDC returned a chunk with length 0");
            if (out[g].offset > len || out[g].length > len - out[g].offset)
                return fail_bounds(len, out[g].offset, out[g].length, "descriptor outside its input");
        }
    }
    return CG_OK;
}

int batch_host(const uint8_t *data, const uint64_t *nar_offsets, size_t n_nars, uint64_t mn, uint64_t avg,
               uint64_t mx, int algo, cg_desc *out, size_t out_cap, uint64_t *nar_first) {
    Opts o;
    int rc = resolve(mn, avg, mx, &o, nullptr, 0);
    if (rc) return rc;
    if ((rc = check_tables())) return rc;
    Workspace *ws = nullptr;
    if ((rc = acquire(&ws))) return rc;
    WsGuard guard{ws};
    const uint64_t lo = n_nars ? nar_offsets[0] : 0, hi = n_nars ? nar_offsets[n_nars] : 0;
    const uint64_t bytes = hi - lo;
    // device copy starts at nar_offsets[0]; offsets are rebased so the flat buffer starts at 0
    std::vector<uint64_t> off(n_nars + 1);
    for (size_t i = 0; i <= n_nars; ++i) off[i] = nar_offsets[i] - lo;
    uint64_t total_cap = 0;
    for (size_t i = 0; i < n_nars; ++i) total_cap += capacity_of(off[i + 1] - off[i], o.min);
    if ((rc = ws->in.ensure(bytes + 256, "input"))) return rc;
    if ((rc = ws->out.ensure((total_cap + 1) * sizeof(cg_desc), "descriptors"))) return rc;
    if (bytes) HIP_TRY(hipMemcpyAsync(ws->in.p, data + lo, bytes, hipMemcpyHostToDevice, ws->stream));
    std::vector<uint64_t> first(n_nars + 1);
    // (the host entry does not join the coalescer: bound by the host link, 1 GiB batches
    // take turns on it when their digests merge -- K = 16 41.7-43.3 GiB/s against 48.2-48.4
    // per batch, profiles/r04_v33_*; and the reference's own call shape, 10 MiB per call,
    // gains nothing in rate and loses in latency -- K = 32 2.08 vs 2.13 GiB/s, p50 127 vs
    // 100 ms, profiles/r05_v2_dropin*)
    rc = run_batch(ws, ws->in.as<uint8_t>(), off.data(), n_nars, o, algo, ws->out.as<cg_desc>(), total_cap,
                   first.data(), ws->stream);
    if (rc) return rc;
    const uint64_t total = first[n_nars];
    if (nar_first) memcpy(nar_first, first.data(), (n_nars + 1) * 8);
    if (total > out_cap) return fail(CG_E_CAPACITY, "descriptor output array too small");
    if (total) {
        HIP_TRY(hipMemcpyAsync(out, ws->out.p, total * sizeof(cg_desc), hipMemcpyDeviceToHost, ws->stream));
        HIP_TRY(hipStreamSynchronize(ws->stream));
    }
    return check_descriptors(out, first.data(), off.data(), n_nars);
}

// Digest-only pipeline over n device spans on `st` (shared by cg_hash_spans_device and cg_hash).
int hash_spans(Workspace *ws, const uint8_t *d_data, const uint64_t *d_offsets, const uint64_t *d_lengths, size_t n,
               int algo, uint8_t *d_digests, hipStream_t st) {
    int rc;
    if ((rc = ws->chunk_abs.ensure((n + 1) * 8, "chunk_abs"))) return rc;
    if ((rc = ws->out.ensure((n + 1) * sizeof(cg_desc), "descriptors"))) return rc;
    if ((rc = ws->nar_first.ensure(16, "total"))) return rc;
    if ((rc = ws->scan_tmp.ensure(cg::exclusive_scan_tmp_elems(n) * 8 + 64, "scan_tmp"))) return rc;
    uint64_t *d_total = ws->nar_first.as<uint64_t>();
    cg::launch_spans_to_desc(d_offsets, d_lengths, n, ws->chunk_abs.as<uint64_t>(), ws->out.p, d_total, st);
    uint8_t *hb = ws->out.as<uint8_t>() + offsetof(cg_desc, hash);
    bool sha_armed = false;
    if (algo == CG_SHA256) {
        // spans are not bounded by a max_size: bucket for the ABI's 16 MiB span cap
        if ((rc = ws->order.ensure(cg::sha256_order_tmp_elems(n) * 4, "order"))) return rc;
        if ((rc = sha_err_arm(ws, st))) return rc;
        sha_armed = true;
        cg::launch_sha256(d_data, ws->chunk_abs.as<uint64_t>(), ws->out.p, d_total, n, n, MAXIMUM_MAX,
                          ws->order.as<uint32_t>(), hb, sizeof(cg_desc), ws->sha_err.as<uint32_t>(), st);
    } else {
        // group-grid bound without reading lengths back: spans are capped at 16 MiB each
        const uint64_t tb = (uint64_t)n * MAXIMUM_MAX;
        const uint64_t gb = cg::blake3_group_bound(tb, n);
        if ((rc = ws->b3_gcount.ensure((n + 1) * 4, "b3_gcount"))) return rc;
        if ((rc = ws->b3_gbase.ensure((n + 1) * 8, "b3_gbase"))) return rc;
        if ((rc = ws->b3_gcv.ensure(cg::blake3_cv_bytes(tb, n, false), "b3_gcv"))) return rc;
        if ((rc = ws->b3_gmap.ensure((gb + 1) * 4, "b3_gmap"))) return rc;
        cg::launch_blake3(d_data, ws->chunk_abs.as<uint64_t>(), ws->out.p, d_total, n, tb, hb, sizeof(cg_desc),
                          ws->b3_gmap.as<uint32_t>(), ws->b3_gbase.as<uint64_t>(), ws->b3_gcount.as<uint32_t>(),
                          ws->scan_tmp.as<uint64_t>(), ws->b3_gcv.as<uint32_t>(), false, st);
    }
    HIP_TRY(hipMemcpy2DAsync(d_digests, 32, hb, sizeof(cg_desc), 32, n, hipMemcpyDeviceToDevice, st));
    HIP_TRY(hipGetLastError());
    if (sha_armed && (rc = sha_err_fetch(ws, st))) return rc;
    HIP_TRY(hipStreamSynchronize(st));
    if (sha_armed && (rc = sha_err_check(ws))) return rc;
    return CG_OK;
}

// ContentId pipeline over n device spans on `st` (cg_cas_ids_device, cg_cas_id).
int cas_spans(Workspace *ws, const uint8_t *d_data, const uint64_t *d_offsets, const uint64_t *d_lengths, size_t n,
              uint32_t kind, uint8_t *d_ids, hipStream_t st) {
    int rc;
    if ((rc = ws->chunk_abs.ensure((n + 1) * 8, "chunk_abs"))) return rc;
    if ((rc = ws->out.ensure((n + 1) * sizeof(cg_desc), "descriptors"))) return rc;
    if ((rc = ws->nar_first.ensure(16, "total"))) return rc;
    if ((rc = ws->cas_order.ensure(cg::sha256_order_tmp_elems(n) * 4, "cas_order"))) return rc;
    uint64_t *d_total = ws->nar_first.as<uint64_t>();
    cg::launch_spans_to_desc(d_offsets, d_lengths, n, ws->chunk_abs.as<uint64_t>(), ws->out.p, d_total, st);
    const uint32_t *ord =
        n > 64 ? cg::launch_len_order(ws->out.p, d_total, n, MAXIMUM_MAX, ws->cas_order.as<uint32_t>(), st) : nullptr;
    cg::launch_cas_ids(d_data, ws->chunk_abs.as<uint64_t>(), ws->out.p, d_total, n, ord, kind, d_ids, 32, st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
    return CG_OK;
}

int check_kind(uint32_t kind) {
    if (kind < CG_KIND_CHUNK || kind > CG_KIND_COMMIT) return fail(CG_E_INVALID_OPTIONS, "unknown object kind");
    return CG_OK;
}

}  // namespace cgrt

using namespace cgrt;

// ---------------------------------------------------------------------------
// PushChunker (src/chunking.rs:753-829) over drain_finalized_chunks (:541-673)
// ---------------------------------------------------------------------------
// The retained bytes live in HBM: each push copies only its new bytes H2D, straight
// from the caller's buffer, after the device-resident tail (no host-side copy of
// the stream); after a drain the tail moves to the front of the other buffer.
struct cg_push {
    Opts o;
    int algo;
    int device = -1;
    DevBuf dbuf[2];
    int cur = 0;
    uint64_t dlen = 0;  // retained bytes in dbuf[cur]
    uint64_t position = 0;
    bool finished = false;
    ~cg_push() {
        if (device >= 0) {
            int prev = 0;
            (void)hipGetDevice(&prev);
            (void)hipSetDevice(device);
            dbuf[0].release();
            dbuf[1].release();
            (void)hipSetDevice(prev);
        }
    }
};

namespace cgrt {

// drain_finalized_chunks (src/chunking.rs:541-673) on the GPU.  The retained buffer
// is staged once; boundaries for all of it come from the device pipeline (the
// reference re-runs FastCDC over the buffer too, :553); the descriptors go back to the
// host, which decides what is final (:579-584); then only the final chunks are
// digested, on the bytes already in HBM -- the retained tail chunk is never hashed
// twice (the reference hashes only emitted chunks, :612-641).
int push_drain(cg_push *h, bool eof, cg_desc *out, size_t out_cap, size_t *n_out) {
    *n_out = 0;
    if (h->dlen == 0 || (h->dlen < h->o.min && !eof)) return CG_OK;
    Workspace *ws = nullptr;
    int rc = acquire(&ws);
    if (rc) return rc;
    WsGuard guard{ws};
    const uint64_t len = h->dlen;
    const uint64_t cap = capacity_of(len, h->o.min);
    hipStream_t st = ws->stream;
    if ((rc = ws->out.ensure((cap + 1) * sizeof(cg_desc), "descriptors"))) return rc;
    const uint8_t *d_in = h->dbuf[h->cur].as<uint8_t>();
    uint64_t offs[2] = {0, len}, first[2] = {0, 0};
    cg_desc *d_out = ws->out.as<cg_desc>();
    if ((rc = run_batch(ws, d_in, offs, 1, h->o, h->algo, d_out, cap, first, st, nullptr, nullptr,
                        /*digest=*/false)))
        return rc;
    const uint64_t total = first[1];
    std::vector<cg_desc> tmp(total);
    if (total) {
        HIP_TRY(hipMemcpyAsync(tmp.data(), d_out, total * sizeof(cg_desc), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    size_t n = 0;
    uint64_t emitted = 0;
    for (uint64_t k = 0; k < total; ++k) {
        const cg_desc &d = tmp[k];
        if (d.length == 0) return fail(CG_E_ZERO_LENGTH_CHUNK, "FastCDC returned a chunk with length 0");
        const bool touches_end = d.offset + d.length == len;
        if (touches_end && !eof && d.length < h->o.max) break;  // retained tail (:579-584)
        ++n;
        emitted += d.length;
    }
    // EOF remainder (:651-670): FastCDC's chunks always cover the buffer, so at EOF
    // every byte has been emitted; anything else is an engine fault, never silent
    if (eof && emitted < len) return fail(CG_E_IO, "push: chunks do not cover the buffer at finish");
    if (n > out_cap) return fail(CG_E_CAPACITY, "push output array too small");
    if (n) {
        // digest descriptors [0, n) in place: the count goes to the device total slot
        uint64_t *d_total = ws->nar_first.as<uint64_t>() + 1;
        if ((rc = ws->stage.ensure(64, /*mapped=*/true))) return rc;
        ws->stage.as<uint64_t>()[0] = n;
        HIP_TRY(hipMemcpyAsync(d_total, ws->stage.p, 8, hipMemcpyHostToDevice, st));
        uint8_t *hb = reinterpret_cast<uint8_t *>(d_out) + offsetof(cg_desc, hash);
        bool sha_armed = false;
        if (h->algo == CG_SHA256) {
            if ((rc = ws->order.ensure(cg::sha256_order_tmp_elems(n) * 4, "order"))) return rc;
            if ((rc = sha_err_arm(ws, st))) return rc;
            sha_armed = true;
            cg::launch_sha256(d_in, ws->chunk_abs.as<uint64_t>(), d_out, d_total, n, n, h->o.max,
                              ws->order.as<uint32_t>(), hb, sizeof(cg_desc), ws->sha_err.as<uint32_t>(), st);
        } else {
            const uint64_t gb = cg::blake3_group_bound(len, n);
            if ((rc = ws->b3_gcount.ensure((n + 1) * 4, "b3_gcount"))) return rc;
            if ((rc = ws->b3_gbase.ensure((n + 1) * 8, "b3_gbase"))) return rc;
            if ((rc = ws->b3_gcv.ensure(cg::blake3_cv_bytes(len, n, true), "b3_gcv"))) return rc;
            if ((rc = ws->b3_gmap.ensure((gb + 1) * 4, "b3_gmap"))) return rc;
            cg::launch_blake3(d_in, ws->chunk_abs.as<uint64_t>(), d_out, d_total, n, len, hb,
                              sizeof(cg_desc), ws->b3_gmap.as<uint32_t>(), ws->b3_gbase.as<uint64_t>(),
                              ws->b3_gcount.as<uint32_t>(), ws->scan_tmp.as<uint64_t>(), ws->b3_gcv.as<uint32_t>(),
                              true, st);
        }
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(out, d_out, n * sizeof(cg_desc), hipMemcpyDeviceToHost, st));
        if (sha_armed && (rc = sha_err_fetch(ws, st))) return rc;
        HIP_TRY(hipStreamSynchronize(st));
        if (sha_armed && (rc = sha_err_check(ws))) return rc;
        for (size_t k = 0; k < n; ++k) out[k].offset += h->position;
    }
    const uint64_t consumed = eof ? len : emitted;
    const uint64_t tail = len - consumed;
    if (tail && consumed) {  // tail to the front of the other buffer (16-B aligned base)
        if ((rc = h->dbuf[1 - h->cur].ensure(std::max(h->dbuf[h->cur].cap, tail + 256), "push buffer"))) return rc;
        HIP_TRY(hipMemcpyAsync(h->dbuf[1 - h->cur].p, d_in + consumed, tail, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));
        h->cur = 1 - h->cur;
    }
    h->dlen = tail;
    h->position += consumed;
    *n_out = n;
    return CG_OK;
}

// Append `len` caller bytes after the device-resident tail (growing the buffer keeps
// the tail: it is copied into the larger other buffer first).
int push_append(cg_push *h, const uint8_t *data, uint64_t len) {
    int dev = 0, rc = current_device(&dev);
    if (rc) return rc;
    if (h->device < 0) h->device = dev;
    if (h->device != dev) return fail(CG_E_IO, "push handle used on another device than the one it started on");
    Workspace *ws = nullptr;
    if ((rc = acquire(&ws))) return rc;
    WsGuard guard{ws};
    hipStream_t st = ws->stream;
    // both buffers always have the same capacity, so a tail move never needs to grow one
    const uint64_t need = h->dlen + len + 256;
    if (need > h->dbuf[h->cur].cap) {
        // grow: the tail moves into the (larger) other buffer, which becomes current as
        // soon as it holds the only copy; a failed allocation leaves a usable handle
        DevBuf &nb = h->dbuf[1 - h->cur];
        nb.release();
        if ((rc = nb.ensure(need, "push buffer"))) return rc;
        if (h->dlen) HIP_TRY(hipMemcpyAsync(nb.p, h->dbuf[h->cur].p, h->dlen, hipMemcpyDeviceToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));
        h->cur = 1 - h->cur;
        DevBuf &ob = h->dbuf[1 - h->cur];
        ob.release();
        if ((rc = ob.ensure(need, "push buffer"))) return rc;  // same request -> same capacity
    }
    HIP_TRY(hipMemcpyAsync(h->dbuf[h->cur].as<uint8_t>() + h->dlen, data, len, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    h->dlen += len;
    return CG_OK;
}

}  // namespace cgrt

extern "C" int cg_test_split_mode(int v) { return cgrt::g_split_mode.exchange(v == 2 ? 2 : 1); }

extern "C" uint32_t cg_test_coalesce(uint32_t v) {  // 0 = every device-entry call digests alone
    return cgrt::g_coalesce.exchange(v ? 1u : 0u);
}

// Coalescer counters of the current device since the process started: out = {groups led,
// batches in them, total leader wait (us), groups launched because the window ran out}.
extern "C" void cg_coalesce_stats(uint64_t out[4]) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    cgrt::Coalescer &C = cgrt::coalescer(dev);
    std::lock_guard<std::mutex> g(C.mu);
    out[0] = C.groups;
    out[1] = C.members;
    out[2] = C.wait_us;
    out[3] = C.window_expired;
}

extern "C" {

uint32_t cg_abi_version(void) { return CG_ABI_VERSION; }

// Test hook: make the n-th device-buffer growth from now fail as out of memory (0 = off);
// returns the previous countdown.
uint32_t cg_test_fail_alloc(uint32_t n) { return cgrt::g_fail_alloc.exchange(n); }

// Test hook: BLAKE3 group map from the walk + assembly (1) or from k_b3_plan (0); returns
// the previous setting.
int cg_test_b3_fused_plan(int on) { return cgrt::g_b3_fused_plan.exchange(on ? 1 : 0); }

// Test hook: BLAKE3 leaves packed across chunks (1) or one group per wave (0); returns the
// previous setting.
int cg_test_b3_packed(int on) { return cgrt::g_b3_packed.exchange(on ? 1 : 0); }

const char *cg_last_error_message(void) { return t_err.c_str(); }

int cg_validate(uint64_t min_size, uint64_t avg_size, uint64_t max_size, char *msg, size_t msg_cap) {
    clear_error();
    Opts o;
    return resolve(min_size, avg_size, max_size, &o, msg, msg_cap);
}

size_t cg_capacity(uint64_t len, uint64_t min_size) { return capacity_of(len, min_size ? min_size : DEF_MIN); }

int cg_chunk_batch(const uint8_t *data, const uint64_t *nar_offsets, size_t n_nars, uint64_t min_size,
                   uint64_t avg_size, uint64_t max_size, int algo, cg_desc *out, size_t out_cap,
                   uint64_t *nar_first) {
    clear_error();
    return batch_host(data, nar_offsets, n_nars, min_size, avg_size, max_size, algo, out, out_cap, nar_first);
}

int cg_chunk_descriptors(const uint8_t *data, uint64_t len, uint64_t min_size, uint64_t avg_size,
                         uint64_t max_size, int algo, cg_desc *out, size_t out_cap, size_t *n_out) {
    clear_error();
    uint64_t offs[2] = {0, len};
    uint64_t first[2] = {0, 0};
    int rc = batch_host(data, offs, 1, min_size, avg_size, max_size, algo, out, out_cap, first);
    if (n_out) *n_out = rc == CG_OK ? first[1] : 0;
    return rc;
}

int cg_chunk_batch_device(const uint8_t *d_data, const uint64_t *nar_offsets, size_t n_nars, uint64_t min_size,
                          uint64_t avg_size, uint64_t max_size, int algo, cg_desc *d_out, size_t out_cap,
                          uint64_t *nar_first, void *stream) {
    clear_error();
    Opts o;
    int rc = resolve(min_size, avg_size, max_size, &o, nullptr, 0);
    if (rc) return rc;
    if (n_nars && nar_offsets[0] != 0)
        return fail_bounds(nar_offsets[n_nars], nar_offsets[0], 0, "device batch offsets must start at 0");
    if ((rc = check_tables())) return rc;
    Workspace *ws = nullptr;
    if ((rc = acquire(&ws))) return rc;
    WsGuard guard{ws};
    // concurrent SHA-256 callers share one digest launch (coalesced_sha256)
    if (algo != CG_SHA256 || !g_coalesce.load(std::memory_order_relaxed))
        return run_batch(ws, d_data, nar_offsets, n_nars, o, algo, d_out, out_cap, nar_first,
                         static_cast<hipStream_t>(stream));
    CoalActive active(ws->device);
    t_coal_active = &active;
    rc = run_batch(ws, d_data, nar_offsets, n_nars, o, algo, d_out, out_cap, nar_first,
                   static_cast<hipStream_t>(stream), nullptr, nullptr, true, true);
    t_coal_active = nullptr;
    active.leave();
    return rc;
}

int cg_chunk_batch_device_async(const uint8_t *d_data, const uint64_t *nar_offsets, size_t n_nars, uint64_t min_size,
                                uint64_t avg_size, uint64_t max_size, int algo, cg_desc *d_out, size_t out_cap,
                                void *stream, cg_batch **batch) {
    return cg_chunk_batch_device_async_after(d_data, nar_offsets, n_nars, min_size, avg_size, max_size, algo, d_out,
                                             out_cap, stream, nullptr, batch);
}

int cg_chunk_batch_device_async_after(const uint8_t *d_data, const uint64_t *nar_offsets, size_t n_nars,
                                      uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo,
                                      cg_desc *d_out, size_t out_cap, void *stream, void *inputs_ready,
                                      cg_batch **batch) {
    clear_error();
    if (!batch) return fail(CG_E_IO, "null batch handle pointer");
    *batch = nullptr;
    Opts o;
    int rc = resolve(min_size, avg_size, max_size, &o, nullptr, 0);
    if (rc) return rc;
    if (n_nars && nar_offsets[0] != 0)
        return fail_bounds(nar_offsets[n_nars], nar_offsets[0], 0, "device batch offsets must start at 0");
    if ((rc = check_tables())) return rc;
    Workspace *ws = nullptr;
    if ((rc = acquire(&ws))) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    BatchLaunch bl;
    rc = launch_batch(ws, d_data, nar_offsets, n_nars, o, algo, d_out, out_cap, st, nullptr, nullptr, true, &bl,
                      false, static_cast<hipEvent_t>(inputs_ready));
    if (rc) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamSynchronize(ws->stream);
        release(ws);
        return rc;
    }
    *batch = new cg_batch{ws, st, bl, nullptr, 0, ws->device};
    return CG_OK;
}

int cg_batch_wait(cg_batch *batch, uint64_t *nar_first) {
    clear_error();
    if (!batch) return fail(CG_E_IO, "null batch handle");
    if (batch->group) return pipeline_wait(batch, nar_first);  // frees the handle
    const int rc = finish_batch(batch->ws, batch->st, batch->bl, nar_first);
    release(batch->ws);
    delete batch;
    return rc;
}

int cg_hash_spans_device(const uint8_t *d_data, const uint64_t *d_offsets, const uint64_t *d_lengths, size_t n,
                         int algo, uint8_t *d_digests, void *stream) {
    clear_error();
    if (algo != CG_BLAKE3 && algo != CG_SHA256) return fail(CG_E_INVALID_OPTIONS, "unknown hash algorithm");
    if (n == 0) return CG_OK;
    Workspace *ws = nullptr;
    int rc = acquire(&ws);
    if (rc) return rc;
    WsGuard guard{ws};
    return hash_spans(ws, d_data, d_offsets, d_lengths, n, algo, d_digests, static_cast<hipStream_t>(stream));
}

int cg_cas_ids_device(const uint8_t *d_data, const uint64_t *d_offsets, const uint64_t *d_lengths, size_t n,
                      uint32_t kind, uint8_t *d_ids, void *stream) {
    clear_error();
    int rc = check_kind(kind);
    if (rc || n == 0) return rc;
    Workspace *ws = nullptr;
    if ((rc = acquire(&ws))) return rc;
    WsGuard guard{ws};
    return cas_spans(ws, d_data, d_offsets, d_lengths, n, kind, d_ids, static_cast<hipStream_t>(stream));
}

int cg_cas_id(const uint8_t *data, uint64_t len, uint32_t kind, uint8_t out[32]) {
    clear_error();
    int rc = check_kind(kind);
    if (rc) return rc;
    Workspace *ws = nullptr;
    if ((rc = acquire(&ws))) return rc;
    WsGuard guard{ws};
    if ((rc = ws->in.ensure(len + 256, "input"))) return rc;
    if ((rc = ws->span_off.ensure(64, "span"))) return rc;
    if ((rc = ws->stage.ensure(64, /*mapped=*/true))) return rc;
    uint64_t *s = ws->stage.as<uint64_t>();
    s[0] = 0;
    s[1] = len;
    if (len) HIP_TRY(hipMemcpyAsync(ws->in.p, data, len, hipMemcpyHostToDevice, ws->stream));
    HIP_TRY(hipMemcpyAsync(ws->span_off.p, s, 16, hipMemcpyHostToDevice, ws->stream));
    const uint64_t *d_off = ws->span_off.as<uint64_t>();
    uint8_t *d_id = reinterpret_cast<uint8_t *>(ws->span_off.as<uint64_t>() + 2);
    if ((rc = cas_spans(ws, ws->in.as<uint8_t>(), d_off, d_off + 1, 1, kind, d_id, ws->stream))) return rc;
    HIP_TRY(hipMemcpyAsync(s + 2, d_id, 32, hipMemcpyDeviceToHost, ws->stream));
    HIP_TRY(hipStreamSynchronize(ws->stream));
    memcpy(out, s + 2, 32);
    return CG_OK;
}

int cg_node_put_batch_device(const uint8_t *d_data, const uint64_t *nar_offsets, size_t n_nars, uint64_t min_size,
                             uint64_t avg_size, uint64_t max_size, cg_desc *d_out, size_t out_cap,
                             uint64_t *nar_first, uint8_t *d_chunk_ids, uint8_t *manifest_ids, void *stream) {
    clear_error();
    Opts o;
    int rc = resolve(min_size, avg_size, max_size, &o, nullptr, 0);
    if (rc) return rc;
    if (!d_chunk_ids) return fail(CG_E_IO, "node put: null chunk id buffer");
    if (n_nars && nar_offsets[0] != 0)
        return fail_bounds(nar_offsets[n_nars], nar_offsets[0], 0, "device batch offsets must start at 0");
    if ((rc = check_tables())) return rc;
    Workspace *ws = nullptr;
    if ((rc = acquire(&ws))) return rc;
    WsGuard guard{ws};
    return run_batch(ws, d_data, nar_offsets, n_nars, o, CG_SHA256, d_out, out_cap, nar_first,
                     static_cast<hipStream_t>(stream), d_chunk_ids, manifest_ids);
}

int cg_node_put(const uint8_t *data, uint64_t len, uint64_t min_size, uint64_t avg_size, uint64_t max_size,
                cg_desc *out, size_t out_cap, size_t *n_out, uint8_t *chunk_ids, uint8_t manifest_id[32]) {
    clear_error();
    if (n_out) *n_out = 0;
    Opts o;
    int rc = resolve(min_size, avg_size, max_size, &o, nullptr, 0);
    if (rc) return rc;
    if ((rc = check_tables())) return rc;
    Workspace *ws = nullptr;
    if ((rc = acquire(&ws))) return rc;
    WsGuard guard{ws};
    const uint64_t cap = capacity_of(len, o.min);
    if ((rc = ws->in.ensure(len + 256, "input"))) return rc;
    if ((rc = ws->out.ensure((cap + 1) * sizeof(cg_desc), "descriptors"))) return rc;
    if ((rc = ws->span_len.ensure((cap + 1) * 32, "chunk ids"))) return rc;
    if (len) HIP_TRY(hipMemcpyAsync(ws->in.p, data, len, hipMemcpyHostToDevice, ws->stream));
    uint64_t offs[2] = {0, len}, first[2] = {0, 0};
    uint8_t man[32];
    rc = run_batch(ws, ws->in.as<uint8_t>(), offs, 1, o, CG_SHA256, ws->out.as<cg_desc>(), cap, first, ws->stream,
                   ws->span_len.as<uint8_t>(), man);
    if (rc) return rc;
    const uint64_t total = first[1];
    if (total > out_cap) return fail(CG_E_CAPACITY, "descriptor output array too small");
    if (total) {
        HIP_TRY(hipMemcpyAsync(out, ws->out.p, total * sizeof(cg_desc), hipMemcpyDeviceToHost, ws->stream));
        if (chunk_ids) HIP_TRY(hipMemcpyAsync(chunk_ids, ws->span_len.p, total * 32, hipMemcpyDeviceToHost, ws->stream));
        HIP_TRY(hipStreamSynchronize(ws->stream));
    }
    if (n_out) *n_out = total;
    if (manifest_id) memcpy(manifest_id, man, 32);
    return CG_OK;
}

int cg_hash(const uint8_t *data, uint64_t len, int algo, uint8_t out[32]) {
    clear_error();
    if (algo != CG_BLAKE3 && algo != CG_SHA256) return fail(CG_E_INVALID_OPTIONS, "unknown hash algorithm");
    if (algo == CG_BLAKE3 && len > MAXIMUM_MAX) return fail(CG_E_BOUNDS, "cg_hash: BLAKE3 input above 16 MiB");
    Workspace *ws = nullptr;
    int rc = acquire(&ws);
    if (rc) return rc;
    WsGuard guard{ws};
    if ((rc = ws->in.ensure(len + 256, "input"))) return rc;
    if ((rc = ws->span_off.ensure(64, "span"))) return rc;
    if ((rc = ws->stage.ensure(64, /*mapped=*/true))) return rc;
    uint64_t *s = ws->stage.as<uint64_t>();
    s[0] = 0;
    s[1] = len;
    if (len) HIP_TRY(hipMemcpyAsync(ws->in.p, data, len, hipMemcpyHostToDevice, ws->stream));
    HIP_TRY(hipMemcpyAsync(ws->span_off.p, s, 16, hipMemcpyHostToDevice, ws->stream));
    const uint64_t *d_off = ws->span_off.as<uint64_t>();
    uint8_t *d_dig = reinterpret_cast<uint8_t *>(ws->span_off.as<uint64_t>() + 2);
    if ((rc = hash_spans(ws, ws->in.as<uint8_t>(), d_off, d_off + 1, 1, algo, d_dig, ws->stream))) return rc;
    HIP_TRY(hipMemcpyAsync(s + 2, d_dig, 32, hipMemcpyDeviceToHost, ws->stream));
    HIP_TRY(hipStreamSynchronize(ws->stream));
    memcpy(out, s + 2, 32);
    return CG_OK;
}

cg_push *cg_push_new(uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo, int *status) {
    clear_error();
    Opts o;
    int rc = resolve(min_size, avg_size, max_size, &o, nullptr, 0);
    if (!rc && algo != CG_BLAKE3 && algo != CG_SHA256) rc = fail(CG_E_INVALID_OPTIONS, "unknown hash algorithm");
    if (status) *status = rc;
    if (rc) return nullptr;
    cg_push *h = new cg_push();
    h->o = o;
    h->algo = algo;
    return h;
}

int cg_push_push(cg_push *h, const uint8_t *data, uint64_t len, cg_desc *out, size_t out_cap, size_t *n_out) {
    clear_error();
    if (n_out) *n_out = 0;
    if (!h) return fail(CG_E_IO, "null push handle");
    if (h->finished) return fail(CG_E_INVALID_OPTIONS, "push called after finish");
    if (len == 0) return CG_OK;
    int rc = check_tables();
    if (rc) return rc;
    const uint64_t dlen0 = h->dlen;
    if ((rc = push_append(h, data, len))) return rc;
    size_t n = 0;
    if ((rc = push_drain(h, false, out, out_cap, &n))) {
        // push_drain changes the handle only on success: dropping the appended bytes
        // leaves it exactly as before this call, so a caller may retry the same slice
        h->dlen = dlen0;
        return rc;
    }
    if (n_out) *n_out = n;
    return CG_OK;
}

int cg_push_finish(cg_push *h, cg_desc *out, size_t out_cap, size_t *n_out) {
    clear_error();
    if (n_out) *n_out = 0;
    if (!h) return fail(CG_E_IO, "null push handle");
    int rc0 = check_tables();
    if (rc0) return rc0;
    h->finished = true;
    size_t n = 0;
    int rc = push_drain(h, true, out, out_cap, &n);
    if (n_out) *n_out = n;
    return rc;
}

uint64_t cg_push_bytes_consumed(const cg_push *h) { return h ? h->position + h->dlen : 0; }

size_t cg_push_out_capacity(const cg_push *h, uint64_t next_len) {
    return h ? capacity_of(h->dlen + next_len, h->o.min) + 1 : 0;
}

void cg_push_free(cg_push *h) { delete h; }

int cg_set_cdc_tables(const uint64_t gear[256], const uint64_t masks[26]) {
    clear_error();
    if (!gear) return fail(CG_E_INVALID_OPTIONS, "null GEAR table");
    auto t = std::make_shared<Tables>();
    memcpy(t->gear, gear, sizeof t->gear);
    if (masks) {
        // the candidate scan's 48-byte window is exact only for masks within bits 0..47
        for (int i = 0; i < 26; ++i)
            if (masks[i] >> 48)
                return fail(CG_E_INVALID_OPTIONS, "MASKS[" + std::to_string(i) +
                                                      "] has bits above 47: unsupported by the windowed GPU scan");
        memcpy(t->masks, masks, sizeof t->masks);
    } else {
        memcpy(t->masks, tables()->masks, sizeof t->masks);
    }
    t->placeholder = CG_GEAR_IS_PLACEHOLDER && memcmp(gear, CG_DEFAULT_GEAR, sizeof t->gear) == 0;
    std::lock_guard<std::mutex> g(g_tab_mu);
    t->epoch = g_tab_epoch.fetch_add(1) + 1;
    g_tab = t;
    return CG_OK;
}

int cg_set_gear_table(const uint64_t gear[256]) { return cg_set_cdc_tables(gear, nullptr); }

void cg_get_cdc_tables(uint64_t gear[256], uint64_t masks[26]) {
    const std::shared_ptr<const Tables> t = tables();
    if (gear) memcpy(gear, t->gear, sizeof t->gear);
    if (masks) memcpy(masks, t->masks, sizeof t->masks);
}

void cg_get_gear_table(uint64_t gear[256]) { cg_get_cdc_tables(gear, nullptr); }

int cg_gear_is_placeholder(void) { return tables()->placeholder ? 1 : 0; }

int cg_selftest(void) {
    clear_error();
    return selftest_gpu();
}

int cg_tables_verified(void) { return g_verified_epoch.load() == tables()->epoch ? 1 : 0; }

int cg_last_error_detail(uint64_t out[3]) {
    if (out) memcpy(out, t_detail, sizeof t_detail);
    return t_status;
}

void cg_set_profiling(int on) { g_profiling.store(on == 2 ? 2 : on ? 1 : 0); }

size_t cg_last_stage_times(double *ms, size_t n) {
    const size_t k = std::min(n, t_stage_ms.size());
    for (size_t i = 0; i < k; ++i) ms[i] = t_stage_ms[i];
    return k;
}

void cg_synth_nars(uint8_t *out, const uint64_t *nar_sizes, size_t n, int zeros, uint64_t first_index) {
    std::vector<uint64_t> off(n + 1, 0);
    for (size_t i = 0; i < n; ++i) off[i + 1] = off[i] + nar_sizes[i];
    auto one = [&](size_t i) {
        uint8_t *p = out + off[i];
        const uint64_t S = nar_sizes[i];
        const uint64_t L = S >= 112 ? S - 112 : 0;  // payload; framing is 112 bytes for a regular file
        uint64_t at = 0;
        auto put_u64 = [&](uint64_t v) {
            memcpy(p + at, &v, 8);
            at += 8;
        };
        auto put_str = [&](const char *s) {
            const uint64_t l = strlen(s);
            put_u64(l);
            memset(p + at, 0, (l + 7) / 8 * 8);
            memcpy(p + at, s, l);
            at += (l + 7) / 8 * 8;
        };
        put_str("nix-archive-1");
        put_str("(");
        put_str("type");
        put_str("regular");
        put_str("contents");
        put_u64(L);
        if (zeros) {
            memset(p + at, 0, L);
        } else {  // xorshift64, crates/node/src/lib.rs:192-203
            uint64_t state = (0x9E3779B97F4A7C15ull ^ (first_index + i)) | 1ull;
            uint64_t k = 0;
            for (; k + 8 <= L; k += 8) {
                state ^= state << 13;
                state ^= state >> 7;
                state ^= state << 17;
                memcpy(p + at + k, &state, 8);
            }
            if (k < L) {
                state ^= state << 13;
                state ^= state >> 7;
                state ^= state << 17;
                memcpy(p + at + k, &state, L - k);
            }
        }
        at += L;
        // payload padded to 8 (L may be unaligned only if S is not a multiple of 8)
        const uint64_t pad = (8 - (L & 7)) & 7;
        memset(p + at, 0, std::min<uint64_t>(pad, S - std::min(S, at)));
        at += pad;
        if (at + 16 <= S) {
            put_str(")");
        }
    };
    const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n <= 1 || nt == 1) {
        for (size_t i = 0; i < n; ++i) one(i);
        return;
    }
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&]() {
            for (size_t i; (i = next.fetch_add(1)) < n;) one(i);
        });
    for (auto &t : th) t.join();
}

}  // extern "C"
