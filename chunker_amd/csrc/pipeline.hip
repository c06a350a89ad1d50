// pipeline.hip -- the digest pipeline (cg_pipeline_*, round 6): batches in flight from one
// caller, their SHA-256 digests merged G at a time into ONE k_sha256 launch.
//
// A device batch's SHA-256 digest is bound by its longest chunk's serial chain (config 2:
// ~55 ms for a 1 GiB batch) and, with the latency tiers, occupies only ~18 workgroups,
// so one caller needs many batches in flight to fill the chip.  Round 5 bought that
// concurrency with one HIP stream per batch in flight (cg_chunk_batch_device_async_after):
// twenty batches needed GPU_MAX_HW_QUEUES=22, HIP's default 4 queues gave 36-60 GiB/s, and
// an RCCL communicator in the same process took queues away (0.70 of the rate).  Here the
// concurrency lives inside one launch instead:
//   * every batch's boundary stages (scan, compaction, walk, assembly) run on the
//     pipeline's one boundary stream, each after its own inputs-ready event;
//   * the batches queued since the last digest form the open group; at G members (or
//     when a member is waited for, or at cg_pipeline_flush) the group's chunk lists are
//     merged (k_pipe_merge) and digested by one k_sha256 on one of the pipeline's L digest
//     lanes (streams), so the next group's boundary stages and digest run beside it;
//   * the digest kernel counts each member down as its chunks finish and raises the
//     member's host-mapped completion word when its last chunk is stored (ShaNotify), so a
//     batch completes when ITS longest chunk does, not when the merged launch ends, and a
//     cg_batch_wait returns as soon as its own digests are in HBM.
// The pipeline holds 1 + L streams (L = 3 by default) however many batches are in flight.  They are
// non-blocking high-priority streams (CHUNKER_AMD_PIPE_STREAMS, below): HIP keeps a pool
// of hardware queues per priority, so they do not share a queue with the process's
// ordinary streams however many of those are busy (scripts/micro/queue_probe.hip,
// profiles/r06_v4_queue_probe.txt: three such streams ran three 40 ms kernels side by side
// beside 16 busy ordinary streams at GPU_MAX_HW_QUEUES=4, where three ordinary streams took
// 5x as long).  A full-CU-mask stream also gets a queue of its own, but HIP creates it as a
// blocking stream (it then synchronises with the legacy null stream, which torch and other
// callers use).  BLAKE3 batches (a digest that fills the chip by itself) run whole on a
// boundary stream (three when the pipeline starts with one: start_streams).
// Replaces, across a caller's consecutive chunk_descriptors_with_hash calls, the
// collect-then-hash sequence of src/chunking.rs:334-368.
#include <chrono>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "runtime.h"

namespace cgrt {

struct PipeMember {
    Workspace *ws = nullptr;
    const uint8_t *d_data = nullptr;
    cg_desc *d_out = nullptr;
    const uint64_t *d_abs = nullptr, *d_total = nullptr;
    uint64_t bound = 0, expected = 0, max_len = 0, bytes = 0;
    volatile uint32_t *flag_host = nullptr;  // mapped: written by the digest kernel
    uint32_t *flag_dev = nullptr;
};

constexpr uint32_t PIPE_MAX_BSTREAMS = 4;

struct PipeGroup {
    std::vector<PipeMember> members;
    hipEvent_t bdone[PIPE_MAX_BSTREAMS] = {}, done = nullptr, t0 = nullptr, t1 = nullptr;
    bool launched = false, timed = false;
    int rc = CG_OK;
    std::string err;
    uint64_t detail[3] = {0, 0, 0};
    uint64_t bytes = 0;
    cg_pipeline *owner = nullptr;  // while the group is open (a wait flushes it)
    ~PipeGroup() {
        for (hipEvent_t e : bdone)
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : {done, t0, t1})
            if (e) (void)hipEventDestroy(e);
    }
};

struct PipeLane {
    hipStream_t st = nullptr;
    DevBuf mdesc, mabs, mdst, mmember, mtotal, morder, remain, merr, mflag, err;
    std::shared_ptr<PipeGroup> last;
};

// Lane staggering (device side).  Lanes whose groups form faster than they digest start
// their launches together -- the fill submits (lanes + 1) groups at once -- and stay in
// phase: completions then come in bursts of `lanes` groups, and any window of one group's
// completions reads anywhere from 0.7x to 1.4x the steady rate (profiles/r06_v36_*).  So each
// lane's launch first waits (k_pipe_stagger, one wave) until `ema / lanes` after the latest
// launch on any lane, ema = the lanes' recent launch durations (k_pipe_end after each merged
// digest).  Times are s_memrealtime ticks (100 MHz); a wait never exceeds 50 ms.
struct PipeClock {
    unsigned long long last_start, ema, start[8];
};

__global__ void k_pipe_stagger(PipeClock *c, uint32_t lane, uint32_t nlanes) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long last = __hip_atomic_load(&c->last_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long ema = __hip_atomic_load(&c->ema, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long target = last + ema / nlanes;
    unsigned long long now = t0;
    while (last && ema && now < target && now - t0 < 5000000ull) {
        __builtin_amdgcn_s_sleep(32);
        now = __builtin_amdgcn_s_memrealtime();
    }
    __hip_atomic_store(&c->start[lane], now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&c->last_start, now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_pipe_end(PipeClock *c, uint32_t lane) {
    if (threadIdx.x != 0) return;
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    const unsigned long long st = __hip_atomic_load(&c->start[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long ema = __hip_atomic_load(&c->ema, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!st || now <= st) return;
    const unsigned long long d = now - st;
    __hip_atomic_store(&c->ema, ema ? (3 * ema + d) / 4 : d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace cgrt

struct cg_pipeline {
    int device = -1;
    uint32_t group_max = 0, nlanes = 0;
    // boundary streams: a submitted batch's stages run on bstream[k % nb] (batch k)
    hipStream_t bstream[cgrt::PIPE_MAX_BSTREAMS] = {};
    uint32_t nb = 0, next_b = 0;  // nb 0: no batch yet (start_streams)
    std::vector<cgrt::PipeLane> lanes;
    uint32_t next_lane = 0;
    cgrt::DevBuf clock;  // PipeClock (lane staggering)
    std::shared_ptr<cgrt::PipeGroup> open;
    std::mutex mu;
    // counters (cg_pipeline_stats)
    uint64_t groups = 0, batches = 0, timed_groups = 0;
    double digest_ms = 0, digest_bytes = 0, last_digest_ms = 0;
    std::deque<std::shared_ptr<cgrt::PipeGroup>> timing;  // timed groups not yet read
};

namespace cgrt {

// Stream kind of the pipeline's streams (CHUNKER_AMD_PIPE_STREAMS, read once): default =
// non-blocking, priority streams: the boundary streams high priority (HIP's high-priority
// queue pool, four queues), the digest lanes too while they all fit there, else low priority
// (the low-priority pool, four more queues); "high" / "split" = lanes always high / low;
// "cumask" = a CU mask over every CU (a queue of its own, but a blocking stream); "plain" =
// ordinary non-blocking streams (the shared pool).  The last three are A/B only.
static int pipe_stream_kind() {
    static const int k = [] {
        const char *e = getenv("CHUNKER_AMD_PIPE_STREAMS");
        if (e && !strcmp(e, "plain")) return 0;
        if (e && !strcmp(e, "cumask")) return 2;
        if (e && !strcmp(e, "split")) return 3;
        if (e && !strcmp(e, "high")) return 4;
        return 1;
    }();
    return k;
}

// Lane staggering off (default) / on (CHUNKER_AMD_PIPE_STAGGER=1, read once; A/B): at three
// lanes the boundary stream spaces the launches by itself; the wait measured neutral on
// config 2 and cost configs 4 / 5 their 20-step lines (profiles/r06_v40_summary.txt).
static bool pipe_stagger() {
    static const bool on = [] {
        const char *e = getenv("CHUNKER_AMD_PIPE_STAGGER");
        return e && e[0] == '1';
    }();
    return on;
}

static int make_stream(hipStream_t *s, bool low) {
    const int kind = pipe_stream_kind();
    if (kind == 1 || kind == 3 || kind == 4) {
        int lo = 0, hi = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIP_TRY(hipStreamCreateWithPriority(s, hipStreamNonBlocking, low ? lo : hi));
    } else if (kind == 2) {
        int dev = 0;
        HIP_TRY(hipGetDevice(&dev));
        int ncu = 0;
        HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0xffffffffu);
        HIP_TRY(hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data()));
    } else {
        HIP_TRY(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
    }
    return CG_OK;
}

// The group's failure, as seen by each of its members' waits.
static int group_fail(PipeGroup &g, int rc) {
    g.rc = rc;
    g.err = cg_last_error_message();
    cg_last_error_detail(g.detail);
    return rc;
}

// Launch the open group's merged digest on the next lane (pipeline lock held).
static int flush_locked(cg_pipeline *p) {
    std::shared_ptr<PipeGroup> g = std::move(p->open);
    p->open.reset();
    if (!g || g->members.empty()) return CG_OK;
    g->owner = nullptr;
    g->launched = true;
    PipeLane &L = p->lanes[p->next_lane];
    p->next_lane = (p->next_lane + 1) % p->nlanes;
    auto launch = [&]() -> int {
        for (uint32_t i = 0; i < p->nb; ++i) {
            HIP_TRY(hipEventRecord(g->bdone[i], p->bstream[i]));
            HIP_TRY(hipStreamWaitEvent(L.st, g->bdone[i], 0));
        }
        cg::PipeTable t{};
        t.n = (uint32_t)g->members.size();
        uint64_t bound = 0, expected = 0, max_len = 0;
        for (uint32_t b = 0; b < t.n; ++b) {
            const PipeMember &m = g->members[b];
            t.data[b] = m.d_data;
            t.abs[b] = m.d_abs;
            t.out[b] = reinterpret_cast<DescRaw *>(m.d_out);
            t.total[b] = m.d_total;
            t.bound[b] = m.bound;
            t.flag[b] = m.flag_dev;
            bound += m.bound;
            expected += m.expected;
            max_len = std::max(max_len, m.max_len);
        }
        // growing a lane buffer frees the old one, which the lane's previous group may
        // still read: wait for it first (only until the buffers have their steady size)
        const uint64_t ord = cg::sha256_order_tmp_elems(bound) * 4;
        const bool grow = L.mdesc.cap < (bound + 1) * sizeof(DescRaw) || L.morder.cap < ord || !L.remain.p;
        if (grow && L.last) HIP_TRY(hipEventSynchronize(L.last->done));
        int rc;
        if ((rc = L.mdesc.ensure((bound + 1) * sizeof(DescRaw), "pipeline descriptors"))) return rc;
        if ((rc = L.mabs.ensure((bound + 1) * 8, "pipeline addresses"))) return rc;
        if ((rc = L.mdst.ensure((bound + 1) * 8, "pipeline destinations"))) return rc;
        if ((rc = L.mmember.ensure((bound + 1) * 4, "pipeline members"))) return rc;
        if ((rc = L.morder.ensure(ord, "pipeline order"))) return rc;
        if ((rc = L.mtotal.ensure(64, "pipeline total"))) return rc;
        if ((rc = L.remain.ensure(CG_PIPE_MAX * 4, "pipeline counters"))) return rc;
        if ((rc = L.merr.ensure(CG_PIPE_MAX * 4, "pipeline counters"))) return rc;
        if ((rc = L.mflag.ensure(CG_PIPE_MAX * 8, "pipeline flags"))) return rc;
        if ((rc = L.err.ensure(64, "pipeline spin guard"))) return rc;
        cg::PipeBufs pb{L.mdesc.as<DescRaw>(),  L.mabs.as<uint64_t>(),  L.mdst.as<uint64_t>(),
                        L.mmember.as<uint32_t>(), L.mtotal.as<uint64_t>(), L.morder.as<uint32_t>(),
                        L.remain.as<uint32_t>(), L.merr.as<uint32_t>(),  L.mflag.as<uint32_t *>(),
                        L.err.as<uint32_t>()};
        const uint32_t lane = (uint32_t)(&L - p->lanes.data());
        PipeClock *clk = p->clock.as<PipeClock>();
        if (clk && pipe_stagger()) hipLaunchKernelGGL(k_pipe_stagger, dim3(1), dim3(64), 0, L.st, clk, lane, p->nlanes);
        cg::launch_sha256_pipe(t, bound, expected, max_len, pb, L.st, g->timed ? g->t0 : nullptr,
                               g->timed ? g->t1 : nullptr);
        if (clk && pipe_stagger()) hipLaunchKernelGGL(k_pipe_end, dim3(1), dim3(64), 0, L.st, clk, lane);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(g->done, L.st));
        return CG_OK;
    };
    const int rc = launch();
    if (rc) {
        // whatever was queued may still read the members' buffers: drain before their
        // waits release the workspaces
        (void)hipStreamSynchronize(L.st);
        for (uint32_t i = 0; i < p->nb; ++i) (void)hipStreamSynchronize(p->bstream[i]);
        return group_fail(*g, rc);
    }
    L.last = g;
    ++p->groups;
    p->batches += g->members.size();
    if (g->timed) p->timing.push_back(g);
    return CG_OK;
}

// Fold the timing of groups that have completed into the counters (pipeline lock held).
static void read_timing(cg_pipeline *p) {
    while (!p->timing.empty()) {
        std::shared_ptr<PipeGroup> g = p->timing.front();
        if (hipEventQuery(g->done) != hipSuccess) break;
        float ms = 0;
        if (hipEventElapsedTime(&ms, g->t0, g->t1) == hipSuccess) {
            p->digest_ms += ms;
            p->digest_bytes += (double)g->bytes;
            p->last_digest_ms = ms;
            ++p->timed_groups;
        }
        p->timing.pop_front();
    }
}

int pipeline_wait(cg_batch *b, uint64_t *nar_first) {
    std::unique_ptr<cg_batch> hold(b);
    std::shared_ptr<PipeGroup> g = b->group;
    WsGuard guard{b->ws};
    int rc = CG_OK;
    if (!g->launched) {  // the batch is in the open group: launch it now
        cg_pipeline *p = g->owner;
        DeviceScope scope;
        if ((rc = scope.set(p->device))) return rc;
        std::lock_guard<std::mutex> lk(p->mu);
        if (!g->launched) rc = flush_locked(p);
    }
    if (g->rc) return fail_detail(g->rc, g->err, g->detail);
    if (rc) return rc;
    const PipeMember &m = g->members[b->member];
    // the member's completion word (ShaNotify): yield for the first ~0.2 ms, then poll
    // every 20 us; the group's end event catches a word that never arrives
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t f = 0;
    for (;;) {
        f = __atomic_load_n(m.flag_host, __ATOMIC_ACQUIRE);
        if (f) break;
        if (hipEventQuery(g->done) == hipSuccess) {
            f = __atomic_load_n(m.flag_host, __ATOMIC_ACQUIRE);
            break;
        }
        if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200))
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    if (f == 0) return fail(CG_E_IO, "digest pipeline: the merged digest ended without completing this batch");
    if (f != 1)
        return fail(CG_E_IO, "SHA-256 digest: a producer/consumer hand-off hit the kernel's spin guard; "
                             "the digests of this call are invalid");
    return finish_batch(b->ws, b->st, b->bl, nar_first);
}

}  // namespace cgrt

using namespace cgrt;

extern "C" {

int cg_pipeline_create(int device, uint32_t group_batches, uint32_t lanes, cg_pipeline **out) {
    clear_error();
    if (!out) return fail(CG_E_IO, "null pipeline handle pointer");
    *out = nullptr;
    if (group_batches > CG_PIPE_MAX) {
        char buf[96];
        snprintf(buf, sizeof buf, "pipeline group must be at most %u batches, got %u", CG_PIPE_MAX, group_batches);
        return fail(CG_E_INVALID_OPTIONS, buf);
    }
    if (lanes > 8) return fail(CG_E_INVALID_OPTIONS, "pipeline lanes must be at most 8");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(CG_E_NO_DEVICE, "no HIP device visible: the chunker engine has no CPU fallback");
    if (device < 0) {
        int cur = 0;
        HIP_TRY(hipGetDevice(&cur));
        device = cur;
    }
    if (device >= n) return fail(CG_E_NO_DEVICE, "pipeline device index out of range");
    DeviceScope scope;
    int rc = scope.set(device);
    if (rc) return rc;
    std::unique_ptr<cg_pipeline> p(new cg_pipeline());
    p->device = device;
    p->group_max = group_batches ? group_batches : 16;
    p->nlanes = lanes ? lanes : 3;
    p->lanes.resize(p->nlanes);
    *out = p.release();  // the streams come with the first batch (start_streams)
    return CG_OK;
}

// The pipeline's streams, made at its first batch (pipeline lock held): one boundary stream
// for SHA-256 (CHUNKER_AMD_PIPE_BSTREAMS=1..4, A/B: two boundary streams and four lanes raise
// config 2's steady rate ~7 % but leave the lanes' phases loose, so a 20-batch window reads
// 0.7-1.1x of it), three for a pipeline that starts with a BLAKE3 batch -- its
// digest runs whole on the boundary stream, so consecutive batches on three streams overlap
// one's scan with another's digest (config 3: 1498-1516 -> 1566-1572 GiB/s, steady window
// 1549-1558 -> 1698-1708, profiles/r06_v42_summary.txt) -- then the lanes.
static int start_streams(cg_pipeline *p, uint64_t batch_bytes, int algo) {
    if (p->nb) return CG_OK;
    (void)batch_bytes;
    uint32_t nb = algo == CG_BLAKE3 ? 3u : 1u;
    if (const char *e = getenv("CHUNKER_AMD_PIPE_BSTREAMS")) nb = std::min<uint32_t>(std::max(atoi(e), 1), PIPE_MAX_BSTREAMS);
    const int kind = pipe_stream_kind();
    const bool low = kind == 3 || (kind == 1 && nb + p->nlanes > 4);
    std::vector<hipStream_t> made;
    int rc = CG_OK;
    for (uint32_t i = 0; i < nb + p->nlanes && !rc; ++i) {
        hipStream_t st = nullptr;
        if (!(rc = make_stream(&st, i >= nb && low))) made.push_back(st);
    }
    if (rc) {  // nothing is kept: the next batch tries again
        for (hipStream_t st : made) (void)hipStreamDestroy(st);
        return rc;
    }
    if ((rc = p->clock.ensure(sizeof(PipeClock), "pipeline clock")) ||
        (rc = hipMemset(p->clock.p, 0, sizeof(PipeClock)) == hipSuccess ? CG_OK : fail(CG_E_IO, "hipMemset failed"))) {
        for (hipStream_t st : made) (void)hipStreamDestroy(st);
        return rc;
    }
    for (uint32_t i = 0; i < nb; ++i) p->bstream[i] = made[i];
    for (uint32_t i = 0; i < p->nlanes; ++i) p->lanes[i].st = made[nb + i];
    p->nb = nb;
    return CG_OK;
}

int cg_pipeline_submit(cg_pipeline *p, const uint8_t *d_data, const uint64_t *nar_offsets, size_t n_nars,
                       uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo, cg_desc *d_out,
                       size_t out_cap, void *inputs_ready, cg_batch **batch) {
    clear_error();
    if (!p || !batch) return fail(CG_E_IO, "null pipeline or batch handle pointer");
    *batch = nullptr;
    if (algo != CG_BLAKE3 && algo != CG_SHA256) return fail(CG_E_INVALID_OPTIONS, "unknown hash algorithm");
    Opts o;
    int rc = resolve(min_size, avg_size, max_size, &o, nullptr, 0);
    if (rc) return rc;
    if (n_nars && nar_offsets[0] != 0)
        return fail_bounds(nar_offsets[n_nars], nar_offsets[0], 0, "device batch offsets must start at 0");
    if ((rc = check_tables())) return rc;
    DeviceScope scope;
    if ((rc = scope.set(p->device))) return rc;
    Workspace *ws = nullptr;
    if ((rc = acquire(&ws))) return rc;
    std::lock_guard<std::mutex> lk(p->mu);
    if ((rc = start_streams(p, n_nars ? nar_offsets[n_nars] : 0, algo))) {
        release(ws);
        return rc;
    }
    hipStream_t bs = p->bstream[p->next_b];
    p->next_b = (p->next_b + 1) % p->nb;
    auto undo = [&](int code) {
        (void)hipStreamSynchronize(bs);
        release(ws);
        return code;
    };
    if (inputs_ready && hipStreamWaitEvent(bs, static_cast<hipEvent_t>(inputs_ready), 0) != hipSuccess)
        return undo(fail(CG_E_IO, "hipStreamWaitEvent(inputs_ready) failed"));
    BatchLaunch bl;
    if (algo == CG_BLAKE3) {  // the whole batch on its boundary stream
        if ((rc = launch_batch(ws, d_data, nar_offsets, n_nars, o, algo, d_out, out_cap, bs, nullptr, nullptr, true,
                               &bl)))
            return undo(rc);
        *batch = new cg_batch{ws, bs, bl, nullptr, 0, p->device};
        return CG_OK;
    }
    if ((rc = ws->done_flag.ensure(64, /*mapped=*/true))) return undo(rc);
    __atomic_store_n(ws->done_flag.as<uint32_t>(), 0u, __ATOMIC_RELEASE);
    // the boundary stages run beside the merged digests, which hold two workgroups on every
    // CU: the lean scan fits there (scan.hip, t_scan_lean)
    cg::t_scan_lean = true;
    rc = launch_batch(ws, d_data, nar_offsets, n_nars, o, algo, d_out, out_cap, bs, nullptr, nullptr,
                      /*digest=*/false, &bl);
    cg::t_scan_lean = false;
    if (rc) return undo(rc);
    // the digest's sizes, as launch_batch's own digest would take them
    uint64_t total_cap = 0;
    for (size_t i = 0; i < n_nars; ++i) total_cap += capacity_of(nar_offsets[i + 1] - nar_offsets[i], o.min);
    const uint64_t total_len = n_nars ? nar_offsets[n_nars] : 0;
    PipeMember m;
    m.ws = ws;
    m.d_data = d_data;
    m.d_out = d_out;
    m.d_abs = ws->chunk_abs.as<uint64_t>();
    m.d_total = ws->nar_first.as<uint64_t>() + n_nars;
    m.bound = std::min<uint64_t>(total_cap, out_cap);
    m.expected = std::min<uint64_t>(m.bound, total_len / (o.min + o.avg) + n_nars);
    m.max_len = o.max;
    m.bytes = total_len;
    m.flag_host = ws->done_flag.as<uint32_t>();
    m.flag_dev = static_cast<uint32_t *>(ws->done_flag.dev);
    if (!p->open) {
        auto g = std::make_shared<PipeGroup>();
        g->timed = g_profiling.load() != 0;
        for (uint32_t i = 0; i < p->nb; ++i)
            if (hipEventCreateWithFlags(&g->bdone[i], hipEventDisableTiming) != hipSuccess)
                return undo(fail(CG_E_IO, "hipEventCreate failed"));
        if (hipEventCreateWithFlags(&g->done, hipEventDisableTiming) != hipSuccess ||
            (g->timed && (hipEventCreate(&g->t0) != hipSuccess || hipEventCreate(&g->t1) != hipSuccess)))
            return undo(fail(CG_E_IO, "hipEventCreate failed"));
        g->owner = p;
        p->open = g;
    }
    std::shared_ptr<PipeGroup> g = p->open;
    g->members.push_back(m);
    g->bytes += total_len;
    *batch = new cg_batch{ws, bs, bl, g, (uint32_t)(g->members.size() - 1), p->device};
    if (g->members.size() >= p->group_max) flush_locked(p);  // a failure reaches every member's wait
    return CG_OK;
}

int cg_pipeline_flush(cg_pipeline *p) {
    clear_error();
    if (!p) return fail(CG_E_IO, "null pipeline handle");
    DeviceScope scope;
    int rc = scope.set(p->device);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(p->mu);
    return flush_locked(p);
}

int cg_batch_event(cg_batch *batch, void **event) {
    clear_error();
    if (!batch || !event) return fail(CG_E_IO, "null batch handle or event pointer");
    *event = nullptr;
    if (!batch->group) {
        *event = batch->bl.done;
        return CG_OK;
    }
    std::shared_ptr<PipeGroup> g = batch->group;
    if (!g->launched) {
        cg_pipeline *p = g->owner;
        DeviceScope scope;
        int rc = scope.set(p->device);
        if (rc) return rc;
        std::lock_guard<std::mutex> lk(p->mu);
        if (!g->launched) flush_locked(p);
    }
    if (g->rc) return fail_detail(g->rc, g->err, g->detail);
    *event = g->done;
    return CG_OK;
}

int cg_pipeline_stats(cg_pipeline *p, double out[6]) {
    clear_error();
    if (!p || !out) return fail(CG_E_IO, "null pipeline handle or output");
    std::lock_guard<std::mutex> lk(p->mu);
    read_timing(p);
    out[0] = (double)p->groups;
    out[1] = (double)p->batches;
    out[2] = (double)p->timed_groups;
    out[3] = p->digest_ms;
    out[4] = p->digest_bytes;
    out[5] = p->last_digest_ms;
    return CG_OK;
}

void cg_pipeline_destroy(cg_pipeline *p) {
    if (!p) return;
    {
        DeviceScope scope;
        (void)scope.set(p->device);
        std::lock_guard<std::mutex> lk(p->mu);
        (void)flush_locked(p);  // a batch still in the open group gets its digest
        for (auto &L : p->lanes)
            if (L.st) (void)hipStreamSynchronize(L.st);
        for (hipStream_t b : p->bstream)
            if (b) (void)hipStreamSynchronize(b);
        p->timing.clear();
        for (auto &L : p->lanes) {
            L.last.reset();
            for (DevBuf *d : {&L.mdesc, &L.mabs, &L.mdst, &L.mmember, &L.mtotal, &L.morder, &L.remain, &L.merr,
                              &L.mflag, &L.err})
                d->release();
            if (L.st) (void)hipStreamDestroy(L.st);
        }
        for (hipStream_t b : p->bstream)
            if (b) (void)hipStreamDestroy(b);
        p->clock.release();
    }
    delete p;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Multi-device batches (cg_multi_*, round 6): north_star's split -- a batch of NARs
// shards one-file-per-GPU across the GPUs of one node, the chunk descriptors gathered to
// one GPU -- behind the C ABI, so a single host process (the reference's node-bin,
// crates/node-bin/src/main.rs:1-25, calling Node::put per PUT, crates/node/src/lib.rs:114-132)
// can drive every GPU.  Each device runs its own digest pipeline on its shard (no data-path
// exchange: FastCDC state never crosses files); the wait gathers the shards' descriptors
// into the caller's array on devices[0] with peer copies over xGMI (hipMemcpyPeerAsync on
// a stream of devices[0]) and concatenates the NAR index on the host.
// ---------------------------------------------------------------------------
namespace cgrt {

struct MultiShard {
    cg_batch *b = nullptr;
    DevBuf *scratch = nullptr;  // descriptors of a shard on devices[k], k > 0 (pooled)
    size_t n_nars = 0;
    bool direct = false;        // shard 0: written straight into the caller's array
};

}  // namespace cgrt

struct cg_multi {
    std::vector<int> devices;
    std::vector<cg_pipeline *> pipes;
    hipStream_t gather = nullptr;  // on devices[0]
    std::mutex mu;
    std::vector<std::vector<std::unique_ptr<cgrt::DevBuf>>> pool;  // free scratch per shard index
};

struct cg_multi_batch {
    cg_multi *m;
    std::vector<cgrt::MultiShard> shards;
    cg_desc *d_out;
    size_t out_cap;
};

namespace cgrt {

static void multi_release(cg_multi_batch *mb) {
    cg_multi *m = mb->m;
    std::lock_guard<std::mutex> lk(m->mu);
    for (size_t k = 0; k < mb->shards.size(); ++k)
        if (mb->shards[k].scratch) m->pool[k].emplace_back(mb->shards[k].scratch);
}

}  // namespace cgrt

extern "C" {

int cg_multi_create(const int *devices, size_t n_dev, uint32_t group_batches, uint32_t lanes, cg_multi **out) {
    clear_error();
    if (!out || !devices || n_dev == 0) return fail(CG_E_IO, "cg_multi_create: null handle pointer or no devices");
    *out = nullptr;
    if (n_dev > 64) return fail(CG_E_INVALID_OPTIONS, "cg_multi_create: at most 64 devices");
    std::unique_ptr<cg_multi> m(new cg_multi());
    m->devices.assign(devices, devices + n_dev);
    m->pool.resize(n_dev);
    auto fail_all = [&](int rc) {
        for (cg_pipeline *p : m->pipes) cg_pipeline_destroy(p);
        m->pipes.clear();
        return rc;
    };
    for (size_t k = 0; k < n_dev; ++k) {
        cg_pipeline *p = nullptr;
        int rc = cg_pipeline_create(devices[k], group_batches, lanes, &p);
        if (rc) return fail_all(rc);
        m->pipes.push_back(p);
    }
    DeviceScope scope;
    int rc = scope.set(devices[0]);
    if (rc) return fail_all(rc);
    // peer access to every other device's HBM (already enabled / same device: fine; without
    // it hipMemcpyPeerAsync still copies, staged by the runtime)
    for (size_t k = 1; k < n_dev; ++k)
        if (devices[k] != devices[0]) {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, devices[0], devices[k]) == hipSuccess && can) {
                const hipError_t e = hipDeviceEnablePeerAccess(devices[k], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return fail_all(hip_fail(e, "peer access"));
                (void)hipGetLastError();
            }
        }
    if (hipStreamCreateWithFlags(&m->gather, hipStreamNonBlocking) != hipSuccess)
        return fail_all(fail(CG_E_IO, "cg_multi_create: gather stream"));
    *out = m.release();
    return CG_OK;
}

int cg_multi_submit(cg_multi *m, const uint8_t *const *d_data, const uint64_t *const *nar_offsets, const size_t *n_nars,
                    uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo, cg_desc *d_out, size_t out_cap,
                    void *const *inputs_ready, cg_multi_batch **batch) {
    clear_error();
    if (!m || !batch || !d_data || !nar_offsets || !n_nars) return fail(CG_E_IO, "cg_multi_submit: null argument");
    *batch = nullptr;
    Opts o;
    int rc = resolve(min_size, avg_size, max_size, &o, nullptr, 0);
    if (rc) return rc;
    const size_t nd = m->devices.size();
    std::unique_ptr<cg_multi_batch> mb(new cg_multi_batch{m, std::vector<MultiShard>(nd), d_out, out_cap});
    auto undo = [&](int code) {
        // shards already submitted: wait for them (their workspaces go back), keep the error
        std::string msg = cg_last_error_message();
        uint64_t det[3];
        cg_last_error_detail(det);
        for (auto &s : mb->shards)
            if (s.b) (void)cg_batch_wait(s.b, nullptr);
        multi_release(mb.get());
        return fail_detail(code, msg, det);
    };
    for (size_t k = 0; k < nd; ++k) {
        MultiShard &s = mb->shards[k];
        s.n_nars = n_nars[k];
        uint64_t cap = 0;
        for (size_t i = 0; i < n_nars[k]; ++i) cap += capacity_of(nar_offsets[k][i + 1] - nar_offsets[k][i], o.min);
        cg_desc *dst = nullptr;
        size_t dst_cap = (size_t)cap;
        if (k == 0) {
            s.direct = true;
            dst = d_out;
            dst_cap = std::min<size_t>(out_cap, (size_t)cap);
        } else {
            {
                std::lock_guard<std::mutex> lk(m->mu);
                if (!m->pool[k].empty()) {
                    s.scratch = m->pool[k].back().release();
                    m->pool[k].pop_back();
                }
            }
            if (!s.scratch) s.scratch = new DevBuf();
            DeviceScope scope;
            if ((rc = scope.set(m->devices[k])) ||
                (rc = s.scratch->ensure((cap + 1) * sizeof(cg_desc), "multi-device shard descriptors")))
                return undo(rc);
            dst = s.scratch->as<cg_desc>();
        }
        if ((rc = cg_pipeline_submit(m->pipes[k], d_data[k], nar_offsets[k], n_nars[k], min_size, avg_size, max_size,
                                     algo, dst, dst_cap, inputs_ready ? inputs_ready[k] : nullptr, &s.b)))
            return undo(rc);
    }
    *batch = mb.release();
    return CG_OK;
}

int cg_multi_wait(cg_multi_batch *batch, uint64_t *nar_first) {
    clear_error();
    if (!batch) return fail(CG_E_IO, "null multi-device batch handle");
    std::unique_ptr<cg_multi_batch> mb(batch);
    cg_multi *m = mb->m;
    int rc = CG_OK;
    std::string err;  // the first failure (each later cg_batch_wait clears the thread's error)
    uint64_t det[3] = {0, 0, 0};
    auto keep = [&](int r) {
        if (r && !rc) {
            rc = r;
            err = cg_last_error_message();
            cg_last_error_detail(det);
        }
    };
    uint64_t base_nar = 0, base_desc = 0;
    std::vector<uint64_t> first;
    // every shard is waited for (and its workspace returned) whatever fails
    for (size_t k = 0; k < mb->shards.size(); ++k) {
        MultiShard &s = mb->shards[k];
        first.assign(s.n_nars + 1, 0);
        keep(cg_batch_wait(s.b, first.data()));
        s.b = nullptr;
        if (rc) continue;
        const uint64_t n = first[s.n_nars];
        if (base_desc + n > mb->out_cap) {
            keep(fail(CG_E_CAPACITY, "descriptor output array too small"));
            continue;
        }
        if (!s.direct && n) {
            DeviceScope scope;
            keep(scope.set(m->devices[0]));
            if (rc) continue;
            const hipError_t e = hipMemcpyPeerAsync(mb->d_out + base_desc, m->devices[0], s.scratch->p, m->devices[k],
                                                    n * sizeof(cg_desc), m->gather);
            if (e != hipSuccess) keep(hip_fail(e, "hipMemcpyPeerAsync (descriptor gather)"));
        }
        if (nar_first)
            for (size_t i = 0; i < s.n_nars; ++i) nar_first[base_nar + i] = base_desc + first[i];
        base_nar += s.n_nars;
        base_desc += n;
    }
    if (nar_first && !rc) nar_first[base_nar] = base_desc;
    {
        DeviceScope scope;
        if (scope.set(m->devices[0]) == CG_OK) {
            const hipError_t e = hipStreamSynchronize(m->gather);
            if (e != hipSuccess) keep(hip_fail(e, "descriptor gather"));
        }
    }
    multi_release(mb.get());
    return rc ? fail_detail(rc, err, det) : CG_OK;
}

int cg_multi_flush(cg_multi *m) {
    clear_error();
    if (!m) return fail(CG_E_IO, "null multi-device handle");
    for (cg_pipeline *p : m->pipes) {
        const int rc = cg_pipeline_flush(p);
        if (rc) return rc;
    }
    return CG_OK;
}

void cg_multi_destroy(cg_multi *m) {
    if (!m) return;
    for (cg_pipeline *p : m->pipes) cg_pipeline_destroy(p);
    {
        DeviceScope scope;
        (void)scope.set(m->devices[0]);
        if (m->gather) {
            (void)hipStreamSynchronize(m->gather);
            (void)hipStreamDestroy(m->gather);
        }
        for (size_t k = 0; k < m->pool.size(); ++k) {
            DeviceScope s2;
            (void)s2.set(m->devices[k]);
            for (auto &b : m->pool[k]) b->release();
        }
    }
    delete m;
}

}  // extern "C"
