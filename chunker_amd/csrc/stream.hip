// stream.hip -- pipelined stream handle (cg_stream_*): ChunkStream (src/chunking.rs:675-740)
// over drain_finalized_chunks (:541-673) with many read slices in flight.
//
// A SHA-256 / BLAKE3 digest costs one serial chain per chunk (~60 ms for a 4 MiB
// chunk on the GPU), so a stream that waits for each slice's digests
// (cg_push_*) runs at slice / 60 ms.  This handle instead keeps the stream's bytes in
// an HBM arena of slots and separates two pipelines:
//   * boundaries, synchronous per pushed slice, on the handle's workspace stream: the
//     slice is copied H2D behind the retained tail (in the slot that holds it), the
//     scan / walk find every cut of [tail, slice), the host applies the reference's
//     retain rule (:579-584), and the retained tail moves D2D to the next slot;
//   * digests, asynchronous: final chunks accumulate in an open group; a group of
//     >= group_bytes is launched on one of a few digest streams and completes later.
// Chunks come out of cg_stream_take strictly in stream order, with the exact
// (offset, length, hash) the reference's ChunkStream / PushChunker yields.  Memory is
// bounded by the arena (slots are reused only after every group reading them has
// completed); when no slot is free a push waits for the oldest group.
//
// Device resources are taken as the stream needs them: the arena starts at two slots at
// the first push and grows to the full in-flight budget only when the pipeline runs out
// of free slots; digest lanes (stream + event + scratch) are created one at a time when
// every existing lane is busy.  A short stream therefore holds two slots and one lane,
// not the whole budget.  (The two-slot arena is kept until the handle is freed: freeing
// device memory waits for the whole device, which would drain the digest pipeline.)  The first failure of push / finish / take poisons the
// handle: every later call returns the same status (a failed push may have left part of
// its slice inside the engine, so nothing after it could be trusted).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <deque>

#include "runtime.h"

namespace cgrt {

// One digest launch in flight: device scratch, pinned staging and its own stream.
// Scratch grows without freeing: hipFree / hipHostFree wait for the whole device, i.e.
// for every digest in flight (a 50-75 ms stall per growth), so a lane keeps the buffers
// it outgrew (at most as much again, growth is by doubling) until it is destroyed.
struct Lane {
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr;
    DevBuf desc, abs, total, order, err, b3_gcount, b3_gbase, b3_gcv, b3_gmap, scan_tmp;
    PinBuf stage;  // [descs | abs | total | err]
    std::vector<void *> old_dev, old_pin;
    bool busy = false;
    int init() {
        HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        return CG_OK;
    }
    int ensure(DevBuf &b, size_t bytes, const char *name) {
        if (bytes <= b.cap) return CG_OK;
        const size_t want = std::max(bytes + 256, 2 * b.cap);
        void *p = nullptr;
        const hipError_t e = test_alloc_fault() ? hipErrorOutOfMemory : hipMalloc(&p, want);
        if (e != hipSuccess) return hip_fail(e, name, want);
        if (b.p) old_dev.push_back(b.p);
        b.p = p;
        b.cap = want;
        return CG_OK;
    }
    int ensure_stage(size_t bytes) {
        if (bytes <= stage.cap) return CG_OK;
        const size_t want = std::max(bytes + 256, 2 * stage.cap);
        void *p = nullptr;
        const hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e != hipSuccess) return hip_fail(e, "hipHostMalloc", want);
        if (stage.p) old_pin.push_back(stage.p);
        stage.p = p;
        stage.cap = want;
        return CG_OK;
    }
    void destroy() {
        if (st) (void)hipStreamSynchronize(st);
        for (DevBuf *b : {&desc, &abs, &total, &order, &err, &b3_gcount, &b3_gbase, &b3_gcv, &b3_gmap, &scan_tmp})
            b->release();
        for (void *p : old_dev) (void)hipFree(p);
        if (stage.p) (void)hipHostFree(stage.p);
        for (void *p : old_pin) (void)hipHostFree(p);
        if (done) (void)hipEventDestroy(done);
        if (st) (void)hipStreamDestroy(st);
    }
};

// The final chunks of a run of consecutive slots [slot_lo, slot_hi], one digest launch.
struct Group {
    std::vector<cg_desc> desc;  // offsets are stream offsets (ChunkMetadata::offset)
    std::vector<uint64_t> abs;  // arena offsets of the same chunks
    const uint8_t *base = nullptr;  // the arena those offsets are into (it may have been retired since)
    uint64_t slot_lo = 0, slot_hi = 0, bytes = 0;
    int lane = -1;
};

// The arena: nslots slots of slot_bytes, allocated exactly (no DevBuf slack).
struct Arena {
    uint8_t *p = nullptr;
    uint64_t nslots = 0;
    int alloc(uint64_t n, uint64_t slot_bytes) {
        const uint64_t bytes = n * slot_bytes;
        hipError_t e = test_alloc_fault() ? hipErrorOutOfMemory : hipMalloc(reinterpret_cast<void **>(&p), bytes);
        if (e != hipSuccess) {
            p = nullptr;
            return hip_fail(e, "stream arena", bytes);
        }
        nslots = n;
        return CG_OK;
    }
    void release() {
        if (p) (void)hipFree(p);  // hipFree waits for the device: no copy or kernel still reads it
        p = nullptr;
        nslots = 0;
    }
};

// Stream shape knobs (test hooks cg_test_stream_group_cap / cg_test_stream_max_lanes):
// 0 = the built-in rule of cg_stream_new.
uint64_t g_stream_group_cap = 0;
uint32_t g_stream_max_lanes = 0;
uint32_t g_stream_eager = 0;  // cg_test_stream_eager: launch a group whenever a lane is idle

}  // namespace cgrt

using namespace cgrt;

struct cg_stream {
    Opts o;
    int algo = CG_SHA256;
    int device = -1;
    Workspace *ws = nullptr;  // boundary pipeline, held for the handle's lifetime
    Arena arena;
    std::vector<Arena> retired;  // the first, two-slot arena once grown (freed with the handle)
    uint64_t slot_bytes = 0, max_slots = 0, group_bytes = 0, group_hard = 0;
    size_t max_lanes = 0;
    int poisoned = CG_OK;  // first failure of push / finish / take, returned by every later call
    std::string poison_msg;
    uint64_t poison_detail[3] = {0, 0, 0};
    uint64_t cur = 0;       // sequence number of the slot holding the retained tail
    uint64_t tail = 0;      // retained bytes at the start of slot `cur`
    uint64_t position = 0;  // stream offset of slot `cur`'s first byte
    uint64_t pushed = 0;
    bool finished = false;
    Group open;
    std::deque<Group> inflight;
    std::deque<cg_desc> ready;
    std::vector<Lane> lanes;  // reserved to max_lanes up front: references stay valid as it grows
    std::vector<cg_desc> scratch;  // boundary descriptors of the current slot
    hipEvent_t ev_bytes = nullptr;  // boundary stream position a digest launch must wait for
    ~cg_stream() {
        if (device < 0) return;
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(device);
        for (Lane &l : lanes) l.destroy();
        if (ws) {
            (void)hipStreamSynchronize(ws->stream);
            release(ws);
        }
        if (ev_bytes) (void)hipEventDestroy(ev_bytes);
        arena.release();
        for (Arena &a : retired) a.release();
        (void)hipSetDevice(prev);
    }
};

namespace cgrt {

uint8_t *slot_ptr(cg_stream *h, uint64_t seq) { return h->arena.p + (seq % h->arena.nslots) * h->slot_bytes; }
uint64_t slot_off(const cg_stream *h, uint64_t seq) { return (seq % h->arena.nslots) * h->slot_bytes; }

// Wait for the oldest launched group, check it, and move its chunks (now with digests)
// to the ready queue.
int complete_oldest(cg_stream *h) {
    Group &g = h->inflight.front();
    Lane &l = h->lanes[g.lane];
    HIP_TRY(hipEventSynchronize(l.done));
    const size_t n = g.desc.size();
    const uint8_t *st = l.stage.as<uint8_t>();
    const uint32_t err = *reinterpret_cast<const uint32_t *>(st + n * sizeof(cg_desc) + n * 8 + 8);
    l.busy = false;
    if (err)
        return fail(CG_E_IO, "stream digest: a producer/consumer hand-off hit the SHA-256 kernel's spin guard");
    const cg_desc *res = reinterpret_cast<const cg_desc *>(st);
    for (size_t k = 0; k < n; ++k) {
        cg_desc d = g.desc[k];
        memcpy(d.hash, res[k].hash, 32);
        h->ready.push_back(d);
    }
    h->inflight.pop_front();
    return CG_OK;
}

// Launch the open group's digests on a free lane (waiting for the oldest group if none).
int launch_open(cg_stream *h) {
    if (h->open.desc.empty()) return CG_OK;
    int rc;
    int li = -1;
    for (;;) {
        for (size_t i = 0; i < h->lanes.size(); ++i)
            if (!h->lanes[i].busy) li = (int)i;
        if (li >= 0) break;
        if (h->lanes.size() < h->max_lanes) {  // every lane busy: open one more
            h->lanes.emplace_back();
            if ((rc = h->lanes.back().init())) {
                h->lanes.back().destroy();
                h->lanes.pop_back();
                if (h->lanes.empty()) return rc;
                h->max_lanes = h->lanes.size();  // the runtime will not give more: wait instead
                clear_error();
                continue;
            }
            li = (int)h->lanes.size() - 1;
            break;
        }
        if ((rc = complete_oldest(h))) return rc;
    }
    Lane &l = h->lanes[li];
    Group g = std::move(h->open);
    h->open = Group();
    const size_t n = g.desc.size();
    const size_t nd = n * sizeof(cg_desc);
    if ((rc = l.ensure_stage(nd + n * 8 + 16))) return rc;
    uint8_t *stg = l.stage.as<uint8_t>();
    memcpy(stg, g.desc.data(), nd);  // the kernels read lengths here and chunk bytes at arena + abs
    memcpy(stg + nd, g.abs.data(), n * 8);
    *reinterpret_cast<uint64_t *>(stg + nd + n * 8) = n;
    *reinterpret_cast<uint32_t *>(stg + nd + n * 8 + 8) = 0;
    if ((rc = l.ensure(l.desc, nd + 64, "stream descriptors"))) return rc;
    if ((rc = l.ensure(l.abs, n * 8 + 64, "stream offsets"))) return rc;
    if ((rc = l.ensure(l.total, 64, "stream total"))) return rc;
    if ((rc = l.ensure(l.err, 64, "stream err"))) return rc;
    // the chunk bytes were written (H2D, tail moves) on the boundary stream
    HIP_TRY(hipEventRecord(h->ev_bytes, h->ws->stream));
    HIP_TRY(hipStreamWaitEvent(l.st, h->ev_bytes, 0));
    HIP_TRY(hipMemcpyAsync(l.desc.p, stg, nd, hipMemcpyHostToDevice, l.st));
    HIP_TRY(hipMemcpyAsync(l.abs.p, stg + nd, n * 8, hipMemcpyHostToDevice, l.st));
    HIP_TRY(hipMemcpyAsync(l.total.p, stg + nd + n * 8, 8, hipMemcpyHostToDevice, l.st));
    HIP_TRY(hipMemsetAsync(l.err.p, 0, 4, l.st));
    uint8_t *hb = l.desc.as<uint8_t>() + offsetof(cg_desc, hash);
    const uint8_t *base = g.base;
    const uint64_t *d_total = l.total.as<uint64_t>();
    if (h->algo == CG_SHA256) {
        if ((rc = l.ensure(l.order, cg::sha256_order_tmp_elems(n) * 4, "order"))) return rc;
        // (no latency tiers: a stream's rate is its groups' chains one after another, and a
        // one-lane chain sharing the CUs with the next slices' scans ran slower than the quad
        // it replaced -- 1 / 4 GiB at 4 queues 9.86 / 10.20 -> 8.92 / 8.74 GiB/s with them,
        // profiles/r05_v36_stream_tiers_ab.txt)
        cg::launch_sha256(base, l.abs.as<uint64_t>(), l.desc.p, d_total, n, n, h->o.max, l.order.as<uint32_t>(), hb,
                          sizeof(cg_desc), l.err.as<uint32_t>(), l.st, /*latency_tiers=*/false);
    } else {
        const uint64_t gb = cg::blake3_group_bound(g.bytes, n);
        if ((rc = l.ensure(l.b3_gcount, (n + 1) * 4, "b3_gcount"))) return rc;
        if ((rc = l.ensure(l.b3_gbase, (n + 1) * 8, "b3_gbase"))) return rc;
        if ((rc = l.ensure(l.b3_gcv, cg::blake3_cv_bytes(g.bytes, n, true), "b3_gcv"))) return rc;
        if ((rc = l.ensure(l.b3_gmap, (gb + 1) * 4, "b3_gmap"))) return rc;
        if ((rc = l.ensure(l.scan_tmp, cg::exclusive_scan_tmp_elems(n) * 8 + 64, "scan_tmp"))) return rc;
        cg::launch_blake3(base, l.abs.as<uint64_t>(), l.desc.p, d_total, n, g.bytes, hb, sizeof(cg_desc),
                          l.b3_gmap.as<uint32_t>(), l.b3_gbase.as<uint64_t>(), l.b3_gcount.as<uint32_t>(),
                          l.scan_tmp.as<uint64_t>(), l.b3_gcv.as<uint32_t>(), true, l.st);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(stg, l.desc.p, nd, hipMemcpyDeviceToHost, l.st));
    HIP_TRY(hipMemcpyAsync(stg + nd + n * 8 + 8, l.err.p, 4, hipMemcpyDeviceToHost, l.st));
    HIP_TRY(hipEventRecord(l.done, l.st));
    l.busy = true;
    g.lane = li;
    h->inflight.push_back(std::move(g));
    return CG_OK;
}

// Grow the arena to the full budget instead of waiting for a slot.  A group never spans
// two arenas, so the open one is launched on the current arena first; the old arena stays
// allocated (launched groups and the pending tail move still read it) until the handle
// is freed.  When the device has no memory for the larger arena the budget shrinks to
// the current size.
int grow_arena(cg_stream *h) {
    int rc;
    if ((rc = launch_open(h))) return rc;
    Arena nb;
    if (nb.alloc(h->max_slots, h->slot_bytes)) {
        clear_error();
        h->max_slots = h->arena.nslots;
        return CG_OK;
    }
    h->retired.push_back(h->arena);
    h->arena = nb;
    return CG_OK;
}

// Make slot `seq` writable: every group reading its previous tenant (seq - nslots) in the
// current arena done (groups launched on a retired arena do not count).
int free_slot(cg_stream *h, uint64_t seq) {
    int rc;
    for (;;) {
        uint64_t oldest = !h->open.desc.empty() ? h->open.slot_lo : h->cur;
        for (const Group &g : h->inflight)
            if (g.base == h->arena.p) {
                oldest = g.slot_lo;
                break;
            }
        if (seq < oldest + h->arena.nslots) return CG_OK;
        if (h->arena.nslots < h->max_slots) {
            if ((rc = grow_arena(h))) return rc;
        } else if (h->inflight.empty()) {
            if ((rc = launch_open(h))) return rc;
        } else if ((rc = complete_oldest(h))) {
            return rc;
        }
    }
}

// drain_finalized_chunks over slot `cur` = [tail | `len` new bytes already copied in].
int stream_drain(cg_stream *h, uint64_t len, bool eof) {
    int rc;
    const uint64_t buf = h->tail + len;
    if (buf == 0 || (buf < h->o.min && !eof)) {
        h->tail = buf;
        return CG_OK;
    }
    Workspace *ws = h->ws;
    const uint64_t cap = capacity_of(buf, h->o.min);
    if ((rc = ws->out.ensure((cap + 1) * sizeof(cg_desc), "descriptors"))) return rc;
    uint64_t offs[2] = {0, buf}, first[2] = {0, 0};
    if ((rc = run_batch(ws, slot_ptr(h, h->cur), offs, 1, h->o, h->algo, ws->out.as<cg_desc>(), cap, first,
                        ws->stream, nullptr, nullptr, /*digest=*/false)))
        return rc;
    const uint64_t total = first[1];
    h->scratch.resize(total);
    if (total) {
        HIP_TRY(hipMemcpyAsync(h->scratch.data(), ws->out.p, total * sizeof(cg_desc), hipMemcpyDeviceToHost,
                               ws->stream));
        HIP_TRY(hipStreamSynchronize(ws->stream));
    }
    uint64_t consumed = 0;
    const uint64_t base = slot_off(h, h->cur);
    for (uint64_t k = 0; k < total; ++k) {
        const cg_desc &d = h->scratch[k];
        if (d.length == 0) return fail(CG_E_ZERO_LENGTH_CHUNK, "FastCDC returned a chunk with length 0");
        if (d.offset + d.length == buf && !eof && d.length < h->o.max) break;  // retained tail (:579-584)
        if (h->open.desc.empty()) {
            h->open.slot_lo = h->cur;
            h->open.base = h->arena.p;
        }
        h->open.slot_hi = h->cur;
        cg_desc c{};
        c.offset = h->position + d.offset;
        c.length = d.length;
        h->open.desc.push_back(c);
        h->open.abs.push_back(base + d.offset);
        h->open.bytes += d.length;
        consumed += d.length;
    }
    if (eof && consumed < buf) return fail(CG_E_IO, "stream: chunks do not cover the buffer at finish");
    const uint64_t rest = buf - consumed;
    if (consumed) {  // the chunks emitted from this slot stay put; the next slice goes to the next slot
        const uint8_t *src = slot_ptr(h, h->cur) + consumed;  // (free_slot may move on to a larger arena)
        if ((rc = free_slot(h, h->cur + 1))) return rc;
        if (rest)  // the retained tail moves to the front of that slot
            HIP_TRY(hipMemcpyAsync(slot_ptr(h, h->cur + 1), src, rest, hipMemcpyDeviceToDevice, ws->stream));
        h->cur += 1;
    }
    h->position += consumed;
    h->tail = rest;
    if (h->open.bytes >= h->group_bytes) {
        // accumulate mode (cg_test_stream_eager(2)): while every lane is busy the group keeps
        // growing -- a SHA-256 group costs one chain (its longest chunk) whatever its size, up
        // to what one launch can spread over the chip -- instead of the push waiting for a lane
        if (g_stream_eager != 2 || h->open.bytes >= h->group_hard) return launch_open(h);
        bool idle = h->lanes.size() < h->max_lanes;
        for (const Lane &l : h->lanes) idle = idle || !l.busy;
        if (!idle && !h->inflight.empty() && hipEventQuery(h->lanes[h->inflight.front().lane].done) == hipSuccess) {
            if ((rc = complete_oldest(h))) return rc;
            idle = true;
        }
        if (idle) return launch_open(h);
        return CG_OK;
    }
    if (g_stream_eager == 1 && !h->open.desc.empty()) {  // launch now if a lane is idle
        bool idle = h->lanes.size() < h->max_lanes;
        for (const Lane &l : h->lanes) idle = idle || !l.busy;
        if (!idle && !h->inflight.empty() && hipEventQuery(h->lanes[h->inflight.front().lane].done) == hipSuccess) {
            if ((rc = complete_oldest(h))) return rc;
            idle = true;
        }
        if (idle) return launch_open(h);
    }
    return CG_OK;
}

}  // namespace cgrt

namespace {
// Hardware queues HIP gives this process: GPU_MAX_HW_QUEUES as the environment held it
// when this library was loaded (HIP's default 4 when unset).  HIP reads the variable once,
// when it initialises, and the library makes no HIP call before it is loaded, so this is
// the value HIP applies -- unless the caller initialised HIP earlier under another value
// (the library never changes the variable on the caller's behalf).
const int g_hw_queues_at_load = [] {
    const char *q = std::getenv("GPU_MAX_HW_QUEUES");
    const int v = q ? std::atoi(q) : 0;
    return v > 0 ? v : 4;
}();
}  // namespace

extern "C" {

// Test/tuning query (not in the header): the hardware-queue count above, which the
// Python depth rule (chunking.default_depth) uses instead of the environment's current value.
int cg_hw_queues(void) { return g_hw_queues_at_load; }

cg_stream *cg_stream_new(uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo, uint64_t slice_bytes,
                         uint64_t inflight_bytes, int *status) {
    clear_error();
    Opts o;
    int rc = resolve(min_size, avg_size, max_size, &o, nullptr, 0);
    if (!rc && algo != CG_BLAKE3 && algo != CG_SHA256) rc = fail(CG_E_INVALID_OPTIONS, "unknown hash algorithm");
    if (!rc) rc = check_tables();
    int dev = 0;
    if (!rc) rc = current_device(&dev);
    if (rc) {
        if (status) *status = rc;
        return nullptr;
    }
    cg_stream *h = new cg_stream();
    h->o = o;
    h->algo = algo;
    h->device = dev;
    // slot = the largest retained tail (< max) + one slice.  Digest lanes: one per
    // hardware queue left beside the workspace stream's and the null stream's
    // (GPU_MAX_HW_QUEUES, HIP's default 4; streams sharing a queue serialise, and a lane
    // on the workspace stream's queue would hold every boundary pass behind a 70 ms
    // chain), 2..8; groups of ~1/(lanes + 1) of the full arena, so every lane can hold
    // one while the next fills.  The arena and the lanes themselves are allocated as the
    // stream needs them (see the file header).
    const uint64_t slice = std::max<uint64_t>(slice_bytes ? slice_bytes : 8ull << 20, 4096);
    h->slot_bytes = (o.max + slice + 256 + 255) & ~255ull;
    const uint64_t budget = inflight_bytes ? inflight_bytes : 2048ull << 20;
    h->max_slots = std::max<uint64_t>(budget / h->slot_bytes, 4);
    // At HIP's default 4 queues ONE lane: a second lane's group chain ran beside the push's
    // boundary passes and slowed them more than it overlapped (1 / 4 GiB streams 9.7 / 10.1
    // GiB/s with one lane against 5.9 / 7.6 with two, profiles/r05_v5_stream_shape_q4.json;
    // at 16 queues 8 lanes still win on long streams: 4 GiB 14.0 against 10.2,
    // r05_v6_stream_shape_q16.json).
    h->max_lanes = g_hw_queues_at_load <= 4 ? 1 : (size_t)std::min(g_hw_queues_at_load - 2, 8);
    if (g_stream_max_lanes) h->max_lanes = g_stream_max_lanes;
    h->lanes.reserve(h->max_lanes);
    // A group's SHA-256 launch takes one CU per 8 chunks (quad workgroups, padded to a CU
    // each while the grid fits the chip), so the groups of all lanes together stay within
    // the 256 CUs: at most 2048 / lanes chunks of the expected min + avg bytes.  Larger
    // groups queue workgroups behind other lanes' 70 ms chains (8 lanes,
    // 455 MiB groups: 4.3 GiB/s; 256 MiB: 9+).
    const uint64_t group_cap = g_stream_group_cap ? g_stream_group_cap
                                                  : (2048 / (uint64_t)h->max_lanes) * (o.min + o.avg);
    h->group_bytes = std::max<uint64_t>(
        std::min<uint64_t>(h->max_slots * h->slot_bytes / (uint64_t)(h->max_lanes + 1), group_cap), slice);
    // the largest group one launch spreads over the chip (quad workgroups for 2048 chunks)
    h->group_hard = std::max<uint64_t>(2048 * (o.min + o.avg), h->group_bytes);
    if (!(rc = acquire(&h->ws))) {
        const hipError_t e = hipEventCreateWithFlags(&h->ev_bytes, hipEventDisableTiming);
        if (e != hipSuccess) rc = hip_fail(e, "hipEventCreate");
    }
    if (rc) {
        delete h;
        if (status) *status = rc;
        return nullptr;
    }
    if (status) *status = CG_OK;
    return h;
}

namespace {

// The first failure poisons the handle; later calls repeat it (status, message, fields).
int poison(cg_stream *h, int rc) {
    if (rc && !h->poisoned) {
        h->poisoned = rc;
        h->poison_msg = cg_last_error_message();
        cg_last_error_detail(h->poison_detail);
    }
    return rc;
}

int check_poisoned(const cg_stream *h) {
    if (!h->poisoned) return CG_OK;
    return fail_detail(h->poisoned, "stream failed earlier and cannot continue: " + h->poison_msg, h->poison_detail);
}

// Size the workspace for the largest boundary pass (a full slot) before any digest is in
// flight: a workspace buffer that grew later would hipFree, which waits for the whole
// device.  Allocation only: nothing is launched over the fresh (uninitialised) arena.
int prime_workspace(cg_stream *h) { return reserve_pass(h->ws, h->slot_bytes - 256, h->o, h->algo); }

int stream_push(cg_stream *h, const uint8_t *data, uint64_t len) {
    int rc;
    if (len && !h->arena.p) {
        if ((rc = h->arena.alloc(std::min<uint64_t>(2, h->max_slots), h->slot_bytes))) return rc;
        if ((rc = prime_workspace(h))) return rc;
    }
    while (len) {  // a slice larger than a slot goes in slot-sized pieces (chunks do not depend on slicing)
        const uint64_t room = h->slot_bytes - 256 - h->tail;
        const uint64_t take = std::min(len, room);
        HIP_TRY(hipMemcpyAsync(slot_ptr(h, h->cur) + h->tail, data, take, hipMemcpyHostToDevice, h->ws->stream));
        if ((rc = stream_drain(h, take, false))) return rc;
        h->pushed += take;
        data += take;
        len -= take;
    }
    // the caller may reuse `data` as soon as push returns: its copy has completed
    HIP_TRY(hipStreamSynchronize(h->ws->stream));
    return CG_OK;
}

int stream_finish(cg_stream *h) {
    h->finished = true;
    int rc = stream_drain(h, 0, true);
    if (rc) return rc;
    return launch_open(h);
}

int stream_take(cg_stream *h, cg_desc *out, size_t out_cap, size_t *n_out, int wait) {
    int rc;
    while (h->ready.empty()) {
        if (!h->inflight.empty()) {
            const Lane &l = h->lanes[h->inflight.front().lane];
            if (!wait && hipEventQuery(l.done) == hipErrorNotReady) break;
            if ((rc = complete_oldest(h))) return rc;
        } else if (wait && !h->open.desc.empty()) {
            if ((rc = launch_open(h))) return rc;
        } else {
            break;
        }
    }
    size_t n = 0;
    while (n < out_cap && !h->ready.empty()) {
        out[n++] = h->ready.front();
        h->ready.pop_front();
    }
    if (n_out) *n_out = n;
    return CG_OK;
}

}  // namespace

int cg_stream_push(cg_stream *h, const uint8_t *data, uint64_t len) {
    clear_error();
    if (!h) return fail(CG_E_IO, "null stream handle");
    int rc = check_poisoned(h);
    if (rc) return rc;
    if (h->finished) return fail(CG_E_INVALID_OPTIONS, "push called after finish");
    if ((rc = check_tables())) return rc;
    return poison(h, stream_push(h, data, len));
}

int cg_stream_finish(cg_stream *h) {
    clear_error();
    if (!h) return fail(CG_E_IO, "null stream handle");
    int rc = check_poisoned(h);
    if (rc) return rc;
    if (h->finished) return CG_OK;
    if ((rc = check_tables())) return rc;
    return poison(h, stream_finish(h));
}

int cg_stream_take(cg_stream *h, cg_desc *out, size_t out_cap, size_t *n_out, int wait) {
    clear_error();
    if (n_out) *n_out = 0;
    if (!h) return fail(CG_E_IO, "null stream handle");
    int rc = check_poisoned(h);
    if (rc) return rc;
    return poison(h, stream_take(h, out, out_cap, n_out, wait));
}

uint64_t cg_stream_pending(const cg_stream *h) {
    if (!h) return 0;
    uint64_t n = h->ready.size() + h->open.desc.size();
    for (const Group &g : h->inflight) n += g.desc.size();
    return n;
}

uint64_t cg_stream_bytes_consumed(const cg_stream *h) { return h ? h->pushed : 0; }

void cg_stream_free(cg_stream *h) { delete h; }

// test hooks: stream shape for streams created afterwards; return the previous value
uint64_t cg_test_stream_group_cap(uint64_t v) {
    const uint64_t old = g_stream_group_cap;
    g_stream_group_cap = v;
    return old;
}
uint32_t cg_test_stream_eager(uint32_t v) {
    const uint32_t old = g_stream_eager;
    g_stream_eager = v;
    return old;
}
uint32_t cg_test_stream_max_lanes(uint32_t v) {
    const uint32_t old = g_stream_max_lanes;
    g_stream_max_lanes = v;
    return old;
}

}  // extern "C"
