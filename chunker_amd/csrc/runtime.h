// runtime.h -- internals shared by the host runtime's translation units (runtime.hip:
// batch pipeline, push handle, tables; stream.hip: the pipelined stream handle).
// Nothing here is part of the C ABI (include/chunker_gpu.h).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/chunker_gpu.h"
#include "common.h"

namespace cgrt {

// reference defaults, src/chunking.rs:179-181
constexpr uint64_t DEF_MIN = 256 * 1024, DEF_AVG = 1024 * 1024, DEF_MAX = 4 * 1024 * 1024;
// fastcdc::v2020 ranges [ext], pinned by src/chunking.rs:1401-1415
constexpr uint64_t MINIMUM_MIN = 64, MINIMUM_MAX = 1048576, AVERAGE_MIN = 256, AVERAGE_MAX = 4194304,
                   MAXIMUM_MIN = 1024, MAXIMUM_MAX = 16777216;

// Failure reporting: status code + thread-local message (cg_last_error_message) and
// the ChunkingError fields (cg_last_error_detail).
int fail(int code, const std::string &msg);
void clear_error();
int fail_bounds(uint64_t data_len, uint64_t offset, uint64_t length, const std::string &what);
int fail_limit(uint64_t attempted, const std::string &what);
int fail_detail(int code, const std::string &msg, const uint64_t detail[3]);  // a failure with given fields
int hip_fail(hipError_t e, const char *what, uint64_t attempted = 0);

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t _e = (expr);                         \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

// FastCDC v2020 tables (runtime.hip): one immutable snapshot per installed set.
struct Tables {
    uint64_t gear[256];
    uint64_t masks[26];
    uint64_t epoch;
    bool placeholder;
};

std::shared_ptr<const Tables> tables();
// Fail-closed gate in front of every chunking entry point.
int check_tables();

// test hook (cg_test_fail_alloc): true when this device allocation is the one to fail
bool test_alloc_fault();

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes, const char *name) {
        if (bytes <= cap) return CG_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 4 + 256;
        hipError_t e = test_alloc_fault() ? hipErrorOutOfMemory : hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return hip_fail(e, name, want);
        }
        cap = want;
        return CG_OK;
    }
    template <class T>
    T *as() const { return static_cast<T *>(p); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct PinBuf {
    void *p = nullptr;
    void *dev = nullptr;  // device address of p (mapped buffers)
    size_t cap = 0;
    // mapped: coherent host memory the GPU writes straight into (uncached, over the link)
    int ensure(size_t bytes, bool mapped = false) {
        if (bytes <= cap && (!mapped || dev)) return CG_OK;  // (a mapped request never gets an unmapped buffer)
        if (bytes < cap) bytes = cap;
        if (p) (void)hipHostFree(p);
        p = dev = nullptr;
        cap = 0;
        size_t want = bytes + bytes / 4 + 256;
        hipError_t e = hipHostMalloc(&p, want, mapped ? (hipHostMallocMapped | hipHostMallocCoherent) : hipHostMallocDefault);
        if (e == hipSuccess && mapped) e = hipHostGetDevicePointer(&dev, p, 0);
        if (e != hipSuccess) {
            if (p) (void)hipHostFree(p);
            p = dev = nullptr;
            return hip_fail(e, "hipHostMalloc", want);
        }
        cap = want;
        return CG_OK;
    }
    template <class T>
    T *as() const { return static_cast<T *>(p); }
};

enum { EV_START, EV_SCAN, EV_COMPACT, EV_WALK, EV_ASSEMBLE, EV_DIGEST, EV_N };

struct Workspace {
    int device = -1;
    hipStream_t stream = nullptr;
    uint64_t gear_epoch = 0;
    DevBuf gear, seg_count, seg_cand, eoff, scan_tmp, entries, nar_off, wchunk, nar_nchunks, nar_first,
        chunk_abs, b3_gcount, b3_gbase, b3_gcv, b3_gmap, in, out, span_off, span_len, order, cas_order, ids,
        man_abs, man_desc, sha_err, pc_first, pc_count, pc_exit, pc_starts, nar_ngroups, b3_lbase, b3_lmap,
        scanq;  // scanq: the persistent scan's work queue (cg::ScanQueue), zeroed once
    bool scanq_zeroed = false;  // the zeroing memset of scanq has been queued
    PinBuf stage, err_stage, first_host;  // first_host: mapped, the assembly writes the NAR index there
    PinBuf done_flag;  // mapped: a pipeline batch's completion word, written by its merged digest
    hipEvent_t ev[EV_N] = {};
    // CAS ids run on side_stream, concurrently with the digest: both stages are bound by
    // their longest chunk's serial chain, not by the chip, so they overlap for free.
    hipStream_t side_stream = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_cas = nullptr;
    // end of a launched batch: its wait syncs this event, not the stream (a batch queued
    // behind it on the same stream must not be waited for too)
    hipEvent_t ev_done = nullptr;
    // A SHA-256 batch queued with an inputs-ready event (cg_chunk_batch_device_async_after)
    // runs on the workspace's own `stream` (idle while an async batch holds the workspace),
    // ordered after that event only, beside the batches queued before it on the caller's
    // stream, which then waits for its done event.  Split mode 1 (A/B): only the boundary
    // stages run there; ev_bdone (recorded after the assembly) holds the digest on the
    // caller's stream back, and ev_dstart (after that wait) opens the digest stage's timing.
    hipEvent_t ev_bdone = nullptr, ev_dstart = nullptr;
    // Streams map onto the process's few hardware queues (GPU_MAX_HW_QUEUES, 4 by default)
    // and two streams on one queue serialise: the side stream exists only where used.
    int ensure_side_stream() {
        if (!side_stream) HIP_TRY(hipStreamCreateWithFlags(&side_stream, hipStreamNonBlocking));
        return CG_OK;
    }
    int init(int dev) {
        device = dev;
        HIP_TRY(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        for (auto &e : ev) HIP_TRY(hipEventCreate(&e));
        HIP_TRY(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
        HIP_TRY(hipEventCreate(&ev_cas));
        HIP_TRY(hipEventCreateWithFlags(&ev_done, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&ev_bdone, hipEventDisableTiming));
        HIP_TRY(hipEventCreate(&ev_dstart));
        return CG_OK;
    }
};

int current_device(int *dev);
int acquire(Workspace **out);
void release(Workspace *ws);
struct WsGuard {
    Workspace *ws;
    ~WsGuard() {
        if (ws) release(ws);
    }
};

struct Opts {
    uint64_t min, avg, max;
};

int resolve(uint64_t mn, uint64_t avg, uint64_t mx, Opts *o, char *msg, size_t cap);
uint64_t capacity_of(uint64_t len, uint64_t mn);
// every workspace buffer a boundary pass over one NAR of len bytes grows, allocated now
int reserve_pass(Workspace *ws, uint64_t len, const Opts &o, int algo);
uint32_t logarithm2(uint32_t v);

// SHA-256 spin-guard word of a workspace: arm before a digest launch, fetch with the
// call's results, check after the stream sync.
int sha_err_arm(Workspace *ws, hipStream_t st);
int sha_err_fetch(Workspace *ws, hipStream_t st);
int sha_err_check(Workspace *ws);

// What a launched batch leaves for finish_batch.
struct BatchLaunch {
    uint64_t *s_first = nullptr;  // pinned staging of the NAR -> first-chunk index (n_nars + 1)
    size_t n_nars = 0, out_cap = 0;
    bool sha_armed = false, node_put = false;
    int pmode = 0;  // profiling mode at launch (stage events recorded)
    hipEvent_t done = nullptr;  // recorded after the batch's last queued operation
    hipEvent_t dstart = nullptr;  // opens the digest stage's timing (profiling)
};
int launch_batch(Workspace *ws, const uint8_t *d_data, const uint64_t *h_nar_off, size_t n_nars, const Opts &o,
                 int algo, cg_desc *d_out, size_t out_cap, hipStream_t st, uint8_t *d_chunk_ids,
                 uint8_t *h_manifest_ids, bool digest, BatchLaunch *bl, bool coalesce = false,
                 hipEvent_t inputs_ready = nullptr);
int finish_batch(Workspace *ws, hipStream_t st, const BatchLaunch &bl, uint64_t *h_nar_first);

// The device pipeline for one batch (scan -> compact -> walk -> assemble -> digest).
int run_batch(Workspace *ws, const uint8_t *d_data, const uint64_t *h_nar_off, size_t n_nars, const Opts &o,
              int algo, cg_desc *d_out, size_t out_cap, uint64_t *h_nar_first, hipStream_t st,
              uint8_t *d_chunk_ids = nullptr, uint8_t *h_manifest_ids = nullptr, bool digest = true,
              bool coalesce = false);

// Digest coalescer (runtime.hip): a SHA-256 device-entry caller is counted as "active" from
// entry (CoalActive) until it submits its chunk list, and as "inside" until it returns, so a
// leader can wait for every caller in the entry to join its group.
struct CoalActive {
    int dev;
    bool left = false;  // submitted, or digesting alone
    bool solo = false;  // digesting alone (counted in Coalescer::solo until it returns)
    explicit CoalActive(int dev);
    void leave();
    void go_solo();
    ~CoalActive();
};
struct CoalGroup;
struct CoalEntry {
    Workspace *ws;
    const uint8_t *d_data;
    const uint64_t *d_abs;
    cg_desc *d_out;
    const uint64_t *d_total;
    uint64_t bound, expected, max_len;
    hipStream_t st;
    CoalActive *active = nullptr;
    hipEvent_t ready = nullptr;
    std::shared_ptr<CoalGroup> group;
    int rc = 0;
};
int coalesced_sha256(CoalEntry *e);
bool coalesce_worth(int dev);

// Which device a call runs on: the device set for the scope, the caller's restored after.
struct DeviceScope {
    int prev = -1;
    int set(int dev) {
        HIP_TRY(hipGetDevice(&prev));
        if (prev != dev) HIP_TRY(hipSetDevice(dev));
        return CG_OK;
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

struct PipeGroup;  // pipeline.hip
extern std::atomic<int> g_profiling;  // cg_set_profiling mode

}  // namespace cgrt

// An asynchronous batch (cg_chunk_batch_device_async, cg_pipeline_submit): its workspace
// stays reserved, and its results unread, until cg_batch_wait.  A pipeline batch also
// names its digest group and its index in it (pipeline.hip).
struct cg_pipeline;
struct cg_batch {
    cgrt::Workspace *ws;
    hipStream_t st;
    cgrt::BatchLaunch bl;
    std::shared_ptr<cgrt::PipeGroup> group;  // pipeline batches only
    uint32_t member = 0;
    int device = -1;
};
namespace cgrt {
int pipeline_wait(cg_batch *b, uint64_t *nar_first);  // pipeline.hip
}
