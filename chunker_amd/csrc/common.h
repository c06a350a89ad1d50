// common.h -- shared definitions of the gfx950 FastCDC + digest engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// One lane of the candidate scan owns SEG consecutive bytes of the flat batch
// buffer, after a HALO-byte warm-up.  Every FastCDC v2020 mask lives in bits <= 47,
// so 48 bytes of history make the rolling Gear hash's tested bits exact
// (SURVEY.md Appendix A.3).
#ifndef CG_SEG
#define CG_SEG 4096u
#endif
#define CG_HALO 48u
#define CG_SCAN_BLOCK 256u

// Compacted candidate entry: (absolute position << 2) | flags.  flags bit1 = the
// position passes mask_s, bit0 = it passes mask_l, 0 = "dense segment" marker
// (the segment had more candidates than the per-segment capacity; the walker
// rescans it exactly).
#define CG_FLAG_S 2u
#define CG_FLAG_L 1u

// Device view of cg_desc (include/chunker_gpu.h): 48 bytes.
struct DescRaw {
    uint64_t offset, length;
    uint8_t hash[32];
};

struct CdcParams {
    uint64_t min, avg, max;
    uint64_t mask_s, mask_l;
};

// Kernel launch wrappers (defined next to their kernels).
namespace cg {

// Block-wide inclusive scan of one u64 per thread (wave64 shuffles + LDS).
__device__ __forceinline__ uint64_t block_inclusive_scan(uint64_t v, uint64_t *s_wave) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    if (lane == 63) s_wave[wave] = v;
    __syncthreads();
    uint64_t add = 0;
    for (uint32_t w = 0; w < wave; ++w) add += s_wave[w];
    __syncthreads();
    return v + add;
}


// Work queue of the persistent candidate scan (scan.hip k_scan_flat32p): one head counter
// per XCD and a leave counter, each on its own 64-B line; zero between launches (the last
// wave of a launch resets it).
struct ScanQueue {
    uint32_t head[8][16];
    uint32_t done[16];
};

// d_queue: a zeroed ScanQueue owned by the caller's workspace (nullptr: the one-shot kernel)
// the calling thread asks launch_scan for the lean one-shot scan (scan.hip; the digest pipeline)
extern thread_local bool t_scan_lean;
void launch_scan(const uint8_t *d_data, uint64_t n, const uint64_t *d_gear, uint64_t mask_s, uint64_t mask_l,
                 uint32_t cap, uint32_t *d_seg_count, uint32_t *d_seg_cand, uint64_t nseg, hipStream_t st,
                 ScanQueue *d_queue = nullptr);
uint64_t scan_resident_wgs();

// Exclusive prefix sum of per-segment entry counts; writes d_out[0..n] (d_out[n] = total).
// `cap` > 0 applies the entry transform (count <= cap ? count : 1).
void launch_exclusive_scan_u32(const uint32_t *d_in, uint64_t *d_out, uint64_t n, uint32_t cap, uint64_t *d_tmp,
                               hipStream_t st);
size_t exclusive_scan_tmp_elems(uint64_t n);
extern uint32_t g_scan_path;  // test hook cg_test_scan_path (scan.hip)

// Exclusive scan of the per-segment candidate counts into d_eoff fused with the compaction of
// the candidate slots into the sorted entry list.
// `si`: host tables copied into HBM by extra blocks of the compaction's first launch.
struct StageIn;
void launch_scan_compact(const uint32_t *d_seg_count, const uint32_t *d_seg_cand, uint64_t *d_eoff, uint32_t cap,
                         uint64_t nseg, uint64_t *d_entries, uint64_t *d_tmp, hipStream_t st, const StageIn &si);

// Piece lists for the walk of large NARs (walk.hip, k_walk_pieces); np = 0: none.
struct WalkPiecesHost {
    const uint64_t *first = nullptr;  // device [n_nars + 1]
    const uint32_t *nar = nullptr;    // device [np]
    const uint64_t *base = nullptr;   // device [np]
    uint32_t *count = nullptr;        // device [np]
    uint64_t *exit = nullptr;         // device [np]
    uint64_t *starts = nullptr;       // device, sum of per-piece capacities
    uint64_t pb = 0, np = 0;
};
// The walk verifies candidate-list walks afterwards (and can use piece lists) when
// mask_s is sparse enough that a cut inside a chunk's 47-byte warm-up is rare.
inline bool walk_is_speculative(const CdcParams &p) { return __builtin_popcountll(p.mask_s) >= 14; }
// d_nar_ngroups (optional, BLAKE3 batches): each NAR's 64-leaf group count, for the
// group map launch_assemble builds
void launch_walk(const uint8_t *d_data, const uint64_t *d_gear, const uint64_t *d_entries, const uint64_t *d_eoff,
                 uint64_t nseg, const uint64_t *d_nar_off, const uint64_t *d_cap_base, uint64_t n_nars,
                 CdcParams p, uint64_t *d_wchunk, uint32_t *d_nar_nchunks, const WalkPiecesHost &pieces,
                 hipStream_t st, uint32_t *d_nar_ngroups = nullptr);

// Up to two host -> HBM copies done by one kernel reading mapped (coherent) host memory.
struct StageIn {
    const void *src[2] = {nullptr, nullptr};  // device addresses of mapped host memory
    void *dst[2] = {nullptr, nullptr};
    uint64_t bytes[2] = {0, 0};  // multiples of 4
    int n = 0;
    void add(const void *s, void *d, uint64_t b) {
        src[n] = s;
        dst[n] = d;
        bytes[n] = b;
        ++n;
    }
};
void launch_stage_in(const StageIn &c, hipStream_t st);
// Blocks per copy when the stage-in rides along another launch (the compaction's first
// kernel), and the copy itself: block b of copy k takes dwords b*T + t, b*T + t + nb*T, ...
#define STAGE_IN_BLOCKS 8u
__device__ __forceinline__ void stage_in_part(const StageIn &c, uint32_t k, uint32_t b, uint32_t nb) {
    const uint32_t *src = static_cast<const uint32_t *>(c.src[k]);
    uint32_t *dst = static_cast<uint32_t *>(c.dst[k]);
    const uint64_t n = c.bytes[k] / 4;
    for (uint64_t i = (uint64_t)b * blockDim.x + threadIdx.x; i < n; i += (uint64_t)nb * blockDim.x) dst[i] = src[i];
}

// A chunk's BLAKE3 64-leaf groups (k_b3_groups work units; an empty chunk is one group).
__device__ __forceinline__ uint32_t b3_leaves_of_len(uint64_t len) { return len ? (uint32_t)((len + 1023) / 1024) : 1u; }
__device__ __forceinline__ uint32_t b3_groups_of_len(uint64_t len) { return (b3_leaves_of_len(len) + 63) / 64; }
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, d, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), d, 64);
        v += ((uint64_t)hi << 32) | lo;
    }
    return v;
}
// The BLAKE3 group map written by the descriptor assembly (launch_blake3 with
// plan_ready): group_base [bound + 1], gmap (one entry per group), from d_nar_ngroups.
// Packed leaves (leaf_base / lmap set): the leaves of all chunks back to back, 64 per
// wave whatever chunk they belong to (no idle lanes at chunk tails); leaf_base [bound + 1]
// = leaves of chunks 0..g-1, lmap[w] = the chunk holding leaf slot 64 w.  nar_ngroups holds
// each NAR's group count at [i] and its leaf count at [n_nars + 1 + i].
struct B3PlanOut {
    const uint32_t *nar_ngroups = nullptr;
    uint64_t *group_base = nullptr;
    uint32_t *gmap = nullptr;
    uint64_t bound = 0;
    uint64_t *leaf_base = nullptr;
    uint32_t *lmap = nullptr;
    uint64_t lmap_cap = 0;
};

// exclusive scan of the per-NAR chunk counts into d_nar_first (total at [n_nars]) + the
// descriptors and absolute chunk offsets of every NAR's chunks
// Returns true when it also built the BLAKE3 group map `b3` (the one-launch form, up to
// 8,192 NARs); otherwise launch_blake3 builds it.  host_first (optional, a device address
// of mapped host memory): the one-launch form also writes the NAR index there and sets
// *wrote_host_first.
bool launch_assemble(const uint64_t *d_nar_off, const uint64_t *d_cap_base, const uint64_t *d_wchunk,
                     const uint32_t *d_nar_nchunks, uint64_t *d_nar_first, uint64_t n_nars, void *d_out,
                     uint64_t out_cap, uint64_t *d_chunk_abs, uint64_t *d_scan_tmp, hipStream_t st,
                     const B3PlanOut *b3, uint64_t *host_first, bool *wrote_host_first);

// Per-member completion of a merged digest (the digest pipeline, pipeline.hip): chunk g of
// the merged list belongs to member[g] and its digest goes to dst[g] (a device address)
// instead of hash_base + g * stride.  Once a workgroup's digests are stored, one lane per
// chunk counts its member down (remain[m]); the lane that takes it to zero writes the
// member's host-mapped completion word *flag[m] = 1, or 2 if a spin guard fired on any of
// the member's chunks (merr[m]).  So a member is done when its own longest chunk is, not
// when the whole merged launch is.
struct ShaNotify {
    const uint64_t *dst = nullptr;
    const uint32_t *member = nullptr;
    uint32_t *remain = nullptr;
    uint32_t *merr = nullptr;
    uint32_t *const *flag = nullptr;
};

// d_order_tmp (sha256_order_tmp_elems(max_chunks) u32, or nullptr = identity order) holds
// the longest-first lane order; max_len bounds every chunk length (bucket width);
// `expected` estimates the chunk count (sizes the workgroup tiers).  d_err (one u32, zeroed
// by the caller) becomes nonzero if a producer/consumer hand-off hit its spin guard.
// `notify` (optional): per-member destinations and completion words (ShaNotify).
void launch_sha256(const uint8_t *d_data, const uint64_t *d_abs, const void *d_desc, const uint64_t *d_total,
                   uint64_t max_chunks, uint64_t expected, uint64_t max_len, uint32_t *d_order_tmp,
                   uint8_t *d_hash_base, size_t hash_stride, uint32_t *d_err, hipStream_t st,
                   bool latency_tiers = true, const ShaNotify *notify = nullptr);
size_t sha256_order_tmp_elems(uint64_t max_chunks);

// The digest pipeline's merged launch (pipeline.hip): up to CG_PIPE_MAX batches of one
// caller, each after its boundary stages, digested by ONE k_sha256 with per-member
// completion.  Member b's chunks are (data[b] + abs[b][i], out[b][i].length) for
// i < min(*total[b], bound[b]); digests land in out[b][i].hash; flag[b] is the device
// address of the member's host-mapped completion word.
#define CG_PIPE_MAX 64
struct PipeTable {
    uint32_t n;
    const uint8_t *data[CG_PIPE_MAX];
    const uint64_t *abs[CG_PIPE_MAX];
    DescRaw *out[CG_PIPE_MAX];
    const uint64_t *total[CG_PIPE_MAX];
    uint64_t bound[CG_PIPE_MAX];
    uint32_t *flag[CG_PIPE_MAX];
};
// The merged arrays a PipeTable launch uses (bound_sum = sum of bound[b]).
struct PipeBufs {
    DescRaw *mdesc;      // bound_sum (lengths only)
    uint64_t *mabs;      // bound_sum: chunk address - data[0]
    uint64_t *mdst;      // bound_sum: digest destination
    uint32_t *mmember;   // bound_sum
    uint64_t *mtotal;    // 1
    uint32_t *morder;    // sha256_order_tmp_elems(bound_sum)
    uint32_t *remain;    // CG_PIPE_MAX
    uint32_t *merr;      // CG_PIPE_MAX
    uint32_t **mflag;    // CG_PIPE_MAX
    uint32_t *err;       // 1: the launch's spin-guard word
};
// start / stop (optional): timing events around the digest kernel alone (after the merge)
void launch_sha256_pipe(const PipeTable &t, uint64_t bound_sum, uint64_t expected, uint64_t max_len,
                        const PipeBufs &b, hipStream_t st, hipEvent_t start = nullptr, hipEvent_t stop = nullptr);

// Coalesced SHA-256 digest (runtime.hip's per-device coalescer of concurrent callers): the
// chunks of up to CG_COAL_MAX batches that are ready at the same time digested by ONE
// launch_sha256.
// Member b's chunks are (data[b] + abs[b][i], out[b][i].length) for i < min(*total[b],
// bound[b]); their digests land in out[b][i].hash and a spin-guard failure in *err[b].
#define CG_COAL_MAX 32
struct CoalTable {
    uint32_t n;
    const uint8_t *data[CG_COAL_MAX];
    const uint64_t *abs[CG_COAL_MAX];
    DescRaw *out[CG_COAL_MAX];
    const uint64_t *total[CG_COAL_MAX];
    uint64_t bound[CG_COAL_MAX];
    uint32_t *err[CG_COAL_MAX];
};
// merged arrays: mdesc / mabs bound_sum entries, mtotal one u64, morder_tmp
// sha256_order_tmp_elems(bound_sum) u32, merr one u32
void launch_sha256_coalesced(const CoalTable &t, uint64_t bound_sum, uint64_t expected, uint64_t max_len,
                             DescRaw *mdesc, uint64_t *mabs, uint64_t *mtotal, uint32_t *morder_tmp, uint32_t *merr,
                             hipStream_t st);

// Longest-first order of the first min(*d_total, max_chunks) descriptors (counting sort
// on SHA-256 block count, max_len bounding every length); returns the order inside
// d_order_tmp (sha256_order_tmp_elems(max_chunks) u32), or nullptr without a buffer.
// d_need (2 u32, optional): the latency-tier counts for k_sha256 (k_len_base).
const uint32_t *launch_len_order(const void *d_desc, const uint64_t *d_total, uint64_t max_chunks, uint64_t max_len,
                                 uint32_t *d_order_tmp, hipStream_t st, uint32_t *d_need = nullptr,
                                 uint32_t quad_pm = 0, uint32_t pair_pm = 0);

// K5: CAS content ids (cas.hip): SHAKE256-256 of the framed span, ContentId::compute
// (crates/core/cas/src/lib.rs:53-69); id of span g -> d_ids + g * id_stride.
void launch_cas_ids(const uint8_t *d_data, const uint64_t *d_abs, const void *d_desc, const uint64_t *d_total,
                    uint64_t max_n, const uint32_t *d_order, uint32_t kind, uint8_t *d_ids, size_t id_stride,
                    hipStream_t st);

// Manifest spans of a batch: span i = bytes [32 first[i], 32 first[i+1]) of the chunk-id
// buffer (crates/node/src/lib.rs:124-129); *d_total = n_nars.
void launch_manifest_spans(const uint64_t *d_first, uint64_t n_nars, uint64_t *d_abs, void *d_desc, uint64_t *d_total,
                           hipStream_t st);

void launch_blake3(const uint8_t *d_data, const uint64_t *d_abs, const void *d_desc, const uint64_t *d_total,
                   uint64_t max_chunks, uint64_t total_bytes, uint8_t *d_hash_base, size_t hash_stride,
                   uint32_t *d_gmap, uint64_t *d_group_base, uint32_t *d_gcount_u32,
                   uint64_t *d_scan_tmp, uint32_t *d_gcv, bool with_lcv, hipStream_t st,
                   bool plan_ready = false, const uint64_t *d_leaf_base = nullptr, const uint32_t *d_lmap = nullptr);
// (plan_ready: d_group_base / d_gmap built by launch_assemble; with d_leaf_base / d_lmap
// from it too, the leaves run packed, k_b3_leaves)
size_t blake3_leaf_wave_bound(uint64_t total_bytes, uint64_t max_chunks);  // lmap entries
size_t blake3_group_bound(uint64_t total_bytes, uint64_t max_chunks);
size_t blake3_cv_bytes(uint64_t total_bytes, uint64_t max_chunks, bool with_lcv);  // launch_blake3's d_gcv

void launch_spans_to_desc(const uint64_t *d_off, const uint64_t *d_len, uint64_t n, uint64_t *d_abs, void *d_desc,
                          uint64_t *d_total, hipStream_t st);

}  // namespace cg
