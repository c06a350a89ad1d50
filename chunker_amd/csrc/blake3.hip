// blake3.hip -- K4: per-chunk BLAKE3 (hash mode, 32-byte output), replacing
// blake3::hash (src/chunking.rs:68-71) called per chunk by compute_hash.
//
// BLAKE3 is a tree over 1 KiB leaves, so unlike SHA-256 it parallelises inside a
// chunk: one lane computes one leaf's chaining value (16 compressions), one wave
// owns 64 consecutive leaves (an aligned 64 KiB subtree) and folds them in LDS,
// and a second kernel folds the <= 256 subtree values of chunks larger than
// 64 KiB.  Level-wise pairing with the odd node carried up is exactly BLAKE3's
// left-complete tree (left subtree = largest power of two < n leaves).
#include "common.h"

namespace cg {

enum : uint32_t { B3_CHUNK_START = 1, B3_CHUNK_END = 2, B3_PARENT = 4, B3_ROOT = 8 };

struct B3Sched {
    uint8_t s[7][16];
    constexpr B3Sched() : s{} {
        constexpr uint8_t perm[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
        for (int i = 0; i < 16; ++i) s[0][i] = (uint8_t)i;
        for (int r = 1; r < 7; ++r)
            for (int i = 0; i < 16; ++i) s[r][i] = s[r - 1][perm[i]];
    }
};
static constexpr B3Sched B3S{};
static constexpr uint32_t B3_IV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                      0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

__device__ __forceinline__ uint32_t rotr32b(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }

#define B3_G(a, b, c, d, x, y)            \
    {                                     \
        v[a] = v[a] + v[b] + (x);         \
        v[d] = rotr32b(v[d] ^ v[a], 16);  \
        v[c] = v[c] + v[d];               \
        v[b] = rotr32b(v[b] ^ v[c], 12);  \
        v[a] = v[a] + v[b] + (y);         \
        v[d] = rotr32b(v[d] ^ v[a], 8);   \
        v[c] = v[c] + v[d];               \
        v[b] = rotr32b(v[b] ^ v[c], 7);   \
    }

// Compress one block; returns the new chaining value in cv (first 8 output words).
__device__ __forceinline__ void b3_compress(uint32_t cv[8], const uint32_t m[16], uint64_t counter, uint32_t blen,
                                            uint32_t flags) {
    uint32_t v[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                      B3_IV[0], B3_IV[1], B3_IV[2], B3_IV[3], (uint32_t)counter, (uint32_t)(counter >> 32),
                      blen, flags};
#pragma unroll
    for (int r = 0; r < 7; ++r) {
        B3_G(0, 4, 8, 12, m[B3S.s[r][0]], m[B3S.s[r][1]]);
        B3_G(1, 5, 9, 13, m[B3S.s[r][2]], m[B3S.s[r][3]]);
        B3_G(2, 6, 10, 14, m[B3S.s[r][4]], m[B3S.s[r][5]]);
        B3_G(3, 7, 11, 15, m[B3S.s[r][6]], m[B3S.s[r][7]]);
        B3_G(0, 5, 10, 15, m[B3S.s[r][8]], m[B3S.s[r][9]]);
        B3_G(1, 6, 11, 12, m[B3S.s[r][10]], m[B3S.s[r][11]]);
        B3_G(2, 7, 8, 13, m[B3S.s[r][12]], m[B3S.s[r][13]]);
        B3_G(3, 4, 9, 14, m[B3S.s[r][14]], m[B3S.s[r][15]]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = v[i] ^ v[i + 8];
}

__device__ __forceinline__ void b3_parent(const uint32_t *l, const uint32_t *r, bool root, uint32_t out[8]) {
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        m[i] = l[i];
        m[i + 8] = r[i];
    }
    uint32_t cv[8] = {B3_IV[0], B3_IV[1], B3_IV[2], B3_IV[3], B3_IV[4], B3_IV[5], B3_IV[6], B3_IV[7]};
    b3_compress(cv, m, 0, 64, B3_PARENT | (root ? B3_ROOT : 0u));
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = cv[i];
}

// Leaf of `n` (0..1024) bytes at p with leaf index ctr.  Words are little-endian;
// p may be unaligned (v_alignbyte realigns aligned dword loads).
__device__ __forceinline__ void b3_leaf(const uint8_t *p, uint32_t n, uint64_t ctr, bool root, uint32_t cv[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = B3_IV[i];
    const uint32_t shift = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *base = reinterpret_cast<const uint32_t *>(p - shift);
    const uint32_t nblk = n ? (n + 63) / 64 : 1;
    const uint8_t *endp = p + n;
    for (uint32_t j = 0; j < nblk; ++j) {
        const uint32_t *q = base + 16 * j;
        const bool last = j + 1 == nblk;
        const uint32_t blen = last ? n - 64 * j : 64u;
        uint32_t dw[17], m[16];
        if (!last) {
#pragma unroll
            for (int i = 0; i < 16; ++i) dw[i] = q[i];
            dw[16] = shift ? q[16] : 0u;
#pragma unroll
            for (int i = 0; i < 16; ++i) m[i] = __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], shift);
        } else {
#pragma unroll
            for (int i = 0; i < 17; ++i) dw[i] = (reinterpret_cast<const uint8_t *>(q + i) < endp) ? q[i] : 0u;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t v = __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], shift);
                const int r = (int)blen - 4 * i;
                m[i] = r >= 4 ? v : (r <= 0 ? 0u : (v & (0xffffffffu >> (32 - 8 * r))));
            }
        }
        uint32_t flags = (j == 0 ? B3_CHUNK_START : 0u) | (last ? B3_CHUNK_END : 0u);
        if (root && last) flags |= B3_ROOT;
        b3_compress(cv, m, ctr, blen, flags);
    }
}

__device__ __forceinline__ uint64_t b3_groups_of(uint64_t len) {
    const uint64_t leaves = len ? (len + 1023) / 1024 : 1;
    return (leaves + 63) / 64;
}

__device__ __forceinline__ void store_digest(uint8_t *dst, const uint32_t cv[8]) {
    uint4 *o = reinterpret_cast<uint4 *>(dst);
    o[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
    o[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
}

__global__ void k_b3_count(const DescRaw *__restrict__ desc, const uint64_t *__restrict__ total_p,
                           uint64_t max_chunks, uint32_t *__restrict__ gcount) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= max_chunks) return;
    uint64_t total = *total_p;
    gcount[g] = g < total ? (uint32_t)b3_groups_of(desc[g].length) : 0u;
}

// Fold the chaining values held one per lane (lanes 0..count-1) level by level,
// the odd last node carried up (BLAKE3's left-complete tree); ROOT on the final
// parent when `root`.  Pure register shuffles: no LDS, no barriers.
__device__ __forceinline__ void b3_wave_fold(uint32_t cv[8], uint32_t count, bool root, uint32_t lane) {
    while (count > 1) {
        const uint32_t half = count >> 1;
        uint32_t l[8], r[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            l[i] = __shfl(cv[i], (int)(2 * lane) & 63, 64);
            r[i] = __shfl(cv[i], (int)(2 * lane + 1) & 63, 64);
        }
        if (lane < half) {
            b3_parent(l, r, root && count == 2, cv);
        } else if ((count & 1u) && lane == half) {
#pragma unroll
            for (int i = 0; i < 8; ++i) cv[i] = l[i];
        }
        count = (count + 1) >> 1;
    }
}

#define B3_WAVES 4u

// One wave per 64-leaf group (4 waves per workgroup for occupancy).
__global__ __launch_bounds__(64 * B3_WAVES) void k_b3_groups(const uint8_t *__restrict__ data,
                                                             const uint64_t *__restrict__ abs,
                                                             const DescRaw *__restrict__ desc,
                                                             const uint64_t *__restrict__ total_p, uint64_t max_chunks,
                                                             const uint64_t *__restrict__ group_base,
                                                             uint8_t *__restrict__ hash_base, size_t stride,
                                                             uint32_t *__restrict__ gcv) {
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    const uint64_t G = (uint64_t)blockIdx.x * B3_WAVES + (threadIdx.x >> 6);
    if (G >= group_base[total]) return;
    // chunk c with group_base[c] <= G < group_base[c+1]
    uint64_t lo = 0, hi = total;
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (group_base[mid] <= G)
            lo = mid;
        else
            hi = mid;
    }
    const uint64_t c = lo;
    const uint64_t len = desc[c].length;
    const uint64_t gi = G - group_base[c];
    const uint64_t ngroups = group_base[c + 1] - group_base[c];
    const uint64_t leaves = len ? (len + 1023) / 1024 : 1;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t count0 = (uint32_t)((leaves - gi * 64) < 64 ? (leaves - gi * 64) : 64);
    const uint64_t leaf = gi * 64 + lane;
    const uint8_t *chunk = data + abs[c];
    uint32_t cv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (lane < count0) {
        const uint64_t off = leaf * 1024;
        const uint32_t n = (uint32_t)((len - off) < 1024 ? (len - off) : 1024);
        b3_leaf(chunk + off, len ? n : 0u, leaf, leaves == 1, cv);
    }
    if (leaves == 1) {
        if (lane == 0) store_digest(hash_base + c * stride, cv);
        return;
    }
    const bool whole = ngroups == 1;
    b3_wave_fold(cv, count0, whole, lane);
    if (lane == 0) {
        if (whole) {
            store_digest(hash_base + c * stride, cv);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) gcv[G * 8 + i] = cv[i];
        }
    }
}

// One wave per chunk with more than one group: fold the subtree chaining values
// (<= 256 of them: chunks are <= 16 MiB).  Levels wider than 64 nodes go through
// LDS; the last six levels are register shuffles (b3_wave_fold).
__global__ __launch_bounds__(64) void k_b3_top(const DescRaw *__restrict__ desc, const uint64_t *__restrict__ total_p,
                                               uint64_t max_chunks, const uint64_t *__restrict__ group_base,
                                               const uint32_t *__restrict__ gcv, uint8_t *__restrict__ hash_base,
                                               size_t stride) {
    __shared__ uint32_t s_cv[256][9];
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    const uint64_t c = blockIdx.x;
    if (c >= total) return;
    const uint64_t g0 = group_base[c];
    uint32_t count = (uint32_t)(group_base[c + 1] - g0);
    if (count <= 1) return;
    const uint32_t lane = threadIdx.x;
    if (count <= 64) {
        uint32_t cv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (lane < count)
#pragma unroll
            for (int i = 0; i < 8; ++i) cv[i] = gcv[(g0 + lane) * 8 + i];
        b3_wave_fold(cv, count, true, lane);
        if (lane == 0) store_digest(hash_base + c * stride, cv);
        return;
    }
    for (uint32_t k = lane; k < count; k += 64)
#pragma unroll
        for (int i = 0; i < 8; ++i) s_cv[k][i] = gcv[(g0 + k) * 8 + i];
    __syncthreads();
    while (count > 64) {
        const uint32_t half = count >> 1;
        uint32_t t[2][8];
        bool wr[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const uint32_t j = lane + 64u * s;
            wr[s] = false;
            if (j < half) {
                b3_parent(s_cv[2 * j], s_cv[2 * j + 1], false, t[s]);
                wr[s] = true;
            } else if ((count & 1u) && j == half) {
#pragma unroll
                for (int i = 0; i < 8; ++i) t[s][i] = s_cv[count - 1][i];
                wr[s] = true;
            }
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 2; ++s)
            if (wr[s])
#pragma unroll
                for (int i = 0; i < 8; ++i) s_cv[lane + 64u * s][i] = t[s][i];
        __syncthreads();
        count = (count + 1) >> 1;
    }
    uint32_t cv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (lane < count)
#pragma unroll
        for (int i = 0; i < 8; ++i) cv[i] = s_cv[lane][i];
    b3_wave_fold(cv, count, true, lane);
    if (lane == 0) store_digest(hash_base + c * stride, cv);
}

size_t blake3_group_bound(uint64_t total_bytes, uint64_t max_chunks) { return total_bytes / 65536 + max_chunks + 1; }

void launch_blake3(const uint8_t *d_data, const uint64_t *d_abs, const void *d_desc, const uint64_t *d_total,
                   uint64_t max_chunks, uint64_t total_bytes, uint8_t *d_hash_base, size_t hash_stride,
                   uint64_t * /*unused*/, uint64_t *d_group_base, uint32_t *d_gcount_u32, uint64_t *d_scan_tmp,
                   uint32_t *d_gcv, hipStream_t st) {
    if (max_chunks == 0) return;
    const DescRaw *desc = (const DescRaw *)d_desc;
    hipLaunchKernelGGL(k_b3_count, dim3((uint32_t)((max_chunks + 255) / 256)), dim3(256), 0, st, desc, d_total,
                       max_chunks, d_gcount_u32);
    launch_exclusive_scan_u32(d_gcount_u32, d_group_base, max_chunks, 0, d_scan_tmp, st);
    const uint64_t gbound = blake3_group_bound(total_bytes, max_chunks);
    hipLaunchKernelGGL(k_b3_groups, dim3((uint32_t)((gbound + B3_WAVES - 1) / B3_WAVES)), dim3(64 * B3_WAVES), 0, st, d_data, d_abs, desc, d_total,
                       max_chunks, d_group_base, d_hash_base, hash_stride, d_gcv);
    hipLaunchKernelGGL(k_b3_top, dim3((uint32_t)max_chunks), dim3(64), 0, st, desc, d_total, max_chunks,
                       d_group_base, d_gcv, d_hash_base, hash_stride);
}

}  // namespace cg
