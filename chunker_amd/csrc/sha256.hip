// sha256.hip -- K3: per-chunk SHA-256 (FIPS 180-4), replacing sha256_hash_raw
// (src/hashing.rs:36-44) called per chunk by compute_hash (src/chunking.rs:65-74)
// on rayon's pool (:340-368).
//
// SHA-256 is Merkle-Damgard: a chunk's 64-byte blocks are strictly serial, so the
// only parallelism is across chunks.  One lane owns one chunk; its blocks are
// loaded as aligned dwords and realigned + byte-swapped with one v_perm_b32 per
// word (chunk offsets are arbitrary bytes).  Rotates are v_alignbit_b32.
#include "common.h"

namespace cg {

static constexpr uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr32(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
// gfx950 v_bitop3_b32: one instruction for any 3-input bitwise function
// (truth-table byte: S0 = 0xF0, S1 = 0xCC, S2 = 0xAA).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) {
    return __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);
}
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
__device__ __forceinline__ uint32_t add3(uint32_t a, uint32_t b, uint32_t c) { return a + b + c; }

#define SHA_S0(a) xor3(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22))
#define SHA_S1(e) xor3(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25))
#define SHA_s0(x) xor3(rotr32(x, 7), rotr32(x, 18), (x) >> 3)
#define SHA_s1(x) xor3(rotr32(x, 17), rotr32(x, 19), (x) >> 10)

// ---------------------------------------------------------------------------
// Producer/consumer SHA-256.  A chunk's compressions are a serial chain, and one
// wave issues one VALU instruction every ~4 cycles (MI355X_MICROARCH.md, "vector-
// instruction ISSUE cost"), so the chain's speed is set by the instructions ONE wave
// must issue per block.  Each workgroup therefore pairs two waves on the same 64
// chunks (one chunk per lane):
//   wave 0 (producer): loads the block, realigns + byte-swaps it (v_perm_b32),
//          builds the final padded block(s), expands the 64-word message schedule
//          (W[t] + K[t]) into a ring of PC_RING LDS slots (one row per lane);
//   wave 1 (consumer): runs only the 64 rounds (14 VALU each), reading the next
//          block's words from LDS into registers half-way through the current one.
// Two LDS counters (s_ready, s_done) with workgroup-scope acquire/release hand the
// slots over; no barrier per block.  The consumer issues ~900 VALU per block instead
// of ~1,400.
// ---------------------------------------------------------------------------
#define PC_ROW 68u  // 64 words + 4 pad per lane: 16 consecutive lanes' 16-B accesses hit distinct banks

// wv = W[i] + K[i], pre-added by the producer (no constant operand in the round)
#define SHA_RNDW(a, b, c, d, e, f, g, h, i, wv)                                  \
    {                                                                            \
        const uint32_t t1 = add3(h, (wv), ch(e, f, g)) + SHA_S1(e);             \
        d += t1;                                                                 \
        h = add3(t1, SHA_S0(a), maj(a, b, c));                                   \
    }

__device__ __forceinline__ uint32_t lds_load_acquire(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_release(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void load_w(uint4 (&w)[16], const uint32_t *row) {
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = *reinterpret_cast<const uint4 *>(row + 4 * i);
}

#define SHA_8RND(i, W)                                       \
    {                                                        \
        const uint4 wa = W[(i) / 4], wb = W[(i) / 4 + 1];    \
        SHA_RNDW(a, b, c, d, e, f, g, h, (i) + 0, wa.x);     \
        SHA_RNDW(h, a, b, c, d, e, f, g, (i) + 1, wa.y);     \
        SHA_RNDW(g, h, a, b, c, d, e, f, (i) + 2, wa.z);     \
        SHA_RNDW(f, g, h, a, b, c, d, e, (i) + 3, wa.w);     \
        SHA_RNDW(e, f, g, h, a, b, c, d, (i) + 4, wb.x);     \
        SHA_RNDW(d, e, f, g, h, a, b, c, (i) + 5, wb.y);     \
        SHA_RNDW(c, d, e, f, g, h, a, b, (i) + 6, wb.z);     \
        SHA_RNDW(b, c, d, e, f, g, h, a, (i) + 7, wb.w);     \
    }

// 64 rounds on `cur`; half-way through, once the producer has published block
// `knext`, the next block's schedule is read from LDS into `nxt`, so its LDS
// latency hides under the remaining 32 rounds.
__device__ __forceinline__ void sha_rounds_pf(uint32_t st[8], const uint4 (&cur)[16], uint4 (&nxt)[16],
                                              const uint32_t *next_row, uint32_t knext, bool prefetch,
                                              const uint32_t *ready, bool active) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    // readiness probe issued now, consumed after 32 rounds: its LDS latency is hidden
    const uint32_t r0 = __hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    SHA_8RND(0, cur);
    SHA_8RND(8, cur);
    SHA_8RND(16, cur);
    SHA_8RND(24, cur);
    if (prefetch) {
        if (__builtin_expect(r0 <= knext, 0))
            while (lds_load_acquire(ready) <= knext) __builtin_amdgcn_s_sleep(1);
        load_w(nxt, next_row);
    }
    SHA_8RND(32, cur);
    SHA_8RND(40, cur);
    SHA_8RND(48, cur);
    SHA_8RND(56, cur);
    // lanes past their last block computed on stale words: keep their state (select,
    // not a branch, so the round code always runs under a full exec mask; the empty asm
    // stops the compiler from sinking the last rounds under an `active` branch)
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    st[0] = active ? st[0] + a : st[0];
    st[1] = active ? st[1] + b : st[1];
    st[2] = active ? st[2] + c : st[2];
    st[3] = active ? st[3] + d : st[3];
    st[4] = active ? st[4] + e : st[4];
    st[5] = active ? st[5] + f : st[5];
    st[6] = active ? st[6] + g : st[6];
    st[7] = active ? st[7] + h : st[7];
}

// Expand w[0..15] into the full schedule and store W[t] + K[t] for all 64 words to
// `row` (LDS): the consumer's round then has no constant operand to materialise.
__device__ __forceinline__ void sha_schedule_store(uint32_t w[16], uint32_t *row) {
#pragma unroll
    for (int i = 0; i < 16; i += 4)
        *reinterpret_cast<uint4 *>(row + i) = make_uint4(w[i] + SHA_K[i], w[i + 1] + SHA_K[i + 1],
                                                         w[i + 2] + SHA_K[i + 2], w[i + 3] + SHA_K[i + 3]);
#pragma unroll
    for (int t = 16; t < 64; t += 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int u = t + j;
            w[u & 15] = add3(w[u & 15], SHA_s0(w[(u - 15) & 15]), w[(u - 7) & 15]) + SHA_s1(w[(u - 2) & 15]);
        }
        *reinterpret_cast<uint4 *>(row + t) =
            make_uint4(w[t & 15] + SHA_K[t], w[(t + 1) & 15] + SHA_K[t + 1], w[(t + 2) & 15] + SHA_K[t + 2],
                       w[(t + 3) & 15] + SHA_K[t + 3]);
    }
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d, 64));
    return v;
}

#define PC_RING 4u  // LDS schedule slots: the producer runs up to 4 blocks ahead

// diag (optional, nullptr in production): per workgroup {producer spin, producer
// total, consumer spin, consumer total} in shader clocks (s_memtime).
__global__ __launch_bounds__(128) void k_sha256(const uint8_t *__restrict__ data, const uint64_t *__restrict__ abs,
                                               const DescRaw *__restrict__ desc, const uint64_t *__restrict__ total_p,
                                               uint64_t max_chunks, const uint32_t *__restrict__ order,
                                               uint8_t *__restrict__ hash_base, size_t stride,
                                               unsigned long long *__restrict__ diag, uint32_t mode) {
    unsigned long long t_start = diag ? __builtin_amdgcn_s_memtime() : 0ull, t_spin = 0;
    __shared__ __attribute__((aligned(16))) uint32_t sW[PC_RING][64 * PC_ROW];
    __shared__ uint32_t s_ready, s_done;  // blocks filled by the producer / consumed by the consumer
    const uint32_t lane = threadIdx.x & 63u;
    const bool producer = threadIdx.x < 64;
    const uint64_t g = (uint64_t)blockIdx.x * 64 + lane;
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    if ((uint64_t)blockIdx.x * 64 >= total) return;  // whole workgroup idle (uniform)
    if (threadIdx.x == 0) {
        s_ready = 0;
        s_done = 0;
    }
    __syncthreads();
    const bool valid = g < total;
    // lane -> chunk through the length order (longest first, see k_len_hist): the 64
    // chunks of a wave have nearly equal block counts and the longest start first
    const uint64_t ci = valid ? (order ? (uint64_t)order[g] : g) : 0;
    const uint64_t len = valid ? desc[ci].length : 0;
    const uint64_t nb = len >> 6;
    const uint32_t rem = (uint32_t)(len & 63u);
    const uint32_t nbt = valid ? (uint32_t)(nb + (rem < 56 ? 1 : 2)) : 0u;  // blocks incl. padding
    // identical in both waves (same 64 chunks); scalar, so the block loops are uniform
    const uint32_t NB = __builtin_amdgcn_readfirstlane(wave_max_u32(nbt));

    if (producer) {
        const uint8_t *p = data + (valid ? abs[ci] : 0);
        const uint32_t shift = (uint32_t)((uintptr_t)p & 3u);
        const uint32_t *base = reinterpret_cast<const uint32_t *>(p - shift);
        const uint32_t sel = (shift << 24) | ((shift + 1) << 16) | ((shift + 2) << 8) | (shift + 3);
        const uint64_t bits = len << 3;
        // One block buffer: block k+1's bytes are requested as soon as block k's words
        // have been realigned out of it, so a whole schedule computation (~2,000
        // cycles) covers their latency and the only loads in flight at the next
        // realign are exactly the ones it needs (vmcnt(0) is then the precise wait).
        uint32_t d[17];
        auto load_full = [&](uint64_t k) {
            const uint32_t *q = base + 16 * k;
#pragma unroll
            for (int i = 0; i < 16; ++i) d[i] = q[i];
            // dword 16 holds chunk bytes whenever shift != 0; for shift == 0 the realign
            // ignores it, so re-read dword 15 (unconditional: keeps vmcnt tracking exact)
            d[16] = q[shift ? 16 : 15];
        };
        auto produce = [&](uint32_t k) {
            // wait for a free slot (wave-uniform spin on an LDS counter)
            if ((int)(k - lds_load_acquire(&s_done)) >= (int)PC_RING) {
                const unsigned long long t0 = diag ? __builtin_amdgcn_s_memtime() : 0ull;
                while ((int)(k - lds_load_acquire(&s_done)) >= (int)PC_RING) __builtin_amdgcn_s_sleep(1);
                if (diag) t_spin += __builtin_amdgcn_s_memtime() - t0;
            }
            if (k < nbt) {
                uint32_t w[16];
                if (k < nb) {
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] = __builtin_amdgcn_perm(d[i + 1], d[i], sel);
                    // keep the realign ahead of the reload so the loads land in d's own
                    // registers (no copies, no wait); the last full block re-reads itself
                    __builtin_amdgcn_sched_barrier(0);
                    load_full(k + 1 < nb ? k + 1 : k);
                } else if (k == nb) {  // tail bytes, 0x80, zeros, [length]
                    const uint32_t *q = base + 16 * nb;
                    const uint8_t *endp = p + len;
                    uint32_t dw[17];
#pragma unroll
                    for (int i = 0; i < 17; ++i)
                        dw[i] = (reinterpret_cast<const uint8_t *>(q + i) < endp) ? q[i] : 0u;
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const uint32_t v = __builtin_amdgcn_perm(dw[i + 1], dw[i], sel);
                        const int r = (int)rem - 4 * i;
                        w[i] = r >= 4 ? v
                                      : (r < 0 ? 0u
                                               : ((r ? (v & (0xffffffffu << (32 - 8 * r))) : 0u) |
                                                  (0x80u << (24 - 8 * r))));
                    }
                    if (rem < 56) {
                        w[14] = (uint32_t)(bits >> 32);
                        w[15] = (uint32_t)bits;
                    }
                } else {  // second padding block
#pragma unroll
                    for (int i = 0; i < 14; ++i) w[i] = 0u;
                    w[14] = (uint32_t)(bits >> 32);
                    w[15] = (uint32_t)bits;
                }
                sha_schedule_store(w, &sW[k % PC_RING][lane * PC_ROW]);
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's schedule writes landed
            if (lane == 0) lds_store_release(&s_ready, k + 1);
        };
        if (mode == 1) {  // diag: no producer work, consumer rounds on stale schedules
            if (lane == 0) lds_store_release(&s_ready, 0xffffffffu);
        } else {
            if (nb > 0) load_full(0);
            for (uint32_t k = 0; k < NB; ++k) produce(k);
        }
        if (diag && lane == 0) {
            diag[4 * blockIdx.x + 0] = t_spin;
            diag[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memtime() - t_start;
        }
    } else {
        uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                          0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        uint4 wA[16], wB[16];
        if (lds_load_acquire(&s_ready) == 0) {
            const unsigned long long t0 = diag ? __builtin_amdgcn_s_memtime() : 0ull;
            while (lds_load_acquire(&s_ready) == 0) __builtin_amdgcn_s_sleep(1);
            if (diag) t_spin += __builtin_amdgcn_s_memtime() - t0;
        }
        load_w(wA, &sW[0][lane * PC_ROW]);
        // Every lane runs every block's rounds (lanes whose chunk is done work on stale
        // words and keep their state by select): with part of the wave masked off, the
        // dependent round chain ran up to 1.7x slower per round on gfx950.
        for (uint32_t k = 0; k < NB; k += 2) {
            // block k from wA, block k+1's schedule prefetched into wB
            sha_rounds_pf(st, wA, wB, &sW[(k + 1) % PC_RING][lane * PC_ROW], k + 1, k + 1 < NB && mode != 2,
                          &s_ready, k < nbt);
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
            if (lane == 0) lds_store_release(&s_done, k + 1);
            if (k + 1 >= NB) break;
            sha_rounds_pf(st, wB, wA, &sW[(k + 2) % PC_RING][lane * PC_ROW], k + 2, k + 2 < NB && mode != 2,
                          &s_ready, k + 1 < nbt);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            if (lane == 0) lds_store_release(&s_done, k + 2);
        }
        if (diag && lane == 0) {
            diag[4 * blockIdx.x + 2] = t_spin;
            diag[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime() - t_start;
        }
        if (valid) {
            uint4 *o = reinterpret_cast<uint4 *>(hash_base + ci * stride);
            o[0] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                              __builtin_bswap32(st[3]));
            o[1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                              __builtin_bswap32(st[7]));
        }
    }
}

// ---------------------------------------------------------------------------
// Length order.  A wave lives as long as its longest chunk, and a batch's digest
// stage as long as its longest chunk, so lanes are handed chunks in descending
// block count: a counting sort on SHA_NBKT buckets of (blocks >> shift), each
// workgroup aggregating in LDS before touching the global counters.  The order
// inside a bucket is arbitrary (atomics); digests land at their chunk's own index,
// so results do not depend on it.
// ---------------------------------------------------------------------------
#define SHA_NBKT 1024u

__device__ __forceinline__ uint32_t len_bucket(uint64_t len, uint32_t shift) {
    const uint64_t nb = (len + 72) >> 6;  // blocks including padding
    const uint64_t b = nb >> shift;
    return SHA_NBKT - 1u - (uint32_t)(b < SHA_NBKT - 1 ? b : SHA_NBKT - 1);  // descending
}

__global__ __launch_bounds__(256) void k_len_hist(const DescRaw *__restrict__ desc, const uint64_t *__restrict__ total_p,
                                                 uint64_t max_chunks, uint32_t shift, uint32_t *__restrict__ bkt) {
    __shared__ uint32_t h[SHA_NBKT];
    for (uint32_t i = threadIdx.x; i < SHA_NBKT; i += 256) h[i] = 0;
    __syncthreads();
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (g < total) atomicAdd(&h[len_bucket(desc[g].length, shift)], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < SHA_NBKT; i += 256)
        if (h[i]) atomicAdd(&bkt[i], h[i]);
}

// one workgroup: bkt[i] <- exclusive prefix sum of the bucket counts
__global__ __launch_bounds__(SHA_NBKT) void k_len_base(uint32_t *__restrict__ bkt) {
    __shared__ uint32_t wsum[SHA_NBKT / 64];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint32_t v = bkt[t];
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if ((int)lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t off = 0;
    for (uint32_t k = 0; k < w; ++k) off += wsum[k];
    bkt[t] = off + x - v;
}

__global__ __launch_bounds__(256) void k_len_scatter(const DescRaw *__restrict__ desc,
                                                    const uint64_t *__restrict__ total_p, uint64_t max_chunks,
                                                    uint32_t shift, uint32_t *__restrict__ bkt,
                                                    uint32_t *__restrict__ order) {
    __shared__ uint32_t h[SHA_NBKT];
    __shared__ uint32_t base[SHA_NBKT];
    for (uint32_t i = threadIdx.x; i < SHA_NBKT; i += 256) h[i] = 0;
    __syncthreads();
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t b = 0, r = 0;
    if (g < total) {
        b = len_bucket(desc[g].length, shift);
        r = atomicAdd(&h[b], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < SHA_NBKT; i += 256)
        if (h[i]) base[i] = atomicAdd(&bkt[i], h[i]);
    __syncthreads();
    if (g < total) order[base[b] + r] = (uint32_t)g;
}

size_t sha256_order_tmp_elems(uint64_t max_chunks) { return max_chunks + SHA_NBKT + 64; }

unsigned long long *g_sha_diag = nullptr;  // set by cg_diag_sha_stats (diagnostics only)
uint32_t g_sha_mode = 0;                    // set by cg_diag_sha_mode (diagnostics only; 0 = product)

void launch_sha256(const uint8_t *d_data, const uint64_t *d_abs, const void *d_desc, const uint64_t *d_total,
                   uint64_t max_chunks, uint64_t max_len, uint32_t *d_order_tmp, uint8_t *d_hash_base,
                   size_t hash_stride, hipStream_t st) {
    if (max_chunks == 0) return;
    const uint32_t nwg = (uint32_t)((max_chunks + 63) / 64);
    const uint32_t *order = nullptr;
    if (d_order_tmp && nwg > 1) {  // one workgroup has nothing to balance
        uint32_t shift = 0;
        while ((((max_len + 72) >> 6) >> shift) >= SHA_NBKT - 1) ++shift;
        uint32_t *bkt = d_order_tmp, *ord = d_order_tmp + SHA_NBKT;
        const uint32_t nb = (uint32_t)((max_chunks + 255) / 256);
        (void)hipMemsetAsync(bkt, 0, SHA_NBKT * sizeof(uint32_t), st);
        hipLaunchKernelGGL(k_len_hist, dim3(nb), dim3(256), 0, st, (const DescRaw *)d_desc, d_total, max_chunks,
                           shift, bkt);
        hipLaunchKernelGGL(k_len_base, dim3(1), dim3(SHA_NBKT), 0, st, bkt);
        hipLaunchKernelGGL(k_len_scatter, dim3(nb), dim3(256), 0, st, (const DescRaw *)d_desc, d_total,
                           max_chunks, shift, bkt, ord);
        order = ord;
    }
    // Latency-bound batches (no more workgroups than CUs): pad the LDS request past half
    // a CU's 160 KiB so no two workgroups share a CU, and a consumer wave never shares a
    // SIMD with another workgroup's wave (which costs it 20-90 % per round).
    const size_t pad = nwg <= 256 ? 16384 : 0;
    hipLaunchKernelGGL(k_sha256, dim3(nwg), dim3(128), pad, st, d_data, d_abs,
                       (const DescRaw *)d_desc, d_total, max_chunks, order, d_hash_base, hash_stride, g_sha_diag,
                       g_sha_mode);
}

}  // namespace cg
