// sha256.hip -- K3: per-chunk SHA-256 (FIPS 180-4), replacing sha256_hash_raw
// (src/hashing.rs:36-44) called per chunk by compute_hash (src/chunking.rs:65-74)
// on rayon's pool (:340-368).
//
// SHA-256 is Merkle-Damgard: a chunk's 64-byte blocks are strictly serial, so the
// only parallelism is across chunks.  One lane owns one chunk; its blocks are
// loaded as aligned dwords and realigned + byte-swapped with one v_perm_b32 per
// word (chunk offsets are arbitrary bytes).  Rotates are v_alignbit_b32.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstddef>

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
// 64 words + 4 pad per row.  One-lane rows: every ds_write_b128 group (8 contiguous lanes,
// bank (a/4) mod 32) and ds_read_b128 group (16 lanes, mod 64) hits distinct banks.  Split
// rows (lo half at word 0, hi at 32) read conflict-free too (split_row), but the pair
// producer's stores are 2-way: lanes 0-3 (lo) and 4-7 (hi) of a store group write the
// same rows, and words 32 apart share a bank modulo 32.  Measured on config 4: conflict
// cycles 0.54 of the LDS-array cycles, yet SQ_WAIT_INST_LDS 0.3 % of wave cycles -- not a
// bound (profiles/r06_v9_pmc_c4_prod.json).
#define PC_ROW 68u

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

__device__ __forceinline__ unsigned long long wait_ready(const uint32_t *ctr, uint32_t k, bool timed);

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
template <bool SEL>
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
    if (__builtin_expect(prefetch && r0 <= knext, 0)) wait_ready(ready, knext, false);
    load_w(nxt, next_row);  // unconditional, as in sha_rounds_split
    SHA_8RND(32, cur);
    SHA_8RND(40, cur);
    SHA_8RND(48, cur);
    SHA_8RND(56, cur);
    // lanes past their last block computed on stale words: keep their state (select,
    // not a branch, so the round code always runs under a full exec mask; the empty asm
    // stops the compiler from sinking the last rounds under an `active` branch)
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
    if (!SEL) active = true;  // every valid lane is inside its chunk (k_sha256's main loop)
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

// LDS schedule ring.  Split (quad / pair) workgroups hold at most 32 chunk rows and use
// PC_RING slots of 32 rows; one-lane workgroups hold 64 rows and use PC_RING1 slots of 64
// rows (68 KiB: two workgroups per CU, one wave per SIMD).  Round 6
// measured smaller one-lane rings for more workgroups per CU: a one-lane consumer holds
// block k + 1's words in registers from the middle of block k on, so with early release
// (SHA_EARLY: it frees both slots at the end of block k) three slots give the producer the
// slack four give without it, at 51 KiB (three workgroups per CU), and two slots fit four.
// None was faster: config 4 793 (3 slots, 3 per CU) / 800 (2 slots, 4 per CU) against 802
// GiB/s (4 slots, 2 per CU), config 5 582 / 620 against 698-710, config 2's merged digest
// 83-86 ms against 69.4 ms; at 2 per CU the 3-slot ring lost 20 % (c4 642)
// (profiles/r06_v8_ring_occupancy.txt, PMC in r06_v9_pmc_c4_*.json).  So the product
// keeps 4 slots; CG_PC_RING1 / CG_SHA_EARLY build the variants (scripts/build_variant.sh).
#define PC_RING 4u  // split tiers: the producer runs up to PC_RING blocks ahead
#ifndef CG_PC_RING1
#define CG_PC_RING1 4u
#endif
#define PC_RING1 CG_PC_RING1  // one-lane tier
#ifndef CG_SHA_EARLY
#define CG_SHA_EARLY 0u
#endif
#define SHA_EARLY CG_SHA_EARLY  // one-lane consumer releases block k + 1's slot at the end of block k
#define SPL_SLOT (32u * PC_ROW)
#define ONE_SLOT (64u * PC_ROW)
#define PC_LDS_WORDS (PC_RING * SPL_SLOT > PC_RING1 * ONE_SLOT ? PC_RING * SPL_SLOT : PC_RING1 * ONE_SLOT)

// Spin guard: no legitimate wait for a ring slot lasts more than a few blocks
// (~10^4 clocks); after `limit` sleeps (2^26 by default, ~2 s) a wait gives up so a
// broken hand-off cannot hang the GPU, and raises the workgroup's timeout flag: the
// kernel then reports the launch as failed (k_sha256 -> *err) and the host returns
// CG_E_IO instead of digests computed from a stale ring slot.
// The workgroup's hand-off words live in LDS in this order; the waits find the flag
// and the limit from the counter they poll.
enum { SY_READY = 0, SY_DONE = 1, SY_TIMEOUT = 2, SY_LIMIT = 3, SY_N = 4 };

__device__ __forceinline__ bool spin_expired(const uint32_t *sync, uint32_t &it) {
    if (++it <= sync[SY_LIMIT]) {
        __builtin_amdgcn_s_sleep(1);
        return false;
    }
    __hip_atomic_store(const_cast<uint32_t *>(sync) + SY_TIMEOUT, 1u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
    return true;
}

// Wait until `*ctr` moved past `k` (consumer: producer filled slot k) -- `ready`
// form -- or until slot k is free (producer: consumer released k - R, R = the ring's slots).
__device__ __forceinline__ unsigned long long wait_ready(const uint32_t *ctr, uint32_t k, bool timed) {
    if (lds_load_acquire(ctr) > k) return 0;
    const unsigned long long t0 = timed ? __builtin_amdgcn_s_memtime() : 0ull;
    const uint32_t *sync = ctr - SY_READY;
    uint32_t it = 0;
    while (lds_load_acquire(ctr) <= k && !spin_expired(sync, it)) {
    }
    return timed ? __builtin_amdgcn_s_memtime() - t0 : 0ull;
}
template <uint32_t R>
__device__ __forceinline__ unsigned long long wait_slot(const uint32_t *done, uint32_t k, bool timed) {
    if ((int)(k - lds_load_acquire(done)) < (int)R) return 0;
    const unsigned long long t0 = timed ? __builtin_amdgcn_s_memtime() : 0ull;
    const uint32_t *sync = done - SY_DONE;
    uint32_t it = 0;
    while ((int)(k - lds_load_acquire(done)) >= (int)R && !spin_expired(sync, it)) {
    }
    return timed ? __builtin_amdgcn_s_memtime() - t0 : 0ull;
}
// This wave's schedule writes for block k have landed: publish k + 1.
// Every lane stores the same value (one ds_write, no exec-mask change around it).
__device__ __forceinline__ void publish(uint32_t *ready, uint32_t k, uint32_t lane) {
    (void)lane;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    lds_store_release(ready, k + 1);
}

// Words of a chunk's tail block (k == nb: tail bytes, 0x80, zeros, [bit length]) or
// of its second padding block (k == nb + 1).  Loads stop at the chunk's end.
__device__ __forceinline__ void sha_pad_words(uint32_t w[16], const uint8_t *p, const uint32_t *base, uint32_t sel,
                                              uint64_t len, uint64_t k) {
    const uint64_t nb = len >> 6;
    const uint32_t rem = (uint32_t)(len & 63u);
    const uint64_t bits = len << 3;
    if (k == nb) {
        const uint32_t *q = base + 16 * nb;
        const uint8_t *endp = p + len;
        uint32_t dw[17];
#pragma unroll
        for (int i = 0; i < 17; ++i) dw[i] = (reinterpret_cast<const uint8_t *>(q + i) < endp) ? q[i] : 0u;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t v = __builtin_amdgcn_perm(dw[i + 1], dw[i], sel);
            const int r = (int)rem - 4 * i;
            w[i] = r >= 4 ? v
                          : (r < 0 ? 0u
                                   : ((r ? (v & (0xffffffffu << (32 - 8 * r))) : 0u) | (0x80u << (24 - 8 * r))));
        }
        if (rem < 56) {
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 14; ++i) w[i] = 0u;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
    }
}

__device__ __forceinline__ uint32_t perm_sel(uint32_t shift) {
    return (shift << 24) | ((shift + 1) << 16) | ((shift + 2) << 8) | (shift + 3);
}

// Producer wave of a one-lane-per-chunk workgroup: for k = 0..NB-1 wait for a free
// ring slot, load + realign + pad block k of this lane's chunk, expand its schedule
// (W[t] + K[t], 64 words) into row `row` of slot k % PC_RING1, publish.
__device__ unsigned long long sha_produce(const uint8_t *p, uint64_t len, uint32_t nbt, uint32_t NB,
                                          uint32_t (*sW)[ONE_SLOT], uint32_t row, uint32_t lane,
                                          uint32_t *s_ready, const uint32_t *s_done, bool timed) {
    unsigned long long t_spin = 0;
    const uint64_t nb = len >> 6;
    const uint32_t shift = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *base = reinterpret_cast<const uint32_t *>(p - shift);
    const uint32_t sel = perm_sel(shift);
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
    if (nb > 0) load_full(0);
    for (uint32_t k = 0; k < NB; ++k) {
        t_spin += wait_slot<PC_RING1>(s_done, k, timed);
        if (k < nbt) {
            uint32_t w[16];
            if (k < nb) {
#pragma unroll
                for (int i = 0; i < 16; ++i) w[i] = __builtin_amdgcn_perm(d[i + 1], d[i], sel);
                // keep the realign ahead of the reload so the loads land in d's own
                // registers (no copies, no wait); the last full block re-reads itself
                __builtin_amdgcn_sched_barrier(0);
                load_full(k + 1 < nb ? k + 1 : k);
            } else {
                sha_pad_words(w, p, base, sel, len, k);
            }
            sha_schedule_store(w, &sW[k % PC_RING1][row * PC_ROW]);
        }
        publish(s_ready, k, lane);
    }
    return t_spin;
}

// ---------------------------------------------------------------------------
// Split-lane workgroups: ONE chunk per PAIR of lanes.
//
// A batch's digest stage lasts as long as its longest chunk, whose 64 rounds per
// block are a chain that one wave issues at ~4.2 clocks per VALU instruction: the
// chain's instruction count per round is the whole cost.  The longest chunks
// therefore run with each round spread over two lanes 4 apart in a DPP row
// ("lo" = banks 0/2, "hi" = banks 1/3).  lo holds e,f,g,h and hi holds a,b,c,d in
// the same four registers X0..X3 (newest first), so one instruction stream
// computes both halves of the round:
//   r1..r3 = rotations of X0       per-lane amounts 6/11/25 (lo), 2/13/22 (hi)
//   x      = X0 ^ (X2 & LM)        LM = 0 (lo), ~0 (hi): e (lo), a^c (hi)
//   S      = r1 ^ r2 ^ r3          Sigma1(e) (lo), Sigma0(a) (hi)
//   F      = x ? X1 : X2           Ch(e,f,g) (lo), Maj(a,b,c) = (a^c) ? b : c (hi)
//   P      = Z + S + F             T1 with Z = h + W[t]+K[t] (lo), T2 with Z = 0 (hi)
//   X3    <- P + d                 lo lanes; d = hi's X3 through DPP row_shl:4 -> new e
//   Z     <- X2 + W[t+1]+K[t+1]    lo lanes (next round's h is this round's g)
//   X3    <- P + T1                hi lanes; T1 = lo's P through DPP row_shr:4 -> new a
// 10 VALU per round instead of 14.  The three partial writes are DPP bank masks
// (0x5 lo, 0xA hi): no exec-mask change.  Every DPP source was written at least two
// instructions earlier (the gfx9 VALU-write -> DPP-read hazard), so the rounds need
// no s_nop.  Per block the pair reads the schedule by parity (see
// sha_produce_pair): lo lanes hold the even words, hi lanes the odd ones, and the
// Z step takes W[t+1] from its own registers (t+1 even) or from hi's through DPP.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t split_slot(uint32_t lane) {
    return ((lane >> 4) << 3) | (((lane >> 3) & 1u) << 2) | (lane & 3u);
}
// LDS row of chunk slot j: rows 8..15 of each 16 swapped in halves, so the 16 lanes
// of every ds_read_b128 lane group (lo at word 0, hi at word 32 of a row) start on
// 16 distinct 4-bank quads.
__device__ __forceinline__ uint32_t split_row(uint32_t j) { return j ^ ((j >> 1) & 4u); }

struct SplitLane {
    uint32_t sh1, sh2, sh3, lm;  // rotation amounts, Maj-select mask
};

template <int I>
__device__ __forceinline__ uint32_t w_at(const uint4 (&W)[8]) {
    if constexpr ((I & 3) == 0)
        return W[I >> 2].x;
    else if constexpr ((I & 3) == 1)
        return W[I >> 2].y;
    else if constexpr ((I & 3) == 2)
        return W[I >> 2].z;
    else
        return W[I >> 2].w;
}

// Every instruction of a round is 8 bytes; the s_nop hipcc puts between asm statements
// (4 bytes) would leave every other 8-round statement at 4 mod 8 -- so each starts on an
// 8-byte boundary (one more s_nop when needed).
#ifndef CG_SHA_ALIGN
#define CG_SHA_ALIGN 1
#endif
#if CG_SHA_ALIGN
#define RALIGN ".p2align 3\n\t"
#else
#define RALIGN ""
#endif

// One split round as asm text, registers named by role: A = X0 (newest) .. D = X3;
// the new X0 is written into D.  ZOP prepares the next round's Z.
#define SR(A, B, C, D, ZOP)                                                               \
    "v_alignbit_b32 %[r1], %[" #A "], %[" #A "], %[s1]\n\t"                               \
    "v_alignbit_b32 %[r2], %[" #A "], %[" #A "], %[s2]\n\t"                               \
    "v_alignbit_b32 %[r3], %[" #A "], %[" #A "], %[s3]\n\t"                               \
    "v_bitop3_b32 %[xx], %[" #A "], %[" #C "], %[lm] bitop3:0x78\n\t"                     \
    "v_bitop3_b32 %[s], %[r1], %[r2], %[r3] bitop3:0x96\n\t"                              \
    "v_bitop3_b32 %[f], %[xx], %[" #B "], %[" #C "] bitop3:0xca\n\t"                      \
    "v_add3_u32 %[p], %[z], %[s], %[f]\n\t"                                               \
    "v_add_u32_dpp %[" #D "], %[" #D "], %[p] row_shl:4 row_mask:0xf bank_mask:0x5\n\t"   \
    ZOP "v_add_u32_dpp %[" #D "], %[p], %[p] row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
// next word from lo's own register / from hi's register (row_shl:4) / none (the
// s_nop keeps two wait states between p's write and its DPP read)
#define ZLO(C, W) "v_add_u32_dpp %[z], %[" #C "], %[" #W "] quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5\n\t"
#define ZHI(C, W) "v_add_u32_dpp %[z], %[" #W "], %[" #C "] row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
#define ZNONE "s_nop 0\n\t"
#define SR8_HEAD                                                                       \
    RALIGN SR(x0, x1, x2, x3, ZHI(x2, w0)) SR(x3, x0, x1, x2, ZLO(x1, w1)) SR(x2, x3, x0, x1, ZHI(x0, w1)) \
    SR(x1, x2, x3, x0, ZLO(x3, w2)) SR(x0, x1, x2, x3, ZHI(x2, w2)) SR(x3, x0, x1, x2, ZLO(x1, w3)) \
    SR(x2, x3, x0, x1, ZHI(x0, w3))
#define SR8_OUTS                                                                                                 \
    [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [z] "+v"(z), [r1] "=&v"(r1), [r2] "=&v"(r2),     \
        [r3] "=&v"(r3), [xx] "=&v"(xx), [s] "=&v"(s), [f] "=&v"(f), [p] "=&v"(p)
#define SR8_INS                                                                                              \
    [s1] "v"(c.sh1), [s2] "v"(c.sh2), [s3] "v"(c.sh3), [lm] "v"(c.lm), [w0] "v"(w_at<T / 2>(W)),             \
        [w1] "v"(w_at<T / 2 + 1>(W)), [w2] "v"(w_at<T / 2 + 2>(W)), [w3] "v"(w_at<T / 2 + 3>(W))

// Rounds T..T+7 of a block in one asm statement (hipcc pads every asm boundary with
// an s_nop, so one statement per round would cost an 11th issue slot).  Round r's
// Z step needs word r+1: odd -> hi's register (r+1-1)/2, even -> lo's (r+1)/2.
template <int T>
__device__ __forceinline__ void spl_round8(uint32_t &x0, uint32_t &x1, uint32_t &x2, uint32_t &x3, uint32_t &z,
                                           const uint4 (&W)[8], const SplitLane &c) {
    uint32_t r1, r2, r3, xx, s, f, p;
    if constexpr (T + 8 < 64) {
        asm volatile(SR8_HEAD SR(x1, x2, x3, x0, ZLO(x3, w4))
                     : SR8_OUTS
                     : SR8_INS, [w4] "v"(w_at<T / 2 + 4>(W)));
    } else {
        asm volatile(SR8_HEAD SR(x1, x2, x3, x0, ZNONE) : SR8_OUTS : SR8_INS);
    }
}

// Quad variant (8 lanes per chunk): each half of the pair is replicated over the 4
// lanes of a DPP bank (lanes 0-2 compute; lane 3 runs isolated garbage).  Sigma
// then takes ONE v_alignbit (per-lane amount, lanes 0-2) and two v_xor_b32 with
// quad_perm rotations of the three rotations, so a round is 9 VALU.  The other
// steps, the bank masks and the schedule words are those of the pair round.
#define QR(A, B, C, D, ZOP)                                                               \
    "v_alignbit_b32 %[r1], %[" #A "], %[" #A "], %[s1]\n\t"                               \
    "v_bitop3_b32 %[xx], %[" #A "], %[" #C "], %[lm] bitop3:0x78\n\t"                     \
    "v_bitop3_b32 %[f], %[xx], %[" #B "], %[" #C "] bitop3:0xca\n\t"                      \
    "v_xor_b32_dpp %[r2], %[r1], %[r1] quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf\n\t" \
    "v_xor_b32_dpp %[s], %[r1], %[r2] quad_perm:[2,0,1,3] row_mask:0xf bank_mask:0xf\n\t"  \
    "v_add3_u32 %[p], %[z], %[s], %[f]\n\t"                                               \
    "v_add_u32_dpp %[" #D "], %[" #D "], %[p] row_shl:4 row_mask:0xf bank_mask:0x5\n\t"   \
    ZOP "v_add_u32_dpp %[" #D "], %[p], %[p] row_shr:4 row_mask:0xf bank_mask:0xa\n\t"
#define QR8_HEAD                                                                       \
    RALIGN QR(x0, x1, x2, x3, ZHI(x2, w0)) QR(x3, x0, x1, x2, ZLO(x1, w1)) QR(x2, x3, x0, x1, ZHI(x0, w1)) \
    QR(x1, x2, x3, x0, ZLO(x3, w2)) QR(x0, x1, x2, x3, ZHI(x2, w2)) QR(x3, x0, x1, x2, ZLO(x1, w3)) \
    QR(x2, x3, x0, x1, ZHI(x0, w3))
#define QR8_OUTS                                                                                              \
    [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [z] "+v"(z), [r1] "=&v"(r1), [r2] "=&v"(r2),  \
        [xx] "=&v"(xx), [s] "=&v"(s), [f] "=&v"(f), [p] "=&v"(p)
#define QR8_INS                                                                                  \
    [s1] "v"(c.sh1), [lm] "v"(c.lm), [w0] "v"(w_at<T / 2>(W)), [w1] "v"(w_at<T / 2 + 1>(W)),     \
        [w2] "v"(w_at<T / 2 + 2>(W)), [w3] "v"(w_at<T / 2 + 3>(W))

template <int T>
__device__ __forceinline__ void quad_round8(uint32_t &x0, uint32_t &x1, uint32_t &x2, uint32_t &x3, uint32_t &z,
                                            const uint4 (&W)[8], const SplitLane &c) {
    uint32_t r1, r2, xx, s, f, p;
    if constexpr (T + 8 < 64) {
        asm volatile(QR8_HEAD QR(x1, x2, x3, x0, ZLO(x3, w4))
                     : QR8_OUTS
                     : QR8_INS, [w4] "v"(w_at<T / 2 + 4>(W)));
    } else {
        asm volatile(QR8_HEAD QR(x1, x2, x3, x0, ZNONE) : QR8_OUTS : QR8_INS);
    }
}

// Z for round 0 of the next block: h (lo's X3 after the state add) + W[0]+K[0], lo lanes only.
__device__ __forceinline__ void spl_z(uint32_t &z, uint32_t h, uint32_t wv0) {
    asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 quad_perm:[0,1,2,3] row_mask:0xf bank_mask:0x5"
                 : "+v"(z)
                 : "v"(h), "v"(wv0));
}

template <bool QUAD, int T>
__device__ __forceinline__ void round8(uint32_t &x0, uint32_t &x1, uint32_t &x2, uint32_t &x3, uint32_t &z,
                                       const uint4 (&W)[8], const SplitLane &c) {
    if constexpr (QUAD)
        quad_round8<T>(x0, x1, x2, x3, z, W, c);
    else
        spl_round8<T>(x0, x1, x2, x3, z, W, c);
}
#define SPL32(T, W)                                         \
    round8<QUAD, (T)>(x0, x1, x2, x3, z, W, c);             \
    round8<QUAD, (T) + 8>(x0, x1, x2, x3, z, W, c);         \
    round8<QUAD, (T) + 16>(x0, x1, x2, x3, z, W, c);        \
    round8<QUAD, (T) + 24>(x0, x1, x2, x3, z, W, c);

__device__ __forceinline__ void load_w8(uint4 (&w)[8], const uint32_t *row) {
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = *reinterpret_cast<const uint4 *>(row + 4 * i);
}

// 64 split rounds on `cur` (this lane's 32 schedule words); half-way through, once
// the producer has published block `knext`, the next block's words are read into `nxt`.
template <bool QUAD, bool SEL = true>
__device__ __forceinline__ void sha_rounds_split(uint32_t st[4], const uint4 (&cur)[8], uint4 (&nxt)[8],
                                                 const uint32_t *next_row, uint32_t knext, bool prefetch,
                                                 const uint32_t *ready, bool active, const SplitLane &c,
                                                 uint32_t &z) {
    uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
    const uint32_t r0 = __hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    SPL32(0, cur)
    if (__builtin_expect(prefetch && r0 <= knext, 0)) wait_ready(ready, knext, false);
    // unconditional (after the last block it reads a stale ring slot nobody uses): a load
    // inside a branch made the compiler drain lgkmcnt at the join, an LDS round trip per block
    load_w8(nxt, next_row);
    SPL32(32, cur)
    if (!SEL) active = true;  // every valid lane is inside its chunk (split_consumer's main loop)
    st[0] = active ? st[0] + x0 : st[0];
    st[1] = active ? st[1] + x1 : st[1];
    st[2] = active ? st[2] + x2 : st[2];
    st[3] = active ? st[3] + x3 : st[3];
}

// Two blocks of split_consumer's select-free main loop (k even, every valid lane inside
// its chunk): one readiness probe for both (the producer normally runs PC_RING - 1 blocks
// ahead; a stale probe only sends the second block to wait_ready, which re-reads), the
// ring rows addressed by the caller's toggled offsets instead of per-block slot
// arithmetic, and no end-of-chunk guard on the prefetch (the producer publishes ~0 after
// its last block).  A wave issues about one instruction per 4 clocks, so each one dropped
// here counts like a VALU op of the round chain.
template <bool QUAD>
__device__ __forceinline__ void split_pair_main(uint32_t st[4], uint4 (&wA)[8], uint4 (&wB)[8], const uint32_t *rowB,
                                                const uint32_t *rowA, uint32_t k, const uint32_t *ready,
                                                uint32_t *done, uint32_t lane, const SplitLane &c, uint32_t &z) {
    uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
    const uint32_t r0 = __hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    SPL32(0, wA)
    if (__builtin_expect(r0 <= k + 1, 0)) wait_ready(ready, k + 1, false);
    load_w8(wB, rowB);
    SPL32(32, wA)
    st[0] += x0;
    st[1] += x1;
    st[2] += x2;
    st[3] += x3;
    spl_z(z, st[3], wB[0].x);
    publish(done, k, lane);
    x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
    SPL32(0, wB)
    if (__builtin_expect(r0 <= k + 2, 0)) wait_ready(ready, k + 2, false);
    load_w8(wA, rowA);
    SPL32(32, wB)
    st[0] += x0;
    st[1] += x1;
    st[2] += x2;
    st[3] += x3;
    spl_z(z, st[3], wA[0].x);
    publish(done, k + 1, lane);
}

// Producer wave of a split workgroup.  The pair shares the message schedule by
// parity: lo lanes own the even words w[2i], hi lanes the odd words w[2i+1].  In
//   w[t] = s1(w[t-2]) + w[t-16] + (w[t-7] + s0(w[t-15]))
// the first two terms have t's parity (own registers) and the bracket the other
// one: the partner computes X = R[i-3] + s0(R[i-7]) on its own words, which is the
// bracket hi needs at step i (lo's X) and lo needs at step i+1 (hi's X), and hands
// it over in one DPP add.  Each lane expands 24 words instead of 48 and stores its
// 32 (+K) to its half of the chunk's row (lo: words 0-31, hi: 32-63).
__device__ __forceinline__ void sha_schedule_pair_store(const uint32_t R0[8], const uint32_t Kp[32], uint32_t *dst) {
    uint32_t R[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) R[i] = R0[i];
#pragma unroll
    for (int i = 0; i < 8; i += 4)
        *reinterpret_cast<uint4 *>(dst + i) =
            make_uint4(R[i] + Kp[i], R[i + 1] + Kp[i + 1], R[i + 2] + Kp[i + 2], R[i + 3] + Kp[i + 3]);
    uint32_t xprev = R[4] + SHA_s0(R[0]);  // X of step 7 (hi's is what lo needs at step 8)
#pragma unroll
    for (int i = 8; i < 32; ++i) {
        const uint32_t x = R[i - 3] + SHA_s0(R[i - 7]);
        const uint32_t y = SHA_s1(R[i - 1]) + R[i - 8];
        uint32_t r;
        asm volatile(
            "s_nop 1\n\t"
            "v_add_u32_dpp %0, %1, %2 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
            "v_add_u32_dpp %0, %3, %2 row_shr:4 row_mask:0xf bank_mask:0xa"
            : "=&v"(r)
            : "v"(xprev), "v"(y), "v"(x));
        R[i] = r;
        xprev = x;
        if ((i & 3) == 3)
            *reinterpret_cast<uint4 *>(dst + i - 3) =
                make_uint4(R[i - 3] + Kp[i - 3], R[i - 2] + Kp[i - 2], R[i - 1] + Kp[i - 1], R[i] + Kp[i]);
    }
}

__device__ unsigned long long sha_produce_pair(const uint8_t *p, uint64_t len, uint32_t nbt, uint32_t NB,
                                               uint32_t (*sW)[SPL_SLOT], uint32_t row, bool hi, uint32_t lane,
                                               uint32_t *s_ready, const uint32_t *s_done, bool timed) {
    unsigned long long t_spin = 0;
    const uint64_t nb = len >> 6;
    const uint32_t shift = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *base = reinterpret_cast<const uint32_t *>(p - shift);
    const uint32_t sel = perm_sel(shift);
    // hi lanes load from one dword further on: their d[i] is the block's dword i+1,
    // so perm(d[2i+1], d[2i]) is word 2i+1 there and word 2i in lo lanes.  The last
    // load is the block's dword 16 in hi lanes when shift != 0, else a re-read
    // inside the block.
    const uint32_t *mine = base + (hi ? 1 : 0);
    const uint32_t last = (hi && shift == 0) ? 14u : 15u;
    uint32_t d[16];
    auto load_full = [&](uint64_t k) {
        const uint32_t *q = mine + 16 * k;
#pragma unroll
        for (int i = 0; i < 15; ++i) d[i] = q[i];
        d[15] = q[last];
    };
    uint32_t Kp[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) Kp[i] = hi ? SHA_K[2 * i + 1] : SHA_K[2 * i];
    uint32_t *const dst0 = &sW[0][row * PC_ROW + (hi ? 32u : 0u)];
    if (nb > 0) load_full(0);
    for (uint32_t k = 0; k < NB; ++k) {
        t_spin += wait_slot<PC_RING>(s_done, k, timed);
        if (k < nbt) {
            uint32_t R[8];
            if (k < nb) {
#pragma unroll
                for (int i = 0; i < 8; ++i) R[i] = __builtin_amdgcn_perm(d[2 * i + 1], d[2 * i], sel);
                __builtin_amdgcn_sched_barrier(0);
                load_full(k + 1 < nb ? k + 1 : k);
            } else {
                uint32_t w[16];
                sha_pad_words(w, p, base, sel, len, k);
#pragma unroll
                for (int i = 0; i < 8; ++i) R[i] = hi ? w[2 * i + 1] : w[2 * i];
            }
            sha_schedule_pair_store(R, Kp, dst0 + (k % PC_RING) * SPL_SLOT);
        }
        publish(s_ready, k, lane);
    }
    publish(s_ready, 0xfffffffeu, lane);  // ~0: every later block "ready" (split_pair_main's guard-free prefetch)
    return t_spin;
}

// Consumer wave of a pair (QUAD = false: lo/hi = banks 0,2 / 1,3 of a DPP row, one
// lane each) or quad (QUAD = true: the same banks, 4 lanes each) workgroup.
template <bool QUAD>
__device__ void split_consumer(uint32_t (*sW)[SPL_SLOT], uint32_t row, bool hi, uint32_t lane, uint32_t NB,
                               uint32_t NBmin, uint32_t nbt, uint32_t *s_ready, uint32_t *s_done, uint32_t st[4],
                               unsigned long long *t_spin, bool timed) {
    SplitLane c;
    if (QUAD) {  // lanes 0-2 of a bank take one rotation each; lane 3 is idle garbage
        const uint32_t q = lane & 3u;
        c.sh1 = hi ? (q == 0 ? 2u : q == 1 ? 13u : q == 2 ? 22u : 0u) : (q == 0 ? 6u : q == 1 ? 11u : q == 2 ? 25u : 0u);
        c.sh2 = c.sh3 = 0;
    } else {
        c.sh1 = hi ? 2u : 6u;
        c.sh2 = hi ? 13u : 11u;
        c.sh3 = hi ? 22u : 25u;
    }
    c.lm = hi ? 0xffffffffu : 0u;
    asm volatile("" : "+v"(c.sh1), "+v"(c.sh2), "+v"(c.sh3), "+v"(c.lm));
    st[0] = hi ? 0x6a09e667u : 0x510e527fu;
    st[1] = hi ? 0xbb67ae85u : 0x9b05688cu;
    st[2] = hi ? 0x3c6ef372u : 0x1f83d9abu;
    st[3] = hi ? 0xa54ff53au : 0x5be0cd19u;
    uint32_t z = 0;  // stays 0 in hi lanes: every write to it is masked to lo lanes
    uint4 wA[8], wB[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) wA[i] = wB[i] = make_uint4(0u, 0u, 0u, 0u);
    const uint32_t off = row * PC_ROW + (hi ? 32u : 0u);
    if (NB > 0) {
        *t_spin += wait_ready(s_ready, 0, timed);
        load_w8(wA, &sW[0][off]);
        spl_z(z, st[3], wA[0].x);
        // block 0's words are all in before the loop: the compiler's wait for them would
        // otherwise sit at the loop head, an LDS round trip on every iteration
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    }
    uint32_t k = 0;
    // blocks every valid lane's chunk still has: no per-lane select of the state.  Blocks
    // k + 1 and k + 2 sit in ring slots (1, 2) and (3, 0) in turn: each row offset toggles
    // by one subtraction from a constant.
    static_assert(PC_RING == 4, "split_pair_main's slot toggling assumes a 4-slot ring");
    constexpr uint32_t SLOT = SPL_SLOT;
    const uint32_t *ring = &sW[0][0];
    uint32_t oB = off + SLOT, oA = off + 2 * SLOT;
    const uint32_t cB = 2 * off + 4 * SLOT, cA = 2 * off + 2 * SLOT;
    if constexpr (QUAD) {  // (the pair tier measured faster with the per-block body below)
        for (; k + 1 < NBmin; k += 2) {
            split_pair_main<QUAD>(st, wA, wB, ring + oB, ring + oA, k, s_ready, s_done, lane, c, z);
            oB = cB - oB;
            oA = cA - oA;
        }
    } else {
        (void)ring, (void)oB, (void)oA, (void)cB, (void)cA;
        for (; k + 1 < NBmin; k += 2) {
            sha_rounds_split<QUAD, false>(st, wA, wB, &sW[(k + 1) % PC_RING][off], k + 1, k + 1 < NB, s_ready, true,
                                          c, z);
            spl_z(z, st[3], wB[0].x);
            publish(s_done, k, lane);
            sha_rounds_split<QUAD, false>(st, wB, wA, &sW[(k + 2) % PC_RING][off], k + 2, k + 2 < NB, s_ready, true,
                                          c, z);
            spl_z(z, st[3], wA[0].x);
            publish(s_done, k + 1, lane);
        }
    }
    for (; k < NB; k += 2) {
        sha_rounds_split<QUAD>(st, wA, wB, &sW[(k + 1) % PC_RING][off], k + 1, k + 1 < NB, s_ready, k < nbt, c, z);
        spl_z(z, st[3], wB[0].x);
        publish(s_done, k, lane);
        if (k + 1 >= NB) break;
        sha_rounds_split<QUAD>(st, wB, wA, &sW[(k + 2) % PC_RING][off], k + 2, k + 2 < NB, s_ready, k + 1 < nbt, c,
                               z);
        spl_z(z, st[3], wA[0].x);
        publish(s_done, k + 1, lane);
    }
}

// Hardware location of the calling wave (diagnostics): HW_ID | XCC_ID << 32.
__device__ __forceinline__ unsigned long long wave_location() {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    return ((unsigned long long)xcc << 32) | hw;
}

__device__ __forceinline__ void sha_diag_consumer(unsigned long long *diag, unsigned long long t_spin,
                                                  unsigned long long t_start, unsigned long long rt_start) {
    diag[8 * blockIdx.x + 2] = t_spin;
    diag[8 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime() - t_start;
    diag[8 * blockIdx.x + 4] = rt_start;
    diag[8 * blockIdx.x + 5] = __builtin_amdgcn_s_memrealtime();
    diag[8 * blockIdx.x + 6] = wave_location();
}

// Any change to this kernel's source -- even code on a path config 2 never takes -- moves
// the register allocation and scheduling of the pinned round code: measure config 2's
// merged launch against the previous build on the same box (round 6: a fused one-lane
// tier for GPU-filling launches made config 2's launches 69.4 -> 79-94 ms and lost on
// config 4 too; removed).
// Workgroup kinds, longest chunks first (the length order): [0, nquad) take 8 chunks
// on 8 lanes each, [nquad, nquad + npair) 32 chunks on lane pairs, the rest 64
// chunks on one lane each.  The quad and pair kinds share the pair producer.
// diag (optional, nullptr in production, diagnostics build only): per workgroup
// {producer spin, producer total, consumer spin, consumer total} in shader clocks
// (s_memtime), then the consumer's start and end on the 100 MHz global clock
// (s_memrealtime) and where the consumer and the producer wave ran
// (HW_ID | XCC_ID << 32: SIMD, CU, shader array, SE, XCD).
__global__ __launch_bounds__(128) void k_sha256(const uint8_t *__restrict__ data, const uint64_t *__restrict__ abs,
                                               const DescRaw *__restrict__ desc, const uint64_t *__restrict__ total_p,
                                               uint64_t max_chunks, const uint32_t *__restrict__ order,
                                               uint8_t *__restrict__ hash_base, size_t stride,
                                               unsigned long long *__restrict__ diag, uint32_t mode,
                                               uint32_t nquad, uint32_t npair, uint32_t spin_limit,
                                               uint32_t *__restrict__ err, const uint32_t *__restrict__ need,
                                               ShaNotify nt) {
    unsigned long long t_start = diag ? __builtin_amdgcn_s_memtime() : 0ull, t_spin = 0;
    const unsigned long long rt_start = diag ? __builtin_amdgcn_s_memrealtime() : 0ull;
    if (need) {  // latency tiers (k_len_base): no more lanes per chunk than its length needs
        const uint32_t nq = (need[0] + 7u) / 8u;
        if (nq < nquad) nquad = nq;
        const uint32_t rest = need[1] > 8u * nquad ? need[1] - 8u * nquad : 0u;
        const uint32_t np = (rest + 31u) / 32u;
        if (np < npair) npair = np;
    }
    __shared__ __attribute__((aligned(16))) uint32_t sLDS[PC_LDS_WORDS];
    uint32_t(*sW)[ONE_SLOT] = reinterpret_cast<uint32_t(*)[ONE_SLOT]>(sLDS);     // one-lane view
    uint32_t(*sWs)[SPL_SLOT] = reinterpret_cast<uint32_t(*)[SPL_SLOT]>(sLDS);    // split view
    // hand-off words (SY_*): blocks filled by the producer / consumed by the consumer,
    // the spin guard's timeout flag and limit
    __shared__ uint32_t s_sync[SY_N];
    uint32_t &s_ready = s_sync[SY_READY], &s_done = s_sync[SY_DONE];
    const uint32_t lane = threadIdx.x & 63u;
    const bool producer = threadIdx.x < 64;
    const uint32_t b = blockIdx.x;
    const bool quad = b < nquad;
    const bool split = b < nquad + npair;  // quad or pair
    const uint64_t wg_base = quad    ? 8ull * b
                             : split ? 8ull * nquad + 32ull * (b - nquad)
                                     : 8ull * nquad + 32ull * npair + 64ull * (b - nquad - npair);
    const uint32_t wg_chunks = quad ? 8u : split ? 32u : 64u;
    const bool hi = split && ((lane >> 2) & 1u);
    // the producer of a quad or pair workgroup pairs lanes as split_slot does (a quad
    // workgroup uses its first 16 lanes); a quad consumer gives chunk j lanes
    // 16r + 8h + 0..7 with j = 2r + h
    const uint32_t slot = !split ? lane
                          : (quad && !producer) ? (((lane >> 4) << 1) | ((lane >> 3) & 1u))
                                                : split_slot(lane);
    const uint32_t row = split ? split_row(slot) : lane;
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    if (wg_base >= total) return;  // whole workgroup idle (uniform)
    if (threadIdx.x == 0) {
        s_ready = 0;
        s_done = 0;
        s_sync[SY_TIMEOUT] = 0;
        s_sync[SY_LIMIT] = spin_limit;
    }
    __syncthreads();
    const uint64_t g = wg_base + slot;
    const bool valid = slot < wg_chunks && g < total;
    // slot -> chunk through the length order (longest first, see k_len_hist): the
    // chunks of a wave have nearly equal block counts and the longest start first
    const uint64_t ci = valid ? (order ? (uint64_t)order[g] : g) : 0;
    const uint64_t len = valid ? desc[ci].length : 0;
    const uint64_t nb = len >> 6;
    const uint32_t rem = (uint32_t)(len & 63u);
    const uint32_t nbt = valid ? (uint32_t)(nb + (rem < 56 ? 1 : 2)) : 0u;  // blocks incl. padding
    // identical in both waves (same chunks); scalar, so the block loops are uniform
    const uint32_t NB = __builtin_amdgcn_readfirstlane(wave_max_u32(nbt));
    // blocks every valid lane's chunk has (the consumers' select-free main loop)
    const uint32_t NBmin = __builtin_amdgcn_readfirstlane(~wave_max_u32(valid ? ~nbt : 0u));

    if (producer) {
        const uint8_t *p = data + (valid ? abs[ci] : 0);
        if (mode == 1) {  // diag: no producer work, consumer rounds on stale schedules
            if (lane == 0) lds_store_release(&s_ready, 0xffffffffu);
        } else if (split) {
            t_spin = sha_produce_pair(p, len, nbt, NB, sWs, row, hi, lane, &s_ready, &s_done, diag != nullptr);
        } else {
            t_spin = sha_produce(p, len, nbt, NB, sW, row, lane, &s_ready, &s_done, diag != nullptr);
        }
        if (diag && lane == 0) {
            diag[8 * blockIdx.x + 0] = t_spin;
            diag[8 * blockIdx.x + 1] = __builtin_amdgcn_s_memtime() - t_start;
            diag[8 * blockIdx.x + 7] = wave_location();
        }
    } else if (split) {
        uint32_t st[4];
        if (quad)
            split_consumer<true>(sWs, row, hi, lane, NB, NBmin, nbt, &s_ready, &s_done, st, &t_spin, diag != nullptr);
        else
            split_consumer<false>(sWs, row, hi, lane, NB, NBmin, nbt, &s_ready, &s_done, st, &t_spin, diag != nullptr);
        if (diag && lane == 0) sha_diag_consumer(diag, t_spin, t_start, rt_start);
        if (valid && (!quad || (lane & 3u) == 0)) {  // hi: H0..H3 (bytes 0-15), lo: H4..H7 (bytes 16-31)
            uint8_t *hb = nt.dst ? reinterpret_cast<uint8_t *>(nt.dst[ci]) : hash_base + ci * stride;
            uint4 *o = reinterpret_cast<uint4 *>(hb + (hi ? 0 : 16));
            *o = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                            __builtin_bswap32(st[3]));
            if (nt.remain) __threadfence();  // visible device-wide before the member is counted down
        }
    } else {
        uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                          0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        uint4 wA[16], wB[16];
        t_spin += wait_ready(&s_ready, 0, diag != nullptr);
        load_w(wA, &sW[0][lane * PC_ROW]);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): as in split_consumer, keep the wait out of the loop head
        // Every lane runs every block's rounds (lanes whose chunk is done work on stale
        // words and keep their state by select): with part of the wave masked off, the
        // dependent round chain ran up to 1.7x slower per round on gfx950.
        // after block k (and the wait that lands block k + 1's words in registers) both
        // their slots are free: release k + 1 + SHA_EARLY
        uint32_t k = 0;
        for (; k + 1 < NBmin; k += 2) {  // blocks every valid lane's chunk has: no select
            sha_rounds_pf<false>(st, wA, wB, &sW[(k + 1) % PC_RING1][lane * PC_ROW], k + 1, k + 1 < NB && mode != 2,
                                 &s_ready, true);
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
            lds_store_release(&s_done, k + 1 + SHA_EARLY);
            sha_rounds_pf<false>(st, wB, wA, &sW[(k + 2) % PC_RING1][lane * PC_ROW], k + 2, k + 2 < NB && mode != 2,
                                 &s_ready, true);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            lds_store_release(&s_done, k + 2 + SHA_EARLY);
        }
        for (; k < NB; k += 2) {
            // block k from wA, block k+1's schedule prefetched into wB
            sha_rounds_pf<true>(st, wA, wB, &sW[(k + 1) % PC_RING1][lane * PC_ROW], k + 1, k + 1 < NB && mode != 2,
                          &s_ready, k < nbt);
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
            lds_store_release(&s_done, k + 1 + SHA_EARLY);
            if (k + 1 >= NB) break;
            sha_rounds_pf<true>(st, wB, wA, &sW[(k + 2) % PC_RING1][lane * PC_ROW], k + 2, k + 2 < NB && mode != 2,
                          &s_ready, k + 1 < nbt);
            __builtin_amdgcn_s_waitcnt(0xc07f);
            lds_store_release(&s_done, k + 2 + SHA_EARLY);
        }
        if (diag && lane == 0) sha_diag_consumer(diag, t_spin, t_start, rt_start);
        if (valid) {
            uint4 *o = reinterpret_cast<uint4 *>(nt.dst ? reinterpret_cast<uint8_t *>(nt.dst[ci]) : hash_base + ci * stride);
            o[0] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                              __builtin_bswap32(st[3]));
            o[1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                              __builtin_bswap32(st[7]));
            if (nt.remain) __threadfence();  // visible device-wide before the member is counted down
        }
    }
    // both waves are past their last wait: report an expired spin guard (vector store)
    __syncthreads();
    const bool timed_out = __hip_atomic_load(&s_sync[SY_TIMEOUT], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
    if (threadIdx.x == 0 && timed_out) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // per-member completion (ShaNotify): one consumer lane per chunk -- the one-lane tier's
    // own lane, a split chunk's hi lane that stored H0..H3 -- counts its member down once
    // every digest of this workgroup is stored and fenced; the last one out raises the
    // member's host-mapped completion word (system scope, vector store)
    if (nt.remain && !producer && valid && (!split || (hi && (!quad || (lane & 3u) == 0)))) {
        const uint32_t m = nt.member[ci];
        if (timed_out) __hip_atomic_fetch_or(&nt.merr[m], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_fetch_sub(&nt.remain[m], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 1u) {
            const uint32_t e = __hip_atomic_load(&nt.merr[m], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence_system();
            __hip_atomic_store(nt.flag[m], e ? 2u : 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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

// one workgroup: bkt[i] <- exclusive prefix sum of the bucket counts.
// With `need` (latency tiers, k_sha256): need[0] = the chunks longer than quad_pm / 1000 of
// the longest one (in buckets), need[1] = those longer than pair_pm / 1000 of it.  A chunk
// runs on one lane unless its one-lane chain (59.4 clocks per round) would outlast the
// longest chunk's quad chain (37.95), and on a lane pair unless its pair chain (42.2) would
// (DESIGN.md §4 "Latency tiers"): the longest chunk still sets the batch's digest time, and
// the other chunks take 1/8 and 1/2 of the SIMD time a quad would give them.
__global__ __launch_bounds__(SHA_NBKT) void k_len_base(uint32_t *__restrict__ bkt, uint32_t *__restrict__ need,
                                                      uint32_t quad_pm, uint32_t pair_pm) {
    __shared__ uint32_t wsum[SHA_NBKT / 64];
    __shared__ uint32_t s_first, s_need[2];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    if (t == 0) {
        s_first = SHA_NBKT;
        s_need[0] = s_need[1] = 0;
    }
    const uint32_t v = bkt[t];
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if ((int)lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (v) atomicMin(&s_first, t);  // the longest chunk's bucket (buckets descend)
    uint32_t off = 0;
    for (uint32_t k = 0; k < w; ++k) off += wsum[k];
    bkt[t] = off + x - v;
    if (!need) return;
    __syncthreads();
    // bucket value (blocks >> shift) of bucket t is SHA_NBKT - 1 - t; the chunks in buckets
    // above a threshold are a prefix of the order, counted by the inclusive prefix sum
    const uint32_t bmax = SHA_NBKT - 1u - min(s_first, SHA_NBKT - 1u), bv = SHA_NBKT - 1u - t;
    if (bv * 1000u > bmax * quad_pm) atomicMax(&s_need[0], off + x);
    if (bv * 1000u > bmax * pair_pm) atomicMax(&s_need[1], off + x);
    __syncthreads();
    if (t == 0) {
        need[0] = max(s_need[0], 1u);
        need[1] = max(s_need[1], s_need[0]);
    }
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

// Latency tiers (k_len_base), in per-mille of the longest chunk's blocks: a chunk longer
// than quad_pm needs a quad (on a pair it would outlast the longest chunk's quad chain:
// 37.95 / 42.2 = 0.899 of it), one longer than pair_pm at least a pair (on one lane:
// 37.95 / 59.4 = 0.639).  [0] a launch that leaves the chip idle but for its chains:
// a little under those ratios; [1] a launch that fills the GPU (sha256_grid's fill
// tiers, config 4), where one lane's SIMD time is what the others queue behind: above
// them (DESIGN.md §4 "Latency tiers", profiles/r05_v24_v26_tiers_ab.txt).  Test hooks
// cg_test_sha_tiers / cg_test_sha_tiers_fill (quad_pm 0 = off: every chunk on the widest
// tier the grid holds).
uint32_t g_sha_tier_quad_pm[2] = {850, 950};
uint32_t g_sha_tier_pair_pm[2] = {600, 700};

const uint32_t *launch_len_order(const void *d_desc, const uint64_t *d_total, uint64_t max_chunks, uint64_t max_len,
                                 uint32_t *d_order_tmp, hipStream_t st, uint32_t *d_need, uint32_t quad_pm,
                                 uint32_t pair_pm) {
    if (!d_order_tmp || max_chunks == 0) return nullptr;
    uint32_t shift = 0;
    while ((((max_len + 72) >> 6) >> shift) >= SHA_NBKT - 1) ++shift;
    uint32_t *bkt = d_order_tmp, *ord = d_order_tmp + SHA_NBKT;
    const uint32_t nb = (uint32_t)((max_chunks + 255) / 256);
    (void)hipMemsetAsync(bkt, 0, SHA_NBKT * sizeof(uint32_t), st);
    hipLaunchKernelGGL(k_len_hist, dim3(nb), dim3(256), 0, st, (const DescRaw *)d_desc, d_total, max_chunks, shift,
                       bkt);
    hipLaunchKernelGGL(k_len_base, dim3(1), dim3(SHA_NBKT), 0, st, bkt, d_need, quad_pm, pair_pm);
    hipLaunchKernelGGL(k_len_scatter, dim3(nb), dim3(256), 0, st, (const DescRaw *)d_desc, d_total, max_chunks,
                       shift, bkt, ord);
    return ord;
}

#ifdef CG_DIAG
unsigned long long *g_sha_diag = nullptr;  // set by cg_diag_sha_stats (diagnostics build only)
uint32_t g_sha_mode = 0;                    // set by cg_diag_sha_mode (diagnostics build only)
#else
constexpr unsigned long long *g_sha_diag = nullptr;
constexpr uint32_t g_sha_mode = 0;
#endif
// Split-lane workgroups per launch (32 longest chunks each): one per CU.  Test hook
// cg_test_sha_split_max (0 = one lane per chunk everywhere).
uint32_t g_sha_split_max = 256;
// Quad workgroups per launch (8 longest chunks each).  Test hook cg_test_sha_quad_max.
uint32_t g_sha_quad_max = 256;
// Quad and pair workgroups when the batch fills the GPU: enough quads for the longest
// chunks (all 256 would hold back the one-lane workgroups queued behind them) and half
// the pair workgroups of a latency-bound batch -- a pair spends 1.4x the SIMD time of one
// lane per chunk, and in a GPU-filling batch the three tiers end together (DESIGN.md §4,
// config 4: 32 quads / 256 pairs 21.7 ms, 64 / 128 19.9-20.3 ms in the same sweep,
// profiles/r03_v2_diag_sha_tiers_c4.json, r03_v3_...).  Test hook cg_test_sha_quad_fill.
uint32_t g_sha_quad_fill = 64;
uint32_t g_sha_pair_fill = 128;
// Spin-guard limit (sleeps per wait) of the producer/consumer hand-off: test hook
// cg_test_sha_spin_limit.
uint32_t g_sha_spin_limit = 1u << 26;

// Workgroup tiers for a launch of up to max_chunks chunks, `expected` of them
// likely (total bytes / (min + avg)).  A quad workgroup holds a whole workgroup's
// LDS for 8 chunks, so up to 256 quads are used only when the one-lane tier left
// behind them fits in one round of workgroups (<= 256 x 64 chunks); on a batch that
// fills the GPU (config 4) only g_sha_quad_fill of them, for the longest chunks.
uint32_t sha256_grid(uint64_t max_chunks, uint64_t expected, uint32_t *nquad_out, uint32_t *npair_out,
                     bool *fill_out) {
    auto tiers = [&](uint64_t qmax, uint64_t pmax, uint64_t &nq, uint64_t &np) {
        nq = (max_chunks + 7) / 8;
        if (nq > qmax) nq = qmax;
        const uint64_t rest = max_chunks > 8 * nq ? max_chunks - 8 * nq : 0;
        np = (rest + 31) / 32;
        if (np > pmax) np = pmax;
    };
    uint64_t nq, np;
    tiers(g_sha_quad_max, g_sha_split_max, nq, np);
    const bool fill = expected > 8 * nq + 32 * np + 256 * 64;
    if (fill_out) *fill_out = fill;
    if (fill)
        tiers(std::min<uint64_t>(g_sha_quad_max, g_sha_quad_fill), std::min<uint64_t>(g_sha_split_max, g_sha_pair_fill),
              nq, np);
    const uint64_t rest = max_chunks > 8 * nq + 32 * np ? max_chunks - 8 * nq - 32 * np : 0;
    if (nquad_out) *nquad_out = (uint32_t)nq;
    if (npair_out) *npair_out = (uint32_t)np;
    return (uint32_t)(nq + np + (rest + 63) / 64);
}

// Workgroups per CU of a launch with more workgroups than CUs: [0] latency-bound (the
// chip mostly idle but for the chains: merged pipeline groups), [1] GPU-filling (config 4 /
// 5 shapes).  Two: the 4-slot ring (68 KiB) admits no more; a 2- or 3-slot ring at 3-4
// per CU measured equal on config 4 and slower on configs 2 / 5 (DESIGN.md §4 round 6,
// profiles/r06_v8_ring_occupancy.txt).  CHUNKER_AMD_SHA_OCC="latency,fill" (read once;
// A/B) or cg_test_sha_occupancy.
uint32_t g_sha_occ[2] = {0, 0};
static uint32_t sha_wgs_per_cu(bool fill) {
    static const bool init = [] {
        uint32_t a = 2, b = 2;
        if (const char *e = getenv("CHUNKER_AMD_SHA_OCC")) (void)sscanf(e, "%u,%u", &a, &b);
        if (!g_sha_occ[0]) g_sha_occ[0] = std::min(std::max(a, 1u), 4u);
        if (!g_sha_occ[1]) g_sha_occ[1] = std::min(std::max(b, 1u), 4u);
        return true;
    }();
    (void)init;
    return g_sha_occ[fill ? 1 : 0];
}
// Dynamic LDS that holds a CU to `n` workgroups: past 160 KiB / (n + 1) in all.
static size_t lds_pad_for(uint32_t n) {
    constexpr size_t ring_bytes = PC_LDS_WORDS * 4 + 64;  // (+ the hand-off words)
    const size_t want = 163840 / (n + 1) + 1024;
    return want > ring_bytes ? want - ring_bytes : 0;
}

// Shape of this thread's last digest launch (cg_last_sha_tiers): quad, pair and
// one-lane workgroups, dynamic LDS pad bytes.
thread_local uint32_t t_sha_tiers[4];

void launch_sha256(const uint8_t *d_data, const uint64_t *d_abs, const void *d_desc, const uint64_t *d_total,
                   uint64_t max_chunks, uint64_t expected, uint64_t max_len, uint32_t *d_order_tmp,
                   uint8_t *d_hash_base, size_t hash_stride, uint32_t *d_err, hipStream_t st,
                   bool latency_tiers, const ShaNotify *notify) {
    if (max_chunks == 0) return;
    uint32_t nquad = 0, npair = 0;
    bool fill = false;
    const uint32_t nwg = sha256_grid(max_chunks, expected, &nquad, &npair, &fill);
    // one workgroup has nothing to balance
    // latency tiers: k_len_base counts the chunks that need a quad / a pair into the two
    // words after the order (sha256_order_tmp_elems' slack)
    const uint32_t qpm = latency_tiers ? g_sha_tier_quad_pm[fill] : 0u, ppm = g_sha_tier_pair_pm[fill];
    uint32_t *need = max_chunks > 8 && d_order_tmp && qpm ? d_order_tmp + SHA_NBKT + max_chunks : nullptr;
    const uint32_t *order = max_chunks > 8
                                ? launch_len_order(d_desc, d_total, max_chunks, max_len, d_order_tmp, st, need, qpm, ppm)
                                : nullptr;
    // Latency-bound batches (no more workgroups than CUs): pad the LDS request past half
    // a CU's 160 KiB so no two workgroups share a CU, and a consumer wave never shares a
    // SIMD with another workgroup's wave (which costs it 20-90 % per round).  Larger
    // launches: at most sha_wgs_per_cu(fill) workgroups per CU (the ring's 34 KiB alone
    // lets four in: two waves per SIMD).
    const uint32_t per_cu = nwg <= 256 ? 1u : sha_wgs_per_cu(fill);
    const size_t pad = lds_pad_for(per_cu);
    t_sha_tiers[0] = nquad;
    t_sha_tiers[1] = npair;
    t_sha_tiers[2] = nwg - nquad - npair;
    t_sha_tiers[3] = (uint32_t)pad;
    hipLaunchKernelGGL(k_sha256, dim3(nwg), dim3(128), pad, st, d_data, d_abs,
                       (const DescRaw *)d_desc, d_total, max_chunks, order, d_hash_base, hash_stride, g_sha_diag,
                       g_sha_mode, nquad, npair, g_sha_spin_limit, d_err, order ? need : nullptr,
                       notify ? *notify : ShaNotify{});
}

// ---------------------------------------------------------------------------
// Coalesced digest of several batches (runtime.hip coalescer, round 4).  One batch's
// digest is a ~55 ms chain of its longest chunk on ~700 waves, so K concurrent callers
// each running their own launch leave the chip mostly idle and serialise on the hardware
// queues; merging the K chunk lists into one launch gives one GPU-filling k_sha256 whose
// length order spreads every batch's chunks over the quad / pair / one-lane tiers.
// k_coal_merge builds the merged list (lengths + addresses relative to member 0's base,
// so an idle lane's address stays inside a real buffer); k_coal_scatter copies the
// digests back into each member's descriptors and the spin-guard word into each member's.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void coal_prefix(const CoalTable &t, uint64_t *pre) {
    if (threadIdx.x == 0) {
        uint64_t s = 0;
        for (uint32_t b = 0; b < t.n; ++b) {
            pre[b] = s;
            const uint64_t c = *t.total[b];
            s += c < t.bound[b] ? c : t.bound[b];
        }
        pre[t.n] = s;
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t coal_member(const uint64_t *pre, uint32_t n, uint64_t g) {
    uint32_t b = 0;
    while (b + 1 < n && pre[b + 1] <= g) ++b;
    return b;
}

__global__ __launch_bounds__(256) void k_coal_merge(CoalTable t, DescRaw *__restrict__ mdesc,
                                                    uint64_t *__restrict__ mabs, uint64_t *__restrict__ mtotal) {
    __shared__ uint64_t pre[CG_COAL_MAX + 1];
    coal_prefix(t, pre);
    const uint64_t total = pre[t.n];
    if (blockIdx.x == 0 && threadIdx.x == 0) *mtotal = total;
    const uint64_t base = (uint64_t)t.data[0];
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += (uint64_t)gridDim.x * 256) {
        const uint32_t b = coal_member(pre, t.n, g);
        const uint64_t i = g - pre[b];
        mdesc[g].length = t.out[b][i].length;
        mabs[g] = (uint64_t)t.data[b] + t.abs[b][i] - base;  // data[0] + mabs[g] = the chunk's address
    }
}

__global__ __launch_bounds__(256) void k_coal_scatter(CoalTable t, const DescRaw *__restrict__ mdesc,
                                                      const uint32_t *__restrict__ merr) {
    __shared__ uint64_t pre[CG_COAL_MAX + 1];
    coal_prefix(t, pre);
    const uint64_t total = pre[t.n];
    if (blockIdx.x == 0 && threadIdx.x < t.n) {
        const uint32_t e = *merr;
        if (e) *t.err[threadIdx.x] = e;
    }
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += (uint64_t)gridDim.x * 256) {
        const uint32_t b = coal_member(pre, t.n, g);
        const uint64_t i = g - pre[b];
        const uint4 *src = reinterpret_cast<const uint4 *>(mdesc[g].hash);
        uint4 *dst = reinterpret_cast<uint4 *>(t.out[b][i].hash);
        dst[0] = src[0];
        dst[1] = src[1];
    }
}

void launch_sha256_coalesced(const CoalTable &t, uint64_t bound_sum, uint64_t expected, uint64_t max_len,
                             DescRaw *mdesc, uint64_t *mabs, uint64_t *mtotal, uint32_t *morder_tmp, uint32_t *merr,
                             hipStream_t st) {
    if (t.n == 0 || bound_sum == 0) return;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((bound_sum + 255) / 256, 1024);
    (void)hipMemsetAsync(merr, 0, sizeof(uint32_t), st);
    hipLaunchKernelGGL(k_coal_merge, dim3(grid), dim3(256), 0, st, t, mdesc, mabs, mtotal);
    launch_sha256(t.data[0], mabs, mdesc, mtotal, bound_sum, expected, max_len, morder_tmp,
                  reinterpret_cast<uint8_t *>(mdesc) + offsetof(DescRaw, hash), sizeof(DescRaw), merr, st);
    hipLaunchKernelGGL(k_coal_scatter, dim3(grid), dim3(256), 0, st, t, mdesc, merr);
}

// ---------------------------------------------------------------------------
// The digest pipeline's merged launch (pipeline.hip, round 6).  One caller's queued
// batches are digested G at a time by ONE k_sha256, so the batches in flight no longer
// need a HIP stream -- a hardware queue -- each: the chip is filled by the merged launch's
// workgroups, not by concurrent launches.  k_pipe_merge builds the merged chunk list
// (lengths, addresses relative to member 0's base, digest destinations inside each
// member's own descriptors, member index) and arms the per-member counters; k_sha256 then
// signals each member as soon as its last chunk is digested (ShaNotify).
// ---------------------------------------------------------------------------
// Member prefix of the chunk counts (n <= CG_PIPE_MAX = one wave): pre[b] = chunks of
// members 0..b-1, pre[n] = all.
__device__ __forceinline__ void pipe_prefix(const PipeTable &t, uint64_t *pre) {
    static_assert(CG_PIPE_MAX <= 64, "one wave scans the member counts");
    if (threadIdx.x < 64) {
        const uint32_t b = threadIdx.x;
        uint64_t c = 0;
        if (b < t.n) {
            c = *t.total[b];
            if (c > t.bound[b]) c = t.bound[b];
        }
        uint64_t x = c;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(x, d, 64);
            if (b >= d) x += y;
        }
        if (b < t.n) pre[b] = x - c;
        if (b == t.n - 1) pre[t.n] = x;
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t pipe_member(const uint64_t *pre, uint32_t n, uint64_t g) {
    uint32_t lo = 0, hi = n - 1;  // the last b with pre[b] <= g
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= g) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ __launch_bounds__(256) void k_pipe_merge(PipeTable t, PipeBufs m) {
    __shared__ uint64_t pre[CG_PIPE_MAX + 1];
    pipe_prefix(t, pre);
    const uint64_t total = pre[t.n];
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            *m.mtotal = total;
            *m.err = 0;
        }
        if (threadIdx.x < t.n) {
            const uint32_t b = threadIdx.x;
            const uint32_t c = (uint32_t)(pre[b + 1] - pre[b]);
            m.remain[b] = c;
            m.merr[b] = 0;
            m.mflag[b] = t.flag[b];
            // a member without chunks (empty NARs only) is complete now
            if (c == 0) __hip_atomic_store(t.flag[b], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    const uint64_t base = (uint64_t)t.data[0];
    for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += (uint64_t)gridDim.x * 256) {
        const uint32_t b = pipe_member(pre, t.n, g);
        const uint64_t i = g - pre[b];
        m.mdesc[g].length = t.out[b][i].length;
        m.mabs[g] = (uint64_t)t.data[b] + t.abs[b][i] - base;  // data[0] + mabs[g] = the chunk's address
        m.mdst[g] = (uint64_t)t.out[b][i].hash;
        m.mmember[g] = b;
    }
}

void launch_sha256_pipe(const PipeTable &t, uint64_t bound_sum, uint64_t expected, uint64_t max_len,
                        const PipeBufs &b, hipStream_t st, hipEvent_t start, hipEvent_t stop) {
    if (t.n == 0) return;
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((bound_sum + 255) / 256, 1024));
    hipLaunchKernelGGL(k_pipe_merge, dim3(grid), dim3(256), 0, st, t, b);
    if (start) (void)hipEventRecord(start, st);
    if (bound_sum) {
        ShaNotify nt;
        nt.dst = b.mdst;
        nt.member = b.mmember;
        nt.remain = b.remain;
        nt.merr = b.merr;
        nt.flag = b.mflag;
        launch_sha256(t.data[0], b.mabs, b.mdesc, b.mtotal, bound_sum, expected, max_len, b.morder, nullptr, 0, b.err,
                      st, true, &nt);
    }
    if (stop) (void)hipEventRecord(stop, st);
}

#ifdef CG_DIAG
// ---------------------------------------------------------------------------
// Diagnostics: cycles per split round for a lone wave (the same round code the
// split consumer runs, schedule words held in registers).
// ---------------------------------------------------------------------------
template <bool QUAD>
__global__ void k_diag_sha_rounds_split(uint32_t iters, uint32_t *out, unsigned long long *cycles) {
    const uint32_t lane = threadIdx.x & 63u;
    const bool hi = (lane >> 2) & 1u;
    const uint32_t q = lane & 3u;
    SplitLane c;
    c.sh1 = QUAD ? (hi ? (q == 0 ? 2u : q == 1 ? 13u : 22u) : (q == 0 ? 6u : q == 1 ? 11u : 25u)) : (hi ? 2u : 6u);
    c.sh2 = hi ? 13u : 11u;
    c.sh3 = hi ? 22u : 25u;
    c.lm = hi ? 0xffffffffu : 0u;
    asm volatile("" : "+v"(c.sh1), "+v"(c.sh2), "+v"(c.sh3), "+v"(c.lm));
    uint4 W[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) W[i] = make_uint4(lane * 32 + 4 * i, lane * 32 + 4 * i + 1, lane + i, lane ^ i);
    uint32_t st[4] = {lane, 1u, 2u, 3u};
    uint32_t z = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t x0 = st[0], x1 = st[1], x2 = st[2], x3 = st[3];
        SPL32(0, W)
        SPL32(32, W)
        st[0] += x0;
        st[1] += x1;
        st[2] += x2;
        st[3] += x3;
        spl_z(z, st[3], W[0].x);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = st[0] ^ st[1] ^ st[2] ^ st[3];
    if (lane == 0) cycles[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

// DPP lane probe: v_add_u32_dpp row_shl:4 with bank_mask 0x5 (the split round's lo
// write): lanes of banks 0/2 get (1000 + lane + 4) + lane, banks 1/3 keep lane.
__global__ void k_diag_dpp_probe(uint32_t *out) {
    const uint32_t lane = threadIdx.x;
    const uint32_t a = 1000u + lane;
    uint32_t b = lane;
    asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %1, %0 row_shl:4 row_mask:0xf bank_mask:0x5" : "+v"(b) : "v"(a));
    out[lane] = b;
}

#endif  // CG_DIAG
}  // namespace cg

#ifdef CG_DIAG
// quad != 0: the 9-VALU quad round; else the 10-VALU pair round
extern "C" int cg_diag_sha_rounds_split(uint32_t iters, uint32_t blocks, uint32_t threads, int quad,
                                        unsigned long long *h_cycles) {
    uint32_t *d_out = nullptr;
    unsigned long long *d_cyc = nullptr;
    const uint32_t waves = blocks * (threads / 64);
    if (hipMalloc(&d_out, (size_t)blocks * threads * 4) != hipSuccess) return 2;
    if (hipMalloc(&d_cyc, waves * 8) != hipSuccess) return 2;
    hipLaunchKernelGGL(quad ? cg::k_diag_sha_rounds_split<true> : cg::k_diag_sha_rounds_split<false>, dim3(blocks),
                       dim3(threads), 0, 0, iters, d_out, d_cyc);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(h_cycles, d_cyc, waves * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    return e == hipSuccess ? 0 : 2;
}

extern "C" int cg_diag_dpp_probe(uint32_t *h_out) {
    uint32_t *d = nullptr;
    if (hipMalloc(&d, 256) != hipSuccess) return 2;
    hipLaunchKernelGGL(cg::k_diag_dpp_probe, dim3(1), dim3(64), 0, 0, d);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(h_out, d, 256, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? 0 : 2;
}

// workgroups the digest launch uses for `max_chunks` (diagnostics: sizes cg_diag_sha_stats)
extern "C" uint32_t cg_diag_sha_grid(uint64_t max_chunks, uint64_t expected) {
    return cg::sha256_grid(max_chunks, expected, nullptr, nullptr, nullptr);
}
#endif  // CG_DIAG

extern "C" int cg_last_sha_tiers(uint32_t out[4]) {
    for (int i = 0; i < 4; ++i) out[i] = cg::t_sha_tiers[i];
    return (cg::t_sha_tiers[0] | cg::t_sha_tiers[1] | cg::t_sha_tiers[2]) ? 1 : 0;
}

// Test hooks: tier caps of the digest launch (the parity tests force every tier mix)
// and the spin-guard limit (a test drives the timeout path); each returns the old value.
extern "C" uint32_t cg_test_sha_split_max(uint32_t v) {
    const uint32_t old = cg::g_sha_split_max;
    cg::g_sha_split_max = v;
    return old;
}

extern "C" uint32_t cg_test_sha_spin_limit(uint32_t v) {
    const uint32_t old = cg::g_sha_spin_limit;
    cg::g_sha_spin_limit = v;
    return old;
}

extern "C" uint32_t cg_test_sha_quad_fill(uint32_t v) {
    const uint32_t old = cg::g_sha_quad_fill;
    cg::g_sha_quad_fill = v;
    return old;
}

extern "C" uint32_t cg_test_sha_pair_fill(uint32_t v) {
    const uint32_t old = cg::g_sha_pair_fill;
    cg::g_sha_pair_fill = v;
    return old;
}

// Latency tiers: per-mille thresholds (quad, pair) of the longest chunk for launches that
// leave the chip idle (cg_test_sha_tiers) and for GPU-filling ones (cg_test_sha_tiers_fill);
// quad_pm 0 = off.  Each returns its previous quad_pm << 16 | pair_pm.
static uint32_t set_sha_tiers(int k, uint32_t quad_pm, uint32_t pair_pm) {
    const uint32_t old = cg::g_sha_tier_quad_pm[k] << 16 | cg::g_sha_tier_pair_pm[k];
    cg::g_sha_tier_quad_pm[k] = quad_pm > 1000u ? 1000u : quad_pm;
    cg::g_sha_tier_pair_pm[k] = pair_pm > cg::g_sha_tier_quad_pm[k] ? cg::g_sha_tier_quad_pm[k] : pair_pm;
    return old;
}
extern "C" uint32_t cg_test_sha_tiers(uint32_t quad_pm, uint32_t pair_pm) { return set_sha_tiers(0, quad_pm, pair_pm); }
extern "C" uint32_t cg_test_sha_tiers_fill(uint32_t quad_pm, uint32_t pair_pm) {
    return set_sha_tiers(1, quad_pm, pair_pm);
}

// Test hook: workgroups per CU of latency-bound (which = 0) / GPU-filling (1) launches with
// more workgroups than CUs (1..4); returns the previous value.
extern "C" uint32_t cg_test_sha_occupancy(uint32_t which, uint32_t v) {
    (void)cg::sha_wgs_per_cu(false);
    const uint32_t k = which ? 1u : 0u, old = cg::g_sha_occ[k];
    cg::g_sha_occ[k] = std::min(std::max(v, 1u), 4u);
    return old;
}

extern "C" uint32_t cg_test_sha_quad_max(uint32_t v) {
    const uint32_t old = cg::g_sha_quad_max;
    cg::g_sha_quad_max = v;
    return old;
}

