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


// The four G functions of a column (or diagonal) step are independent, each a
// strictly serial chain of 12 VALU ops (2 v_add3, 2 v_add, 4 xor, 4 v_alignbit: no
// shorter form exists on gfx950).  They are interleaved op by op so that each op's
// producer is 4 instructions back.
#define B3_G4(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3, mi)                                   \
    {                                                                                                               \
        v[a0] = v[a0] + v[b0] + m[mi[0]];                                                                           \
        v[a1] = v[a1] + v[b1] + m[mi[2]];                                                                           \
        v[a2] = v[a2] + v[b2] + m[mi[4]];                                                                           \
        v[a3] = v[a3] + v[b3] + m[mi[6]];                                                                           \
        v[d0] = rotr32b(v[d0] ^ v[a0], 16);                                                                         \
        v[d1] = rotr32b(v[d1] ^ v[a1], 16);                                                                         \
        v[d2] = rotr32b(v[d2] ^ v[a2], 16);                                                                         \
        v[d3] = rotr32b(v[d3] ^ v[a3], 16);                                                                         \
        v[c0] = v[c0] + v[d0];                                                                                      \
        v[c1] = v[c1] + v[d1];                                                                                      \
        v[c2] = v[c2] + v[d2];                                                                                      \
        v[c3] = v[c3] + v[d3];                                                                                      \
        v[b0] = rotr32b(v[b0] ^ v[c0], 12);                                                                         \
        v[b1] = rotr32b(v[b1] ^ v[c1], 12);                                                                         \
        v[b2] = rotr32b(v[b2] ^ v[c2], 12);                                                                         \
        v[b3] = rotr32b(v[b3] ^ v[c3], 12);                                                                         \
        v[a0] = v[a0] + v[b0] + m[mi[1]];                                                                           \
        v[a1] = v[a1] + v[b1] + m[mi[3]];                                                                           \
        v[a2] = v[a2] + v[b2] + m[mi[5]];                                                                           \
        v[a3] = v[a3] + v[b3] + m[mi[7]];                                                                           \
        v[d0] = rotr32b(v[d0] ^ v[a0], 8);                                                                          \
        v[d1] = rotr32b(v[d1] ^ v[a1], 8);                                                                          \
        v[d2] = rotr32b(v[d2] ^ v[a2], 8);                                                                          \
        v[d3] = rotr32b(v[d3] ^ v[a3], 8);                                                                          \
        v[c0] = v[c0] + v[d0];                                                                                      \
        v[c1] = v[c1] + v[d1];                                                                                      \
        v[c2] = v[c2] + v[d2];                                                                                      \
        v[c3] = v[c3] + v[d3];                                                                                      \
        v[b0] = rotr32b(v[b0] ^ v[c0], 7);                                                                          \
        v[b1] = rotr32b(v[b1] ^ v[c1], 7);                                                                          \
        v[b2] = rotr32b(v[b2] ^ v[c2], 7);                                                                          \
        v[b3] = rotr32b(v[b3] ^ v[c3], 7);                                                                          \
    }

// The same step with every op pinned by its own asm statement (CG_B3_PINNED): the op
// groups stay in the order above and v_xor_b32 / v_add_u32 write a register none of their
// sources holds (early-clobber).  In the issue microbenchmark this stream issues 15-20 % of
// its VALU instructions in pairs (two waves, one quad-cycle) where the compiler's schedule
// of the same ops pairs 0.5 %: 3.82 vs 4.05 clocks per VALU at 4 waves per SIMD, 2,570 vs
// 2,724 clocks per compression (scripts/micro/issue_rates.hip kinds 100 / 125,
// profiles/r05_v6_b3_dual_issue.json).
// On config 3 the pinned stream is the product: 1,342-1,371 vs 1,332-1,344 GiB/s, same box,
// three alternating rounds (profiles/r05_v7_b3_pinned_ab.txt).
#ifndef CG_B3_PINNED
#define CG_B3_PINNED 1
#endif
#define B3P_ADD3(d, x, y, z) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(x), "v"(y), "v"(z))
#define B3P_XOR(d, x, y) asm volatile("v_xor_b32 %0, %1, %2" : "=&v"(d) : "v"(x), "v"(y))
#define B3P_ADD(d, x, y) asm volatile("v_add_u32 %0, %1, %2" : "=&v"(d) : "v"(x), "v"(y))
#define B3P_ROT(d, x, n) asm volatile("v_alignbit_b32 %0, %1, %1, " #n : "=v"(d) : "v"(x))
#define B3_G4P(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3, mi)                                  \
    {                                                                                                               \
        B3P_ADD3(v[a0], v[a0], v[b0], m[mi[0]]);                                                                    \
        B3P_ADD3(v[a1], v[a1], v[b1], m[mi[2]]);                                                                    \
        B3P_ADD3(v[a2], v[a2], v[b2], m[mi[4]]);                                                                    \
        B3P_ADD3(v[a3], v[a3], v[b3], m[mi[6]]);                                                                    \
        B3P_XOR(v[d0], v[d0], v[a0]);                                                                               \
        B3P_XOR(v[d1], v[d1], v[a1]);                                                                               \
        B3P_XOR(v[d2], v[d2], v[a2]);                                                                               \
        B3P_XOR(v[d3], v[d3], v[a3]);                                                                               \
        B3P_ROT(v[d0], v[d0], 16);                                                                                  \
        B3P_ROT(v[d1], v[d1], 16);                                                                                  \
        B3P_ROT(v[d2], v[d2], 16);                                                                                  \
        B3P_ROT(v[d3], v[d3], 16);                                                                                  \
        B3P_ADD(v[c0], v[c0], v[d0]);                                                                               \
        B3P_ADD(v[c1], v[c1], v[d1]);                                                                               \
        B3P_ADD(v[c2], v[c2], v[d2]);                                                                               \
        B3P_ADD(v[c3], v[c3], v[d3]);                                                                               \
        B3P_XOR(v[b0], v[b0], v[c0]);                                                                               \
        B3P_XOR(v[b1], v[b1], v[c1]);                                                                               \
        B3P_XOR(v[b2], v[b2], v[c2]);                                                                               \
        B3P_XOR(v[b3], v[b3], v[c3]);                                                                               \
        B3P_ROT(v[b0], v[b0], 12);                                                                                  \
        B3P_ROT(v[b1], v[b1], 12);                                                                                  \
        B3P_ROT(v[b2], v[b2], 12);                                                                                  \
        B3P_ROT(v[b3], v[b3], 12);                                                                                  \
        B3P_ADD3(v[a0], v[a0], v[b0], m[mi[1]]);                                                                    \
        B3P_ADD3(v[a1], v[a1], v[b1], m[mi[3]]);                                                                    \
        B3P_ADD3(v[a2], v[a2], v[b2], m[mi[5]]);                                                                    \
        B3P_ADD3(v[a3], v[a3], v[b3], m[mi[7]]);                                                                    \
        B3P_XOR(v[d0], v[d0], v[a0]);                                                                               \
        B3P_XOR(v[d1], v[d1], v[a1]);                                                                               \
        B3P_XOR(v[d2], v[d2], v[a2]);                                                                               \
        B3P_XOR(v[d3], v[d3], v[a3]);                                                                               \
        B3P_ROT(v[d0], v[d0], 8);                                                                                   \
        B3P_ROT(v[d1], v[d1], 8);                                                                                   \
        B3P_ROT(v[d2], v[d2], 8);                                                                                   \
        B3P_ROT(v[d3], v[d3], 8);                                                                                   \
        B3P_ADD(v[c0], v[c0], v[d0]);                                                                               \
        B3P_ADD(v[c1], v[c1], v[d1]);                                                                               \
        B3P_ADD(v[c2], v[c2], v[d2]);                                                                               \
        B3P_ADD(v[c3], v[c3], v[d3]);                                                                               \
        B3P_XOR(v[b0], v[b0], v[c0]);                                                                               \
        B3P_XOR(v[b1], v[b1], v[c1]);                                                                               \
        B3P_XOR(v[b2], v[b2], v[c2]);                                                                               \
        B3P_XOR(v[b3], v[b3], v[c3]);                                                                               \
        B3P_ROT(v[b0], v[b0], 7);                                                                                   \
        B3P_ROT(v[b1], v[b1], 7);                                                                                   \
        B3P_ROT(v[b2], v[b2], 7);                                                                                   \
        B3P_ROT(v[b3], v[b3], 7);                                                                                   \
    }

// CG_B3_PINNED=2: each G4 step (48 ops, the order above) as ONE asm statement.  The compiler
// pads between inline-asm statements with an s_nop (its hazard model cannot see inside
// them): one per op group with per-op statements (~170 per compression, an issue slot
// each), one per step here.
#define B3A_BODY(R1, R2)                                                                                            \
    "v_add3_u32 %[a0], %[a0], %[b0], %[x0]\n v_add3_u32 %[a1], %[a1], %[b1], %[x1]\n"                            \
    " v_add3_u32 %[a2], %[a2], %[b2], %[x2]\n v_add3_u32 %[a3], %[a3], %[b3], %[x3]\n"                           \
    " v_xor_b32 %[d0], %[d0], %[a0]\n v_xor_b32 %[d1], %[d1], %[a1]\n"                                           \
    " v_xor_b32 %[d2], %[d2], %[a2]\n v_xor_b32 %[d3], %[d3], %[a3]\n"                                           \
    " v_alignbit_b32 %[d0], %[d0], %[d0], " R1 "\n v_alignbit_b32 %[d1], %[d1], %[d1], " R1 "\n"                 \
    " v_alignbit_b32 %[d2], %[d2], %[d2], " R1 "\n v_alignbit_b32 %[d3], %[d3], %[d3], " R1 "\n"                 \
    " v_add_u32 %[c0], %[c0], %[d0]\n v_add_u32 %[c1], %[c1], %[d1]\n"                                           \
    " v_add_u32 %[c2], %[c2], %[d2]\n v_add_u32 %[c3], %[c3], %[d3]\n"                                           \
    " v_xor_b32 %[b0], %[b0], %[c0]\n v_xor_b32 %[b1], %[b1], %[c1]\n"                                           \
    " v_xor_b32 %[b2], %[b2], %[c2]\n v_xor_b32 %[b3], %[b3], %[c3]\n"                                           \
    " v_alignbit_b32 %[b0], %[b0], %[b0], " R2 "\n v_alignbit_b32 %[b1], %[b1], %[b1], " R2 "\n"                 \
    " v_alignbit_b32 %[b2], %[b2], %[b2], " R2 "\n v_alignbit_b32 %[b3], %[b3], %[b3], " R2 "\n"
#define B3_G4A(A0, B0, C0, D0, A1, B1, C1, D1, A2, B2, C2, D2, A3, B3, C3, D3, MI)                                  \
    {                                                                                                               \
        asm volatile(B3A_BODY("16", "12")                                                                          \
                     : [a0] "+v"(v[A0]), [b0] "+v"(v[B0]), [c0] "+v"(v[C0]), [d0] "+v"(v[D0]), [a1] "+v"(v[A1]), \
                       [b1] "+v"(v[B1]), [c1] "+v"(v[C1]), [d1] "+v"(v[D1]), [a2] "+v"(v[A2]), [b2] "+v"(v[B2]), \
                       [c2] "+v"(v[C2]), [d2] "+v"(v[D2]), [a3] "+v"(v[A3]), [b3] "+v"(v[B3]), [c3] "+v"(v[C3]), \
                       [d3] "+v"(v[D3])                                                                          \
                     : [x0] "v"(m[MI[0]]), [x1] "v"(m[MI[2]]), [x2] "v"(m[MI[4]]), [x3] "v"(m[MI[6]]));         \
        asm volatile(B3A_BODY("8", "7")                                                                            \
                     : [a0] "+v"(v[A0]), [b0] "+v"(v[B0]), [c0] "+v"(v[C0]), [d0] "+v"(v[D0]), [a1] "+v"(v[A1]), \
                       [b1] "+v"(v[B1]), [c1] "+v"(v[C1]), [d1] "+v"(v[D1]), [a2] "+v"(v[A2]), [b2] "+v"(v[B2]), \
                       [c2] "+v"(v[C2]), [d2] "+v"(v[D2]), [a3] "+v"(v[A3]), [b3] "+v"(v[B3]), [c3] "+v"(v[C3]), \
                       [d3] "+v"(v[D3])                                                                          \
                     : [x0] "v"(m[MI[1]]), [x1] "v"(m[MI[3]]), [x2] "v"(m[MI[5]]), [x3] "v"(m[MI[7]]));         \
    }

// Compress one block; returns the new chaining value in cv (first 8 output words).
__device__ __forceinline__ void b3_compress(uint32_t cv[8], const uint32_t m[16], uint64_t counter, uint32_t blen,
                                            uint32_t flags) {
    uint32_t v[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                      B3_IV[0], B3_IV[1], B3_IV[2], B3_IV[3], (uint32_t)counter, (uint32_t)(counter >> 32),
                      blen, flags};
#pragma unroll
    for (int r = 0; r < 7; ++r) {
#if CG_B3_PINNED == 2
        B3_G4A(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15, B3S.s[r]);
        B3_G4A(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14, (B3S.s[r] + 8));
#elif CG_B3_PINNED
        B3_G4P(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15, B3S.s[r]);
        B3_G4P(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14, (B3S.s[r] + 8));
#else
        B3_G4(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15, B3S.s[r]);
        B3_G4(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14, (B3S.s[r] + 8));
#endif
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
// p may be unaligned (v_alignbyte realigns dword-aligned loads: dwordx4 loads from the
// unaligned address instead, 16 fewer VALU per block, made the digest stage 15 % slower,
// profiles/r03_v15_ab_c3_b3_plan_unaligned.jsonl).  Blocks lying
// wholly inside the leaf are fetched as four 16-byte loads (+ the dword after them
// when p is unaligned), one block ahead of the compression that uses them (the lanes
// of a wave sit 1 KiB apart, each on its own cache line).  With loads removed
// altogether (NOLOAD) the kernel is only ~10 % faster: it is bound by the ~700 VALU
// of each compression (scripts/diag_b3.py).
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
// NOLOAD (diagnostics only): compress lane-dependent register words instead of
// loading the leaf, to time the compression alone.
template <bool NOLOAD = false>
__device__ __forceinline__ void b3_leaf(const uint8_t *p, uint32_t n, uint64_t ctr, bool root, uint32_t cv[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = B3_IV[i];
    const uint32_t shift = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *base = reinterpret_cast<const uint32_t *>(p - shift);
    const uint32_t nblk = n ? (n + 63) / 64 : 1;
    const uint32_t nfull = n / 64;  // blocks with all 64 bytes inside the leaf
    const uint8_t *endp = p + n;
    auto flags_of = [&](uint32_t j) {
        const bool last = j + 1 == nblk;
        return (j == 0 ? B3_CHUNK_START : 0u) | (last ? B3_CHUNK_END : 0u) | (root && last ? B3_ROOT : 0u);
    };
    // One full block: realigned and compressed.
    auto full_block = [&](const u32x4_a4 *v, uint32_t v16, uint32_t j) {
        uint32_t m[16];
        if (NOLOAD) {
#pragma unroll
            for (int i = 0; i < 16; ++i) m[i] = (uint32_t)ctr * 0x9E3779B9u + (uint32_t)(i * 0x01010101) + j;
        } else {
            const uint32_t dw[17] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                                     v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w, v16};
#pragma unroll
            for (int i = 0; i < 16; ++i) m[i] = __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], shift);
        }
        b3_compress(cv, m, ctr, 64u, flags_of(j));
    };
    const uint32_t npair = nfull / 2;
    if (npair) {
        // Full blocks two at a time: a lane reads whole 128-byte lines (one block at a time left
        // the other half of each line to a later read, often after L2 had dropped it: 1.55 GB
        // fetched per 1.07 GB, profiles/r02_v15_pmc_c3.json).  The loop body is one basic
        // block: the next pair loads into pn on every iteration (the last re-reads its own
        // pair), pinned before the compressions by a sched_barrier, and moves into px after
        // them behind another, so the loads' wait sits there; the empty asm on px keeps the
        // compiler from rotating the loads to the top of the iteration that consumes them.
        // (With the tail block inside the loop and a conditional prefetch the compiler had
        // waited for the just-issued loads before every compression: ~15 % of the stage.)
        // Two buffers take turns (the loop body holds two pairs), so no pair is ever moved
        // between registers: 33 v_mov per pair (~2.5 % of the VALU) gone.
        u32x4_a4 pa[8], pb[8];
        uint32_t pa32 = 0, pb32 = 0;
        auto fetch2 = [&](u32x4_a4 (&v)[8], uint32_t &v32, uint32_t jp) {
            const uint32_t *q = base + 32 * (jp < npair ? jp : npair - 1);  // past the end: re-read the last pair
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const u32x4_a4 *>(q + 4 * i);
            // the dword after the pair starts inside the leaf whenever shift != 0 (ignored by
            // the realignment when shift == 0: the load re-reads the pair's last dword)
            v32 = q[shift ? 32 : 31];
        };
        auto pin = [&](u32x4_a4 (&v)[8], uint32_t &v32) {  // the loads stay where they were issued
            asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
                         "+v"(v[7]), "+v"(v32));
        };
        if (!NOLOAD) fetch2(pa, pa32, 0);
#pragma unroll 1
        for (uint32_t jp = 0; jp < npair; jp += 2) {
            if (!NOLOAD) fetch2(pb, pb32, jp + 1);
            __builtin_amdgcn_sched_barrier(0);  // issued before the compressions, not sunk after them
            full_block(pa, pa[4].x, 2 * jp);
            full_block(pa + 4, pa32, 2 * jp + 1);
            __builtin_amdgcn_sched_barrier(0);
            if (!NOLOAD) pin(pb, pb32);
            if (jp + 1 == npair) break;
            if (!NOLOAD) fetch2(pa, pa32, jp + 2);
            __builtin_amdgcn_sched_barrier(0);
            full_block(pb, pb[4].x, 2 * jp + 2);
            full_block(pb + 4, pb32, 2 * jp + 3);
            __builtin_amdgcn_sched_barrier(0);
            if (!NOLOAD) pin(pa, pa32);
        }
    }
    if (nfull & 1u) {  // an odd last full block
        const uint32_t j = nfull - 1;
        u32x4_a4 v[4];
        uint32_t v16 = 0;
        if (!NOLOAD) {
            const uint32_t *q = base + 16 * j;
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const u32x4_a4 *>(q + 4 * i);
            v16 = q[shift ? 16 : 15];
        }
        full_block(v, v16, j);
    }
    if (nblk > nfull) {  // the partial last block (or the one empty block of n == 0)
        const uint32_t j = nfull;
        const uint32_t *q = base + 16 * j;
        const uint32_t blen = n - 64 * j;
        uint32_t dw[17], m[16];
        if (NOLOAD) {
#pragma unroll
            for (int i = 0; i < 16; ++i) m[i] = (uint32_t)ctr * 0x9E3779B9u + (uint32_t)(i * 0x01010101) + j;
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
        b3_compress(cv, m, ctr, blen, flags_of(j));
    }
}

#ifndef CG_B3_LDS_REALIGN
#define CG_B3_LDS_REALIGN 1
#endif
#ifndef CG_B3_HOLD_TAIL
#define CG_B3_HOLD_TAIL 1
#endif
#if CG_B3_LDS_REALIGN
// Leaf with every load a whole 64-byte-aligned segment (k_b3_leaves, the product since round
// 6; CG_B3_LDS_REALIGN=0 builds the round-5 b3_leaf loads there).
// b3_leaf reads each block pair from the leaf's own (unaligned) address, so a 128-byte line
// is read twice -- by the pair that ends in it and the next one, and the leaf's last line by
// the right neighbour's first pair ~16 compressions earlier -- and by then L2 has often
// dropped it (1.40x the batch's bytes, profiles/r05_v10_pmc_c3.json).  Here segment k of the
// leaf's aligned span is loaded once, two blocks ahead, into a per-lane LDS ring of 48 dwords
// (segments j and j + 1 at 0 / 16 for even j, 16 / 32 for odd j: the even slot is mirrored at
// 32 so a block's 17 dwords never wrap), and block j is read back at the lane's dword offset
// with constant-offset LDS reads, then realigned by byte as before.  Measured on config 3
// (profiles/r06_v18_b3_lds_realign_ab.txt): fetched 1.41x -> 1.22x the batch (what is left:
// the leaf's last 128-byte line, which the right neighbour's lane read ~16 compressions
// earlier), kernel time equal (0.406 / 0.410 ms): the kernel is VALU-issue bound.  53 KiB
// of LDS per 4-wave workgroup: 3 waves per SIMD instead of 4, no loss at this issue rate.
// With that last line loaded at the start, beside the neighbour's request for it, and held
// in registers (CG_B3_HOLD_TAIL, 32 VGPRs): 1.09x, 0.405 -> 0.412 ms, config 3 equal
// (profiles/r06_v20_b3_hold_tail_ab.txt).
#define B3_RING 52u  // dwords per lane: 48 + 4 pad (8 consecutive lanes' b128 stores on distinct banks)
__device__ __forceinline__ void b3_leaf_lds(const uint8_t *p, uint32_t n, uint64_t ctr, bool root, uint32_t cv[8],
                                            uint32_t *ring) {
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = B3_IV[i];
    const uint32_t off = (uint32_t)((uintptr_t)p & 63u);
    const uint32_t shift = off & 3u;
    const uint4 *seg0 = reinterpret_cast<const uint4 *>(p - off);
    const uint32_t nblk = n ? (n + 63) / 64 : 1;
    const uint32_t nfull = n / 64;
    const uint32_t last_seg = (off + (n ? n : 1u) - 1u) >> 6;  // the last segment holding leaf bytes
    uint32_t *rl = ring + (off >> 2);                           // this lane's block reads start here
    uint4 r0, r1, r2, r3;  // the segment in flight (four named registers: an array went to scratch)
#if CG_B3_HOLD_TAIL
    // The leaf's last 128-byte line (its last segment, and the one before when both share the
    // line) is the right neighbour lane's first: loaded now, at the same time as the
    // neighbour's, and held in registers until the last blocks need it.
    const uint32_t hold_from =
        (last_seg > 0 && (((uintptr_t)(seg0 + 4 * last_seg)) & 64u)) ? last_seg - 1 : last_seg;
    const uint4 *qa = seg0 + 4 * hold_from, *qb = seg0 + 4 * last_seg;
    const uint4 ha0 = qa[0], ha1 = qa[1], ha2 = qa[2], ha3 = qa[3];
    const uint4 hb0 = qb[0], hb1 = qb[1], hb2 = qb[2], hb3 = qb[3];
    auto load_seg = [&](uint32_t k) {  // past the leaf: its last segment again (never read)
        if (k < hold_from) {
            const uint4 *q = seg0 + 4 * k;
            r0 = q[0];
            r1 = q[1];
            r2 = q[2];
            r3 = q[3];
        } else if (k == hold_from) {
            r0 = ha0;
            r1 = ha1;
            r2 = ha2;
            r3 = ha3;
        } else {
            r0 = hb0;
            r1 = hb1;
            r2 = hb2;
            r3 = hb3;
        }
    };
#else
    auto load_seg = [&](uint32_t k) {  // past the leaf: re-read its last segment (never read)
        const uint4 *q = seg0 + 4 * (k < last_seg ? k : last_seg);
        r0 = q[0];
        r1 = q[1];
        r2 = q[2];
        r3 = q[3];
    };
#endif
    auto store_seg = [&](uint32_t at) {
        uint4 *d = reinterpret_cast<uint4 *>(ring + at);
        d[0] = r0;
        d[1] = r1;
        d[2] = r2;
        d[3] = r3;
    };
    auto flags_of = [&](uint32_t j) {
        const bool last = j + 1 == nblk;
        return (j == 0 ? B3_CHUNK_START : 0u) | (last ? B3_CHUNK_END : 0u) | (root && last ? B3_ROOT : 0u);
    };
    load_seg(0);
    store_seg(0);
    store_seg(32);
    load_seg(1);
    store_seg(16);
    load_seg(2);
    // one block: its 17 dwords from the ring at `base` (0: even j, 16: odd j); segment j's
    // slot then takes segment j + 2 (already in r) and segment j + 3 is requested
    auto block = [&](uint32_t j, uint32_t base, bool full) {
        uint32_t dw[17], m[16];
#pragma unroll
        for (int i = 0; i < 17; ++i) dw[i] = rl[base + i];
        const uint32_t blen = full ? 64u : n - 64 * j;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t v = __builtin_amdgcn_alignbyte(dw[i + 1], dw[i], shift);
            if (full) {
                m[i] = v;
            } else {
                const int rr = (int)blen - 4 * i;
                m[i] = rr >= 4 ? v : (rr <= 0 ? 0u : (v & (0xffffffffu >> (32 - 8 * rr))));
            }
        }
        store_seg(base);
        if (base == 0) store_seg(32);
        load_seg(j + 3);
        __builtin_amdgcn_sched_barrier(0);  // the next segment's load is issued before the compression
        b3_compress(cv, m, ctr, blen, flags_of(j));
    };
    uint32_t j = 0;
#pragma unroll 1
    for (; j + 1 < nfull; j += 2) {
        block(j, 0, true);
        block(j + 1, 16, true);
    }
    if (j < nfull) {
        block(j, 0, true);
        ++j;
    }
    if (j < nblk) block(j, (j & 1u) ? 16u : 0u, false);  // the partial last block (or n == 0)
}
#endif

// Leaves per lane in k_b3_groups: a lane hashes B3_LPL consecutive leaves and folds
// them itself (full exec mask), so a wave covers a 64 x B3_LPL-leaf subtree and its
// shuffle fold (6 levels, one wave-wide compression each, mostly idle lanes) is paid
// once per 256 leaves instead of once per 64 (the fold was ~23 % of the
// stage with one leaf per lane).
#define B3_LPL 4u
template <uint32_t LPL>
__device__ __forceinline__ uint64_t b3_groups_of(uint64_t len) {
    const uint64_t leaves = len ? (len + 1023) / 1024 : 1;
    return (leaves + 64 * LPL - 1) / (64 * LPL);
}

__device__ __forceinline__ void store_digest(uint8_t *dst, const uint32_t cv[8]) {
    uint4 *o = reinterpret_cast<uint4 *>(dst);
    o[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
    o[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
}

template <uint32_t LPL>
__global__ void k_b3_count(const DescRaw *__restrict__ desc, const uint64_t *__restrict__ total_p,
                           uint64_t max_chunks, uint32_t *__restrict__ gcount) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= max_chunks) return;
    uint64_t total = *total_p;
    gcount[g] = g < total ? (uint32_t)b3_groups_of<LPL>(desc[g].length) : 0u;
}

// Fold the chaining values held one per lane (lanes 0..count-1) level by level,
// the odd last node carried up (BLAKE3's left-complete tree); ROOT on the final
// parent when `root`.  Pure register shuffles: no LDS, no barriers.  FULL: every lane
// compresses (the surplus lanes' results are dropped by a select), so the levels run
// under a full exec mask -- partial masks slow a VALU chain on gfx950.
template <bool FULL = false>
__device__ __forceinline__ void b3_wave_fold(uint32_t cv[8], uint32_t count, bool root, uint32_t lane) {
    while (count > 1) {
        const uint32_t half = count >> 1;
        uint32_t l[8], r[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            l[i] = __shfl(cv[i], (int)(2 * lane) & 63, 64);
            r[i] = __shfl(cv[i], (int)(2 * lane + 1) & 63, 64);
        }
        if constexpr (FULL) {
            uint32_t p[8];
            b3_parent(l, r, root && count == 2, p);
            const bool take = lane < half, carry = (count & 1u) && lane == half;
#pragma unroll
            for (int i = 0; i < 8; ++i) cv[i] = take ? p[i] : (carry ? l[i] : cv[i]);
        } else if (lane < half) {
            b3_parent(l, r, root && count == 2, cv);
        } else if ((count & 1u) && lane == half) {
#pragma unroll
            for (int i = 0; i < 8; ++i) cv[i] = l[i];
        }
        count = (count + 1) >> 1;
    }
}

#define B3_WAVES 4u

// group -> chunk map: thread c writes c into its chunk's group slots
__global__ __launch_bounds__(256) void k_b3_map(const uint64_t *__restrict__ group_base,
                                                const uint64_t *__restrict__ total_p, uint64_t max_chunks,
                                                uint32_t *__restrict__ gmap) {
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    const uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (c >= total) return;
    for (uint64_t g = group_base[c]; g < group_base[c + 1]; ++g) gmap[g] = (uint32_t)c;
}

// k_b3_count + the exclusive scan + k_b3_map in one single-block launch, for batches of
// up to B3_PLAN_MAX chunk slots (config 3: ~4,400): 1024 threads, 8 consecutive chunks
// each per pass, group counts scanned with a carry between passes, each thread then
// writes its chunks' group -> chunk entries.  group_base[max_chunks] = the group total,
// as the scan writes.  (Interleaving the chunks over the threads -- coalesced descriptor
// loads, one chunk's entries per thread per 1024-chunk slice, 8 block scans per pass --
// took 41 us per config-3 batch against this form's 12.6 and the three kernels' 14.)
#define B3_PLAN_T 1024u
#define B3_PLAN_ITEMS 8u
#define B3_PLAN_MAX (4u * B3_PLAN_T * B3_PLAN_ITEMS)
template <uint32_t LPL>
__global__ __launch_bounds__(B3_PLAN_T) void k_b3_plan(const DescRaw *__restrict__ desc,
                                                       const uint64_t *__restrict__ total_p, uint64_t max_chunks,
                                                       uint64_t *__restrict__ group_base, uint32_t *__restrict__ gmap) {
    __shared__ uint64_t s_wave[B3_PLAN_T / 64];
    __shared__ uint64_t s_carry;
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    uint64_t carry = 0;
    for (uint64_t b = 0; b < max_chunks; b += (uint64_t)B3_PLAN_T * B3_PLAN_ITEMS) {
        const uint64_t c0 = b + threadIdx.x * B3_PLAN_ITEMS;
        uint32_t cnt[B3_PLAN_ITEMS];
        uint64_t s = 0;
#pragma unroll
        for (uint32_t k = 0; k < B3_PLAN_ITEMS; ++k) {
            cnt[k] = c0 + k < total ? (uint32_t)b3_groups_of<LPL>(desc[c0 + k].length) : 0u;
            s += cnt[k];
        }
        const uint64_t inc = block_inclusive_scan(s, s_wave);
        uint64_t run = carry + inc - s;
#pragma unroll
        for (uint32_t k = 0; k < B3_PLAN_ITEMS; ++k) {
            if (c0 + k < max_chunks) group_base[c0 + k] = run;
            for (uint32_t g = 0; g < cnt[k]; ++g) gmap[run + g] = (uint32_t)(c0 + k);
            run += cnt[k];
        }
        if (threadIdx.x == B3_PLAN_T - 1) s_carry = carry + inc;
        __syncthreads();
        carry = s_carry;
        __syncthreads();
    }
    if (threadIdx.x == 0) group_base[max_chunks] = carry;
}

// The chaining value of leaves [leaf0, leaf0 + r) of a chunk (r = 1..4, the subtree of
// one lane): leaf CVs folded pairwise, the odd third leaf paired last (left-complete);
// ROOT on the last compression when the chunk is this subtree (`root`).
template <bool NOLOAD>
__device__ __forceinline__ void b3_lane4(const uint8_t *chunk, uint64_t len, uint64_t leaf0, uint32_t r, bool root,
                                         uint32_t cv[8]) {
    auto leaf = [&](uint32_t k, uint32_t out[8]) {
        const uint64_t off = (leaf0 + k) * 1024;
        const uint32_t n = (uint32_t)((len - off) < 1024 ? (len - off) : 1024);
        b3_leaf<NOLOAD>(chunk + off, len ? n : 0u, leaf0 + k, root && r == 1, out);
    };
    leaf(0, cv);
    if (r == 1) return;
    uint32_t c1[8];
    leaf(1, c1);
    b3_parent(cv, c1, root && r == 2, cv);
    if (r == 2) return;
    uint32_t c2[8];
    leaf(2, c2);
    if (r == 3) {
        b3_parent(cv, c2, root, cv);
        return;
    }
    uint32_t c3[8];
    leaf(3, c3);
    b3_parent(c2, c3, false, c2);
    b3_parent(cv, c2, root, cv);
}

// One wave per group of 64 x LPL leaves (4 waves per workgroup for occupancy).  MODE
// (diagnostics): bit 0 no leaf loads (compress register words: garbage digests), bit 1
// the full-exec fold, bit 2 no fold at all (garbage digests: the fold's share of the time).
//
// DEFER (the product, one leaf per lane): no fold here -- each lane stores its leaf's
// chaining value into lcv (64 per group) and k_b3_fold folds 16 groups per wave with
// every lane busy.  The in-wave fold costs six wave-wide compressions per 64-leaf group
// (with 32, 16, .. 1 lanes doing useful work) against 16 for the leaves.
template <int MODE = 0, uint32_t LPL = B3_LPL, bool DEFER = false>
__global__ __launch_bounds__(64 * B3_WAVES) void k_b3_groups(const uint8_t *__restrict__ data,
                                                             const uint64_t *__restrict__ abs,
                                                             const DescRaw *__restrict__ desc,
                                                             const uint64_t *__restrict__ total_p, uint64_t max_chunks,
                                                             const uint64_t *__restrict__ group_base,
                                                             const uint32_t *__restrict__ gmap,
                                                             uint8_t *__restrict__ hash_base, size_t stride,
                                                             uint32_t *__restrict__ gcv, uint32_t *__restrict__ lcv) {
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    const uint64_t G = (uint64_t)blockIdx.x * B3_WAVES + (threadIdx.x >> 6);
    if (G >= group_base[total]) return;
    const uint64_t c = gmap[G];  // chunk c with group_base[c] <= G < group_base[c+1]
    const uint64_t len = desc[c].length;
    const uint64_t gi = G - group_base[c];
    const uint64_t ngroups = group_base[c + 1] - group_base[c];
    const uint64_t leaves = len ? (len + 1023) / 1024 : 1;
    const uint32_t lane = threadIdx.x & 63u;
    static_assert(LPL == 1 || LPL == 4, "one leaf per lane or a 4-leaf lane subtree");
    const uint64_t gleaves64 = leaves - gi * 64 * LPL;
    const uint32_t gleaves = (uint32_t)(gleaves64 < 64 * LPL ? gleaves64 : 64 * LPL);
    const uint32_t count0 = (gleaves + LPL - 1) / LPL;  // lanes holding a subtree
    const uint64_t leaf = (gi * 64 + lane) * LPL;
    const uint8_t *chunk = data + abs[c];
    uint32_t cv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (lane < count0) {
        if constexpr (LPL == 1) {
            const uint64_t off = leaf * 1024;
            const uint32_t n = (uint32_t)((len - off) < 1024 ? (len - off) : 1024);
            b3_leaf<(MODE & 1) != 0>(chunk + off, len ? n : 0u, leaf, leaves == 1, cv);
        } else {
            const uint32_t r = gleaves - lane * LPL < LPL ? gleaves - lane * LPL : LPL;
            b3_lane4<(MODE & 1) != 0>(chunk, len, leaf, r, leaves <= LPL, cv);
        }
    }
    if (leaves <= LPL) {  // the chunk is lane 0's subtree: cv is its digest
        if (lane == 0) store_digest(hash_base + c * stride, cv);
        return;
    }
    if constexpr (DEFER) {
        static_assert(LPL == 1, "deferred folds take one leaf per lane");
        if (lane < count0) {
            uint4 *o = reinterpret_cast<uint4 *>(lcv + (G * 64 + lane) * 8);
            o[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
            o[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
        }
        return;
    }
    const bool whole = ngroups == 1;
    if constexpr ((MODE & 4) == 0) b3_wave_fold<(MODE & 2) != 0>(cv, count0, whole, lane);
    if (lane == 0) {
        if (whole) {
            store_digest(hash_base + c * stride, cv);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) gcv[G * 8 + i] = cv[i];
        }
    }
}

// Packed leaves (the product when the group map comes from the descriptor assembly): the
// leaves of all chunks back to back, lane = leaf slot, so a wave covers 64 leaves whatever
// chunk they belong to and no lane idles at a chunk's partial last group (the
// one-group-per-wave form above idles ~32 lanes per chunk: ~3 % of the leaf compressions on
// config 3, more for smaller chunks).  lmap[w] is the chunk of the wave's first slot; a
// lane past that chunk's leaves steps to the next chunk (chunks of fewer than 64 leaves
// make it several steps).  A one-leaf chunk's lane writes the digest (ROOT); every other
// leaf value goes to its group's slot in lcv, folded by k_b3_fold as before.
__global__ __launch_bounds__(64 * B3_WAVES) void k_b3_leaves(const uint8_t *__restrict__ data,
                                                             const uint64_t *__restrict__ abs,
                                                             const DescRaw *__restrict__ desc,
                                                             const uint64_t *__restrict__ total_p,
                                                             uint64_t max_chunks,
                                                             const uint64_t *__restrict__ group_base,
                                                             const uint64_t *__restrict__ leaf_base,
                                                             const uint32_t *__restrict__ lmap,
                                                             uint8_t *__restrict__ hash_base, size_t stride,
                                                             uint32_t *__restrict__ lcv) {
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    const uint64_t W = (uint64_t)blockIdx.x * B3_WAVES + (threadIdx.x >> 6);
    const uint64_t T = leaf_base[total];
    if (W * 64 >= T) return;  // uniform per wave
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t s = W * 64 + lane;
    if (s >= T) return;  // the batch's last wave
    uint64_t c = lmap[W];
    while (s >= leaf_base[c + 1]) ++c;
    const uint64_t len = desc[c].length;
    const uint64_t leaves = len ? (len + 1023) / 1024 : 1;
    const uint64_t l = s - leaf_base[c];
    const uint64_t off = l * 1024;
    const uint32_t n = len ? (uint32_t)((len - off) < 1024 ? (len - off) : 1024) : 0u;
    uint32_t cv[8];
#if CG_B3_LDS_REALIGN
    __shared__ __attribute__((aligned(16))) uint32_t s_ring[B3_WAVES * 64 * B3_RING];
    b3_leaf_lds(data + abs[c] + off, n, l, leaves == 1, cv, s_ring + (threadIdx.x * B3_RING));
#else
    b3_leaf<false>(data + abs[c] + off, n, l, leaves == 1, cv);
#endif
    if (leaves == 1) {
        store_digest(hash_base + c * stride, cv);
    } else {
        uint4 *o = reinterpret_cast<uint4 *>(lcv + ((group_base[c] + l / 64) * 64 + l % 64) * 8);
        o[0] = make_uint4(cv[0], cv[1], cv[2], cv[3]);
        o[1] = make_uint4(cv[4], cv[5], cv[6], cv[7]);
    }
}

// Fold the leaf chaining values of B3_FOLD_G consecutive 64-leaf groups per wave, level
// by level in LDS: at each level every (group, parent) slot is a lane, so a level of the
// 16 groups costs (16 x parents) / 64 wave-wide compressions instead of one per group
// (~17 compressions per 16 groups against 6 per group in b3_wave_fold).  Same pairing
// as b3_wave_fold (odd node carried up; ROOT on the last parent of a single-group chunk);
// the group's value goes to the digest (single-group chunks) or gcv (k_b3_top).
#ifndef B3_FOLD_G
#define B3_FOLD_G 16u
#endif
#ifndef B3_FOLD_T
#define B3_FOLD_T 256u  // 4 waves: level-1 loads all in flight at once, level slots over 4 waves
#endif
__global__ __launch_bounds__(B3_FOLD_T) void k_b3_fold(const DescRaw *__restrict__ desc,
                                                       const uint64_t *__restrict__ total_p, uint64_t max_chunks,
                                                       const uint64_t *__restrict__ group_base,
                                                       const uint32_t *__restrict__ gmap,
                                                       const uint32_t *__restrict__ lcv, uint8_t *__restrict__ hash_base,
                                                       size_t stride, uint32_t *__restrict__ gcv) {
    // level-1 results only (32 per group): level 1 reads its children straight from lcv,
    // so the block needs 18 KiB of LDS and a CU holds six blocks (one dispatch round at
    // 1 GiB; the 64-node layout took 37 KiB and two rounds)
    __shared__ uint32_t s_node[B3_FOLD_G][32][9];  // 9: a CV's 8 words + 1 (bank spread)
    __shared__ uint32_t s_cnt[B3_FOLD_G];          // nodes at the current level (0: skip)
    __shared__ uint32_t s_whole[B3_FOLD_G];
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    const uint64_t ng = group_base[total];
    const uint64_t g0 = (uint64_t)blockIdx.x * B3_FOLD_G;
    if (g0 >= ng) return;  // uniform over the block
    const uint32_t t = threadIdx.x;
    if (t < B3_FOLD_G) {
        const uint64_t g = g0 + t;
        uint32_t cnt = 0, whole = 0;
        if (g < ng) {
            const uint64_t c = gmap[g];
            const uint64_t len = desc[c].length;
            const uint64_t leaves = len ? (len + 1023) / 1024 : 1;
            const uint64_t left = leaves - (g - group_base[c]) * 64;
            // a one-leaf chunk was digested by k_b3_groups
            cnt = leaves == 1 ? 0u : (uint32_t)(left < 64 ? left : 64);
            whole = group_base[c + 1] - group_base[c] == 1;
        }
        s_cnt[t] = cnt;
        s_whole[t] = whole;
    }
    __syncthreads();
    // level 1: slot (group gl, parent j) pairs leaves 2j and 2j + 1 of lcv
    constexpr uint32_t L1 = B3_FOLD_G * 32 / B3_FOLD_T;  // slots per thread
    uint4 lv[L1][2][2];
#pragma unroll
    for (uint32_t i = 0; i < L1; ++i) {
        const uint32_t sl = t + B3_FOLD_T * i, gl = sl / 32, j = sl % 32, cnt = s_cnt[gl];
#pragma unroll
        for (uint32_t h = 0; h < 2; ++h) {
            if (2 * j + h < cnt) {
                const uint4 *q = reinterpret_cast<const uint4 *>(lcv + ((g0 + gl) * 64 + 2 * j + h) * 8);
                lv[i][h][0] = q[0];
                lv[i][h][1] = q[1];
            } else {
                lv[i][h][0] = lv[i][h][1] = make_uint4(0u, 0u, 0u, 0u);
            }
        }
    }
#pragma unroll
    for (uint32_t i = 0; i < L1; ++i) {
        const uint32_t sl = t + B3_FOLD_T * i, gl = sl / 32, j = sl % 32, cnt = s_cnt[gl];
        const uint32_t l[8] = {lv[i][0][0].x, lv[i][0][0].y, lv[i][0][0].z, lv[i][0][0].w,
                               lv[i][0][1].x, lv[i][0][1].y, lv[i][0][1].z, lv[i][0][1].w};
        const uint32_t r[8] = {lv[i][1][0].x, lv[i][1][0].y, lv[i][1][0].z, lv[i][1][0].w,
                               lv[i][1][1].x, lv[i][1][1].y, lv[i][1][1].z, lv[i][1][1].w};
        uint32_t p[8];
        b3_parent(l, r, s_whole[gl] && cnt == 2, p);  // every lane (full exec mask)
        const bool pair = j < cnt / 2, carry = (cnt & 1u) && j == cnt / 2 && cnt > 1;
        if (pair || carry)
#pragma unroll
            for (int k = 0; k < 8; ++k) s_node[gl][j][k] = pair ? p[k] : l[k];
    }
    __syncthreads();
    if (t < B3_FOLD_G) {
        const uint32_t c0 = s_cnt[t];
        if (c0 == 1) {  // a one-leaf group (a chunk's last 1 KiB) has no level-1 parent: its leaf is node 0
            const uint4 *q = reinterpret_cast<const uint4 *>(lcv + (g0 + t) * 64 * 8);
            const uint4 x = q[0], y = q[1];
            uint32_t *d = s_node[t][0];
            d[0] = x.x, d[1] = x.y, d[2] = x.z, d[3] = x.w, d[4] = y.x, d[5] = y.y, d[6] = y.z, d[7] = y.w;
        }
        s_cnt[t] = c0 > 1 ? (c0 + 1) >> 1 : c0;
    }
    __syncthreads();
    // levels 2..6 in LDS: (32 >> (L - 1)) parent slots per group.  (Rotating which of the 4
    // waves are live at levels 3-6 by the block index, so that the blocks sharing a CU would
    // use different SIMDs, measured 48.3 against 47.0 us per config-3 batch: not the limit.)
    const uint32_t tr = t;
#pragma unroll 1
    for (uint32_t lvl = 2; lvl <= 6; ++lvl) {
        const uint32_t per = 64u >> lvl;
        const uint32_t slots = B3_FOLD_G * per;
#pragma unroll 1
        for (uint32_t base = 0; base < slots; base += B3_FOLD_T) {
            const uint32_t sl = base + tr, gl = (sl / per) % B3_FOLD_G, j = sl % per;
            const uint32_t cnt = sl < slots ? s_cnt[gl] : 0u;
            const bool pair = j < cnt / 2, carry = (cnt & 1u) && j == cnt / 2 && cnt > 1;
            uint32_t l[8], p[8];
            // waves wholly past the level's slots skip the compression (uniform per wave)
            const bool wave_live = base + (tr & ~63u) < slots;
            if (wave_live) {
                uint32_t r[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    l[i] = s_node[gl][(2 * j) & 31][i];
                    r[i] = s_node[gl][(2 * j + 1) & 31][i];
                }
                // every lane of a live wave compresses (full exec mask); pair lanes keep it
                b3_parent(l, r, s_whole[gl] && cnt == 2, p);
            }
            __syncthreads();
            if (pair || carry)
#pragma unroll
                for (int i = 0; i < 8; ++i) s_node[gl][j][i] = pair ? p[i] : l[i];
            __syncthreads();
        }
        if (t < B3_FOLD_G) s_cnt[t] = (s_cnt[t] + 1) >> 1;
        __syncthreads();
    }
    if (t < B3_FOLD_G) {
        const uint64_t g = g0 + t;
        if (g < ng && s_cnt[t]) {  // 1 node left
            const uint32_t *w = s_node[t][0];
            const uint32_t cv[8] = {w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7]};
            if (s_whole[t]) {
                store_digest(hash_base + (uint64_t)gmap[g] * stride, cv);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) gcv[g * 8 + i] = cv[i];
            }
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
        b3_wave_fold<true>(cv, count, true, lane);  // full exec mask: the wave is alone on its SIMD
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
    b3_wave_fold<true>(cv, count, true, lane);
    if (lane == 0) store_digest(hash_base + c * stride, cv);
}

#ifdef CG_DIAG
uint32_t g_b3_diag = 0;  // set by cg_diag_b3_mode (diagnostics build only)

// Compression throughput microbenchmark (diagnostics): K independent compression chains
// per lane, interleaved op by op, no memory traffic.
template <int K>
__device__ __forceinline__ void b3_compress_k(uint32_t (&cv)[K][8], const uint32_t (&mm)[K][16], uint32_t ctr) {
    uint32_t v[K][16];
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            v[k][i] = cv[k][i];
            v[k][i + 8] = B3_IV[i];
        }
        v[k][12] = ctr;
        v[k][13] = 0;
        v[k][14] = 64;
        v[k][15] = 0;
    }
    auto g = [&](int a, int b, int c, int d, int x, int y) {
#pragma unroll
        for (int k = 0; k < K; ++k) v[k][a] = v[k][a] + v[k][b] + mm[k][x];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k][d] = rotr32b(v[k][d] ^ v[k][a], 16);
#pragma unroll
        for (int k = 0; k < K; ++k) v[k][c] = v[k][c] + v[k][d];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k][b] = rotr32b(v[k][b] ^ v[k][c], 12);
#pragma unroll
        for (int k = 0; k < K; ++k) v[k][a] = v[k][a] + v[k][b] + mm[k][y];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k][d] = rotr32b(v[k][d] ^ v[k][a], 8);
#pragma unroll
        for (int k = 0; k < K; ++k) v[k][c] = v[k][c] + v[k][d];
#pragma unroll
        for (int k = 0; k < K; ++k) v[k][b] = rotr32b(v[k][b] ^ v[k][c], 7);
    };
#pragma unroll
    for (int r = 0; r < 7; ++r) {
        const uint8_t *s = B3S.s[r];
        g(0, 4, 8, 12, s[0], s[1]);
        g(1, 5, 9, 13, s[2], s[3]);
        g(2, 6, 10, 14, s[4], s[5]);
        g(3, 7, 11, 15, s[6], s[7]);
        g(0, 5, 10, 15, s[8], s[9]);
        g(1, 6, 11, 12, s[10], s[11]);
        g(2, 7, 8, 13, s[12], s[13]);
        g(3, 4, 9, 14, s[14], s[15]);
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) cv[k][i] = v[k][i] ^ v[k][i + 8];
}

template <int K>
__global__ void k_diag_b3_chain(uint32_t iters, uint32_t *out) {
    uint32_t cv[K][8], mm[K][16];
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int i = 0; i < 8; ++i) cv[k][i] = threadIdx.x * 0x9E3779B9u + i + 131 * k;
#pragma unroll
        for (int i = 0; i < 16; ++i) mm[k][i] = (threadIdx.x ^ blockIdx.x) * 0x85EBCA6Bu + i * 0x01010101u + k;
    }
    for (uint32_t it = 0; it < iters; ++it) b3_compress_k<K>(cv, mm, it);
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) x ^= cv[k][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// the macro-interleaved product compression (B3_G4), one chain per lane
__global__ void k_diag_b3_chain_g4(uint32_t iters, uint32_t *out) {
    uint32_t cv[8], m[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = threadIdx.x * 0x9E3779B9u + i;
#pragma unroll
    for (int i = 0; i < 16; ++i) m[i] = (threadIdx.x ^ blockIdx.x) * 0x85EBCA6Bu + i * 0x01010101u;
    for (uint32_t it = 0; it < iters; ++it) b3_compress(cv, m, it, 64, 0);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= cv[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
#endif

size_t blake3_leaf_wave_bound(uint64_t total_bytes, uint64_t max_chunks) {
    return (total_bytes / 1024 + max_chunks + 63) / 64 + 1;
}
size_t blake3_group_bound(uint64_t total_bytes, uint64_t max_chunks) {
    return total_bytes / 65536 + max_chunks + 1;  // an upper bound for every leaves-per-lane setting
}
// group chaining values (gcv), then 64 leaf chaining values per group (lcv, the deferred
// folds of launch_blake3 with with_lcv)
size_t blake3_cv_bytes(uint64_t total_bytes, uint64_t max_chunks, bool with_lcv) {
    return (blake3_group_bound(total_bytes, max_chunks) + 1) * 32 * (with_lcv ? 65 : 1);
}

void launch_blake3(const uint8_t *d_data, const uint64_t *d_abs, const void *d_desc, const uint64_t *d_total,
                   uint64_t max_chunks, uint64_t total_bytes, uint8_t *d_hash_base, size_t hash_stride,
                   uint32_t *d_gmap, uint64_t *d_group_base, uint32_t *d_gcount_u32, uint64_t *d_scan_tmp,
                   uint32_t *d_gcv, bool with_lcv, hipStream_t st, bool plan_ready, const uint64_t *d_leaf_base,
                   const uint32_t *d_lmap) {
    if (max_chunks == 0) return;
    const DescRaw *desc = (const DescRaw *)d_desc;
    const uint32_t cblocks = (uint32_t)((max_chunks + 255) / 256);
    // product: one leaf per lane, folds deferred to k_b3_fold when the caller sized d_gcv
    // for the leaf values (with_lcv), else folded in-wave
    auto count = k_b3_count<1>;
    auto plan = k_b3_plan<1>;
    bool defer = with_lcv;
    auto groups = defer ? k_b3_groups<0, 1, true> : k_b3_groups<0, 1>;
    uint64_t gbound = blake3_group_bound(total_bytes, max_chunks);
    uint32_t *d_lcv = d_gcv + (gbound + 1) * 8;
#ifdef CG_DIAG
    // 1 / 5: no leaf loads (deferred / in-wave fold); 2 / 4: in-wave fold, full-exec / none;
    // 8: in-wave fold (round-2 v11); 16: 4-leaf lane subtrees + in-wave fold
    if (g_b3_diag) defer = with_lcv && g_b3_diag == 1;
    switch (g_b3_diag) {
    case 1: groups = defer ? k_b3_groups<1, 1, true> : k_b3_groups<1, 1>; break;
    case 2: groups = k_b3_groups<2, 1>; break;
    case 4: groups = k_b3_groups<4, 1>; break;
    case 5: groups = k_b3_groups<1, 1>; break;
    case 8: groups = k_b3_groups<0, 1>; break;
    case 16:
        groups = k_b3_groups<0, 4>;
        count = k_b3_count<4>;
        plan = k_b3_plan<4>;
        gbound = total_bytes / (65536 * 4) + max_chunks + 1;
        break;
    default: break;
    }
#endif
    // (a forced scan path, cg_test_scan_path, takes the three-kernel form so tests reach it)
    if (plan_ready) {
        // group_base / gmap came with the descriptor assembly (k_assemble_counts)
    } else if (max_chunks <= B3_PLAN_MAX && g_scan_path == 0) {
        hipLaunchKernelGGL(plan, dim3(1), dim3(B3_PLAN_T), 0, st, desc, d_total, max_chunks, d_group_base, d_gmap);
    } else {
        hipLaunchKernelGGL(count, dim3(cblocks), dim3(256), 0, st, desc, d_total, max_chunks, d_gcount_u32);
        launch_exclusive_scan_u32(d_gcount_u32, d_group_base, max_chunks, 0, d_scan_tmp, st);
        hipLaunchKernelGGL(k_b3_map, dim3(cblocks), dim3(256), 0, st, d_group_base, d_total, max_chunks, d_gmap);
    }
    if (plan_ready && d_leaf_base && defer) {
        // packed leaves: at most total_bytes / 1 KiB + one partial leaf per chunk
        const uint64_t wbound = (total_bytes / 1024 + max_chunks + 63) / 64;
        hipLaunchKernelGGL(k_b3_leaves, dim3((uint32_t)((wbound + B3_WAVES - 1) / B3_WAVES)), dim3(64 * B3_WAVES), 0, st,
                           d_data, d_abs, desc, d_total, max_chunks, d_group_base, d_leaf_base, d_lmap, d_hash_base,
                           hash_stride, d_lcv);
    } else {
        hipLaunchKernelGGL(groups, dim3((uint32_t)((gbound + B3_WAVES - 1) / B3_WAVES)), dim3(64 * B3_WAVES), 0, st,
                           d_data, d_abs, desc, d_total, max_chunks, d_group_base, d_gmap, d_hash_base, hash_stride,
                           d_gcv, d_lcv);
    }
    if (defer)
        hipLaunchKernelGGL(k_b3_fold, dim3((uint32_t)((gbound + B3_FOLD_G - 1) / B3_FOLD_G)), dim3(B3_FOLD_T), 0, st, desc,
                           d_total, max_chunks, d_group_base, d_gmap, d_lcv, d_hash_base, hash_stride, d_gcv);
    hipLaunchKernelGGL(k_b3_top, dim3((uint32_t)max_chunks), dim3(64), 0, st, desc, d_total, max_chunks,
                       d_group_base, d_gcv, d_hash_base, hash_stride);
}

}  // namespace cg

#ifdef CG_DIAG
// ms for `blocks` x `threads` lanes each running `iters` x K compressions (kind 0: the
// product's B3_G4 compression, K = 1; kind K = 1, 2, 4: K interleaved chains)
extern "C" float cg_diag_b3_chain(int kind, uint32_t blocks, uint32_t threads, uint32_t iters) {
    uint32_t *d_out = nullptr;
    if (hipMalloc(&d_out, (size_t)blocks * threads * 4) != hipSuccess) return -1.f;
    auto k = kind == 0 ? cg::k_diag_b3_chain_g4
             : kind == 1 ? cg::k_diag_b3_chain<1>
             : kind == 2 ? cg::k_diag_b3_chain<2>
                         : cg::k_diag_b3_chain<4>;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, iters / 8 + 1, d_out);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, iters, d_out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(d_out);
    return ms;
}
#endif
