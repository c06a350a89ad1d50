// cas.hip -- K5: CAS content identifiers, the second per-chunk
// digest of the reference's ingest path.  Node::put (crates/node/src/lib.rs:114-132)
// stores every chunk under
//   ContentId::compute(kind, payload) = SHAKE256-256("flakecache-cas" || 0x00 ||
//       kind || u16le(FORMAT_VERSION = 1) || u64le(payload.len()) || payload)
// (crates/core/cas/src/lib.rs:23-26, :53-69; shake256_256 in
// crates/core/crypto/src/hash.rs:34-41), and the manifest (the ordered chunk ids)
// under kind Level1Manifest (crates/node/src/lib.rs:124-129).
//
// One lane absorbs one span: a Keccak-f[1600] sponge (FIPS 202; rate 136 B, SHAKE
// padding 0x1F .. 0x80) with the 25 lanes of state as 50 dword registers, every
// 64-bit rotation two v_alignbit, theta's parities and the a ^= d fold as
// v_bitop3 xor3, chi as one v_bitop3 per dword.  The sponge is serial per span, so
// like SHA-256 this stage is bound by the chain of its longest span; lanes take spans
// longest first (the SHA-256 length order) so a wave's lanes finish together.
#include "common.h"

namespace cg {

namespace {

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// a ^ (~b & c)
__device__ __forceinline__ uint32_t chi3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xD2);
}

// rotl64 on (lo, hi) by a compile-time r in [1, 63]
template <int R>
__device__ __forceinline__ void rot(uint32_t lo, uint32_t hi, uint32_t &olo, uint32_t &ohi) {
    if constexpr (R == 0) {
        olo = lo;
        ohi = hi;
    } else if constexpr (R < 32) {
        ohi = __builtin_amdgcn_alignbit(hi, lo, 32 - R);
        olo = __builtin_amdgcn_alignbit(lo, hi, 32 - R);
    } else if constexpr (R == 32) {
        olo = hi;
        ohi = lo;
    } else {
        ohi = __builtin_amdgcn_alignbit(lo, hi, 64 - R);
        olo = __builtin_amdgcn_alignbit(hi, lo, 64 - R);
    }
}

__constant__ uint32_t KRC_LO[24] = {0x00000001u, 0x00008082u, 0x0000808au, 0x80008000u, 0x0000808bu, 0x80000001u,
                                    0x80008081u, 0x00008009u, 0x0000008au, 0x00000088u, 0x80008009u, 0x8000000au,
                                    0x8000808bu, 0x0000008bu, 0x00008089u, 0x00008003u, 0x00008002u, 0x00000080u,
                                    0x0000800au, 0x8000000au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
__constant__ uint32_t KRC_HI[24] = {0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u,
                                    0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u,
                                    0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u,
                                    0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};

// rho offsets r[x + 5y] (FIPS 202 Table 2)
#define KR(i) ((i) == 0 ? 0 : (i) == 1 ? 1 : (i) == 2 ? 62 : (i) == 3 ? 28 : (i) == 4 ? 27 : (i) == 5 ? 36 \
    : (i) == 6 ? 44 : (i) == 7 ? 6 : (i) == 8 ? 55 : (i) == 9 ? 20 : (i) == 10 ? 3 : (i) == 11 ? 10 : (i) == 12 ? 43 \
    : (i) == 13 ? 25 : (i) == 14 ? 39 : (i) == 15 ? 41 : (i) == 16 ? 45 : (i) == 17 ? 15 : (i) == 18 ? 21 \
    : (i) == 19 ? 8 : (i) == 20 ? 18 : (i) == 21 ? 2 : (i) == 22 ? 61 : (i) == 23 ? 56 : 14)

// rho + pi for lane i = x + 5y: B[y + 5((2x + 3y) % 5)] = rot(A[i], r[i])
template <int I>
__device__ __forceinline__ void rho_pi(const uint32_t *lo, const uint32_t *hi, uint32_t *blo, uint32_t *bhi) {
    constexpr int x = I % 5, y = I / 5, j = y + 5 * ((2 * x + 3 * y) % 5);
    rot<KR(I)>(lo[I], hi[I], blo[j], bhi[j]);
    if constexpr (I < 24) rho_pi<I + 1>(lo, hi, blo, bhi);
}

// Keccak-f[1600] on (lo[25], hi[25]), lanes A[x + 5y].  Fully unrolled: with the
// rounds in a loop the B -> A renaming costs ~70 v_mov_b64 per round.
__device__ __forceinline__ void keccak_f(uint32_t lo[25], uint32_t hi[25]) {
#pragma unroll
    for (int round = 0; round < 24; ++round) {
        uint32_t clo[5], chi_[5], blo[25], bhi[25];
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            clo[x] = x3(x3(lo[x], lo[x + 5], lo[x + 10]), lo[x + 15], lo[x + 20]);
            chi_[x] = x3(x3(hi[x], hi[x + 5], hi[x + 10]), hi[x + 15], hi[x + 20]);
        }
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            uint32_t rlo, rhi;
            rot<1>(clo[(x + 1) % 5], chi_[(x + 1) % 5], rlo, rhi);
#pragma unroll
            for (int y = 0; y < 5; ++y) {
                lo[x + 5 * y] = x3(lo[x + 5 * y], clo[(x + 4) % 5], rlo);
                hi[x + 5 * y] = x3(hi[x + 5 * y], chi_[(x + 4) % 5], rhi);
            }
        }
        rho_pi<0>(lo, hi, blo, bhi);
#pragma unroll
        for (int y = 0; y < 5; ++y)
#pragma unroll
            for (int x = 0; x < 5; ++x) {
                lo[x + 5 * y] = chi3(blo[x + 5 * y], blo[(x + 1) % 5 + 5 * y], blo[(x + 2) % 5 + 5 * y]);
                hi[x + 5 * y] = chi3(bhi[x + 5 * y], bhi[(x + 1) % 5 + 5 * y], bhi[(x + 2) % 5 + 5 * y]);
            }
        lo[0] ^= KRC_LO[round];
        hi[0] ^= KRC_HI[round];
    }
}

// ---------------------------------------------------------------------------
// Pair tier: one span on a lane pair, lane h = 0 holding the low dwords of the 25
// state lanes and h = 1 the high dwords.  Every 64-bit rotation is then the same
// instruction on both lanes, new_own = alignbit(own, other) (r < 32) or
// alignbit(other, own) (r > 32), with `other` the partner's half through one DPP
// quad_perm swap; theta's parities, the a ^= d fold and chi touch only the lane's own
// half.  ~120 VALU per round instead of ~180, so the longest span's chain is ~1.5x
// shorter.
// ---------------------------------------------------------------------------
// The partner's value (quad_perm [1,0,3,2]).  A v_mov_b32 -- DPP or not -- issues in ~8
// clocks on gfx950 against ~4.9 for a DPP ALU op (scripts/diag_ops.py,
// profiles/r02_v7_diag_ops_mov.json), so the move is written as an add of an opaque
// zero, which the compiler's DPP combine turns into one v_add_u32_dpp.
__device__ __forceinline__ uint32_t partner(uint32_t v, uint32_t zero) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true) + zero;
}

template <int R>
__device__ __forceinline__ uint32_t rot_pair(uint32_t own, uint32_t zero) {
    if constexpr (R == 0) {
        return own;
    } else if constexpr (R < 32) {
        return __builtin_amdgcn_alignbit(own, partner(own, zero), 32 - R);
    } else if constexpr (R == 32) {
        return partner(own, zero);
    } else {
        return __builtin_amdgcn_alignbit(partner(own, zero), own, 64 - R);
    }
}

template <int I>
__device__ __forceinline__ void rho_pi_pair(const uint32_t *a, uint32_t *b, uint32_t zero) {
    constexpr int x = I % 5, y = I / 5, j = y + 5 * ((2 * x + 3 * y) % 5);
    b[j] = rot_pair<KR(I)>(a[I], zero);
    if constexpr (I < 24) rho_pi_pair<I + 1>(a, b, zero);
}

// hmask = 0 on the low lane, ~0 on the high lane
__device__ __forceinline__ void keccak_f_pair(uint32_t a[25], uint32_t hmask) {
    uint32_t zero = 0;
    asm volatile("" : "+v"(zero));  // a VGPR the compiler cannot fold away (see partner)
#pragma unroll
    for (int round = 0; round < 24; ++round) {
        uint32_t c[5], b[25];
#pragma unroll
        for (int x = 0; x < 5; ++x) c[x] = x3(x3(a[x], a[x + 5], a[x + 10]), a[x + 15], a[x + 20]);
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            const uint32_t d = rot_pair<1>(c[(x + 1) % 5], zero);
#pragma unroll
            for (int y = 0; y < 5; ++y) a[x + 5 * y] = x3(a[x + 5 * y], c[(x + 4) % 5], d);
        }
        rho_pi_pair<0>(a, b, zero);
#pragma unroll
        for (int y = 0; y < 5; ++y)
#pragma unroll
            for (int x = 0; x < 5; ++x)
                a[x + 5 * y] = chi3(b[x + 5 * y], b[(x + 1) % 5 + 5 * y], b[(x + 2) % 5 + 5 * y]);
        // iota: own half of RC = lo ^ ((lo ^ hi) & hmask)
        a[0] ^= KRC_LO[round] ^ ((KRC_LO[round] ^ KRC_HI[round]) & hmask);
    }
}

constexpr uint32_t CAS_HDR = 26;   // "flakecache-cas" 0x00 kind u16le(1) u64le(len)
constexpr uint32_t CAS_RATE = 136; // SHAKE256 rate in bytes (17 lanes)

// Message byte m of a span's framed message (header, then payload); 0 past the end.
__device__ __forceinline__ uint32_t msg_byte(const uint8_t *pay, uint64_t len, uint32_t kind, uint64_t m) {
    if (m >= CAS_HDR) return m - CAS_HDR < len ? pay[m - CAS_HDR] : 0u;
    constexpr char dom[15] = "flakecache-cas";
    if (m < 14) return (uint8_t)dom[m];
    if (m == 14) return 0u;
    if (m == 15) return kind;
    if (m == 16) return 1u;  // FORMAT_VERSION = 1, u16 little-endian
    if (m == 17) return 0u;
    return (uint32_t)(len >> (8 * (m - 18))) & 0xFFu;
}

// Block k (k >= 1) lies wholly inside the payload: its 136 bytes start at payload
// byte 136k - 26.  The 35 aligned dwords covering them are loaded once and realigned
// with v_alignbyte (the byte shift is the same for every block since 136 % 4 == 0).
__device__ __forceinline__ bool whole_block(uint64_t k, uint64_t mlen) {
    return k > 0 && (k + 1) * CAS_RATE <= mlen;
}

}  // namespace

// Absorb-and-permute of one span.  PAIR: the calling lane holds half `h` of the
// state (see keccak_f_pair); otherwise the whole state.  Writes the 32-byte id.
template <bool PAIR>
__device__ __forceinline__ void cas_span(const uint8_t *pay, uint64_t len, uint32_t kind, uint32_t h, uint8_t *id) {
    const uint64_t mlen = CAS_HDR + len;
    const uint64_t nblk = mlen / CAS_RATE + 1;  // the pad block always exists (mlen % rate < rate)
    const uint32_t shift = (uint32_t)((uintptr_t)pay & 3u);
    const uint32_t *base0 = reinterpret_cast<const uint32_t *>(pay - shift);
    const uint32_t sh = (shift + 2u) & 3u;
    constexpr int NW = PAIR ? 25 : 50;  // state dwords held by this lane
    constexpr int ND = PAIR ? 34 : 35;  // block dwords loaded by this lane
    uint32_t a[NW], dw[ND];
#pragma unroll
    for (int i = 0; i < NW; ++i) a[i] = 0;
    // Aligned dwords of whole block k: payload bytes [136k - 26, 136k + 110) start
    // at dword (136k - 26 + shift) / 4 of base0, byte sh = (shift + 2) & 3 of it (136k - 26
    // is 2 mod 4).  The last dword is needed only when sh > 0 and then lies inside the
    // payload, so no load leaves the span.  A pair lane reads its stream one dword later
    // on the high lane, so its halves are dw[2i], dw[2i + 1] on both lanes.
    auto load_whole = [&](uint64_t k) {
        const uint32_t *b = base0 + ((k * CAS_RATE - CAS_HDR + shift) >> 2) + h;
#pragma unroll
        for (int i = 0; i < ND - 1; ++i) dw[i] = __builtin_nontemporal_load(b + i);
        dw[ND - 1] = (sh || (PAIR && !h)) ? __builtin_nontemporal_load(b + ND - 1) : 0u;
    };
    if (whole_block(1, mlen)) load_whole(1);
    for (uint64_t k = 0; k < nblk; ++k) {
        if (whole_block(k, mlen)) {
#pragma unroll
            for (int i = 0; i < 17; ++i) {
                if constexpr (PAIR) {
                    a[i] ^= __builtin_amdgcn_alignbyte(dw[2 * i + 1], dw[2 * i], sh);
                } else {
                    a[2 * i] ^= __builtin_amdgcn_alignbyte(dw[2 * i + 1], dw[2 * i], sh);
                    a[2 * i + 1] ^= __builtin_amdgcn_alignbyte(dw[2 * i + 2], dw[2 * i + 1], sh);
                }
            }
        } else {  // header block, last partial block or the pad block: byte by byte
            const uint64_t m0 = k * CAS_RATE;
            for (uint32_t i = 0; i < CAS_RATE; ++i) {
                const uint32_t w = i >> 2;  // message dword; state dword w = half (w & 1) of lane w / 2
                if (PAIR && (w & 1u) != h) continue;
                const uint64_t m = m0 + i;
                uint32_t v = m < mlen ? msg_byte(pay, len, kind, m) : 0u;
                if (m == mlen) v ^= 0x1Fu;                          // SHAKE domain bits + first pad bit
                if (k == nblk - 1 && i == CAS_RATE - 1) v ^= 0x80u;  // last pad bit
                const uint32_t sb = 8 * (i & 3);
                if constexpr (PAIR) {
#pragma unroll
                    for (int j = 0; j < 17; ++j)
                        if ((uint32_t)j == (w >> 1)) a[j] ^= v << sb;
                } else {
#pragma unroll
                    for (int j = 0; j < 34; ++j)
                        if ((uint32_t)j == w) a[j] ^= v << sb;
                }
            }
        }
        if (whole_block(k + 1, mlen)) load_whole(k + 1);  // in flight during the permutation
        if constexpr (PAIR) {
            keccak_f_pair(a, h ? ~0u : 0u);
        } else {
            uint32_t lo[25], hi[25];
#pragma unroll
            for (int i = 0; i < 25; ++i) {
                lo[i] = a[2 * i];
                hi[i] = a[2 * i + 1];
            }
            keccak_f(lo, hi);
#pragma unroll
            for (int i = 0; i < 25; ++i) {
                a[2 * i] = lo[i];
                a[2 * i + 1] = hi[i];
            }
        }
    }
    uint32_t *o = reinterpret_cast<uint32_t *>(id);
    if constexpr (PAIR) {
#pragma unroll
        for (int i = 0; i < 4; ++i) o[2 * i + h] = a[i];
    } else {
        reinterpret_cast<uint4 *>(id)[0] = make_uint4(a[0], a[1], a[2], a[3]);
        reinterpret_cast<uint4 *>(id)[1] = make_uint4(a[4], a[5], a[6], a[7]);
    }
}

// Slots take spans in the SHA-256 length order (longest first; `order` may be null).
// Workgroups [0, npair_wg) run the pair tier on slots [0, 32 npair_wg), the rest one
// lane per span.  Span g: bytes data[abs[g] .. abs[g] + desc[g].length); its id ->
// ids + g * id_stride.
__global__ __launch_bounds__(64) void k_cas_ids(const uint8_t *__restrict__ data, const uint64_t *__restrict__ abs,
                                                const DescRaw *__restrict__ desc, const uint64_t *__restrict__ total_p,
                                                uint64_t max_n, const uint32_t *__restrict__ order, uint32_t kind,
                                                uint8_t *__restrict__ ids, uint64_t id_stride, uint32_t npair_wg) {
    uint64_t total = *total_p;
    if (total > max_n) total = max_n;
    const bool pair = blockIdx.x < npair_wg;
    const uint64_t slot = pair ? (uint64_t)blockIdx.x * 32 + (threadIdx.x >> 1)
                               : (uint64_t)npair_wg * 32 + (uint64_t)(blockIdx.x - npair_wg) * 64 + threadIdx.x;
    if (slot >= total) return;  // pair lanes leave together: both halves share the slot
    const uint64_t g = order ? (uint64_t)order[slot] : slot;
    const uint8_t *pay = data + abs[g];
    if (pair)
        cas_span<true>(pay, desc[g].length, kind, threadIdx.x & 1u, ids + id_stride * g);
    else
        cas_span<false>(pay, desc[g].length, kind, 0, ids + id_stride * g);
}

uint64_t g_cas_wave_budget = 1024;  // SIMDs of the chip
int64_t g_cas_pair_max = -1;        // diagnostics/tests: cap on pair-tier spans (-1 = none)

void launch_cas_ids(const uint8_t *d_data, const uint64_t *d_abs, const void *d_desc, const uint64_t *d_total,
                    uint64_t max_n, const uint32_t *d_order, uint32_t kind, uint8_t *d_ids, size_t id_stride,
                    hipStream_t st) {
    if (max_n == 0) return;
    // Pair tier for the longest spans while the whole grid still fits one wave per SIMD
    // (256 CUs x 4): npair spans cost npair / 64 extra waves over the one-lane grid.
    const uint64_t single_waves = (max_n + 63) / 64;
    uint64_t npair = single_waves < g_cas_wave_budget ? 64 * (g_cas_wave_budget - single_waves) : 0;
    if (npair > max_n) npair = max_n;
    if (g_cas_pair_max >= 0 && npair > (uint64_t)g_cas_pair_max) npair = (uint64_t)g_cas_pair_max;
    const uint32_t npair_wg = (uint32_t)((npair + 31) / 32);
    const uint64_t rest = max_n > 32 * (uint64_t)npair_wg ? max_n - 32 * (uint64_t)npair_wg : 0;
    const uint32_t nwg = npair_wg + (uint32_t)((rest + 63) / 64);
    hipLaunchKernelGGL(k_cas_ids, dim3(nwg), dim3(64), 0, st, d_data, d_abs, (const DescRaw *)d_desc, d_total, max_n,
                       d_order, kind, d_ids, (uint64_t)id_stride, npair_wg);
}

// Manifest spans (crates/node/src/lib.rs:124-129): NAR i's manifest is the
// concatenation of its chunk ids, i.e. bytes [32 first[i], 32 first[i+1]) of the id
// buffer.  Writes the (abs, desc.length) span view the CAS kernel reads.
__global__ void k_manifest_spans(const uint64_t *__restrict__ first, uint64_t n_nars, uint64_t *__restrict__ abs,
                                 DescRaw *__restrict__ desc, uint64_t *__restrict__ total) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *total = n_nars;
    if (i >= n_nars) return;
    abs[i] = 32 * first[i];
    desc[i].offset = 32 * first[i];
    desc[i].length = 32 * (first[i + 1] - first[i]);
}

void launch_manifest_spans(const uint64_t *d_first, uint64_t n_nars, uint64_t *d_abs, void *d_desc, uint64_t *d_total,
                           hipStream_t st) {
    hipLaunchKernelGGL(k_manifest_spans, dim3((uint32_t)(n_nars ? (n_nars + 255) / 256 : 1)), dim3(256), 0, st,
                       d_first, n_nars, d_abs, (DescRaw *)d_desc, d_total);
}

}  // namespace cg

// Test hook: cap the pair tier (-1 = budget only, 0 = one lane per span everywhere) so
// the parity tests can force every tier mix; returns the previous cap.
extern "C" int64_t cg_test_cas_pair_max(int64_t v) {
    const int64_t old = cg::g_cas_pair_max;
    cg::g_cas_pair_max = v;
    return old;
}
