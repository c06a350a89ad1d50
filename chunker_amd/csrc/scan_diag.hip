// scan_diag.hip -- diagnostics build only (make diag; -DCG_DIAG): the alternative K1
// candidate-scan kernels kept for the A/B measurements recorded in DESIGN.md §4
// (scripts/diag_scan.py, tests/test_gpu_parity.py::test_diag_scan_variants_agree):
// k_scan_flat (16-byte lane blocks, the round-2 v3..v12 product, by FORM), the round-1
// quad-transpose kernel k_scan_quad, the LDS-staged k_scan_lds and the page-per-wave
// k_scan_wave.  The product kernels live in scan.hip.
#include <algorithm>
#include <cstdlib>

#include "scan_common.h"

#ifdef CG_DIAG
namespace cg {

uint32_t g_scan_diag = 0;     // set by cg_diag_scan_mode (quad-kernel diag modes)
uint32_t g_scan_variant = 0;  // set by cg_diag_scan_variant: 1 quad, 2 LDS-staged, 3 page per wave, 4 k_scan, 5 flat rows
uint32_t g_scan_spw_max = 0;  // set by cg_diag_scan_spw_max: k_scan_flat's segments-per-wave cap (0 = default)

// ---------------------------------------------------------------------------
// K1, flat form: the product kernel for prefilterable masks (k_scan<false> for the
// rest).  k_scan gives every lane
// its own 4 KiB stream, and 64 per-lane streams read HBM at ~4.4-4.9 TB/s whatever the
// run length (scripts/diag_scan.py read patterns); whole 1 KiB rows per wave-instruction
// read at ~5.8-6.4.  So here a wave walks a run of `spw` consecutive segments as 1 KiB
// rows, lane L holding bytes [16 L, 16 L + 16) of each row (one dwordx4, the row
// contiguous), and the hash crosses lanes by linearity instead of by a warm-up:
//  * in the shifted representation H' = H << 16 (k_scan), a byte k positions back
//    contributes GEAR'[b] << k, which vanishes mod 2^64 for k >= 48: H' at any position
//    is exactly the sum over the 48 bytes before it (SURVEY.md App. A.3's window);
//  * lane L forms P_L = sum_j GEAR'[b_j] << (15 - j) over its 16 bytes (16 lookups, a
//    shift-add chain), and the state entering its block is
//    C_L = P_{L-1} + (P_{L-2} << 16) + (P_{L-3} << 32): three DPP wave_ror:1 rotations,
//    lanes 0..2 taking the previous row's lanes 61..63 from the rotation kept over from
//    the previous row (one v_bitop3 select each);
//  * from C_L the lane re-runs its 16 steps with the prefilter (one v_and_b32 + 1/2
//    v_min3_u32 per byte, as k_scan);
//  * a row where any lane's prefilter fires (wave-uniform branch, rare) re-runs the 16
//    steps exactly from the registers into per-lane S / L position masks, places the
//    candidates with a wave prefix sum into a per-wave LDS slot list (no global stores inside the row loop: vmcnt keeps counting
//    the load ring exactly), and every 4th row flushes the finished segment's slots and
//    count.
// Per byte: 1 SDWA mov + 1 ds_read_b64 + 2 v_lshl_add_u64 + 1 v_and_b32 + 1/2 v_min3_u32,
// plus 5 DPP adds + 5 selects + ~4 VALU per 16 bytes.
// Round-2 v11/v12 product form (FORM 5; since v13 the product is k_scan_flat32, below,
// which takes the same steps over 32-byte lane blocks): the 16 steps as split chains (split_partials: 6 + 4 dependent
// v_lshl_add_u64 per row instead of 15 + 16), rows handled in pairs -- both rows' lookups,
// chains and prefilters, then ONE wave-uniform verdict branch; the rare exact path redoes
// a row's lookups from its ring slot, so only C stays live across the branch -- an 8-row
// ring re-issued after each pair, runs of <= 32 segments per wave (launch_scan): config 2
// 0.237 -> 0.203-0.206 ms per GiB, 5.2-5.8 TB/s on configs 2, 4 and 5
// (profiles/r02_v10_diag_scan_split.json).
// ---------------------------------------------------------------------------
#define FLAT_ROW 1024u  // bytes per wave row (64 lanes x 16 B)
#define FLAT_RPS (CG_SEG / FLAT_ROW)  // rows per segment
static_assert(CG_SEG % FLAT_ROW == 0, "whole rows per segment");// the 16 table entries of one lane's 16-byte block
__device__ __forceinline__ void block_lookups(const char *gbase, uint32_t (&ad)[2][4], const uint4 v,
                                              uint64_t (&g)[4][4]) {
    lookup4(gbase, ad[0], v.x, g[0]);
    lookup4(gbase, ad[1], v.y, g[1]);
    lookup4(gbase, ad[0], v.z, g[2]);
    lookup4(gbase, ad[1], v.w, g[3]);
}
__device__ __forceinline__ uint64_t block_partial(const uint64_t (&g)[4][4]) {
    uint64_t P = g[0][0];
#pragma unroll
    for (int i = 1; i < 16; ++i) P = shl1_add(P, g[i >> 2][i & 3]);
    return P;
}
// Split chains: the 16 steps of a lane block as four independent 4-byte chains.
// q[k][b] = sum_{i<=b} GEAR'[byte 4k+i] << (b-i) (q[k][0] = g[k][0]); the block partial
// P = ((q0 << 4 + q1) << 4 + q2) << 4 + q3 (the [3] entries), and from the incoming state C
// the hash after byte 4k+b is (E_{k-1} << (b+1)) + q[k][b] with E_{-1} = C and
// E_k = (E_{k-1} << 4) + q[k][3] -- the same 31 v_lshl_add_u64 as two 16-step chains, but
// 6 + 4 deep instead of 15 + 16.
__device__ __forceinline__ void split_partials(uint64_t (&q)[4][4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        q[k][1] = shl1_add(q[k][0], q[k][1]);
        q[k][2] = shl1_add(q[k][1], q[k][2]);
        q[k][3] = shl1_add(q[k][2], q[k][3]);
    }
}
__device__ __forceinline__ uint64_t split_block(const uint64_t (&q)[4][4]) {
    return shl_add<4>(shl_add<4>(shl_add<4>(q[0][3], q[1][3]), q[2][3]), q[3][3]);
}
// FORM 0 (round-2 v3..v8 product) issues a ring slot's next load after the row; FORM 1 (diagnostics) as soon
// as the row's lookup addresses have consumed its bytes (in flight during the row's hash work:
// measured the same, with 123 VGPRs instead of 114); FORM 2 (diagnostics) loads the rows and
// hashes nothing -- the ceiling of this read schedule (6.6-6.7 TB/s,
// profiles/r02_v8_diag_scan_forms.json); FORM 3 is FORM 0 with split hash chains
// (split_partials), FORM 4 FORM 1 with split chains, FORM 5 (the product) split chains in
// row pairs with one verdict branch per pair, FORM 6 the same in row quads.
template <uint32_t FLAT_D, bool NT, int FORM = 0>
__global__ __launch_bounds__(SCAN2_T, 4) void k_scan_flat(const uint8_t *data, uint64_t n,
                                                      const uint64_t *__restrict__ gear_g, uint64_t mask_s,
                                                      uint64_t mask_l, uint32_t cap, uint32_t *__restrict__ seg_count,
                                                      uint32_t *__restrict__ seg_cand, uint64_t nseg, uint32_t spw) {
    __shared__ __attribute__((aligned(16))) uint64_t s_gear[256 * GEAR_COPIES];
    __shared__ uint32_t s_slots[SCAN2_T / 64][64];  // the open segment's candidate slots, per wave
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t seg0 = ((uint64_t)blockIdx.x * (SCAN2_T / 64) + (threadIdx.x >> 6)) * spw;
    const bool active = seg0 < nseg;  // whole wave (uniform)
    const uint64_t r0 = seg0 * CG_SEG;
    const uint64_t nrow64 = (uint64_t)spw * FLAT_RPS;  // a multiple of FLAT_D (spw even)
    // Loads are unconditional and never leave the batch: a block past its end reads the last
    // block holding a batch byte (a cache hit), so the compiler counts vmcnt exactly through
    // the ring.
    const uint64_t last_abs = (n - 1) & ~(uint64_t)15;
    auto blk = [&](uint64_t row) {
        const uint64_t a = r0 + row * FLAT_ROW + 16u * lane;
        typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
        const u32x4_t *q = reinterpret_cast<const u32x4_t *>(data + (a < last_abs ? a : last_abs));
        const u32x4_t x = NT ? __builtin_nontemporal_load(q) : *q;
        return uint4{x.x, x.y, x.z, x.w};
    };
    static_assert(FLAT_D % FLAT_RPS == 0, "a ring trip ends on a segment boundary");
    // this thread's Gear entry, then the row before the run (lanes 61..63 feed this run's
    // first row) and the first FLAT_D rows: one memory round trip before the table fill
    static_assert(SCAN2_T == 2 * 256 && GEAR_COPIES == 32, "two threads per Gear entry, 16 copies each");
    const uint32_t ge = threadIdx.x >> 1;
    const uint64_t gv = gear_g[ge] << SCAN_SHIFT;
    uint4 ring[FLAT_D];
#pragma unroll
    for (uint32_t i = 0; i < FLAT_D; ++i) ring[i] = blk(active ? i : 0);
    const bool has_pro = active && r0 >= FLAT_ROW;
    const uint4 pro = *reinterpret_cast<const uint4 *>(data + (has_pro ? r0 - FLAT_ROW + 16u * lane : 0));
    __builtin_amdgcn_sched_barrier(0);  // every load above is issued before the fill waits for gv
    // copies rotated by the entry so the 32 threads of a parity write 32 distinct banks
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) s_gear[ge * GEAR_COPIES + (((threadIdx.x & 1u) * 16u + j + ge) & 31u)] = gv;
    __syncthreads();
    if (!active) return;
    const char *gbase = reinterpret_cast<const char *>(s_gear);
    uint32_t *slots = s_slots[threadIdx.x >> 6];
    const uint32_t lo8 = (threadIdx.x & 31u) * 8u;
    uint32_t ad[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int b = 0; b < 4; ++b) ad[i][b] = lo8;
    const uint64_t ms = mask_s << SCAN_SHIFT, ml = mask_l << SCAN_SHIFT;
    const uint32_t mh = (uint32_t)((mask_s & mask_l) >> (32 - SCAN_SHIFT));
    const uint32_t m0 = lane == 0 ? 0xffffffffu : 0u;  // lane-0 select mask (bitop3 0xCA: m ? a : b)
    uint32_t zero = 0;
    asm volatile("" : "+v"(zero));  // a VGPR the compiler cannot fold away (wave_ror1_add)
    const uint32_t ms_lo = (uint32_t)ms, ms_hi = (uint32_t)(ms >> 32), ml_lo = (uint32_t)ml, ml_hi = (uint32_t)(ml >> 32);
    const uint64_t end_rel = n - r0;  // rows reaching past it hold the batch end (a partial block)

    // zero state at the batch start, as the crate's hash restart
    uint64_t R1 = 0, R2 = 0;
    uint32_t R3 = 0;
    if (has_pro) {
        uint64_t g[4][4];
        block_lookups(gbase, ad, pro, g);
        const uint64_t P = block_partial(g);
        R1 = ((uint64_t)wave_ror1((uint32_t)(P >> 32)) << 32) | wave_ror1((uint32_t)P);
        R2 = ((uint64_t)wave_ror1((uint32_t)(R1 >> 32)) << 32) | wave_ror1((uint32_t)R1);
        R3 = wave_ror1((uint32_t)R2);
    }

    uint32_t segc = 0;  // wave-uniform: candidates of the open segment so far
    uint32_t sink = 0;  // FORM 2: the loaded bytes, kept live
    struct RowState {
        uint64_t g[4][4];  // Gear' entries of the lane's 16 bytes (FORM >= 3: split partials q)
        uint64_t C;        // hash state entering the lane's block
        uint32_t acc;      // prefilter: min over the block of (H bits 16..47) & mh
    };
    // the hash after byte j of a lane block, for j = 0, 1, .. in order, x starting at the
    // state entering the block (FORM >= 3: x is E_{k-1})
    auto step = [&](const uint64_t(&g)[4][4], uint64_t &x, uint32_t j) -> uint64_t {
        if constexpr (FORM >= 3) {
            const uint64_t qj = g[j >> 2][j & 3];
            switch (j & 3) {
            case 0: return shl_add<1>(x, qj);
            case 1: return shl_add<2>(x, qj);
            case 2: return shl_add<3>(x, qj);
            default: return x = shl_add<4>(x, qj);
            }
        } else {
            return x = shl1_add(x, g[j >> 2][j & 3]);
        }
    };
    auto next_row = [&](uint64_t row) { return row + FLAT_D < nrow64 ? row + FLAT_D : nrow64 - 1; };
    // lookups, block partial, the cross-lane state C and the prefilter of ring slot u (= row)
    auto front = [&](uint32_t u, uint64_t row, RowState &st) {
        block_lookups(gbase, ad, ring[u], st.g);
        if constexpr (FORM == 1 || FORM == 4) ring[u] = blk(next_row(row));
        uint64_t P;
        if constexpr (FORM >= 3) {
            split_partials(st.g);  // g[k][b] now holds q[k][b]
            P = split_block(st.g);
        } else {
            P = block_partial(st.g);
        }
        // P_{L-1}, P_{L-2}, low dword of P_{L-3}; lanes 0.. take the previous row's
        const uint32_t a_lo = wave_ror1_add((uint32_t)P, zero), a_hi = wave_ror1_add((uint32_t)(P >> 32), zero);
        const uint32_t p1_lo = __builtin_amdgcn_bitop3_b32(m0, (uint32_t)R1, a_lo, 0xCA);
        const uint32_t p1_hi = __builtin_amdgcn_bitop3_b32(m0, (uint32_t)(R1 >> 32), a_hi, 0xCA);
        R1 = ((uint64_t)a_hi << 32) | a_lo;
        const uint32_t b_lo = wave_ror1_add(p1_lo, zero), b_hi = wave_ror1_add(p1_hi, zero);
        const uint32_t p2_lo = __builtin_amdgcn_bitop3_b32(m0, (uint32_t)R2, b_lo, 0xCA);
        const uint32_t p2_hi = __builtin_amdgcn_bitop3_b32(m0, (uint32_t)(R2 >> 32), b_hi, 0xCA);
        R2 = ((uint64_t)b_hi << 32) | b_lo;
        const uint32_t c_lo = wave_ror1_add(p2_lo, zero);
        const uint32_t p3_lo = __builtin_amdgcn_bitop3_b32(m0, R3, c_lo, 0xCA);
        R3 = c_lo;
        // C = P_{L-1} + (P_{L-2} << 16) + (P_{L-3} << 32), the shifted P_{L-2} by dwords
        const uint32_t s_hi = __builtin_amdgcn_alignbit(p2_hi, p2_lo, 16) + p3_lo;
        st.C = (((uint64_t)p1_hi << 32) | p1_lo) + (((uint64_t)s_hi << 32) | (p2_lo << 16));
        uint32_t acc = 0xffffffffu;
        if constexpr (FORM >= 3) {
            uint64_t E = st.C;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t h0 = shl_add<1>(E, st.g[k][0]), h1 = shl_add<2>(E, st.g[k][1]);
                const uint64_t h2 = shl_add<3>(E, st.g[k][2]), h3 = shl_add<4>(E, st.g[k][3]);
                acc = min(min(acc, (uint32_t)(h0 >> 32) & mh), (uint32_t)(h1 >> 32) & mh);
                acc = min(min(acc, (uint32_t)(h2 >> 32) & mh), (uint32_t)(h3 >> 32) & mh);
                E = h3;
            }
        } else {
            uint64_t h = st.C;
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                h = shl1_add(h, st.g[i >> 2][i & 3]);
                const uint32_t t0 = (uint32_t)(h >> 32) & mh;
                h = shl1_add(h, st.g[(i + 1) >> 2][(i + 1) & 3]);
                const uint32_t t1 = (uint32_t)(h >> 32) & mh;
                acc = min(min(acc, t0), t1);  // v_min3_u32
            }
        }
        st.acc = acc;
    };
    // the row's verdict: a fired prefilter (or the batch's last rows) is checked against
    // the full masks and, if a candidate exists, re-walked exactly into the slot list
    auto back = [&](uint32_t u, uint64_t row, RowState &st) {
        const bool tail = (row + 1) * FLAT_ROW > end_rel;  // uniform
        if (__builtin_amdgcn_ballot_w64(st.acc == 0) == 0 && !tail) return;
        if constexpr (FORM >= 5) {  // the group forms keep only C: redo the row's lookups
            block_lookups(gbase, ad, ring[u], st.g);
            split_partials(st.g);
        }
        bool exact = tail;
        if (!tail) {
            // the prefilter fired somewhere in the row (mostly on bits below 16 it cannot
            // see): does any byte pass the full S or L mask?  2 VALU per mask per byte
            uint32_t ex = 0xffffffffu;
            uint64_t x = st.C;
#pragma unroll
            for (uint32_t j = 0; j < 16; ++j) {
                const uint64_t hx = step(st.g, x, j);
                const uint32_t lo = (uint32_t)hx, hi = (uint32_t)(hx >> 32);
                ex = min(ex, min((lo & ms_lo) | (hi & ms_hi), (lo & ml_lo) | (hi & ml_hi)));
            }
            exact = __builtin_amdgcn_ballot_w64(ex == 0) != 0;
        }
        if (!exact) return;
        // exact pass from C over the 16 entries still in registers: per-lane bit masks of
        // the S / L positions (no branches, no LDS), a wave prefix sum (ballot + mbcnt when
        // no lane holds two), candidates into the slot list in (row, lane, byte) = position
        // order
        const uint64_t prel = row * FLAT_ROW + 16u * lane;
        const uint32_t nb = prel < end_rel ? (end_rel - prel < 16 ? (uint32_t)(end_rel - prel) : 16u) : 0u;
        uint32_t sm = 0, lm = 0;
        uint64_t x = st.C;
#pragma unroll
        for (uint32_t j = 0; j < 16; ++j) {
            const uint64_t hx = step(st.g, x, j);
            const uint64_t zs = hx & ms, zl = hx & ml;
            const uint32_t ts = (uint32_t)zs | (uint32_t)(zs >> 32), tl = (uint32_t)zl | (uint32_t)(zl >> 32);
            sm |= (1u - min(ts, 1u)) << j;
            lm |= (1u - min(tl, 1u)) << j;
        }
        const uint32_t vm = nb >= 16 ? 0xffffu : (1u << nb) - 1u;
        sm &= vm;
        lm &= vm;
        const uint32_t any = sm | lm, c = (uint32_t)__builtin_popcount(any);
        uint32_t excl, total;
        if (__builtin_amdgcn_ballot_w64(c > 1) == 0) {
            const uint64_t bal = __builtin_amdgcn_ballot_w64(c != 0);
            excl = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
            total = (uint32_t)__builtin_popcountll(bal);
        } else {
            uint32_t incl = c;
#pragma unroll
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
                if (lane >= d) incl += y;
            }
            excl = incl - c;
            total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        const uint32_t pos0 = (uint32_t)(row % FLAT_RPS) * FLAT_ROW + 16u * lane;
        uint32_t idx = segc + excl;
        for (uint32_t m = any; m; m &= m - 1) {
            const uint32_t j = (uint32_t)__builtin_ctz(m);
            const uint32_t f = (((sm >> j) & 1u) * CG_FLAG_S) | (((lm >> j) & 1u) * CG_FLAG_L);
            if (idx < cap) slots[idx] = ((pos0 + j) << 2) | f;
            ++idx;
        }
        segc += total;
    };
    // after ring slot u's row: at a segment end, flush its slots and count
    auto flush = [&](uint32_t u, uint64_t row) {
        if (u % FLAT_RPS == FLAT_RPS - 1) {
            const uint64_t seg = seg0 + row / FLAT_RPS;
            if (seg < nseg) {
                if (lane < min(segc, cap)) seg_cand[seg * cap + lane] = slots[lane];
                if (lane == 0) seg_count[seg] = segc;
            }
            segc = 0;
        }
    };
    static_assert(FLAT_RPS % 2 == 0, "row pairs never straddle a segment");
#pragma unroll 1
    for (uint64_t r = 0; r < nrow64; r += FLAT_D) {
        if constexpr (FORM >= 5) {
            // row groups (pairs, FORM 6 quads): the rows' lookups and chains before one
            // combined verdict branch; the rare exact path redoes a row's lookups from its
            // ring slot, re-issued only after the group
            constexpr uint32_t GRP = FORM == 6 ? 4u : 2u;
            static_assert(FLAT_D % GRP == 0 && FLAT_RPS % GRP == 0, "groups never straddle a segment");
#pragma unroll
            for (uint32_t u = 0; u < FLAT_D; u += GRP) {
                RowState st[GRP];
                uint32_t acc = 0xffffffffu;
#pragma unroll
                for (uint32_t i = 0; i < GRP; ++i) {
                    front(u + i, r + u + i, st[i]);
                    acc = min(acc, st[i].acc);
                }
                const bool tail = (r + u + GRP) * FLAT_ROW > end_rel;
                if (__builtin_amdgcn_ballot_w64(acc == 0) != 0 || tail) {
#pragma unroll
                    for (uint32_t i = 0; i < GRP; ++i) {
                        back(u + i, r + u + i, st[i]);
                        if (i + 1 < GRP) flush(u + i, r + u + i);
                    }
                }
#pragma unroll
                for (uint32_t i = 0; i < GRP; ++i) ring[u + i] = blk(next_row(r + u + i));
                flush(u + GRP - 1, r + u + GRP - 1);
            }
        } else {
#pragma unroll
            for (uint32_t u = 0; u < FLAT_D; ++u) {
                const uint64_t row = r + u;
                if constexpr (FORM == 2) {
                    sink ^= ring[u].x ^ ring[u].y ^ ring[u].z ^ ring[u].w;
                    ring[u] = blk(next_row(row));
                } else {
                    RowState st;
                    front(u, row, st);
                    back(u, row, st);
                    if constexpr (FORM == 0 || FORM == 3) ring[u] = blk(next_row(row));
                }
                flush(u, row);
            }
        }
    }
    if constexpr (FORM == 2)
        if (sink == 0x9e3779b9u && lane == 0) seg_count[seg0] = sink;  // never true for the diag inputs
}

// ===========================================================================
// Alternative scan kernels, kept in the diagnostics build for the A/B measurements
// recorded in DESIGN.md §4 (scripts/diag_scan.py --variants).
// ===========================================================================
// v_perm_b32 selector producing (byte b of `w`) << 8 | (byte 0 of `lo8`): the LDS
// address of entry w.byte[b] in this lane's copy, in one instruction.
__device__ __forceinline__ uint32_t gear_addr(uint32_t w, uint32_t lo8, int b) {
    return __builtin_amdgcn_perm(w, lo8, 0x0C0C0000u | ((4u + (uint32_t)b) << 8));
}


// 4x4 transpose of 16-byte elements inside each quad of lanes: on entry lane i
// holds v[j] = quarter i of lane j's 64-byte piece; on exit lane i holds v[j] =
// quarter j of its own piece.  Two rounds of DPP quad_perm swaps (lane^1, lane^2),
// each a v_mov_dpp + select per dword.
template <int CTRL, int BIT>
__device__ __forceinline__ void quad_swap(uint4 v[4], uint32_t lane) {
    uint4 t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint4 src = v[j ^ BIT];
        t[j].x = __builtin_amdgcn_mov_dpp(src.x, CTRL, 0xf, 0xf, false);
        t[j].y = __builtin_amdgcn_mov_dpp(src.y, CTRL, 0xf, 0xf, false);
        t[j].z = __builtin_amdgcn_mov_dpp(src.z, CTRL, 0xf, 0xf, false);
        t[j].w = __builtin_amdgcn_mov_dpp(src.w, CTRL, 0xf, 0xf, false);
    }
    // select by a lane-constant all-ones/zero VGPR mask with v_bitop3 (m ? t : v):
    // v_cndmask on an SGPR lane mask cost ~13 cycles per wave-instruction per SIMD at
    // 4 waves/SIMD in our measurements (scripts/diag_ops.py), bitop3 ~1.6
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t m = 0u - (((lane ^ (uint32_t)j) & BIT) != 0 ? 1u : 0u);
        asm volatile("" : "+v"(m));  // keep the mask in a VGPR (no re-derivation into an SGPR lane mask)
        v[j].x = __builtin_amdgcn_bitop3_b32(m, t[j].x, v[j].x, 0xCA);
        v[j].y = __builtin_amdgcn_bitop3_b32(m, t[j].y, v[j].y, 0xCA);
        v[j].z = __builtin_amdgcn_bitop3_b32(m, t[j].z, v[j].z, 0xCA);
        v[j].w = __builtin_amdgcn_bitop3_b32(m, t[j].w, v[j].w, 0xCA);
    }
}

__device__ __forceinline__ void quad_transpose(uint4 v[4], uint32_t lane) {
    quad_swap<0xB1, 1>(v, lane);  // quad_perm [1,0,3,2]
    quad_swap<0x4E, 2>(v, lane);  // quad_perm [2,3,0,1]
}


// K1.  Each lane owns CG_SEG bytes of the flat batch buffer.  Bytes arrive in 64-B
// pieces loaded cooperatively by the 4 lanes of a quad (each dwordx4 instruction
// reads 16 whole 64-B runs instead of 64 scattered 16-B pieces) and transposed in
// registers; two pieces are in flight ahead of the one being hashed.
// PRE = prefilter mode: per byte only (h & (mask_s & mask_l)) is folded into a
// running min (5 VALU + 1 LDS read per byte); a piece whose min hits 0 in some lane
// is re-walked exactly for that lane.  Used when mask_s & mask_l has >= 15 bits
// (hits are rarer than ~1 per 32 KiB); otherwise every byte is tested exactly.
// DIAG (diagnostics build only, 0 = product): 1 = loads only, 2 = loads + transpose,
// 3 = hashing on register-resident bytes without loads, 4 = as 3 without LDS reads;
// + 8 = non-temporal loads.
template <bool PRE, int DIAG = 0>
__global__ __launch_bounds__(SCAN2_T) void k_scan_quad(const uint8_t *__restrict__ data, uint64_t n,
                                                  const uint64_t *__restrict__ gear_g, uint64_t mask_s,
                                                  uint64_t mask_l, uint32_t cap, uint32_t *__restrict__ seg_count,
                                                  uint32_t *__restrict__ seg_cand, uint64_t nseg) {
    __shared__ __attribute__((aligned(16))) uint64_t s_gear[256 * GEAR_COPIES];
    for (uint32_t i = threadIdx.x; i < 256 * GEAR_COPIES; i += SCAN2_T) s_gear[i] = gear_g[i / GEAR_COPIES];
    __syncthreads();
    const char *gbase = reinterpret_cast<const char *>(s_gear);

    const uint32_t lane = threadIdx.x & 63u, qi = lane & 3u;
    const uint64_t seg = (uint64_t)blockIdx.x * SCAN2_T + threadIdx.x;
    // whole waves stay active through the cooperative loop (DPP needs every lane)
    const uint64_t wave_first = seg - lane;
    if (wave_first >= nseg) return;
    const bool active = seg < nseg;
    const uint32_t lo8 = (threadIdx.x & 31u) * 8u;
    const uint64_t start = seg * CG_SEG;
    const uint64_t end = active ? (start + CG_SEG < n ? start + CG_SEG : n) : start;
    const uint32_t npieces = active ? (uint32_t)((end - start) / QPIECE) : 0u;
    const uint64_t mask_c = mask_s & mask_l;
    const uint32_t ml = (uint32_t)mask_c, mh = (uint32_t)(mask_c >> 32);

    // the quad's 4 owners: segments seg - qi + j; this lane loads quarter qi of each
    uint64_t own_start[4];
    uint32_t own_np[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        own_start[j] = __shfl(start, (int)((lane & ~3u) + j), 64);
        own_np[j] = __shfl(npieces, (int)((lane & ~3u) + j), 64);
    }

    uint64_t h = 0;
    if (active && start >= CG_HALO) {  // warm-up over the 48 bytes before the segment
        const uint4 *hp = reinterpret_cast<const uint4 *>(data + start - CG_HALO);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint4 v = hp[k];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int b = 0; b < 4; ++b) h = (h << 1) + lds_gear(gbase, gear_addr(w[j], lo8, b));
        }
    }

    uint32_t count = 0;
    uint64_t hits = 0;  // PRE: bit r = piece r may hold a candidate (CG_SEG / QPIECE <= 64 pieces)
    uint32_t *cand = seg_cand + seg * cap;
    const uint32_t rounds = CG_SEG / QPIECE;  // wave-uniform trip count
    static_assert(CG_SEG / QPIECE <= 64 && CG_SEG % (4 * QPIECE) == 0, "hits mask / ring loop geometry");
    uint4 buf[4][4];
    // Loads are unconditional (a piece index past the owner's last piece is clamped to
    // a valid address and its bytes are never hashed): with no exec-masked loads the
    // compiler counts vmcnt exactly and waits only for the piece about to be hashed,
    // keeping the two pieces behind it in flight.
    // Per owner: base address of this lane's quarter and the last valid piece index, so
    // a load address is one v_min_u32 + one v_lshl_add_u64 (no lane-mask selects).
    const uint8_t *own_base[4];
    uint32_t own_last[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        own_base[j] = own_np[j] ? data + own_start[j] + 16u * qi : data;
        own_last[j] = own_np[j] ? own_np[j] - 1u : 0u;
    }
    auto issue = [&](uint4(&v)[4], uint32_t r) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t rj = min(r, own_last[j]);
            const uint8_t *a = own_base[j] + (uint64_t)rj * QPIECE;
            if constexpr ((DIAG & 8) != 0) {
                typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(a));
                v[j] = make_uint4(t.x, t.y, t.z, t.w);
            } else {
                v[j] = *reinterpret_cast<const uint4 *>(a);
            }
        }
    };
    issue(buf[0], 0);
    issue(buf[1], 1);
    // 4-deep register ring.  Pieces are fetched in pairs -- both 64-B halves of each
    // segment's 128-B line in one burst, so no line is requested twice (a lone half
    // re-requested a piece later was re-fetched from HBM: +22 % traffic) -- two to
    // three pieces ahead of the one being hashed.  The trip count is a multiple of the
    // unroll, so the body has one path and the compiler's vmcnt waits are exact.
#pragma unroll 1
    for (uint32_t r = 0; r < rounds; r += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t rr = r + u;
            if constexpr ((DIAG & 7) < 3) {
                if ((u & 1) == 0) {
                    issue(buf[(u + 2) & 3], rr + 2);
                    issue(buf[(u + 3) & 3], rr + 3);
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // keep each piece's loads in program order
            uint4 v[4] = {buf[u][0], buf[u][1], buf[u][2], buf[u][3]};
            if constexpr ((DIAG & 7) >= 3) {
#pragma unroll
                for (int k = 0; k < 4; ++k) v[k] = make_uint4(lane * 0x01010101u + rr, (uint32_t)h, k, rr * 77u);
            }
            if constexpr ((DIAG & 7) != 1) quad_transpose(v, lane);
            if constexpr ((DIAG & 7) == 1 || (DIAG & 7) == 2) {
                uint32_t x = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) x ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
                h += x;
                hits |= (x == 0x12345678u) ? 1ull : 0ull;
            } else if (PRE) {
                // Branch-free: fold (h & mask_s & mask_l) into a running min; a piece
                // whose min reaches 0 only sets its bit in `hits` and is re-walked
                // exactly after the loop.  No stores inside the loop, so the compiler's
                // vmcnt stays exact and two pieces stay in flight.
                uint64_t hn = h;
                uint32_t acc = 0xffffffffu;
                const uint32_t wd[16] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                                         v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
                // Gear lookups run GRP bytes ahead of the shift-add chain (two groups of
                // LDS reads in flight per wave instead of four reads).
                constexpr int GRP = 4;
                uint64_t g[2][GRP];
                auto fetch = [&](uint64_t(&dst)[GRP], int grp) {
#pragma unroll
                    for (int t = 0; t < GRP; ++t) {
                        const int byte = grp * GRP + t;
                        if constexpr ((DIAG & 7) == 4) {
                            const uint32_t a = gear_addr(wd[byte >> 2], lo8, byte & 3);
                            dst[t] = ((uint64_t)a << 32) | a;
                        } else {
                            dst[t] = lds_gear(gbase, gear_addr(wd[byte >> 2], lo8, byte & 3));
                        }
                    }
                };
                fetch(g[0], 0);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int grp = 0; grp < QPIECE / GRP; ++grp) {
                    if (grp + 1 < QPIECE / GRP) fetch(g[(grp + 1) & 1], grp + 1);
                    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the chain
#pragma unroll
                    for (int t = 0; t < GRP; ++t) {
                        hn = (hn << 1) + g[grp & 1][t];
                        // (lo & ml) | (hi & mh) in two ops: v_and + v_bitop3 (S0&S1)|S2
                        acc = min(acc, (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(hn >> 32), mh, (uint32_t)hn & ml, 0xEA));
                    }
                }
                const bool live = rr < npieces;
                h = live ? hn : h;
                hits |= (live && acc == 0) ? (1ull << rr) : 0ull;
            } else if (rr < npieces) {
                const uint64_t p = start + (uint64_t)rr * QPIECE;
                {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
                        for (int j = 0; j < 4; ++j)
#pragma unroll
                            for (int b = 0; b < 4; ++b) {
                                h = (h << 1) + lds_gear(gbase, gear_addr(w[j], lo8, b));
                                const uint32_t f = gear_flags(h, mask_s, mask_l);
                                if (f) {
                                    if (count < cap)
                                        cand[count] = ((uint32_t)(p - start + 16 * k + 4 * j + b) << 2) | f;
                                    ++count;
                                }
                            }
                    }
                }
            }
        }
    }
    if (!active) return;
    if (PRE) {
        // Exact re-walk of the flagged pieces, in order, from L2/MALL-resident bytes.
        // The hash restarts 48 bytes before the piece (or at 0 for the batch's first
        // bytes, where the scan itself started): the tested bits (<= 47) equal the
        // scan's, which restarted at the segment's own halo.
        while (hits) {
            const uint32_t r = (uint32_t)__builtin_ctzll(hits);
            hits &= hits - 1;
            const uint64_t p = start + (uint64_t)r * QPIECE;
            const uint64_t q0 = p >= CG_HALO ? p - CG_HALO : 0;
            uint64_t hh = 0;
            for (uint64_t q = q0; q < p; q += 16) {
                const uint4 x = *reinterpret_cast<const uint4 *>(data + q);
                const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int b = 0; b < 4; ++b) hh = (hh << 1) + lds_gear(gbase, gear_addr(w[j], lo8, b));
            }
            for (uint32_t k = 0; k < QPIECE; k += 16) {
                const uint4 x = *reinterpret_cast<const uint4 *>(data + p + k);
                const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
                        hh = (hh << 1) + lds_gear(gbase, gear_addr(w[j], lo8, b));
                        const uint32_t f = gear_flags(hh, mask_s, mask_l);
                        if (f) {
                            if (count < cap) cand[count] = ((uint32_t)(p - start + k + 4 * j + b) << 2) | f;
                            ++count;
                        }
                    }
            }
        }
    }
    for (uint64_t p = start + (uint64_t)npieces * QPIECE; p < end; ++p) {  // ragged tail (< 64 bytes)
        h = (h << 1) + lds_gear(gbase, ((uint32_t)data[p] << 8) | lo8);
        const uint32_t f = gear_flags(h, mask_s, mask_l);
        if (f) {
            if (count < cap) cand[count] = ((uint32_t)(p - start) << 2) | f;
            ++count;
        }
    }
    seg_count[seg] = count;
}

// ---------------------------------------------------------------------------
// K1, LDS-staged form (diagnostics build: measured slower).  HBM efficiency depends on the read pattern far more than on
// the hashing: a wave reading its 64 lanes' segments in 64-128 B runs per lane reaches
// ~4.4-4.8 TB/s, in 256 B runs ~5.1-5.5 TB/s (scripts/diag_scan.py read patterns,
// profiles/r02_diag_scan.json).  So each wave stages its segments through LDS:
//  * a phase moves 256 B of each of the wave's 64 segments (16 KiB) with 16 LDS-DMA
//    instructions (global_load_lds_dwordx4), each reading four whole 256-B runs (16
//    lanes per run, so every 128-B line is requested whole by one instruction);
//  * the per-lane SOURCE addresses are permuted so that the lane-linear LDS image puts
//    segment o's 16-B chunk m at 1024 (o % 16) + 256 (o / 16) + 16 ((m + o) % 16):
//    every ds_read_b128 lane group then reads 16 distinct bank quads (no conflicts);
//  * the wave copies its phase into registers, issues the next phase's DMA at once,
//    and hashes the 256 B from registers while it lands (one 16-KiB buffer per wave);
//  * 8 waves per CU (one 512-thread workgroup, persistent over 64-segment tasks) share
//    one 16-copy GEAR table (32 KiB; lanes c and c+16 share a copy: ~1.5-way bank
//    conflicts on lookups), 8 x 16 KiB staging + 32 KiB = the CU's 160 KiB of LDS.
// Hash representation and prefilter as k_scan (H' = H << 16).
// ---------------------------------------------------------------------------
#define LW 8u                        // waves per workgroup (one workgroup per CU)
#define LCOPIES 16u                  // GEAR table copies
#define LPHASE 256u                  // bytes per segment per phase
#define LSTAGE (64u * LPHASE)        // staging bytes per wave
static_assert(LCOPIES * 256u * 8u + LW * LSTAGE <= 163840u, "LDS budget of one CU");
static_assert(CG_SEG % LPHASE == 0 && LPHASE % QPIECE == 0, "phase geometry");

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

// lookup address of byte B of w: (byte << 7) | copy offset (entry stride 128 B = 16 copies)
template <int B>
__device__ __forceinline__ uint32_t addr16(uint32_t w, uint32_t sh7, uint32_t cbase) {
    uint32_t a;
    if constexpr (B == 0)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
            : "=v"(a) : "v"(sh7), "v"(w));
    else if constexpr (B == 1)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
            : "=v"(a) : "v"(sh7), "v"(w));
    else if constexpr (B == 2)
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2"
            : "=v"(a) : "v"(sh7), "v"(w));
    else
        asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3"
            : "=v"(a) : "v"(sh7), "v"(w));
    return a | cbase;
}

__device__ __forceinline__ void lookup4x16(const char *gbase, uint32_t w, uint32_t sh7, uint32_t cbase,
                                           uint64_t (&g)[4]) {
    const uint32_t a0 = addr16<0>(w, sh7, cbase), a1 = addr16<1>(w, sh7, cbase);
    const uint32_t a2 = addr16<2>(w, sh7, cbase), a3 = addr16<3>(w, sh7, cbase);
    g[0] = lds_gear(gbase, a0);
    g[1] = lds_gear(gbase, a1);
    g[2] = lds_gear(gbase, a2);
    g[3] = lds_gear(gbase, a3);
}

template <bool PRE>
__global__ __launch_bounds__(64 * LW) void k_scan_lds(const uint8_t *__restrict__ data, uint64_t n,
                                                      const uint64_t *__restrict__ gear_g, uint64_t mask_s,
                                                      uint64_t mask_l, uint32_t cap, uint32_t *__restrict__ seg_count,
                                                      uint32_t *__restrict__ seg_cand, uint64_t nseg) {
    __shared__ __attribute__((aligned(16))) uint64_t s_gear[256 * LCOPIES];
    __shared__ __attribute__((aligned(16))) uint8_t s_stage[LW][LSTAGE];
    for (uint32_t i = threadIdx.x; i < 256 * LCOPIES; i += 64 * LW) s_gear[i] = gear_g[i / LCOPIES] << SCAN_SHIFT;
    __syncthreads();
    const char *gbase = reinterpret_cast<const char *>(s_gear);
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    uint32_t sh7 = 7, cbase = (lane & 15u) * 8u;
    asm volatile("" : "+v"(sh7), "+v"(cbase));  // VGPR operands of the SDWA shifts
    uint8_t *stage = s_stage[wave];
    // this lane's chunk m of the staged phase sits at rd + 16 ((m + lane) % 16)
    const uint8_t *rd = stage + 1024u * (lane & 15u) + 256u * (lane >> 4);
    const uint64_t ms = mask_s << SCAN_SHIFT, ml = mask_l << SCAN_SHIFT;
    const uint32_t mh = (uint32_t)((mask_s & mask_l) >> (32 - SCAN_SHIFT));
    const uint64_t ntask = (nseg + 63) / 64;
    const uint32_t phases = CG_SEG / LPHASE;
    static_assert(CG_SEG / QPIECE <= 64, "hits mask holds one bit per piece");

    for (uint64_t task = (uint64_t)blockIdx.x * LW + wave; task < ntask; task += (uint64_t)gridDim.x * LW) {
        const uint64_t seg = task * 64 + lane;
        const bool active = seg < nseg;
        const uint64_t start = seg * CG_SEG;
        const uint64_t end = active ? (start + CG_SEG < n ? start + CG_SEG : n) : start;
        const uint32_t npieces = active ? (uint32_t)((end - start) / QPIECE) : 0u;
        // DMA role: instruction i reads chunk ((lane % 16) - i) % 16 of segment 16 (lane / 16) + i
        const uint64_t grp = (task * 64 + 16u * (lane >> 4)) * CG_SEG;
        auto dma_phase = [&](uint32_t ph) {
#pragma unroll
            for (uint32_t i = 0; i < 16; ++i) {
                uint64_t src = grp + (uint64_t)i * CG_SEG + ph * LPHASE + 16u * ((lane - i) & 15u);
                src = src + 16 <= n ? src : 0;  // past the batch: any readable bytes (never hashed)
                __builtin_amdgcn_global_load_lds((gbl_void *)(data + src), (lds_void *)(stage + 1024u * i), 16, 0,
                                                 0);
            }
        };

        uint64_t h = 0;
        if (active && start >= CG_HALO) {  // warm-up over the 48 bytes before the segment
            const uint4 *hp = reinterpret_cast<const uint4 *>(data + start - CG_HALO);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint4 v = hp[k];
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    uint64_t g[4];
                    lookup4x16(gbase, w[j], sh7, cbase, g);
#pragma unroll
                    for (int b = 0; b < 4; ++b) h = (h << 1) + g[b];
                }
            }
        }
        uint32_t count = 0;
        uint64_t hits = 0;
        uint32_t *cand = seg_cand + seg * cap;
        dma_phase(0);
#pragma unroll 1
        for (uint32_t ph = 0; ph < phases; ++ph) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of phase ph has landed
            uint4 d[16];
#pragma unroll
            for (uint32_t m = 0; m < 16; ++m) d[m] = *reinterpret_cast<const uint4 *>(rd + 16u * ((m + lane) & 15u));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging read out: the next phase may land
            if (ph + 1 < phases) dma_phase(ph + 1);
#pragma unroll
            for (uint32_t q = 0; q < LPHASE / QPIECE; ++q) {
                const uint32_t rr = ph * (LPHASE / QPIECE) + q;  // piece index in the segment
                const uint32_t wd[16] = {d[4 * q].x,     d[4 * q].y,     d[4 * q].z,     d[4 * q].w,
                                         d[4 * q + 1].x, d[4 * q + 1].y, d[4 * q + 1].z, d[4 * q + 1].w,
                                         d[4 * q + 2].x, d[4 * q + 2].y, d[4 * q + 2].z, d[4 * q + 2].w,
                                         d[4 * q + 3].x, d[4 * q + 3].y, d[4 * q + 3].z, d[4 * q + 3].w};
                if (PRE) {
                    uint64_t hn = h;
                    uint32_t acc = 0xffffffffu;
                    uint64_t g[2][4];
                    lookup4x16(gbase, wd[0], sh7, cbase, g[0]);
#pragma unroll
                    for (int k = 0; k < 16; ++k) {
                        if (k + 1 < 16) lookup4x16(gbase, wd[k + 1], sh7, cbase, g[(k + 1) & 1]);
                        hn = (hn << 1) + g[k & 1][0];
                        const uint32_t t0 = (uint32_t)(hn >> 32) & mh;
                        hn = (hn << 1) + g[k & 1][1];
                        const uint32_t t1 = (uint32_t)(hn >> 32) & mh;
                        acc = min(min(acc, t0), t1);  // v_min3_u32
                        hn = (hn << 1) + g[k & 1][2];
                        const uint32_t t2 = (uint32_t)(hn >> 32) & mh;
                        hn = (hn << 1) + g[k & 1][3];
                        const uint32_t t3 = (uint32_t)(hn >> 32) & mh;
                        acc = min(min(acc, t2), t3);
                    }
                    const bool live = rr < npieces;
                    h = live ? hn : h;
                    hits |= (live && acc == 0) ? (1ull << rr) : 0ull;
                } else if (rr < npieces) {
                    const uint64_t p = start + (uint64_t)rr * QPIECE;
#pragma unroll
                    for (int k = 0; k < 16; ++k) {
                        uint64_t g[4];
                        lookup4x16(gbase, wd[k], sh7, cbase, g);
#pragma unroll
                        for (int b = 0; b < 4; ++b) {
                            h = (h << 1) + g[b];
                            const uint32_t f = gear_flags64(h, ms, ml);
                            if (f) {
                                if (count < cap) cand[count] = ((uint32_t)(p - start + 4 * k + b) << 2) | f;
                                ++count;
                            }
                        }
                    }
                }
            }
        }
        if (!active) continue;
        if (PRE) {  // exact re-walk of the flagged pieces (as k_scan)
            while (hits) {
                const uint32_t r = (uint32_t)__builtin_ctzll(hits);
                hits &= hits - 1;
                const uint64_t p = start + (uint64_t)r * QPIECE;
                const uint64_t q0 = p >= CG_HALO ? p - CG_HALO : 0;
                uint64_t hh = 0;
                for (uint64_t q = q0; q < p; q += 16) {
                    const uint4 x = *reinterpret_cast<const uint4 *>(data + q);
                    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        uint64_t g[4];
                        lookup4x16(gbase, w[j], sh7, cbase, g);
#pragma unroll
                        for (int b = 0; b < 4; ++b) hh = (hh << 1) + g[b];
                    }
                }
                for (uint32_t k = 0; k < QPIECE; k += 16) {
                    const uint4 x = *reinterpret_cast<const uint4 *>(data + p + k);
                    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        uint64_t g[4];
                        lookup4x16(gbase, w[j], sh7, cbase, g);
#pragma unroll
                        for (int b = 0; b < 4; ++b) {
                            hh = (hh << 1) + g[b];
                            const uint32_t f = gear_flags64(hh, ms, ml);
                            if (f) {
                                if (count < cap) cand[count] = ((uint32_t)(p - start + k + 4 * j + b) << 2) | f;
                                ++count;
                            }
                        }
                    }
                }
            }
        }
        for (uint64_t p = start + (uint64_t)npieces * QPIECE; p < end; ++p) {  // ragged tail (< 64 bytes)
            h = (h << 1) + lds_gear(gbase, ((uint32_t)data[p] << 7) | cbase);
            const uint32_t f = gear_flags64(h, ms, ml);
            if (f) {
                if (count < cap) cand[count] = ((uint32_t)(p - start) << 2) | f;
                ++count;
            }
        }
        seg_count[seg] = count;
    }
}

// ---------------------------------------------------------------------------
// K1, page-per-wave form (diagnostics build: measured slower).  What limits the other forms is the
// HBM read pattern, not the hashing: one stream per lane (64 streams per wave, each
// advancing 64-128 B at a time) reads at ~4.4 TB/s, whole 4 KiB pages per wave at
// ~6.0 TB/s (scripts/diag_scan.py read patterns, profiles/r02_diag_scan.json).  So
// here a wave walks its own run of PPW consecutive 4 KiB pages (= CG_SEG segments) in
// order, and in each page lane L takes bytes [64 L, 64 L + 64):
//  * the page arrives as 4 dwordx4 loads per lane (stride 64 B: the 4 instructions
//    cover the page), two pages ahead of the one being hashed;
//  * the 48 bytes before lane L's piece -- the window the masked bits depend on
//     -- are lane L-1's last 48 bytes, moved over by 12 DPP
//    wave_ror:1 movs; lane 0 takes the previous page's lane 63 (the rotation's value
//    kept from one page to the next) and, on a run's first page, loads them;
//  * a piece is hashed from the restart: 48 warm-up steps (lookup + shift-add) and 64
//    tested steps, so the hash state never crosses lanes;
//  * prefilter as k_scan (H' = H << 16, one v_and_b32 + 1/2 v_min3_u32 per byte);
//    a lane whose piece may hold a candidate re-walks it exactly from registers, and the
//    page's candidates are compacted in lane (= position) order by a wave prefix sum.
// Per byte: 1.75 lookups (SDWA mov + ds_read_b64 + v_lshl_add_u64), 1 v_and_b32,
// 1/2 v_min3_u32.
// ---------------------------------------------------------------------------
#define PPW 66u  // pages per wave: a multiple of the 3-page load ring (one loop path: exact vmcnt waits)
static_assert(CG_SEG == 64u * QPIECE, "a page is one 64-B piece per lane");

// Exact test of every position of this lane's piece (nbytes at src, re-read from
// L2: the rare path) from the warm-up state h0; counts the candidates and, with `out`,
// writes them ((page offset << 2) | flags) up to `room`.  Out of line: it runs only for
// the few pieces the prefilter flags, and inlined it would cost the hot loop registers.
__device__ __noinline__ uint32_t exact_piece(const char *gbase, uint32_t lo8, const uint8_t *src, uint64_t h0,
                                             uint32_t nbytes, uint64_t ms, uint64_t ml, uint32_t pos0,
                                             uint32_t *out, uint32_t room) {
    uint32_t w[16];
    if (nbytes == 64) {  // whole piece: four 16-B loads in flight together (one L2 round trip)
        const uint4 *q = reinterpret_cast<const uint4 *>(src);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = q[k];
            w[4 * k] = v.x;
            w[4 * k + 1] = v.y;
            w[4 * k + 2] = v.z;
            w[4 * k + 3] = v.w;
        }
    } else {  // the batch's ragged last piece: never read past its end
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = 0;
        for (uint32_t j = 0; j < nbytes; ++j) w[j >> 2] |= (uint32_t)src[j] << (8 * (j & 3));
    }
    uint64_t h = h0;
    uint32_t c = 0;
#pragma unroll
    for (uint32_t j = 0; j < 64; ++j) {
        h = (h << 1) + lds_gear(gbase, (((w[j >> 2] >> (8 * (j & 3))) & 0xffu) << 8) | lo8);
        const uint32_t f = j < nbytes ? gear_flags64(h, ms, ml) : 0u;
        if (f) {
            if (out && c < room) out[c] = ((pos0 + j) << 2) | f;
            ++c;
        }
    }
    return c;
}

template <bool PRE>
__global__ __launch_bounds__(SCAN2_T, 4) void k_scan_wave(const uint8_t *__restrict__ data, uint64_t n,
                                                       const uint64_t *__restrict__ gear_g, uint64_t mask_s,
                                                       uint64_t mask_l, uint32_t cap, uint32_t *__restrict__ seg_count,
                                                       uint32_t *__restrict__ seg_cand, uint64_t nseg) {
    __shared__ __attribute__((aligned(16))) uint64_t s_gear[256 * GEAR_COPIES];
    for (uint32_t i = threadIdx.x; i < 256 * GEAR_COPIES; i += SCAN2_T)
        s_gear[i] = gear_g[i / GEAR_COPIES] << SCAN_SHIFT;
    __syncthreads();
    const char *gbase = reinterpret_cast<const char *>(s_gear);
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t page0 = ((uint64_t)blockIdx.x * (SCAN2_T / 64) + (threadIdx.x >> 6)) * PPW;
    if (page0 >= nseg) return;  // whole wave (uniform)
    // pages of the run past the batch are walked as empty pages (no output), so every run
    // has PPW pages and the ring loop one path
    const uint64_t page_end = page0 + PPW < nseg ? page0 + PPW : nseg;
    const uint32_t lo8 = (threadIdx.x & 31u) * 8u;
    uint32_t ad[2][4];  // lookup address registers: bits 0..7 stay this lane's copy offset
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int b = 0; b < 4; ++b) ad[i][b] = lo8;
    const uint64_t ms = mask_s << SCAN_SHIFT, ml = mask_l << SCAN_SHIFT;
    const uint32_t mh = (uint32_t)((mask_s & mask_l) >> (32 - SCAN_SHIFT));

    // Loads are unconditional: a page past the run re-reads the run's last page, a piece
    // past the batch end reads the batch's first bytes (never hashed as data).
    auto issue = [&](uint4(&v)[4], uint64_t p) {
        const uint64_t q = p < page_end ? p : page_end - 1;
        const uint64_t a = q * CG_SEG + 64u * lane;
        const uint4 *src = reinterpret_cast<const uint4 *>(data + (a + 64 <= n ? a : 0));
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = src[j];
    };
    uint4 buf[3][4];
    issue(buf[0], page0);
    issue(buf[1], page0 + 1);
    // lane 0's window before the run's first page (wave-uniform: scalar registers)
    uint32_t carry[12];
    {
        const uint64_t a = page0 * CG_SEG;
        const uint32_t *src = reinterpret_cast<const uint32_t *>(data + (a >= CG_HALO ? a - CG_HALO : 0));
#pragma unroll
        for (int j = 0; j < 12; ++j) carry[j] = __builtin_amdgcn_readfirstlane(src[j]);
    }

    static_assert(PPW % 3 == 0, "the ring loop hashes three pages per trip");
#pragma unroll 1
    for (uint64_t p = page0; p < page0 + PPW; p += 3) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const uint64_t pg = p + u;
            const bool live = pg < page_end;  // uniform
            issue(buf[(u + 2) % 3], pg + 2);
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t wd[16] = {buf[u][0].x, buf[u][0].y, buf[u][0].z, buf[u][0].w,
                                     buf[u][1].x, buf[u][1].y, buf[u][1].z, buf[u][1].w,
                                     buf[u][2].x, buf[u][2].y, buf[u][2].z, buf[u][2].w,
                                     buf[u][3].x, buf[u][3].y, buf[u][3].z, buf[u][3].w};
            const uint64_t pstart = pg * CG_SEG;
            const uint64_t mine = pstart + 64u * lane;
            const uint32_t nbytes = (!live || mine >= n) ? 0u : (n - mine >= 64 ? 64u : (uint32_t)(n - mine));
            // the 48 bytes before this lane's piece: lane L-1's last 12 dwords
            uint32_t prev[12];
#pragma unroll
            for (int k = 0; k < 12; ++k) {
                // lane L <- lane L-1 (DPP), lane 0 <- the previous page's lane 63 (SGPR)
                uint32_t v = wave_ror1(wd[4 + k]);
                asm("v_writelane_b32 %0, %1, 0" : "+v"(v) : "s"(carry[k]));
                prev[k] = v;
                carry[k] = (uint32_t)__builtin_amdgcn_readlane((int)wd[4 + k], 63);
            }
            uint64_t h0 = 0;
#pragma unroll
            for (int k = 0; k < 12; ++k) {
                uint64_t g[4];
                lookup4(gbase, ad[k & 1], prev[k], g);
#pragma unroll
                for (int b = 0; b < 4; ++b) h0 = (h0 << 1) + g[b];
            }
            if (mine == 0) h0 = 0;  // the batch's first byte: no history (as the crate's restart)
            bool hit;
            if (PRE) {
                uint64_t hn = h0;
                uint32_t acc = 0xffffffffu;
                uint64_t g[2][4];
                lookup4(gbase, ad[0], wd[0], g[0]);
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    if (k + 1 < 16) lookup4(gbase, ad[(k + 1) & 1], wd[k + 1], g[(k + 1) & 1]);
                    hn = (hn << 1) + g[k & 1][0];
                    const uint32_t t0 = (uint32_t)(hn >> 32) & mh;
                    hn = (hn << 1) + g[k & 1][1];
                    const uint32_t t1 = (uint32_t)(hn >> 32) & mh;
                    acc = min(min(acc, t0), t1);  // v_min3_u32
                    hn = (hn << 1) + g[k & 1][2];
                    const uint32_t t2 = (uint32_t)(hn >> 32) & mh;
                    hn = (hn << 1) + g[k & 1][3];
                    const uint32_t t3 = (uint32_t)(hn >> 32) & mh;
                    acc = min(min(acc, t2), t3);
                }
                hit = (acc == 0 && nbytes) || (nbytes && nbytes < 64);  // a ragged piece is always exact
            } else {
                hit = nbytes != 0;
            }
            const uint64_t any = __ballot(hit);
            uint32_t total = 0;
            if (any) {  // exact pass for the flagged pieces, then compaction in lane order
                const uint8_t *src = data + (hit ? mine : 0);
                const uint32_t c =
                    hit ? exact_piece(gbase, lo8, src, h0, nbytes, ms, ml, 64u * lane, nullptr, 0) : 0u;
                uint32_t incl = c;  // inclusive prefix over lanes (position order)
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
                    if ((int)lane >= d) incl += y;
                }
                total = (uint32_t)__shfl((int)incl, 63, 64);
                const uint32_t before = incl - c;
                if (c && before < cap)
                    exact_piece(gbase, lo8, src, h0, nbytes, ms, ml, 64u * lane, seg_cand + pg * cap + before,
                                cap - before);
            }
            if (lane == 0 && live) seg_count[pg] = total;
        }
    }
}


using ScanFlatKernel = void (*)(const uint8_t *, uint64_t, const uint64_t *, uint64_t, uint64_t, uint32_t, uint32_t *,
                                uint32_t *, uint64_t, uint32_t);
ScanFlatKernel scan_flat32_variant(uint32_t mode);
void launch_k_scan_pre(const uint8_t *d_data, uint64_t n, const uint64_t *d_gear, uint64_t mask_s, uint64_t mask_l,
                       uint32_t cap, uint32_t *d_seg_count, uint32_t *d_seg_cand, uint64_t nseg, hipStream_t st);

// Variants 1-4 and the quad-kernel modes; false = the product path (or variant 5) runs.
bool launch_scan_diag(const uint8_t *d_data, uint64_t n, const uint64_t *d_gear, uint64_t mask_s, uint64_t mask_l,
                      uint32_t cap, uint32_t *d_seg_count, uint32_t *d_seg_cand, uint64_t nseg, hipStream_t st) {
    const uint64_t blocks = (nseg + SCAN2_T - 1) / SCAN2_T;
    const bool pre = __builtin_popcountll((mask_s & mask_l) >> SCAN_SHIFT) >= 14;
    const bool pre_quad = __builtin_popcountll(mask_s & mask_l) >= 15;
    if (g_scan_diag && pre_quad && g_scan_variant != 5) {
        auto k = g_scan_diag == 1   ? k_scan_quad<true, 1>
                 : g_scan_diag == 2 ? k_scan_quad<true, 2>
                 : g_scan_diag == 3 ? k_scan_quad<true, 3>
                 : g_scan_diag == 4 ? k_scan_quad<true, 4>
                 : g_scan_diag == 8 ? k_scan_quad<true, 8>
                                    : k_scan_quad<true, 9>;
        hipLaunchKernelGGL(k, dim3((uint32_t)blocks), dim3(SCAN2_T), 0, st, d_data, n, d_gear, mask_s, mask_l, cap,
                           d_seg_count, d_seg_cand, nseg);
        return true;
    }
    if (g_scan_variant == 1) {
        hipLaunchKernelGGL(pre_quad ? k_scan_quad<true> : k_scan_quad<false>, dim3((uint32_t)blocks), dim3(SCAN2_T),
                           0, st, d_data, n, d_gear, mask_s, mask_l, cap, d_seg_count, d_seg_cand, nseg);
        return true;
    }
    if (g_scan_variant == 2) {
        int dev = 0, cus = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const uint64_t ntask = (nseg + 63) / 64;
        const uint32_t grid = (uint32_t)std::min<uint64_t>(cus > 0 ? cus : 256, (ntask + LW - 1) / LW);
        hipLaunchKernelGGL(pre ? k_scan_lds<true> : k_scan_lds<false>, dim3(grid), dim3(64 * LW), 0, st, d_data, n,
                           d_gear, mask_s, mask_l, cap, d_seg_count, d_seg_cand, nseg);
        return true;
    }
    if (g_scan_variant == 3) {
        const uint64_t waves = (nseg + PPW - 1) / PPW;
        const uint64_t wgs = (waves + SCAN2_T / 64 - 1) / (SCAN2_T / 64);
        hipLaunchKernelGGL(pre ? k_scan_wave<true> : k_scan_wave<false>, dim3((uint32_t)wgs), dim3(SCAN2_T), 0, st,
                           d_data, n, d_gear, mask_s, mask_l, cap, d_seg_count, d_seg_cand, nseg);
        return true;
    }
    if (g_scan_variant == 4 && pre) {  // (without the prefilter the product already runs k_scan<false>)
        launch_k_scan_pre(d_data, n, d_gear, mask_s, mask_l, cap, d_seg_count, d_seg_cand, nseg, st);
        return true;
    }
    return false;
}

ScanFlatKernel scan_flat_diag_kernel(ScanFlatKernel k) {
    // variant 5 by g_scan_diag: k_scan_flat<ring rows, nt, FORM> (1: <8, nt>, 2: <16, cached>,
    // 3: <16, nt>, 4: <8, nt, 1>, 5: <8, nt, 2> loads only, 6-8: split chains <8|4|16, nt, 3>,
    // 9: <4, nt, 4>, 10: <4, nt, 2>, 11: <4, cached, 3>, 12-15: row pairs / quads <4|8, nt, 5|6>,
    // other: <8, cached>), 20-22: k_scan_flat32 <2, nt> (product) / <4, nt> / <2, cached>
    if (g_scan_variant == 5 && g_scan_diag >= 20) {
        k = scan_flat32_variant(g_scan_diag);
    } else if (g_scan_variant == 5) {
        k = g_scan_diag == 1    ? k_scan_flat<8, true>
            : g_scan_diag == 2  ? k_scan_flat<16, false>
            : g_scan_diag == 3  ? k_scan_flat<16, true>
            : g_scan_diag == 4  ? k_scan_flat<8, true, 1>
            : g_scan_diag == 5  ? k_scan_flat<8, true, 2>
            : g_scan_diag == 6  ? k_scan_flat<8, true, 3>
            : g_scan_diag == 7  ? k_scan_flat<4, true, 3>
            : g_scan_diag == 8  ? k_scan_flat<16, true, 3>
            : g_scan_diag == 9  ? k_scan_flat<4, true, 4>
            : g_scan_diag == 10 ? k_scan_flat<4, true, 2>
            : g_scan_diag == 11 ? k_scan_flat<4, false, 3>
            : g_scan_diag == 12 ? k_scan_flat<4, true, 5>
            : g_scan_diag == 13 ? k_scan_flat<8, true, 5>
            : g_scan_diag == 14 ? k_scan_flat<8, true, 6>
            : g_scan_diag == 15 ? k_scan_flat<4, true, 6>
                                : k_scan_flat<8, false>;
    }
    return k;
}

}  // namespace cg
#endif  // CG_DIAG
