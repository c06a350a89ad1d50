// scan.hip -- K1: data-parallel FastCDC v2020 boundary-candidate scan, and the
// device prefix sum + compaction that turn per-segment candidates into one sorted
// candidate list for the cut walk (K2, walk.hip).
//
// Replaces the serial Gear loop inside fastcdc's `cut_gear` [ext], called from
// chunk_descriptors_with_hash (src/chunking.rs:334-336).  The rolling hash
// h = (h << 1) + GEAR[b] is evaluated for every byte of the flat batch buffer with
// a 48-byte warm-up per lane segment; because every mask lives in bits <= 47,
// the tested bits equal those of the crate's per-chunk hash for every position at
// least 47 bytes past the chunk's hash start.  The 47
// positions before that are recomputed exactly by the walker.
#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "scan_common.h"

// Segment flush: the product lets the compiler form the flush addresses,
// which it hoists out of the row loop and, at 128 VGPRs, spills (3 VGPRs, 16 B of scratch;
// each reload waits vmcnt and so drains the row ring on segments holding a candidate).
// CG_SCAN_FLUSH_INPLACE=1 makes them in place from an opaque lane id (scan_common.h
// flush_slots): no spill, no scratch -- and measured no faster: same box, three alternating
// rounds, c2 0.1964-0.1967 vs 0.1943-0.1950 ms, c4 3.30-3.40 vs 3.24-3.29, c5 3.39-3.48 vs
// 3.42-3.46 (profiles/r05_v5_scan_flush_ab.txt): the drain costs less than the extra live
// registers of the in-place form.
#ifndef CG_SCAN_FLUSH_INPLACE
#define CG_SCAN_FLUSH_INPLACE 0
#endif

namespace cg {

template <bool PRE, int RING = 4>
__global__ __launch_bounds__(SCAN2_T) void k_scan(const uint8_t *__restrict__ data, uint64_t n,
                                                      const uint64_t *__restrict__ gear_g, uint64_t mask_s,
                                                      uint64_t mask_l, uint32_t cap, uint32_t *__restrict__ seg_count,
                                                      uint32_t *__restrict__ seg_cand, uint64_t nseg) {
    __shared__ __attribute__((aligned(16))) uint64_t s_gear[256 * GEAR_COPIES];
    for (uint32_t i = threadIdx.x; i < 256 * GEAR_COPIES; i += SCAN2_T)
        s_gear[i] = gear_g[i / GEAR_COPIES] << SCAN_SHIFT;
    __syncthreads();
    const char *gbase = reinterpret_cast<const char *>(s_gear);

    const uint64_t seg = (uint64_t)blockIdx.x * SCAN2_T + threadIdx.x;
    if (seg - (threadIdx.x & 63u) >= nseg) return;  // whole wave past the end
    const bool active = seg < nseg;
    const uint32_t lo8 = (threadIdx.x & 31u) * 8u;
    const uint64_t start = seg * CG_SEG;
    const uint64_t end = active ? (start + CG_SEG < n ? start + CG_SEG : n) : start;
    const uint32_t npieces = active ? (uint32_t)((end - start) / QPIECE) : 0u;
    const uint64_t ms = mask_s << SCAN_SHIFT, ml = mask_l << SCAN_SHIFT;
    const uint32_t mh = (uint32_t)((mask_s & mask_l) >> (32 - SCAN_SHIFT));  // H bits 16..47 = H' high dword

    uint32_t ad[2][4];  // lookup address registers: bits 0..7 stay this lane's copy offset
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int b = 0; b < 4; ++b) ad[i][b] = lo8;

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
                lookup4(gbase, ad[0], w[j], g);
#pragma unroll
                for (int b = 0; b < 4; ++b) h = (h << 1) + g[b];
            }
        }
    }

    uint32_t count = 0;
    uint64_t hits = 0;  // PRE: bit r = piece r may hold a candidate
    uint32_t *cand = seg_cand + seg * cap;
    const uint32_t rounds = CG_SEG / QPIECE;  // wave-uniform trip count
    static_assert(CG_SEG / QPIECE <= 64, "hits mask holds one bit per piece");
    // RING pieces in registers; loads go out BURST = RING / 2 pieces (RING / 2 x 64 B of
    // one segment) at a time, RING / 2 .. RING - 1 pieces ahead of the one being hashed
    constexpr int BURST = RING / 2;
    static_assert(CG_SEG % (RING * QPIECE) == 0, "the ring loop hashes RING pieces per trip");
    // Loads are unconditional (a piece past the last full one re-reads the last one, or
    // the buffer's first bytes for a segment without a full piece): the compiler then
    // counts vmcnt exactly and waits only for the piece about to be hashed.
    const uint8_t *base = npieces ? data + start : data;
    const uint32_t last = npieces ? npieces - 1u : 0u;
    uint4 buf[RING][4];
    auto issue = [&](uint4(&v)[4], uint32_t r) {
        const uint4 *a = reinterpret_cast<const uint4 *>(base + (uint64_t)min(r, last) * QPIECE);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = a[j];
    };
#pragma unroll
    for (int i = 0; i < BURST; ++i) issue(buf[i], i);
#pragma unroll 1
    for (uint32_t r = 0; r < rounds; r += RING) {
#pragma unroll
        for (int u = 0; u < RING; ++u) {
            const uint32_t rr = r + u;
            if ((u % BURST) == 0) {  // whole 128-B lines of the segment in one burst
#pragma unroll
                for (int i = 0; i < BURST; ++i) issue(buf[(u + BURST + i) % RING], rr + BURST + i);
            }
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t wd[16] = {buf[u][0].x, buf[u][0].y, buf[u][0].z, buf[u][0].w,
                                     buf[u][1].x, buf[u][1].y, buf[u][1].z, buf[u][1].w,
                                     buf[u][2].x, buf[u][2].y, buf[u][2].z, buf[u][2].w,
                                     buf[u][3].x, buf[u][3].y, buf[u][3].z, buf[u][3].w};
            if (PRE) {
                uint64_t hn = h;
                uint32_t acc = 0xffffffffu;
                uint64_t g[2][4];
                lookup4(gbase, ad[0], wd[0], g[0]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    if (k + 1 < 16) lookup4(gbase, ad[(k + 1) & 1], wd[k + 1], g[(k + 1) & 1]);
                    __builtin_amdgcn_sched_barrier(0);  // keep the lookups one dword ahead of the chain
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
                    lookup4(gbase, ad[k & 1], wd[k], g);
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
                for (int j = 0; j < 4; ++j) {
                    uint64_t g[4];
                    lookup4(gbase, ad[0], w[j], g);
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
                    lookup4(gbase, ad[0], w[j], g);
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
        h = (h << 1) + lds_gear(gbase, ((uint32_t)data[p] << 8) | lo8);
        const uint32_t f = gear_flags64(h, ms, ml);
        if (f) {
            if (count < cap) cand[count] = ((uint32_t)(p - start) << 2) | f;
            ++count;
        }
    }
    seg_count[seg] = count;
}

// ---------------------------------------------------------------------------
// K1, the product kernel for prefilterable masks (launch_scan; k_scan<false> takes the
// dense ones): flat form with 32-byte lane blocks (2 KiB rows, lane L: bytes [32 L, 32 L + 32) as
// two dwordx4).  The 48-byte window then spans one and a half lane blocks, so the state
// entering lane L's block is C_L = P_{L-1} + (P_{L-2} << 32) -- three DPP rotations and
// three selects per 32 bytes instead of five and five (plus the dword shuffle) per 16 --
// and a row's verdict branch covers 2 KiB, as a row pair of k_scan_flat did.  A 2-row
// ring (4 KiB per wave in flight), each slot re-issued as soon as its lookup addresses are
// formed; split chains as k_scan_flat's FORM 3+.  Same-box A/B vs the v12 row pairs:
// config 2 0.229 -> 0.218 ms, one 1 GiB NAR 0.226 -> 0.213, config 4 shape equal
// (profiles/r02_v13_diag_scan_flat32.json).
// VALU per 32 bytes: 32 SDWA addresses, 24 + 7 (partials, P), 32 (hashes), 32 ands +
// 16 min3 (prefilter), 7 (exchange) ~= 150, against ~186 for two 16-byte blocks.
// ---------------------------------------------------------------------------
// Issue priority from a row's start to its slot re-issue (round 4): a wave that has its row's
// bytes forms its lookup addresses and re-issues the slot ahead of the waves hashing, so
// loads go out sooner and more bytes are in flight.  Same-box A/B, 3 alternating rounds
// (profiles/r04_v12_*): config 2 0.2005-0.2026 -> 0.194-0.196 ms, the 16 GiB shapes
// 3.24-3.45 / 3.37-3.53 -> 3.15-3.30 / 3.33-3.51 ms; levels 1, 2 and 3 alike.
#ifndef CG_SCAN_PRIO
#define CG_SCAN_PRIO 2
#endif
#define F32_ROW 2048u
#define F32_RPS (CG_SEG / F32_ROW)  // rows per segment
static_assert(CG_SEG % F32_ROW == 0 && F32_RPS == 2, "two 2 KiB rows per segment");

template <uint32_t RING, bool NT, uint32_t GC = GEAR_COPIES, uint32_t T = SCAN2_T>
__global__ __launch_bounds__(T, 4) void k_scan_flat32(const uint8_t *data, uint64_t n,
                                                          const uint64_t *__restrict__ gear_g, uint64_t mask_s,
                                                          uint64_t mask_l, uint32_t cap,
                                                          uint32_t *__restrict__ seg_count,
                                                          uint32_t *__restrict__ seg_cand, uint64_t nseg, uint32_t spw) {
    __shared__ __attribute__((aligned(16))) uint64_t s_gear[256 * GC];
    __shared__ uint32_t s_slots[T / 64][64];  // the open segment's candidate slots, per wave
    const uint32_t lane = threadIdx.x & 63u;
    // the wave index through readfirstlane: the run's base, bounds and buffer resource
    // are then scalar (SGPRs), not per-lane copies
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t seg0 = ((uint64_t)blockIdx.x * (T / 64) + wv) * spw;
    const bool active = seg0 < nseg;  // whole wave (uniform)
    const uint64_t r0 = seg0 * CG_SEG;
    const uint64_t nrow = (uint64_t)spw * F32_RPS;  // a multiple of RING (spw a multiple of 4)
    static_assert(RING % F32_RPS == 0 && 8 % RING == 0, "ring trips end on segment boundaries");
    // The run's rows are read through a buffer resource based at the run (wave-uniform, in
    // SGPRs) whose size ends at the batch end: a row's address is an SGPR offset plus the
    // lane's constant 32 L, and a load past the batch end returns zeros instead of
    // faulting, so no per-lane address arithmetic or clamp is left in the row loop (the
    // bytes past the end only feed candidates the tail rows mask off).
    typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
    // The range ends at the batch end rounded up to its 16-byte granule (the input is
    // 16-byte aligned, so the granule is allocated): a dwordx4 load of the last granule
    // then returns its bytes whatever the hardware's range check does with a partial one.
    const uint64_t run_bytes = nrow * F32_ROW;  // <= spw x 4 KiB: 32-bit offsets
    const uint64_t avail = active ? ((n - r0 + 15) & ~15ull) : 0;
    const __amdgpu_buffer_rsrc_t run_rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(data + (active ? r0 : 0)), (short)0, (int)(avail < run_bytes ? avail : run_bytes),
        0x00027000);
    const uint32_t lane_off = 32u * lane;
    auto blk = [&](uint64_t row, uint4 (&v)[2]) {
        const uint32_t so = (uint32_t)(row * F32_ROW);
        const u32x4_t x0 = __builtin_amdgcn_raw_buffer_load_b128(run_rs, lane_off, so, NT ? 2 : 0);  // aux 2: nt
        const u32x4_t x1 = __builtin_amdgcn_raw_buffer_load_b128(run_rs, lane_off + 16u, so, NT ? 2 : 0);
        v[0] = uint4{x0.x, x0.y, x0.z, x0.w};
        v[1] = uint4{x1.x, x1.y, x1.z, x1.w};
    };
    static_assert(T == 2 * 256 || (T == 256 && GC == GEAR_COPIES_LEAN), "two threads per Gear entry, or one (lean)");
    const uint32_t ge = T == 256 ? threadIdx.x : threadIdx.x >> 1;
    const uint64_t gv = gear_g[ge] << SCAN_SHIFT;
    uint4 ring[RING][2];
#pragma unroll
    for (uint32_t i = 0; i < RING; ++i) blk(active ? i : 0, ring[i]);
    const bool has_pro = active && r0 >= F32_ROW;
    uint4 pro[2];
    {
        // only lanes 62 and 63 of the row before the run feed the hash (C_0 and C_1 take
        // P_63 and P_62), so the other lanes read nothing
        pro[0] = pro[1] = uint4{0, 0, 0, 0};
        if (has_pro && lane >= 62) {
            const uint64_t a = r0 - F32_ROW + 32u * lane;
            pro[0] = *reinterpret_cast<const uint4 *>(data + a);
            pro[1] = *reinterpret_cast<const uint4 *>(data + a + 16);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (T == 256) {
#pragma unroll
        for (uint32_t j = 0; j < GC; ++j) s_gear[ge * GC + ((j + ge) & (GC - 1))] = gv;
    } else {
        gear_fill<GC>(s_gear, gv, ge, threadIdx.x);
    }
    __syncthreads();
    if (!active) return;
    const char *gbase = reinterpret_cast<const char *>(s_gear);
    uint32_t *slots = s_slots[wv];
    const uint32_t lo8 = (threadIdx.x & (GC - 1)) * 8u;
    uint32_t ad[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int b = 0; b < 4; ++b) ad[i][b] = lo8;
    const uint64_t ms = mask_s << SCAN_SHIFT, ml = mask_l << SCAN_SHIFT;
    const uint32_t mh = (uint32_t)((mask_s & mask_l) >> (32 - SCAN_SHIFT));
    const uint32_t m0 = lane == 0 ? 0xffffffffu : 0u;
    uint32_t zero = 0;
    asm volatile("" : "+v"(zero));
    const uint32_t ms_lo = (uint32_t)ms, ms_hi = (uint32_t)(ms >> 32), ml_lo = (uint32_t)ml, ml_hi = (uint32_t)(ml >> 32);
    const uint64_t end_rel = n - r0;

    // q[k][b]: split partials of the lane's 8 dwords (k), byte b
    auto partials = [&](const uint4 (&v)[2], uint64_t (&q)[8][4]) {
        gear_look<GC>(gbase, ad[0], lo8, v[0].x, q[0]);
        gear_look<GC>(gbase, ad[0], lo8, v[0].y, q[1]);
        gear_look<GC>(gbase, ad[0], lo8, v[0].z, q[2]);
        gear_look<GC>(gbase, ad[0], lo8, v[0].w, q[3]);
        gear_look<GC>(gbase, ad[0], lo8, v[1].x, q[4]);
        gear_look<GC>(gbase, ad[0], lo8, v[1].y, q[5]);
        gear_look<GC>(gbase, ad[0], lo8, v[1].z, q[6]);
        gear_look<GC>(gbase, ad[0], lo8, v[1].w, q[7]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            q[k][1] = shl1_add(q[k][0], q[k][1]);
            q[k][2] = shl1_add(q[k][1], q[k][2]);
            q[k][3] = shl1_add(q[k][2], q[k][3]);
        }
    };
    auto block_p = [&](const uint64_t (&q)[8][4]) {
        uint64_t P = q[0][3];
#pragma unroll
        for (int k = 1; k < 8; ++k) P = shl_add<4>(P, q[k][3]);
        return P;
    };
    // zero state at the batch start, as the crate's hash restart
    uint64_t R1 = 0;
    uint32_t R2 = 0;
    if (has_pro) {
        uint64_t q[8][4];
        partials(pro, q);
        const uint64_t P = block_p(q);
        R1 = ((uint64_t)wave_ror1((uint32_t)(P >> 32)) << 32) | wave_ror1((uint32_t)P);
        R2 = wave_ror1((uint32_t)R1);
    }
    uint32_t segc = 0;
    // row limits as 32-bit scalars (a run has at most 128 rows): the first row that reaches
    // past the batch end (tail path) and the run's segments inside the batch, so the per-row
    // tests are SALU compares rather than 64-bit VALU ones
    const uint32_t nrow32 = (uint32_t)nrow;
    const uint32_t tail_row = (uint32_t)std::min<uint64_t>(end_rel / F32_ROW, 0x7fffffffu);
    const uint32_t seg_lim = (uint32_t)std::min<uint64_t>(nseg - seg0, 0x7fffffffu);
#pragma unroll 1
    for (uint32_t r = 0; r < nrow32; r += RING) {
#pragma unroll
        for (uint32_t u = 0; u < RING; ++u) {
            const uint32_t row = r + u;
            const uint32_t next = row + RING < nrow32 ? row + RING : nrow32 - 1;
            uint64_t q[8][4];
            if (CG_SCAN_PRIO) __builtin_amdgcn_s_setprio(CG_SCAN_PRIO);
            partials(ring[u], q);
            blk(next, ring[u]);  // the slot's bytes are in the lookups: re-issue it now
            if (CG_SCAN_PRIO) __builtin_amdgcn_s_setprio(0);
            const uint64_t P = block_p(q);
            const uint32_t a_lo = wave_ror1_add((uint32_t)P, zero), a_hi = wave_ror1_add((uint32_t)(P >> 32), zero);
            const uint32_t p1_lo = __builtin_amdgcn_bitop3_b32(m0, (uint32_t)R1, a_lo, 0xCA);
            const uint32_t p1_hi = __builtin_amdgcn_bitop3_b32(m0, (uint32_t)(R1 >> 32), a_hi, 0xCA);
            R1 = ((uint64_t)a_hi << 32) | a_lo;
            const uint32_t b_lo = wave_ror1_add(p1_lo, zero);
            const uint32_t p2_lo = __builtin_amdgcn_bitop3_b32(m0, R2, b_lo, 0xCA);
            R2 = b_lo;
            // C = P_{L-1} + (P_{L-2} << 32)
            const uint64_t C = ((uint64_t)(p1_hi + p2_lo) << 32) | p1_lo;
            uint32_t acc = 0xffffffffu;
            {
                uint64_t E = C;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint64_t h0 = shl_add<1>(E, q[k][0]), h1 = shl_add<2>(E, q[k][1]);
                    const uint64_t h2 = shl_add<3>(E, q[k][2]), h3 = shl_add<4>(E, q[k][3]);
                    acc = min(min(acc, (uint32_t)(h0 >> 32) & mh), (uint32_t)(h1 >> 32) & mh);
                    acc = min(min(acc, (uint32_t)(h2 >> 32) & mh), (uint32_t)(h3 >> 32) & mh);
                    E = h3;
                }
            }
            auto step = [&](uint64_t &x, uint32_t j) -> uint64_t {
                const uint64_t qj = q[j >> 2][j & 3];
                switch (j & 3) {
                case 0: return shl_add<1>(x, qj);
                case 1: return shl_add<2>(x, qj);
                case 2: return shl_add<3>(x, qj);
                default: return x = shl_add<4>(x, qj);
                }
            };
            const bool tail = row >= tail_row;  // (row + 1) x 2 KiB > end_rel; uniform
            if (__builtin_amdgcn_ballot_w64(acc == 0) != 0 || tail) {
                bool exact = tail;
                if (!tail) {
                    uint32_t ex = 0xffffffffu;
                    uint64_t x = C;
#pragma unroll
                    for (uint32_t j = 0; j < 32; ++j) {
                        const uint64_t hx = step(x, j);
                        const uint32_t lo = (uint32_t)hx, hi = (uint32_t)(hx >> 32);
                        ex = min(ex, min((lo & ms_lo) | (hi & ms_hi), (lo & ml_lo) | (hi & ml_hi)));
                    }
                    exact = __builtin_amdgcn_ballot_w64(ex == 0) != 0;
                }
                if (exact) {
                    const uint64_t prel = (uint64_t)row * F32_ROW + 32u * lane;
                    const uint32_t nb = prel < end_rel ? (end_rel - prel < 32 ? (uint32_t)(end_rel - prel) : 32u) : 0u;
                    uint32_t sm = 0, lm = 0;
                    uint64_t x = C;
#pragma unroll
                    for (uint32_t j = 0; j < 32; ++j) {
                        const uint64_t hx = step(x, j);
                        const uint64_t zs = hx & ms, zl = hx & ml;
                        const uint32_t ts = (uint32_t)zs | (uint32_t)(zs >> 32), tl = (uint32_t)zl | (uint32_t)(zl >> 32);
                        sm |= (1u - min(ts, 1u)) << j;
                        lm |= (1u - min(tl, 1u)) << j;
                    }
                    const uint32_t vm = nb >= 32 ? 0xffffffffu : (1u << nb) - 1u;
                    sm &= vm;
                    lm &= vm;
                    const uint32_t any = sm | lm, c = (uint32_t)__builtin_popcount(any);
                    uint32_t excl, total;
                    if (__builtin_amdgcn_ballot_w64(c > 1) == 0) {
                        const uint64_t bal = __builtin_amdgcn_ballot_w64(c != 0);
                        excl = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
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
                    const uint32_t pos0 = (uint32_t)(row % F32_RPS) * F32_ROW + 32u * lane;
                    uint32_t idx = segc + excl;
                    for (uint32_t m = any; m; m &= m - 1) {
                        const uint32_t j = (uint32_t)__builtin_ctz(m);
                        const uint32_t f = (((sm >> j) & 1u) * CG_FLAG_S) | (((lm >> j) & 1u) * CG_FLAG_L);
                        if (idx < cap) slots[idx] = ((pos0 + j) << 2) | f;
                        ++idx;
                    }
                    segc += total;
                }
            }
            if (u % F32_RPS == F32_RPS - 1) {  // segment end: flush its slots and count
                const uint64_t seg = seg0 + row / F32_RPS;
                if (row / F32_RPS < seg_lim) {
#if !CG_SCAN_FLUSH_INPLACE  // (see CG_SCAN_FLUSH_INPLACE at the top)
                    if (lane < min(segc, cap)) seg_cand[seg * cap + lane] = slots[lane];
#else
                    flush_slots(seg_cand + seg * cap, slots, min(segc, cap));
#endif
                    if (lane == 0) seg_count[seg] = segc;
                }
                segc = 0;
            }
        }
    }
}


// ---------------------------------------------------------------------------
// K1, persistent form (round 4, the product for prefilterable masks): the row work of
// k_scan_flat32 above, but the grid is only the workgroups the chip holds at once and every
// wave takes units of SPU segments (32 KiB at SPU = 8) from a queue until it is empty.
//
// Why: a one-shot grid (one run per wave, 8,192 waves at 1 GiB) kept only ~2.5 of the 4
// resident waves per SIMD busy on average (SQ_WAVE_CYCLES / kernel cycles,
// profiles/r04_pmc_sq_c2.json): a 512-thread workgroup's LDS is held until its slowest
// wave ends, and waves on one SIMD finish at different times (the oldest gets the VALU
// first), so dispatch rounds drain unevenly.  Here all waves live until the queue is
// empty, and the tail is at most one unit per wave.
//
// Queue: the batch's units split into 8 contiguous ranges, one per XCD (HW_REG_XCC_ID);
// a wave takes from its own XCD's range first (consecutive units stay in one L2, so a
// unit's halo row -- the row before it, read by the wave that took the previous unit a
// moment earlier -- is usually an L2 hit), then from the others'.  One returning agent-
// scope atomic per unit, dequeued a unit ahead so its latency hides behind the current
// unit's rows; the next unit's halo row and first two rows are in flight when the current
// unit's last rows are hashed.  The last wave to leave resets the counters, so every launch
// starts from zero without a memset.
// ---------------------------------------------------------------------------
#ifndef CG_SCAN_SPU
#define CG_SCAN_SPU 16u
#endif
#ifndef CG_SCAN_STATIC
#define CG_SCAN_STATIC 0
#endif
#ifndef CG_SCAN_LOADS_ONLY  // diagnostics A/B: the persistent schedule's loads without the hashing
#define CG_SCAN_LOADS_ONLY 0
#endif
#ifndef CG_SCAN_RESOLVE_LATE  // read the next unit's ticket at the unit's last row pair (else half-way)
#define CG_SCAN_RESOLVE_LATE 1
#endif
static_assert(sizeof(ScanQueue) == 9 * 64, "one 64-B line per counter");

template <uint32_t SPU, uint32_t GC = GEAR_COPIES, uint32_t T = SCAN2_T>
__global__ __launch_bounds__(T, 4) void k_scan_flat32p(const uint8_t *data, uint64_t n,
                                                           const uint64_t *__restrict__ gear_g, uint64_t mask_s,
                                                           uint64_t mask_l, uint32_t cap,
                                                           uint32_t *__restrict__ seg_count,
                                                           uint32_t *__restrict__ seg_cand, uint64_t nseg,
                                                           ScanQueue *queue, uint32_t nunits) {
    __shared__ __attribute__((aligned(16))) uint64_t s_gear[256 * GC];
    __shared__ uint32_t s_slots[T / 64][64];  // the open segment's candidate slots, per wave
    constexpr uint32_t R = SPU * F32_RPS;           // rows per unit
    constexpr uint32_t UNIT = SPU * CG_SEG;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    xcc &= 7u;
    typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
    // A unit's rows through a buffer resource based at its halo row (the row before the unit;
    // at the batch start, the unit itself), its size ending at the batch end rounded up to the
    // 16-byte granule (k_scan_flat32).  The halo is entry 0 of the unit's stream, data row j
    // entry j + 1 at byte hoff + j x 2 KiB of the resource.
    struct UnitRs {
        __amdgpu_buffer_rsrc_t rs;
        uint32_t hoff;  // 2 KiB, or 0 for the batch's first unit (no halo: its "halo" is row 0, unused)
    };
    auto unit_rs = [&](uint32_t u) {
        const uint64_t r0 = (uint64_t)u * UNIT;
        const uint64_t base = r0 >= F32_ROW ? r0 - F32_ROW : 0;
        const uint64_t avail = base < n ? ((n - base + 15) & ~15ull) : 0;
        const uint64_t span = UNIT + (r0 - base);
        return UnitRs{__builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(data + (base < n ? base : 0)), (short)0,
                                                        (int)(avail < span ? avail : span), 0x00027000),
                      (uint32_t)(r0 - base)};
    };
    const uint32_t lane_off = 32u * lane;
    // A halo row feeds the hash only through lanes 62 and 63 (C_0 and C_1 take P_63 and
    // P_62), so its other lanes read at an offset past every resource's size: zeros, no
    // memory request (PMC: the halo rows were +3 % of the unit bytes in HBM reads).
    const uint32_t halo_off = lane >= 62 ? lane_off : 0x80000000u;
    auto blk = [&](__amdgpu_buffer_rsrc_t rs, uint32_t so, uint4 (&v)[2], uint32_t voff) {
        const u32x4_t x0 = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, so, 2);  // aux 2: nt
        const u32x4_t x1 = __builtin_amdgcn_raw_buffer_load_b128(rs, voff + 16u, so, 2);
        v[0] = uint4{x0.x, x0.y, x0.z, x0.w};
        v[1] = uint4{x1.x, x1.y, x1.z, x1.w};
    };
    // One unit index, wave-uniform; nunits when every range is empty.  The add on this XCD's
    // head is issued at a unit's start and read half a unit later (the compiler's atomic
    // optimizer is off for this file, so the returning atomic is one instruction and the
    // wait for it lands at the read); only once this XCD's range is empty are the other
    // heads tried, one at a time.
    const uint32_t own_lo = (uint32_t)((uint64_t)nunits * xcc / 8);
    const uint32_t own_n = (uint32_t)((uint64_t)nunits * (xcc + 1) / 8) - own_lo;
    uint32_t tick = 0;
#if CG_SCAN_STATIC
    // (A/B form: no queue; wave g of the grid takes units g, g + W, g + 2W, ...)
    uint32_t snext = blockIdx.x * (T / 64) + wv;
    const uint32_t sstride = gridDim.x * (T / 64);
    auto dq_issue = [&]() {};
#else
    auto dq_issue = [&]() {
        if (lane == 0) tick = __hip_atomic_fetch_add(&queue->head[xcc][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
#endif
    // `dep`: a value of the row loop, so the read stays where it is written (without it the
    // compiler hoists the read out of the row loop, to right after the issue)
    auto dq_resolve = [&](uint32_t dep) -> uint32_t {
#if CG_SCAN_STATIC
        (void)dep;
        const uint32_t si = snext;
        snext += sstride;
        return si < nunits ? si : nunits;
#else
        (void)0;
#endif
        asm volatile("" : "+v"(tick) : "v"(dep));
        const uint32_t i = __builtin_amdgcn_readfirstlane(tick);
        if (i < own_n) return own_lo + i;
        for (uint32_t k = 1; k < 8; ++k) {
            const uint32_t x = (xcc + k) & 7u;
            const uint32_t lo = (uint32_t)((uint64_t)nunits * x / 8), hi = (uint32_t)((uint64_t)nunits * (x + 1) / 8);
            if (lo == hi) continue;
            uint32_t j = 0;
            if (lane == 0) j = __hip_atomic_fetch_add(&queue->head[x][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            j = __builtin_amdgcn_readfirstlane(j);
            if (j < hi - lo) return lo + j;
        }
        return nunits;
    };

    static_assert(T == 2 * 256 || (T == 256 && GC == GEAR_COPIES_LEAN), "two threads per Gear entry, or one (lean)");
    const uint32_t ge = T == 256 ? threadIdx.x : threadIdx.x >> 1;
    const uint64_t gv = gear_g[ge] << SCAN_SHIFT;
    dq_issue();
    uint32_t u = dq_resolve(0u);
    const bool any = u < nunits;
    UnitRs ur = unit_rs(any ? u : 0);
    // the ring: two stream entries in flight; a unit starts with its halo in slot 0 and its
    // row 0 in slot 1
    uint4 ring[2][2];
    blk(ur.rs, 0, ring[0], halo_off);
    blk(ur.rs, ur.hoff, ring[1], lane_off);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (T == 256) {
#pragma unroll
        for (uint32_t j = 0; j < GC; ++j) s_gear[ge * GC + ((j + ge) & (GC - 1))] = gv;
    } else {
        gear_fill<GC>(s_gear, gv, ge, threadIdx.x);
    }
    __syncthreads();
    const char *gbase = reinterpret_cast<const char *>(s_gear);
    uint32_t *slots = s_slots[wv];
    const uint32_t lo8 = (threadIdx.x & (GC - 1)) * 8u;
    uint32_t ad[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int b = 0; b < 4; ++b) ad[i][b] = lo8;
    const uint64_t ms = mask_s << SCAN_SHIFT, ml = mask_l << SCAN_SHIFT;
    const uint32_t mh = (uint32_t)((mask_s & mask_l) >> (32 - SCAN_SHIFT));
    const uint32_t m0 = lane == 0 ? 0xffffffffu : 0u;
    uint32_t zero = 0;
    asm volatile("" : "+v"(zero));
    const uint32_t ms_lo = (uint32_t)ms, ms_hi = (uint32_t)(ms >> 32), ml_lo = (uint32_t)ml, ml_hi = (uint32_t)(ml >> 32);

    auto partials = [&](const uint4 (&v)[2], uint64_t (&q)[8][4]) {
        gear_look<GC>(gbase, ad[0], lo8, v[0].x, q[0]);
        gear_look<GC>(gbase, ad[0], lo8, v[0].y, q[1]);
        gear_look<GC>(gbase, ad[0], lo8, v[0].z, q[2]);
        gear_look<GC>(gbase, ad[0], lo8, v[0].w, q[3]);
        gear_look<GC>(gbase, ad[0], lo8, v[1].x, q[4]);
        gear_look<GC>(gbase, ad[0], lo8, v[1].y, q[5]);
        gear_look<GC>(gbase, ad[0], lo8, v[1].z, q[6]);
        gear_look<GC>(gbase, ad[0], lo8, v[1].w, q[7]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            q[k][1] = shl1_add(q[k][0], q[k][1]);
            q[k][2] = shl1_add(q[k][1], q[k][2]);
            q[k][3] = shl1_add(q[k][2], q[k][3]);
        }
    };
    auto block_p = [&](const uint64_t (&q)[8][4]) {
        uint64_t P = q[0][3];
#pragma unroll
        for (int k = 1; k < 8; ++k) P = shl_add<4>(P, q[k][3]);
        return P;
    };

#if CG_SCAN_LOADS_ONLY
    uint32_t sink = 0;
#endif
    while (any) {
        const uint64_t r0 = (uint64_t)u * UNIT;
        const uint64_t seg0 = (uint64_t)u * SPU;
        const uint64_t end_rel = n - r0;  // > 0: units start inside the batch
        // 32-bit scalar row limits (SALU compares in the row loop): the first row reaching past
        // the batch end, and the unit's segments inside the batch
        const uint32_t tail_row = (uint32_t)std::min<uint64_t>(end_rel / F32_ROW, 0x7fffffffu);
        const uint32_t seg_lim = (uint32_t)std::min<uint64_t>(nseg - seg0, 0x7fffffffu);
        // the next unit: its head add issued now and read half a unit later, its halo and row
        // 0 issued as this unit's last two rows free their slots
        dq_issue();
        uint32_t un = nunits;
        bool more = false;
        UnitRs urn = ur;
        // halo (slot 0): zero state at the batch start, as the crate's hash restart
        uint64_t R1 = 0;
        uint32_t R2 = 0;
        {
            uint64_t q[8][4];
            partials(ring[0], q);
            blk(ur.rs, ur.hoff + F32_ROW, ring[0], lane_off);  // row 1
            if (r0 >= F32_ROW) {
                const uint64_t P = block_p(q);
                R1 = ((uint64_t)wave_ror1((uint32_t)(P >> 32)) << 32) | wave_ror1((uint32_t)P);
                R2 = wave_ror1((uint32_t)R1);
            }
        }
        uint32_t segc = 0;
#pragma unroll 1
        for (uint32_t r = 0; r < R; r += 2) {
            if (r == (CG_SCAN_RESOLVE_LATE ? R - 2 : ((R / 2) & ~1u))) {  // uniform: read the next unit's index
                un = dq_resolve((uint32_t)R1);
                more = un < nunits;
                urn = unit_rs(more ? un : u);
            }
#pragma unroll
            for (uint32_t uu = 0; uu < 2; ++uu) {
                const uint32_t row = r + uu;
                const uint32_t slot = uu ^ 1u;  // data row j sits in slot (j + 1) & 1
                // the entry two ahead: row + 2 of this unit, else the next unit's halo / row 0
                const uint32_t e = row + 2;
                const __amdgpu_buffer_rsrc_t nrs = e < R ? ur.rs : urn.rs;
                const uint32_t nso = e < R ? ur.hoff + e * F32_ROW : (e == R ? 0u : urn.hoff);
                // (a row past the batch end -- the last unit's -- takes the tail path below with
                // every position masked: the slot's loads stay on one code path, so the compiler
                // counts vmcnt exactly)
                const uint64_t rowb = (uint64_t)row * F32_ROW;
#if CG_SCAN_LOADS_ONLY
                // diagnostics form: the same schedule with the hashing removed (no candidates)
                sink ^= ring[slot][0].x ^ ring[slot][0].y ^ ring[slot][0].z ^ ring[slot][0].w ^ ring[slot][1].x ^
                        ring[slot][1].y ^ ring[slot][1].z ^ ring[slot][1].w;
                blk(nrs, nso, ring[slot], e == R ? halo_off : lane_off);
                (void)rowb;
                if (uu == 1) {
                    const uint64_t seg = seg0 + row / F32_RPS;
                    if (seg < nseg && lane == 0) seg_count[seg] = 0;
                }
                continue;
#endif
                uint64_t q[8][4];
                if (CG_SCAN_PRIO) __builtin_amdgcn_s_setprio(CG_SCAN_PRIO);
                partials(ring[slot], q);
                blk(nrs, nso, ring[slot], e == R ? halo_off : lane_off);  // re-issue the slot now
                if (CG_SCAN_PRIO) __builtin_amdgcn_s_setprio(0);
                const uint64_t P = block_p(q);
                const uint32_t a_lo = wave_ror1_add((uint32_t)P, zero), a_hi = wave_ror1_add((uint32_t)(P >> 32), zero);
                const uint32_t p1_lo = __builtin_amdgcn_bitop3_b32(m0, (uint32_t)R1, a_lo, 0xCA);
                const uint32_t p1_hi = __builtin_amdgcn_bitop3_b32(m0, (uint32_t)(R1 >> 32), a_hi, 0xCA);
                R1 = ((uint64_t)a_hi << 32) | a_lo;
                const uint32_t b_lo = wave_ror1_add(p1_lo, zero);
                const uint32_t p2_lo = __builtin_amdgcn_bitop3_b32(m0, R2, b_lo, 0xCA);
                R2 = b_lo;
                // C = P_{L-1} + (P_{L-2} << 32)
                const uint64_t C = ((uint64_t)(p1_hi + p2_lo) << 32) | p1_lo;
                uint32_t acc = 0xffffffffu;
                {
                    uint64_t E = C;
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const uint64_t h0 = shl_add<1>(E, q[k][0]), h1 = shl_add<2>(E, q[k][1]);
                        const uint64_t h2 = shl_add<3>(E, q[k][2]), h3 = shl_add<4>(E, q[k][3]);
                        acc = min(min(acc, (uint32_t)(h0 >> 32) & mh), (uint32_t)(h1 >> 32) & mh);
                        acc = min(min(acc, (uint32_t)(h2 >> 32) & mh), (uint32_t)(h3 >> 32) & mh);
                        E = h3;
                    }
                }
                auto step = [&](uint64_t &x, uint32_t j) -> uint64_t {
                    const uint64_t qj = q[j >> 2][j & 3];
                    switch (j & 3) {
                    case 0: return shl_add<1>(x, qj);
                    case 1: return shl_add<2>(x, qj);
                    case 2: return shl_add<3>(x, qj);
                    default: return x = shl_add<4>(x, qj);
                    }
                };
                const bool tail = row >= tail_row;  // rowb + 2 KiB > end_rel; uniform
                if (__builtin_amdgcn_ballot_w64(acc == 0) != 0 || tail) {
                    bool exact = tail;
                    if (!tail) {
                        uint32_t ex = 0xffffffffu;
                        uint64_t x = C;
#pragma unroll
                        for (uint32_t j = 0; j < 32; ++j) {
                            const uint64_t hx = step(x, j);
                            const uint32_t lo = (uint32_t)hx, hi = (uint32_t)(hx >> 32);
                            ex = min(ex, min((lo & ms_lo) | (hi & ms_hi), (lo & ml_lo) | (hi & ml_hi)));
                        }
                        exact = __builtin_amdgcn_ballot_w64(ex == 0) != 0;
                    }
                    if (exact) {
                        const uint64_t prel = rowb + 32u * lane;
                        const uint32_t nb = prel < end_rel ? (end_rel - prel < 32 ? (uint32_t)(end_rel - prel) : 32u) : 0u;
                        uint32_t sm = 0, lm = 0;
                        uint64_t x = C;
#pragma unroll
                        for (uint32_t j = 0; j < 32; ++j) {
                            const uint64_t hx = step(x, j);
                            const uint64_t zs = hx & ms, zl = hx & ml;
                            const uint32_t ts = (uint32_t)zs | (uint32_t)(zs >> 32), tl = (uint32_t)zl | (uint32_t)(zl >> 32);
                            sm |= (1u - min(ts, 1u)) << j;
                            lm |= (1u - min(tl, 1u)) << j;
                        }
                        const uint32_t vm = nb >= 32 ? 0xffffffffu : (1u << nb) - 1u;
                        sm &= vm;
                        lm &= vm;
                        const uint32_t anyb = sm | lm, c = (uint32_t)__builtin_popcount(anyb);
                        uint32_t excl, total;
                        if (__builtin_amdgcn_ballot_w64(c > 1) == 0) {
                            const uint64_t bal = __builtin_amdgcn_ballot_w64(c != 0);
                            excl = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
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
                        const uint32_t pos0 = (row % F32_RPS) * F32_ROW + 32u * lane;
                        uint32_t idx = segc + excl;
                        for (uint32_t m = anyb; m; m &= m - 1) {
                            const uint32_t j = (uint32_t)__builtin_ctz(m);
                            const uint32_t f = (((sm >> j) & 1u) * CG_FLAG_S) | (((lm >> j) & 1u) * CG_FLAG_L);
                            if (idx < cap) slots[idx] = ((pos0 + j) << 2) | f;
                            ++idx;
                        }
                        segc += total;
                    }
                }
                if (uu == 1) {  // segment end: flush its slots and count
                    const uint64_t seg = seg0 + row / F32_RPS;
                    if (row / F32_RPS < seg_lim) {
#if !CG_SCAN_FLUSH_INPLACE  // (see CG_SCAN_FLUSH_INPLACE at the top)
                        if (lane < min(segc, cap)) seg_cand[seg * cap + lane] = slots[lane];
#else
                        flush_slots(seg_cand + seg * cap, slots, min(segc, cap));
#endif
                        if (lane == 0) seg_count[seg] = segc;
                    }
                    segc = 0;
                }
            }
        }
        if (!more) break;
        // the next unit's halo went to slot 1 and its row 0 to slot 0: swap them into place
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint4 t = ring[0][k];
            ring[0][k] = ring[1][k];
            ring[1][k] = t;
        }
        u = un;
        ur = urn;
    }
#if CG_SCAN_LOADS_ONLY
    if (sink == 0x9e3779b9u && nseg == 0) seg_count[0] = sink;  // keeps the loads alive
#endif
    // leave: the last wave of the grid resets the queue for the next launch.  Relaxed:
    // a wave counts itself done only after its last dequeue has returned, the counter
    // guards no data, and the kernel's end publishes the reset.  (An acquire-release
    // count made every wave write back and invalidate its XCD's L2 on the way out --
    // buffer_wbl2 / buffer_inv sc1 -- dropping the lines the running waves had fetched.)
    if (lane == 0) {
        const uint32_t waves = gridDim.x * (T / 64);
        const uint32_t old = __hip_atomic_fetch_add(&queue->done[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == waves - 1) {
#pragma unroll
            for (int x = 0; x < 8; ++x) __hip_atomic_store(&queue->head[x][0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&queue->done[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

#ifdef CG_DIAG
// diagnostics build (scan_diag.hip): the alternative scan kernels of DESIGN.md §4's A/B
extern uint32_t g_scan_spw_max, g_scan_variant;
bool launch_scan_diag(const uint8_t *d_data, uint64_t n, const uint64_t *d_gear, uint64_t mask_s, uint64_t mask_l,
                      uint32_t cap, uint32_t *d_seg_count, uint32_t *d_seg_cand, uint64_t nseg, hipStream_t st);
using ScanFlatKernel = void (*)(const uint8_t *, uint64_t, const uint64_t *, uint64_t, uint64_t, uint32_t, uint32_t *,
                                uint32_t *, uint64_t, uint32_t);
ScanFlatKernel scan_flat_diag_kernel(ScanFlatKernel product);
// k_scan_flat32 forms the diagnostics build selects (variant 5, modes 21 / 22)
ScanFlatKernel scan_flat32_variant(uint32_t mode) {
    return mode == 21 ? k_scan_flat32<4, true> : mode == 22 ? k_scan_flat32<2, false> : k_scan_flat32<2, true>;
}
// k_scan<true> (variant 4: the prefiltered own-segment kernel)
void launch_k_scan_pre(const uint8_t *d_data, uint64_t n, const uint64_t *d_gear, uint64_t mask_s, uint64_t mask_l,
                       uint32_t cap, uint32_t *d_seg_count, uint32_t *d_seg_cand, uint64_t nseg, hipStream_t st) {
    hipLaunchKernelGGL(k_scan<true>, dim3((uint32_t)((nseg + SCAN2_T - 1) / SCAN2_T)), dim3(SCAN2_T), 0, st, d_data, n,
                       d_gear, mask_s, mask_l, cap, d_seg_count, d_seg_cand, nseg);
}
#endif

// test hook (cg_test_scan_kernel): 0 = the product's choice (below), 1 = the one-shot
// k_scan_flat32, 2 = the persistent k_scan_flat32p at any size
uint32_t g_scan_kernel = 0;
// test hook (cg_test_scan_grid): workgroups of the persistent scan (0 = the resident count)
uint64_t g_scan_grid = 0;

// Lean one-shot scan (256-thread workgroups, GEAR_COPIES_LEAN table, 17 KiB of LDS): the
// digest pipeline's boundary stream asks for it (t_scan_lean, pipeline.hip), because there
// every CU already holds two k_sha256 workgroups of the merged launches, and a 512-thread,
// 128-VGPR scan workgroup does not fit beside them (the per-SIMD register file: two digest
// waves of 136 VGPRs leave room for one 128-VGPR wave on that SIMD, and the SPI gives a
// 512-thread workgroup two per SIMD; profiles/r06_v28_hol_probe.txt).  So the boundary stages
// of the next group waited 0.5-26 ms per scan for a digest workgroup to end
// (profiles/r06_v22_*), and the lanes starved.  The lean scan alone is ~10 % slower (0.23 vs
// 0.21 ms per GiB cold: two VALU per lookup address, 2-way bank conflicts), but runs beside the
// digests (1.0-1.3 ms under load, against 0.5-26).  CHUNKER_AMD_SCAN_LEAN=0/1 (read once)
// forces it off / on for every one-shot scan (A/B).
thread_local bool t_scan_lean = false;
static bool scan_lean() {
    static const int forced = [] {
        const char *e = getenv("CHUNKER_AMD_SCAN_LEAN");
        return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
    }();
    return forced >= 0 ? forced == 1 : t_scan_lean;
}

void launch_scan(const uint8_t *d_data, uint64_t n, const uint64_t *d_gear, uint64_t mask_s, uint64_t mask_l,
                 uint32_t cap, uint32_t *d_seg_count, uint32_t *d_seg_cand, uint64_t nseg, hipStream_t st,
                 ScanQueue *d_queue) {
    if (nseg == 0) return;
    const bool lean = scan_lean();
    const uint64_t blocks = (nseg + SCAN2_T - 1) / SCAN2_T;
    // prefilter when the bits of mask_s & mask_l it tests leave hits rarer than ~1 per 16 KiB
    // (averages >= 64 KiB with the v2020 masks)
    const bool pre = __builtin_popcountll((mask_s & mask_l) >> SCAN_SHIFT) >= 14;
#ifdef CG_DIAG
    if (launch_scan_diag(d_data, n, d_gear, mask_s, mask_l, cap, d_seg_count, d_seg_cand, nseg, st)) return;
#endif
    // k_scan_flat re-walks a whole 1 KiB row whenever its prefilter fires, k_scan only the
    // lane's 64-B piece; with split chains the flat kernel is faster at 16 prefilter bits
    // (config 2: 0.205 vs 0.27 ms per GiB) and at 14 (config 4: 0.20 vs 0.237;
    // profiles/r02_v10_diag_scan_split.json), so k_scan only takes the dense masks
    if (!pre) {
        hipLaunchKernelGGL(k_scan<false>, dim3((uint32_t)blocks), dim3(SCAN2_T), 0, st, d_data, n, d_gear, mask_s,
                           mask_l, cap, d_seg_count, d_seg_cand, nseg);
        return;
    }
    // segments per wave: 4..32 below 4 GiB (two dispatch rounds of waves at 1 GiB, runs of at
    // most 128 KiB: 256 KiB runs were 2-5 % slower at configs 2 and 5 in round 2), 64 from
    // 4 GiB on -- runs short enough that the waves in flight (one stream each, advancing
    // together) stay within a window of ~1 GiB rather than spread at a power-of-two stride
    // of several MiB (4 MiB runs at config 4 read ~20 % slower).  Same box, alternating
    // builds (profiles/r03_v37_ab_scan_runs.txt): 256 KiB runs read the 16 GiB configs 4 / 5
    // in 3.63 / 3.76 ms against 3.76 / 3.85 for 128 KiB (5 and 3 pairs); 64 KiB runs 3-5 %
    // slower, 512 KiB mixed; config 3's 1 GiB equal within the box's spread
    uint64_t spw = (nseg + 4095) / 4096;
#ifndef CG_SCAN_SPW_MAX
#define CG_SCAN_SPW_MAX (nseg >= (1ull << 20) ? 64 : 32)
#endif
    uint64_t spw_max = CG_SCAN_SPW_MAX;
#ifdef CG_DIAG
    if (g_scan_spw_max) spw_max = g_scan_spw_max;
#endif
    spw = spw < 4 ? 4 : (spw > spw_max ? spw_max : (spw + 3) & ~3ull);
    const uint64_t waves = (nseg + spw - 1) / spw;
    const uint64_t wgs = (waves + SCAN2_T / 64 - 1) / (SCAN2_T / 64);
    // product: the persistent form (k_scan_flat32p) from 4 GiB on when the caller passes its
    // queue, the one-shot k_scan_flat32 below (cg_test_scan_kernel forces either).  Same-process
    // A/B, 5 reps each (profiles/r04_v5_scan_ab*.json): 16 GiB of 1 GiB NARs (configs 4 / 5)
    // 3.36-3.42 / 3.48-3.57 ms persistent against 3.44-3.57 / 3.54-3.70 one-shot; 1 GiB of
    // 4 MiB NARs (config 2) 0.23-0.27 against 0.203 -- there the one-shot grid is only two
    // dispatch rounds and the queue's per-unit cost shows.  The 16-byte row forms of
    // k_scan_flat are the diagnostics build's A/B
#ifdef CG_DIAG
    const bool diag_variant = g_scan_variant == 5;
#else
    const bool diag_variant = false;
#endif
    const bool persistent = g_scan_kernel == 2 || (g_scan_kernel == 0 && nseg >= (1ull << 20));
    if (d_queue && persistent && !diag_variant) {
        const uint64_t nunits = (nseg + CG_SCAN_SPU - 1) / CG_SCAN_SPU;
        // the lean form: 256-thread workgroups (4 waves), twice as many for the same waves
        const uint32_t t = lean ? 256u : SCAN2_T;
        const uint64_t resident = scan_resident_wgs() * (lean ? 2 : 1);
        const uint64_t want = (nunits + t / 64 - 1) / (t / 64);  // >= one unit per wave
        uint64_t grid = std::max<uint64_t>(1, std::min(want, resident));
        if (g_scan_grid) grid = g_scan_grid;
        auto kp = lean ? k_scan_flat32p<CG_SCAN_SPU, GEAR_COPIES_LEAN, 256> : k_scan_flat32p<CG_SCAN_SPU>;
        hipLaunchKernelGGL(kp, dim3((uint32_t)grid), dim3(t), 0, st, d_data, n, d_gear, mask_s, mask_l, cap,
                           d_seg_count, d_seg_cand, nseg, d_queue, (uint32_t)nunits);
        return;
    }
    if (lean) {  // 256-thread workgroups, 18 KiB: beside two digest workgroups per CU
        auto kl = k_scan_flat32<2, true, GEAR_COPIES_LEAN, 256>;
        hipLaunchKernelGGL(kl, dim3((uint32_t)((waves + 3) / 4)), dim3(256), 0, st, d_data, n, d_gear, mask_s, mask_l,
                           cap, d_seg_count, d_seg_cand, nseg, (uint32_t)spw);
        return;
    }
    auto k = k_scan_flat32<2, true>;
#ifdef CG_DIAG
    if (diag_variant) k = scan_flat_diag_kernel(k);
#endif
    hipLaunchKernelGGL(k, dim3((uint32_t)wgs), dim3(SCAN2_T), 0, st, d_data, n, d_gear, mask_s, mask_l, cap,
                       d_seg_count, d_seg_cand, nseg, (uint32_t)spw);
}

// Workgroups of k_scan_flat32p the current device holds at once (CUs x the occupancy
// query), cached per device.
uint64_t scan_resident_wgs() {
    static std::atomic<uint64_t> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    uint64_t v = cache[dev].load(std::memory_order_relaxed);
    if (v) return v;
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_scan_flat32p<CG_SCAN_SPU>, SCAN2_T, 0) != hipSuccess ||
        per_cu <= 0)
        per_cu = 2;
    v = (uint64_t)cus * (uint64_t)per_cu;
    cache[dev].store(v, std::memory_order_relaxed);
    return v;
}
// ---------------------------------------------------------------------------
// Exclusive prefix sum u32 -> u64 (one launch for small inputs; tile sums + apply otherwise).
// ---------------------------------------------------------------------------
#define SCAN_T 256u
#define SCAN_ITEMS 8u
#define SCAN_TILE (SCAN_T * SCAN_ITEMS)

__device__ __forceinline__ uint64_t xform(uint32_t v, uint32_t cap) { return cap ? (v <= cap ? v : 1u) : v; }

__global__ __launch_bounds__(SCAN_T) void k_tile_sums(const uint32_t *__restrict__ in, uint64_t n, uint32_t cap,
                                                      uint64_t *__restrict__ tile_sum, StageIn si) {
    __shared__ uint64_t s_wave[SCAN_T / 64];
    const uint32_t ntiles = (uint32_t)((n + SCAN_TILE - 1) / SCAN_TILE);
    if (blockIdx.x >= ntiles) {  // stage-in blocks (uniform per block)
        const uint32_t e = blockIdx.x - ntiles;
        stage_in_part(si, e / STAGE_IN_BLOCKS, e % STAGE_IN_BLOCKS, STAGE_IN_BLOCKS);
        return;
    }
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_ITEMS; ++k)
        if (base + k < n) s += xform(in[base + k], cap);
    const uint64_t inc = block_inclusive_scan(s, s_wave);
    if (threadIdx.x == SCAN_T - 1) tile_sum[blockIdx.x] = inc;
}

// Single block: exclusive scan of tile sums in place; total to tile_sum[ntiles].
__global__ __launch_bounds__(1024) void k_top_scan(uint64_t *__restrict__ tile_sum, uint64_t ntiles) {
    __shared__ uint64_t s_wave[16];
    __shared__ uint64_t s_carry;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (uint64_t b = 0; b < ntiles; b += 1024) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t v = i < ntiles ? tile_sum[i] : 0;
        const uint64_t inc = block_inclusive_scan(v, s_wave);
        const uint64_t carry = s_carry;
        if (i < ntiles) tile_sum[i] = carry + inc - v;
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = carry + inc;
        __syncthreads();
    }
    if (threadIdx.x == 0) tile_sum[ntiles] = s_carry;
}

// Optional fused compaction: the scan input is the per-segment candidate count and the
// output its entry offset, so the thread that owns a segment's offset also moves that
// segment's candidate slots into the sorted entry list (what k_compact did in its own launch).
struct CompactArgs {
    const uint32_t *cand;  // nseg * cap candidate slots (scan.hip k_scan_flat32 / k_scan)
    uint64_t *entries;     // sorted entry list (position << 2 | tier)
};

__device__ __forceinline__ void compact_segment(uint64_t seg, uint32_t count, uint64_t base, uint32_t cap,
                                                const CompactArgs &ca) {
    if (count == 0) return;
    const uint64_t start = seg * CG_SEG;
    if (count <= cap) {
        for (uint32_t k = 0; k < count; ++k) {
            const uint32_t e = ca.cand[seg * cap + k];
            ca.entries[base + k] = ((start + (e >> 2)) << 2) | (e & 3u);
        }
    } else {
        ca.entries[base] = start << 2;  // dense-segment marker
    }
}

// Second pass of the tiled scan.  REDUCE: tile_sum holds each tile's own total (k_tile_sums)
// and a block sums its predecessors' (at most SCAN_REDUCE_MAX tiles, all L2-resident), so
// the single-block k_top_scan launch is not needed; otherwise tile_sum is already the
// exclusive scan of the tiles with the total at [ntiles].
#define SCAN_REDUCE_MAX 4096u
template <bool COMPACT, bool REDUCE>
__global__ __launch_bounds__(SCAN_T) void k_scan_apply(const uint32_t *__restrict__ in, uint64_t n, uint32_t cap,
                                                       const uint64_t *__restrict__ tile_sum,
                                                       uint64_t *__restrict__ out, uint64_t ntiles, CompactArgs ca) {
    __shared__ uint64_t s_wave[SCAN_T / 64];
    __shared__ uint64_t s_pre;
    uint64_t tile_pre;
    if (REDUCE) {
        uint64_t p = 0;
        for (uint64_t i = threadIdx.x; i < blockIdx.x; i += SCAN_T) p += tile_sum[i];
        const uint64_t incp = block_inclusive_scan(p, s_wave);
        if (threadIdx.x == SCAN_T - 1) s_pre = incp;
        __syncthreads();
        tile_pre = s_pre;
    } else {
        tile_pre = tile_sum[blockIdx.x];
    }
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    uint32_t raw[SCAN_ITEMS];
    uint64_t v[SCAN_ITEMS];
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_ITEMS; ++k) {
        raw[k] = base + k < n ? in[base + k] : 0u;
        v[k] = xform(raw[k], cap);
        s += v[k];
    }
    const uint64_t inc = block_inclusive_scan(s, s_wave);
    uint64_t run = tile_pre + inc - s;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_ITEMS; ++k) {
        if (base + k < n) {
            out[base + k] = run;
            if (COMPACT) compact_segment(base + k, raw[k], run, cap, ca);
        }
        run += v[k];
    }
    if (REDUCE) {
        if (blockIdx.x == ntiles - 1 && threadIdx.x == SCAN_T - 1) out[n] = tile_pre + inc;
    } else if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[n] = tile_sum[ntiles];
    }
}

// Whole scan in one block (n up to SCAN_SMALL_MAX): 1024 threads × SCAN_ITEMS per pass,
// carry between passes.  Used for the per-NAR chunk counts, the BLAKE3 group counts and
// small batches' segment counts, where three launches cost more than the work.
#define SCAN_SMALL_T 1024u
#define SCAN_SMALL_MAX (4u * SCAN_SMALL_T * SCAN_ITEMS)
template <bool COMPACT>
__global__ __launch_bounds__(SCAN_SMALL_T) void k_scan_small(const uint32_t *__restrict__ in, uint64_t n, uint32_t cap,
                                                             uint64_t *__restrict__ out, CompactArgs ca, StageIn si) {
    __shared__ uint64_t s_wave[SCAN_SMALL_T / 64];
    __shared__ uint64_t s_carry;
    if (blockIdx.x > 0) {  // stage-in blocks (uniform per block)
        const uint32_t e = blockIdx.x - 1;
        stage_in_part(si, e / STAGE_IN_BLOCKS, e % STAGE_IN_BLOCKS, STAGE_IN_BLOCKS);
        return;
    }
    uint64_t carry = 0;
    for (uint64_t b = 0; b < n; b += (uint64_t)SCAN_SMALL_T * SCAN_ITEMS) {
        const uint64_t base = b + threadIdx.x * SCAN_ITEMS;
        uint32_t raw[SCAN_ITEMS];
        uint64_t v[SCAN_ITEMS];
        uint64_t s = 0;
#pragma unroll
        for (uint32_t k = 0; k < SCAN_ITEMS; ++k) {
            raw[k] = base + k < n ? in[base + k] : 0u;
            v[k] = xform(raw[k], cap);
            s += v[k];
        }
        const uint64_t inc = block_inclusive_scan(s, s_wave);
        uint64_t run = carry + inc - s;
#pragma unroll
        for (uint32_t k = 0; k < SCAN_ITEMS; ++k) {
            if (base + k < n) {
                out[base + k] = run;
                if (COMPACT) compact_segment(base + k, raw[k], run, cap, ca);
            }
            run += v[k];
        }
        if (threadIdx.x == SCAN_SMALL_T - 1) s_carry = carry + inc;
        __syncthreads();
        carry = s_carry;
        __syncthreads();
    }
    if (threadIdx.x == 0) out[n] = carry;
}

size_t exclusive_scan_tmp_elems(uint64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

// One launch for n ≤ SCAN_SMALL_MAX, two up to SCAN_REDUCE_MAX tiles, three beyond.
// Test hook (cg_test_scan_path): 0 = by size, 1 = one block, 2 = tile sums + reducing
// apply, 3 = tile sums + top scan + apply, so a test reaches every path at small sizes.
uint32_t g_scan_path = 0;

template <bool COMPACT>
static void launch_scan_impl(const uint32_t *d_in, uint64_t *d_out, uint64_t n, uint32_t cap, uint64_t *d_tmp,
                             CompactArgs ca, hipStream_t st, const StageIn &si = StageIn{}) {
    const uint32_t extra = (uint32_t)si.n * STAGE_IN_BLOCKS;
    if (n == 0) {
        (void)hipMemsetAsync(d_out, 0, sizeof(uint64_t), st);
        launch_stage_in(si, st);
        return;
    }
    const uint32_t path = g_scan_path;
    if (path == 1 || (path == 0 && n <= SCAN_SMALL_MAX)) {
        hipLaunchKernelGGL(k_scan_small<COMPACT>, dim3(1 + extra), dim3(SCAN_SMALL_T), 0, st, d_in, n, cap, d_out, ca,
                           si);
        return;
    }
    const uint64_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    hipLaunchKernelGGL(k_tile_sums, dim3((uint32_t)ntiles + extra), dim3(SCAN_T), 0, st, d_in, n, cap, d_tmp, si);
    if (path == 2 || (path == 0 && ntiles <= SCAN_REDUCE_MAX)) {
        hipLaunchKernelGGL((k_scan_apply<COMPACT, true>), dim3((uint32_t)ntiles), dim3(SCAN_T), 0, st, d_in, n, cap,
                           d_tmp, d_out, ntiles, ca);
    } else {
        hipLaunchKernelGGL(k_top_scan, dim3(1), dim3(1024), 0, st, d_tmp, ntiles);
        hipLaunchKernelGGL((k_scan_apply<COMPACT, false>), dim3((uint32_t)ntiles), dim3(SCAN_T), 0, st, d_in, n, cap,
                           d_tmp, d_out, ntiles, ca);
    }
}

void launch_exclusive_scan_u32(const uint32_t *d_in, uint64_t *d_out, uint64_t n, uint32_t cap, uint64_t *d_tmp,
                               hipStream_t st) {
    launch_scan_impl<false>(d_in, d_out, n, cap, d_tmp, CompactArgs{nullptr, nullptr}, st);
}

// ---------------------------------------------------------------------------
// Compaction: per-segment candidate slots -> one sorted entry list, fused into the
// exclusive scan of the per-segment counts (eoff = each segment's first entry).
// ---------------------------------------------------------------------------
void launch_scan_compact(const uint32_t *d_seg_count, const uint32_t *d_seg_cand, uint64_t *d_eoff, uint32_t cap,
                         uint64_t nseg, uint64_t *d_entries, uint64_t *d_tmp, hipStream_t st, const StageIn &si) {
    launch_scan_impl<true>(d_seg_count, d_eoff, nseg, cap, d_tmp, CompactArgs{d_seg_cand, d_entries}, st, si);
}

}  // namespace cg

// grid override of the persistent scan (0 = resident workgroups); returns the resident count
extern "C" uint64_t cg_test_scan_grid(uint64_t v) {
    cg::g_scan_grid = v;
    return cg::scan_resident_wgs();
}

extern "C" uint32_t cg_test_scan_kernel(uint32_t v) {
    const uint32_t old = cg::g_scan_kernel;
    cg::g_scan_kernel = v <= 2 ? v : 0u;
    return old;
}

extern "C" uint32_t cg_test_scan_path(uint32_t v) {
    const uint32_t old = cg::g_scan_path;
    cg::g_scan_path = v <= 3 ? v : 0;
    return old;
}
