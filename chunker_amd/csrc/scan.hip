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
#include "common.h"

namespace cg {

// One Gear step + both mask tests for one byte.  Returns the 2-bit flag set.
__device__ __forceinline__ uint32_t gear_flags(uint64_t h, uint64_t mask_s, uint64_t mask_l) {
    return (((h & mask_s) == 0) ? CG_FLAG_S : 0u) | (((h & mask_l) == 0) ? CG_FLAG_L : 0u);
}

// LDS Gear table, replicated 32x in a transposed layout: entry v, copy c lives at
// byte (v*32 + c)*8.  Lane l of a 32-lane ds_read_b64 group reads copy l, i.e. the
// bank pair {2l, 2l+1} whatever byte value it looks up: random lookups are
// conflict-free (MI355X_MICROARCH.md §LDS: ds_read_b64 banks are (a/4) mod 64,
// lanes {0-31} and {32-63} are separate groups).  64 KiB per workgroup.
#define GEAR_COPIES 32u
#define SCAN2_T 512u
#define PIECE 128u

// v_perm_b32 selector producing (byte b of `w`) << 8 | (byte 0 of `lo8`): the LDS
// address of entry w.byte[b] in this lane's copy, in one instruction.
__device__ __forceinline__ uint32_t gear_addr(uint32_t w, uint32_t lo8, int b) {
    return __builtin_amdgcn_perm(w, lo8, 0x0C0C0000u | ((4u + (uint32_t)b) << 8));
}

__device__ __forceinline__ uint64_t lds_gear(const char *base, uint32_t addr) {
    return *reinterpret_cast<const uint64_t *>(base + addr);
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

#define QPIECE 64u

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
__global__ __launch_bounds__(SCAN2_T) void k_scan(const uint8_t *__restrict__ data, uint64_t n,
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
    uint64_t hits = 0;  // PRE: bit r = piece r may hold a candidate (CG_SEG / QPIECE == 64 pieces)
    uint32_t *cand = seg_cand + seg * cap;
    const uint32_t rounds = CG_SEG / QPIECE;  // wave-uniform trip count
    static_assert(CG_SEG / QPIECE == 64, "hits mask holds one bit per piece");
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

#ifdef CG_DIAG
uint32_t g_scan_diag = 0;  // set by cg_diag_scan_mode (diagnostics build only)
#endif

void launch_scan(const uint8_t *d_data, uint64_t n, const uint64_t *d_gear, uint64_t mask_s, uint64_t mask_l,
                 uint32_t cap, uint32_t *d_seg_count, uint32_t *d_seg_cand, uint64_t nseg, hipStream_t st) {
    if (nseg == 0) return;
    const uint64_t blocks = (nseg + SCAN2_T - 1) / SCAN2_T;
#ifdef CG_DIAG
    if (g_scan_diag && __builtin_popcountll(mask_s & mask_l) >= 15) {
        auto k = g_scan_diag == 1   ? k_scan<true, 1>
                 : g_scan_diag == 2 ? k_scan<true, 2>
                 : g_scan_diag == 3 ? k_scan<true, 3>
                 : g_scan_diag == 4 ? k_scan<true, 4>
                 : g_scan_diag == 8 ? k_scan<true, 8>
                                    : k_scan<true, 9>;
        hipLaunchKernelGGL(k, dim3((uint32_t)blocks), dim3(SCAN2_T), 0, st, d_data, n, d_gear, mask_s, mask_l, cap,
                           d_seg_count, d_seg_cand, nseg);
        return;
    }
#endif
    if (__builtin_popcountll(mask_s & mask_l) >= 15)
        hipLaunchKernelGGL(k_scan<true>, dim3((uint32_t)blocks), dim3(SCAN2_T), 0, st, d_data, n, d_gear, mask_s,
                           mask_l, cap, d_seg_count, d_seg_cand, nseg);
    else
        hipLaunchKernelGGL(k_scan<false>, dim3((uint32_t)blocks), dim3(SCAN2_T), 0, st, d_data, n, d_gear, mask_s,
                           mask_l, cap, d_seg_count, d_seg_cand, nseg);
}

// ---------------------------------------------------------------------------
// Exclusive prefix sum u32 -> u64 (three launches: tile sums, top scan, apply).
// ---------------------------------------------------------------------------
#define SCAN_T 256u
#define SCAN_ITEMS 8u
#define SCAN_TILE (SCAN_T * SCAN_ITEMS)

__device__ __forceinline__ uint64_t xform(uint32_t v, uint32_t cap) { return cap ? (v <= cap ? v : 1u) : v; }

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

__global__ __launch_bounds__(SCAN_T) void k_tile_sums(const uint32_t *__restrict__ in, uint64_t n, uint32_t cap,
                                                      uint64_t *__restrict__ tile_sum) {
    __shared__ uint64_t s_wave[SCAN_T / 64];
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

__global__ __launch_bounds__(SCAN_T) void k_scan_apply(const uint32_t *__restrict__ in, uint64_t n, uint32_t cap,
                                                       const uint64_t *__restrict__ tile_sum,
                                                       uint64_t *__restrict__ out, uint64_t ntiles) {
    __shared__ uint64_t s_wave[SCAN_T / 64];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    uint64_t v[SCAN_ITEMS];
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_ITEMS; ++k) {
        v[k] = base + k < n ? xform(in[base + k], cap) : 0;
        s += v[k];
    }
    const uint64_t inc = block_inclusive_scan(s, s_wave);
    uint64_t run = tile_sum[blockIdx.x] + inc - s;
#pragma unroll
    for (uint32_t k = 0; k < SCAN_ITEMS; ++k) {
        if (base + k < n) out[base + k] = run;
        run += v[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = tile_sum[ntiles];
}

size_t exclusive_scan_tmp_elems(uint64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

void launch_exclusive_scan_u32(const uint32_t *d_in, uint64_t *d_out, uint64_t n, uint32_t cap, uint64_t *d_tmp,
                               hipStream_t st) {
    const uint64_t ntiles = n ? (n + SCAN_TILE - 1) / SCAN_TILE : 0;
    if (ntiles == 0) {
        (void)hipMemsetAsync(d_out, 0, sizeof(uint64_t), st);
        return;
    }
    hipLaunchKernelGGL(k_tile_sums, dim3((uint32_t)ntiles), dim3(SCAN_T), 0, st, d_in, n, cap, d_tmp);
    hipLaunchKernelGGL(k_top_scan, dim3(1), dim3(1024), 0, st, d_tmp, ntiles);
    hipLaunchKernelGGL(k_scan_apply, dim3((uint32_t)ntiles), dim3(SCAN_T), 0, st, d_in, n, cap, d_tmp, d_out,
                       ntiles);
}

// ---------------------------------------------------------------------------
// Compaction: per-segment candidate slots -> one sorted entry list.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_compact(const uint32_t *__restrict__ seg_count,
                                                 const uint32_t *__restrict__ seg_cand,
                                                 const uint64_t *__restrict__ eoff, uint32_t cap, uint64_t nseg,
                                                 uint64_t *__restrict__ entries) {
    const uint64_t seg = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (seg >= nseg) return;
    const uint32_t count = seg_count[seg];
    if (count == 0) return;
    const uint64_t base = eoff[seg];
    const uint64_t start = seg * CG_SEG;
    if (count <= cap) {
        for (uint32_t k = 0; k < count; ++k) {
            const uint32_t e = seg_cand[seg * cap + k];
            entries[base + k] = ((start + (e >> 2)) << 2) | (e & 3u);
        }
    } else {
        entries[base] = start << 2;  // dense-segment marker
    }
}

void launch_compact(const uint32_t *d_seg_count, const uint32_t *d_seg_cand, const uint64_t *d_eoff, uint32_t cap,
                    uint64_t nseg, uint64_t *d_entries, hipStream_t st) {
    if (nseg == 0) return;
    hipLaunchKernelGGL(k_compact, dim3((uint32_t)((nseg + 255) / 256)), dim3(256), 0, st, d_seg_count, d_seg_cand,
                       d_eoff, cap, nseg, d_entries);
}

}  // namespace cg
