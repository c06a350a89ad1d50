// walk.hip -- K2: per-NAR cut resolution (the sequential part of the FastCDC
// iterator [ext], src/chunking.rs:334-336) and descriptor assembly.
//
// For a chunk starting at c the crate's cut_gear tests, with the hash restarted at
// s = c + 2*floor(min/2), positions [s, 2*floor(center/2)) against mask_s and then
// positions up to 2*floor(R/2) against mask_l, and cuts at R if none hits
// (SURVEY.md Appendix A.2).  The walker recomputes the 47 positions [s, s+47) with
// the exact (restarted) hash and takes every later position's verdict from the
// sorted candidate list produced by K1; "dense" segments (more candidates than
// the per-segment slots) are rescanned exactly here.
#include <algorithm>

#include "common.h"

namespace cg {

#define NONE (~0ull)

// Re-read of a value this wave stored earlier in the launch: an agent-scope load
// is served from L2, never from a possibly stale L1 line.
__device__ __forceinline__ uint64_t ld_l2(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t rd_u64(uint64_t v, int lane) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// Chunk geometry of cut_gear [ext] for a chunk starting at c with rem bytes left
// (SURVEY.md Appendix A.2): hash restarts at s; [s, cs) is tested with mask_s,
// [cs, ce) with mask_l; no hit -> cut at c + R.
struct Geo {
    uint64_t R, s, cs, ce;
};
__device__ __forceinline__ Geo geometry(uint64_t c, uint64_t rem, const CdcParams &P) {
    uint64_t R = rem, center = P.avg;
    if (R > P.max)
        R = P.max;
    else if (R < center)
        center = R;
    Geo g;
    g.R = R;
    g.s = c + 2 * (P.min / 2);
    g.cs = c + 2 * (center / 2);
    g.ce = c + 2 * (R / 2);
    return g;
}

// Exact restarted hash over the first 47 tested positions [s, min(s+47, ce)),
// lane-parallel: lane j loads byte s+j and an inclusive shift-add scan
// (A_j = sum_i g_i << (j-i)) gives the crate's hash at s+j.  First hit or NONE.
__device__ __forceinline__ uint64_t warmup_exact(const uint8_t *__restrict__ data, const uint64_t *gear, const Geo &g,
                                                 const CdcParams &P, uint32_t lane) {
    const uint64_t wend = g.s + 47 < g.ce ? g.s + 47 : g.ce;
    if (wend <= g.s) return NONE;
    const uint64_t p = g.s + lane;
    const bool in = p < wend;
    uint64_t a = in ? gear[data[p]] : 0ull;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t t = __shfl_up(a, d, 64);
        if (lane >= d) a += t << d;
    }
    const uint64_t m = p < g.cs ? P.mask_s : P.mask_l;
    const uint64_t hits = __ballot(in && (a & m) == 0);
    return hits ? g.s + (uint64_t)__builtin_ctzll(hits) : NONE;
}

// The same warm-up for one chunk on ONE lane (the speculative walk's verification,
// one lane per chunk), in two halves so a lane can hold several chunks' loads in
// flight at once.  warm_load: the 13 dwords covering [s, s + 52), never reading at
// or past `lim` (one memory round trip; byte loads in the hash would make it 47
// dependent ones).  warm_cut: first cut among the n <= 47 positions from s (the
// first n_s of them under mask_s), or NONE -- branch-free, so the 47 gear lookups
// issue back to back instead of one LDS round trip per byte.
#ifndef CG_VERIFY_U
#define CG_VERIFY_U 4  // chunks per lane per verification pass
#endif
struct WarmWin {
    uint32_t w[13];
    uint64_t s;
    uint32_t n, n_s;
};
__device__ __forceinline__ void warm_load(WarmWin &v, const uint8_t *__restrict__ data, uint64_t s, uint32_t n,
                                          uint32_t n_s, uint64_t lim) {
    v.s = s;
    v.n = n;
    v.n_s = n_s;
    const uint64_t a0 = s & ~3ull;
    const uint32_t *q = reinterpret_cast<const uint32_t *>(data + a0);
#pragma unroll
    for (int i = 0; i < 13; ++i) v.w[i] = n && a0 + 4 * i + 4 <= lim ? q[i] : 0u;
    if (n && a0 + 52 > lim) {  // the NAR's last bytes: finish the partial dword byte by byte
        const uint64_t full = (lim - a0) / 4;
        if (full < 13) {
            uint32_t x = 0;
            for (uint64_t b = a0 + 4 * full; b < lim; ++b) x |= (uint32_t)data[b] << (8 * (uint32_t)(b & 3));
#pragma unroll
            for (uint32_t i = 0; i < 13; ++i)
                if (i == full) v.w[i] = x;  // static indices keep w[] in registers
        }
    }
}
__device__ __forceinline__ uint64_t warm_cut(const WarmWin &v, const uint64_t *gear, const CdcParams &P) {
    const uint32_t sh = (uint32_t)(v.s & 3u);
    uint32_t a[12];  // the window realigned to s
#pragma unroll
    for (int i = 0; i < 12; ++i) a[i] = __builtin_amdgcn_alignbyte(v.w[i + 1], v.w[i], sh);
    uint64_t h = 0, hits = 0;
#pragma unroll
    for (uint32_t i = 0; i < 47; ++i) {
        h = (h << 1) + gear[(a[i >> 2] >> (8 * (i & 3))) & 0xffu];
        const uint64_t m = i < v.n_s ? P.mask_s : P.mask_l;
        hits |= (uint64_t)((h & m) == 0) << i;
    }
    hits &= v.n >= 64 ? ~0ull : (1ull << v.n) - 1;
    return hits ? v.s + (uint64_t)__builtin_ctzll(hits) : NONE;
}

// Windowed (48-byte) hash verdict for positions [lo, hi) of a dense segment,
// 64 positions per pass; first hit or NONE.  Only reached for inputs with more
// candidates than the per-segment slots.
__device__ uint64_t dense_rescan(const uint8_t *__restrict__ data, const uint64_t *gear, uint64_t lo, uint64_t hi,
                                 uint64_t cs, const CdcParams &P, uint32_t lane) {
    for (uint64_t b = lo; b < hi; b += 64) {
        const uint64_t p = b + lane;
        bool hit = false;
        if (p < hi) {
            uint64_t h = 0;
            for (uint64_t q = p - 47; q <= p; ++q) h = (h << 1) + gear[data[q]];
            hit = (h & (p < cs ? P.mask_s : P.mask_l)) == 0;
        }
        const uint64_t bal = __ballot(hit);
        if (bal) return b + (uint64_t)__builtin_ctzll(bal);
    }
    return NONE;
}

// Window of 64 sorted candidate entries held one per lane.
struct EntryWin {
    uint64_t base;  // index of lane 0's entry
    uint64_t e;     // this lane's entry (or ~0 past the end)
};
__device__ __forceinline__ void win_load(EntryWin &w, const uint64_t *__restrict__ entries, uint64_t n_entries,
                                         uint32_t lane) {
    const uint64_t i = w.base + lane;
    w.e = i < n_entries ? entries[i] : ~0ull;
}

// First position in [q0, ce) whose verdict from the candidate list is a cut
// (mask_s below cs, mask_l from cs), rescanning dense segments exactly.
__device__ uint64_t list_search(EntryWin &w, const uint64_t *__restrict__ entries, uint64_t n_entries,
                                const uint8_t *__restrict__ data, const uint64_t *gear, uint64_t q0, uint64_t cs,
                                uint64_t ce, const CdcParams &P, uint32_t lane) {
    for (;;) {
        if (q0 >= ce) return NONE;
        const uint64_t pos = w.e >> 2;
        const uint32_t f = (uint32_t)(w.e & 3u);
        const bool valid = w.e != ~0ull;
        const uint64_t cover_end = f ? pos + 1 : pos + CG_SEG;
        const bool relevant = valid && cover_end > q0;
        const bool hit = relevant && pos < ce && (f ? (f & (pos < cs ? CG_FLAG_S : CG_FLAG_L)) != 0 : true);
        const uint64_t hb = __ballot(hit);
        if (hb) {
            const int L = __builtin_ctzll(hb);
            const uint64_t e = rd_u64(w.e, L);
            const uint64_t epos = e >> 2;
            if (e & 3u) return epos;
            const uint64_t lo = epos > q0 ? epos : q0;
            const uint64_t hi = epos + CG_SEG < ce ? epos + CG_SEG : ce;
            const uint64_t r = dense_rescan(data, gear, lo, hi, cs, P, lane);
            if (r != NONE) return r;
            q0 = hi;  // marker exhausted; continue after it
            continue;
        }
        // no hit in this window: advance only if every entry is below ce
        const uint64_t last = rd_u64(w.e, 63);
        if (last == ~0ull || (last >> 2) >= ce) return NONE;
        w.base += 64;
        win_load(w, entries, n_entries, lane);
    }
}

// Position the entry window at the first entry of the segment holding c (entries are
// sorted by position, segment seg's at [eoff[seg], eoff[seg + 1])): one load.
__device__ __forceinline__ void win_seek(EntryWin &w, const uint64_t *__restrict__ entries, uint64_t n_entries,
                                         const uint64_t *__restrict__ eoff, uint64_t c, uint32_t lane) {
    w.base = eoff[c / CG_SEG];
    win_load(w, entries, n_entries, lane);
}

// Length of the chunk starting at c (NAR end `end`): exact warm-up or candidate list
// only (spec), then the candidate list.
__device__ __forceinline__ uint64_t chunk_len(const uint8_t *__restrict__ data, const uint64_t *gear, EntryWin &w,
                                              const uint64_t *__restrict__ entries, uint64_t n_entries, uint64_t c,
                                              uint64_t end, const CdcParams &P, bool exact, uint32_t lane) {
    const uint64_t rem = end - c;
    if (rem <= P.min) return rem;
    const Geo g = geometry(c, rem, P);
    uint64_t cut = exact ? warmup_exact(data, gear, g, P, lane) : NONE;
    if (cut == NONE) {
        const uint64_t q0 = g.s + 47 < g.ce ? g.s + 47 : g.ce;
        cut = list_search(w, entries, n_entries, data, gear, q0, g.cs, g.ce, P, lane);
    }
    return cut == NONE ? g.R : cut - c;
}

// Speculative piece walks (large NARs).  A NAR of several piece lengths (pb bytes;
// the last piece takes the remainder) is walked piece by piece in parallel: the wave of
// piece k starts at the piece's first byte as if a chunk started there, and records the
// start of every chunk it finds below the piece end plus the first start at or past it
// (`exit`).  Cut sequences are a function of the previous cut alone, so once the NAR's
// true sequence reaches any recorded start it follows that piece's list to its exit:
// k_walk uses the lists as a cache of "the chunks from here", and walks normally only
// until it lands on a cached start (typically one or two chunks into each piece).
struct WalkPieces {
    const uint64_t *first;   // [n_nars + 1] piece range of each NAR (empty: no pieces)
    const uint32_t *nar;     // [np] the NAR of each piece
    const uint64_t *base;    // [np] start of each piece's list in `starts`
    uint32_t *count;         // [np] chunks recorded per piece
    uint64_t *exit;          // [np] first chunk start at or past the piece end
    uint64_t *starts;        // recorded chunk starts (absolute)
    uint64_t pb;             // piece bytes
    uint64_t np;             // pieces in the batch (0: no cache)
};

__global__ __launch_bounds__(64) void k_walk_pieces(const uint8_t *__restrict__ data,
                                                    const uint64_t *__restrict__ gear_g,
                                                    const uint64_t *__restrict__ entries,
                                                    const uint64_t *__restrict__ eoff, uint64_t nseg,
                                                    const uint64_t *__restrict__ nar_off, CdcParams P, WalkPieces wp) {
    __shared__ uint64_t gear[256];
    for (uint32_t i = threadIdx.x; i < 256; i += 64) gear[i] = gear_g[i];
    __syncthreads();
    const uint64_t g = blockIdx.x;
    if (g >= wp.np) return;
    const uint32_t lane = threadIdx.x;
    const uint32_t nar = wp.nar[g];
    const uint64_t c0 = nar_off[nar], end = nar_off[nar + 1];
    const uint64_t k = g - wp.first[nar], npc = wp.first[nar + 1] - wp.first[nar];
    const uint64_t b = c0 + k * wp.pb, e = k + 1 < npc ? b + wp.pb : end;
    const uint64_t n_entries = eoff[nseg];
    uint64_t *out = wp.starts + wp.base[g];
    EntryWin w;
    win_seek(w, entries, n_entries, eoff, b, lane);
    uint64_t c = b;
    uint32_t cnt = 0;
    while (c < e) {
        const uint64_t len = chunk_len(data, gear, w, entries, n_entries, c, end, P, false, lane);
        if (lane == 0) out[cnt] = c;
        ++cnt;
        c += len;
    }
    if (lane == 0) {
        wp.count[g] = cnt;
        wp.exit[g] = c;
    }
}

// K2: one wave per NAR.  spec = 1: walk with the candidate list only, then verify
// every chunk's 47-position warm-up in parallel (one lane per chunk) and re-walk
// from the first chunk whose warm-up holds a cut (rare when mask_s has >= 14
// bits; falls back to exact mode after 4 re-walks).  spec = 0: exact warm-up per
// chunk.  Both produce the crate's cut sequence exactly.  With piece lists (wp.np,
// spec only) the walk takes whole runs of chunks from them (k_walk_pieces); they come
// from the same candidate-list walk, so the verification below covers them too.
#ifdef CG_DIAG
// diagnostics build: per-NAR walk phase clocks {walk, verify, chunks, piece runs, re-walks,
// piece-search, piece-copy, chunk_len} (cg_diag_walk_stats)
unsigned long long *g_walk_diag = nullptr;
#define WALK_DIAG(expr) expr
#else
#define WALK_DIAG(expr)
#endif

__global__ __launch_bounds__(64) void k_walk(const uint8_t *__restrict__ data, const uint64_t *__restrict__ gear_g,
                                             const uint64_t *__restrict__ entries,
                                             const uint64_t *__restrict__ eoff, uint64_t nseg,
                                             const uint64_t *__restrict__ nar_off,
                                             const uint64_t *__restrict__ cap_base, uint64_t n_nars, CdcParams P,
                                             uint64_t *__restrict__ wchunk, uint32_t *__restrict__ nar_nchunks,
                                             int spec, WalkPieces wp, uint32_t *__restrict__ nar_ngroups,
                                             unsigned long long *__restrict__ wdiag) {
    unsigned long long t_walk = 0, t_ver = 0, t_srch = 0, t_copy = 0, t_len = 0, n_runs = 0, t0 = 0, t1 = 0;
    (void)t_walk, (void)t_ver, (void)t_srch, (void)t_copy, (void)t_len, (void)n_runs, (void)t0, (void)t1;
    __shared__ uint64_t gear[256];
    for (uint32_t i = threadIdx.x; i < 256; i += 64) gear[i] = gear_g[i];
    __syncthreads();
    const uint64_t nar = blockIdx.x;
    if (nar >= n_nars) return;
    const uint32_t lane = threadIdx.x;
    const uint64_t n_entries = eoff[nseg];
    const uint64_t c0 = nar_off[nar], end = nar_off[nar + 1];
    uint64_t *out = wchunk + 2 * cap_base[nar];
    const uint64_t pk0 = wp.np ? wp.first[nar] : 0, npc = wp.np ? wp.first[nar + 1] - pk0 : 0;

    EntryWin w;
    win_seek(w, entries, n_entries, eoff, c0, lane);

    uint64_t k = 0, c = c0;
    uint32_t rewalks = 0;
    bool exact = spec == 0;
    for (;;) {
        WALK_DIAG(if (wdiag) t0 = __builtin_amdgcn_s_memtime());
        const uint64_t k_start = k;
        uint64_t cur = ~0ull, ci = 0;  // piece being searched, and the search cursor in its list
        uint64_t wbase = ~0ull, wv = ~0ull;  // the 64 list entries from wbase, one per lane
        bool seek = false;
        while (c < end) {
            if (npc && !exact) {
                const uint64_t kp = (c - c0) / wp.pb < npc ? (c - c0) / wp.pb : npc - 1;
                if (kp != cur) {
                    cur = kp;
                    ci = 0;
                    wbase = ~0ull;
                }
                const uint64_t pg = pk0 + kp;
                const uint64_t *lst = wp.starts + wp.base[pg];
                const uint64_t m = wp.count[pg];
                // c among the piece's recorded starts (sorted) from the cursor on, 64 per
                // wave-load, the loaded window kept while the cursor stays inside it
                uint64_t hit = NONE;
                WALK_DIAG(if (wdiag) t1 = __builtin_amdgcn_s_memtime());
                while (ci < m) {
                    const uint64_t blk = ci & ~63ull;
                    if (blk != wbase) {
                        wbase = blk;
                        wv = blk + lane < m ? lst[blk + lane] : ~0ull;
                    }
                    const bool live = blk + lane >= ci;
                    const uint64_t eq = __ballot(live && wv == c);
                    if (eq) {
                        hit = blk + (uint64_t)__builtin_ctzll(eq);
                        break;
                    }
                    const uint64_t gt = __ballot(live && wv > c);
                    if (gt) {
                        ci = blk + (uint64_t)__builtin_ctzll(gt);
                        break;
                    }
                    ci = blk + 64;
                }
                WALK_DIAG(if (wdiag) { const unsigned long long t = __builtin_amdgcn_s_memtime(); t_srch += t - t1; t1 = t; });
                if (hit != NONE) {  // the rest of the piece's list is the NAR's sequence
                    const uint64_t ex = wp.exit[pg];
                    for (uint64_t t = hit; t < m; t += 64) {
                        const uint64_t i = t + lane;
                        if (i < m) {
                            const uint64_t a = lst[i], nx = i + 1 < m ? lst[i + 1] : ex;
                            out[2 * (k + i - hit)] = a;
                            out[2 * (k + i - hit) + 1] = nx - a;
                        }
                    }
                    k += m - hit;
                    c = ex;
                    WALK_DIAG(if (wdiag) { t_copy += __builtin_amdgcn_s_memtime() - t1; ++n_runs; });
                    seek = true;  // the entry window is behind c now
                    continue;
                }
            }
            if (seek) {
                win_seek(w, entries, n_entries, eoff, c, lane);
                seek = false;
            }
            WALK_DIAG(if (wdiag) t1 = __builtin_amdgcn_s_memtime());
            const uint64_t len = chunk_len(data, gear, w, entries, n_entries, c, end, P, exact, lane);
            WALK_DIAG(if (wdiag) t_len += __builtin_amdgcn_s_memtime() - t1);
            if (lane == 0) {
                out[2 * k] = c;
                out[2 * k + 1] = len;
            }
            ++k;
            c += len;
        }
        WALK_DIAG(if (wdiag) { t1 = __builtin_amdgcn_s_memtime(); t_walk += t1 - t0; });
        if (exact) break;
        // verify warm-ups of chunks [k_start, k): lane i takes chunks b + i + 64u, u < VU,
        // all VU chunks' loads in flight together
        __syncthreads();  // out[] written by other lanes is read below
        uint64_t bad = NONE, bad_cut = 0;
        constexpr uint32_t VU = CG_VERIFY_U;
        for (uint64_t b = k_start; b < k && bad == NONE; b += 64 * VU) {
            uint64_t cj[VU];
#pragma unroll
            for (uint32_t u = 0; u < VU; ++u) {
                const uint64_t j = b + 64 * u + lane;
                cj[u] = j < k ? ld_l2(out + 2 * j) : end;
            }
            WarmWin v[VU];
#pragma unroll
            for (uint32_t u = 0; u < VU; ++u) {
                const uint64_t rem = end - cj[u];
                uint32_t n = 0, n_s = 0;
                uint64_t s = cj[u];
                if (rem > P.min) {
                    const Geo g = geometry(cj[u], rem, P);
                    const uint64_t wend = g.s + 47 < g.ce ? g.s + 47 : g.ce;
                    s = g.s;
                    n = (uint32_t)(wend - g.s);
                    n_s = g.cs > g.s ? (uint32_t)(g.cs - g.s < 47 ? g.cs - g.s : 47) : 0;
                }
                warm_load(v[u], data, s, n, n_s, end);
            }
#pragma unroll
            for (uint32_t u = 0; u < VU; ++u) {
                if (b + 64 * u >= k) break;  // uniform
                const uint64_t my_cut = warm_cut(v[u], gear, P);
                const uint64_t bal = __ballot(my_cut != NONE);
                if (bal) {
                    const int L = __builtin_ctzll(bal);
                    bad = b + 64 * u + (uint64_t)L;
                    bad_cut = rd_u64(my_cut, L);
                    break;
                }
            }
        }
        WALK_DIAG(if (wdiag) t_ver += __builtin_amdgcn_s_memtime() - t1);
        if (bad == NONE) break;
        // chunk `bad` really ends at bad_cut: fix it and re-walk from there
        const uint64_t cb = rd_u64(lane == 0 ? ld_l2(out + 2 * bad) : 0ull, 0);
        if (lane == 0) out[2 * bad + 1] = bad_cut - cb;
        k = bad + 1;
        c = bad_cut;
        win_seek(w, entries, n_entries, eoff, c, lane);  // entries are sorted: restart at c's segment
        if (++rewalks >= 4) exact = true;
        __syncthreads();
    }
    if (lane == 0) nar_nchunks[nar] = (uint32_t)k;
    WALK_DIAG(if (wdiag && lane == 0) {
        unsigned long long *d = wdiag + 8 * nar;
        d[0] = t_walk; d[1] = t_ver; d[2] = k; d[3] = n_runs; d[4] = rewalks; d[5] = t_srch; d[6] = t_copy; d[7] = t_len;
    });
    if (nar_ngroups) {  // BLAKE3 batches: the NAR's 64-leaf groups and leaves, for the fused maps (k_assemble_counts)
        __syncthreads();  // out[] lengths written by lane 0 / other lanes are read below
        uint32_t ng = 0, nl = 0;
        for (uint64_t j = lane; j < k; j += 64) {
            const uint64_t len = ld_l2(out + 2 * j + 1);
            ng += b3_groups_of_len(len);
            nl += b3_leaves_of_len(len);
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            ng += (uint32_t)__shfl_xor((int)ng, d, 64);
            nl += (uint32_t)__shfl_xor((int)nl, d, 64);
        }
        if (lane == 0) {
            nar_ngroups[nar] = ng;
            nar_ngroups[n_nars + 1 + nar] = nl;
        }
    }
}

void launch_walk(const uint8_t *d_data, const uint64_t *d_gear, const uint64_t *d_entries, const uint64_t *d_eoff,
                 uint64_t nseg, const uint64_t *d_nar_off, const uint64_t *d_cap_base, uint64_t n_nars,
                 CdcParams p, uint64_t *d_wchunk, uint32_t *d_nar_nchunks, const WalkPiecesHost &pieces,
                 hipStream_t st, uint32_t *d_nar_ngroups) {
    if (n_nars == 0) return;
    const int spec = walk_is_speculative(p) ? 1 : 0;
    WalkPieces wp{pieces.first, pieces.nar, pieces.base, pieces.count, pieces.exit, pieces.starts, pieces.pb,
                  spec ? pieces.np : 0};
    if (wp.np)
        hipLaunchKernelGGL(k_walk_pieces, dim3((uint32_t)wp.np), dim3(64), 0, st, d_data, d_gear, d_entries, d_eoff,
                           nseg, d_nar_off, p, wp);
    hipLaunchKernelGGL(k_walk, dim3((uint32_t)n_nars), dim3(64), 0, st, d_data, d_gear, d_entries, d_eoff, nseg,
                       d_nar_off, d_cap_base, n_nars, p, d_wchunk, d_nar_nchunks, spec, wp, d_nar_ngroups,
#ifdef CG_DIAG
                       g_walk_diag
#else
                       nullptr
#endif
    );
}

// One wave per NAR: copy the walker's (abs offset, length) list into the caller's
// descriptor array (NAR-relative offsets, src/chunking.rs:362-366) and the
// absolute-offset array the digest kernels read.
__global__ __launch_bounds__(64) void k_assemble(const uint64_t *__restrict__ nar_off,
                                                 const uint64_t *__restrict__ cap_base,
                                                 const uint64_t *__restrict__ wchunk,
                                                 const uint64_t *__restrict__ nar_first, uint64_t n_nars,
                                                 DescRaw *__restrict__ out, uint64_t out_cap,
                                                 uint64_t *__restrict__ chunk_abs) {
    const uint64_t i = blockIdx.x;
    if (i >= n_nars) return;
    const uint64_t first = nar_first[i], cnt = nar_first[i + 1] - first;
    const uint64_t *w = wchunk + 2 * cap_base[i];
    const uint64_t base = nar_off[i];
    for (uint64_t k = threadIdx.x; k < cnt; k += 64) {
        const uint64_t g = first + k;
        if (g >= out_cap) break;
        const uint64_t abs = w[2 * k];
        out[g].offset = abs - base;
        out[g].length = w[2 * k + 1];
        chunk_abs[g] = abs;
    }
}

// k_assemble with the exclusive scan of the per-NAR chunk counts folded in: NAR i's wave
// sums the counts of NARs 0..i-1 itself (at most ASM_FUSED_MAX - 1 of them, L2-resident)
// and writes nar_first[i] (the last NAR also the total, nar_first[n_nars]), so batches of
// up to ASM_FUSED_MAX NARs take one launch instead of the scan's and the assembly's.
#define ASM_FUSED_MAX 8192u
__global__ __launch_bounds__(64) void k_assemble_counts(const uint64_t *__restrict__ nar_off,
                                                        const uint64_t *__restrict__ cap_base,
                                                        const uint64_t *__restrict__ wchunk,
                                                        const uint32_t *__restrict__ nar_nchunks,
                                                        uint64_t *__restrict__ nar_first, uint64_t n_nars,
                                                        DescRaw *__restrict__ out, uint64_t out_cap,
                                                        uint64_t *__restrict__ chunk_abs, B3PlanOut b3,
                                                        uint64_t *__restrict__ host_first) {
    const uint64_t i = blockIdx.x;
    if (i >= n_nars) return;
    const uint32_t lane = threadIdx.x;
    uint64_t pre = 0, pre_g = 0, pre_l = 0;
    for (uint64_t j = lane; j < i; j += 64) {
        pre += nar_nchunks[j];
        if (b3.group_base) pre_g += b3.nar_ngroups[j];
        if (b3.leaf_base) pre_l += b3.nar_ngroups[n_nars + 1 + j];
    }
    pre = wave_sum_u64(pre);
    const uint64_t first = pre, cnt = nar_nchunks[i];
    if (lane == 0) {
        nar_first[i] = first;
        if (i == n_nars - 1) nar_first[n_nars] = first + cnt;
        if (host_first) {  // the caller's copy, straight into mapped host memory (no D2H copy)
            host_first[i] = first;
            if (i == n_nars - 1) host_first[n_nars] = first + cnt;
        }
    }
    const uint64_t *w = wchunk + 2 * cap_base[i];
    const uint64_t base = nar_off[i];
    for (uint64_t k = lane; k < cnt; k += 64) {
        const uint64_t g = first + k;
        if (g >= out_cap) break;
        const uint64_t abs = w[2 * k];
        out[g].offset = abs - base;
        out[g].length = w[2 * k + 1];
        chunk_abs[g] = abs;
    }
    if (!b3.group_base) return;
    // BLAKE3 group map (what k_b3_plan builds from the descriptors): group_base[g] = the
    // 64-leaf groups of chunks 0..g-1 for every chunk index g <= bound, and gmap[q] = g
    // for each group q of chunk g < bound
    pre_g = wave_sum_u64(pre_g);
    uint64_t run = pre_g;
    for (uint64_t kb = 0; kb < cnt; kb += 64) {
        const uint64_t k = kb + lane, g = first + k;
        const uint32_t gc = k < cnt ? b3_groups_of_len(w[2 * k + 1]) : 0u;
        uint32_t inc = gc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= (uint32_t)d) inc += t;
        }
        const uint64_t gb = run + inc - gc;
        if (k < cnt && g <= b3.bound) b3.group_base[g] = gb;
        if (k < cnt && g < b3.bound)
            for (uint32_t q = 0; q < gc; ++q) b3.gmap[gb + q] = (uint32_t)g;
        run += (uint32_t)__shfl((int)inc, 63, 64);
    }
    if (i == n_nars - 1 && lane == 0 && first + cnt <= b3.bound) b3.group_base[first + cnt] = run;
    if (!b3.leaf_base) return;
    // packed leaves: leaf_base[g] for g <= bound, lmap[w] = g for every wave w whose first
    // slot 64 w lies in chunk g's leaves
    uint64_t run_l = wave_sum_u64(pre_l);
    for (uint64_t kb = 0; kb < cnt; kb += 64) {
        const uint64_t k = kb + lane, g = first + k;
        const uint32_t lc = k < cnt ? b3_leaves_of_len(w[2 * k + 1]) : 0u;
        uint32_t inc = lc;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= (uint32_t)d) inc += t;
        }
        const uint64_t lb = run_l + inc - lc;
        if (k < cnt && g <= b3.bound) b3.leaf_base[g] = lb;
        if (k < cnt && g < b3.bound)
            for (uint64_t wv = (lb + 63) / 64; wv * 64 < lb + lc && wv < b3.lmap_cap; ++wv) b3.lmap[wv] = (uint32_t)g;
        run_l += (uint32_t)__shfl((int)inc, 63, 64);
    }
    if (i == n_nars - 1 && lane == 0 && first + cnt <= b3.bound) b3.leaf_base[first + cnt] = run_l;
}

bool launch_assemble(const uint64_t *d_nar_off, const uint64_t *d_cap_base, const uint64_t *d_wchunk,
                     const uint32_t *d_nar_nchunks, uint64_t *d_nar_first, uint64_t n_nars, void *d_out,
                     uint64_t out_cap, uint64_t *d_chunk_abs, uint64_t *d_scan_tmp, hipStream_t st,
                     const B3PlanOut *b3, uint64_t *host_first, bool *wrote_host_first) {
    *wrote_host_first = false;
    // (a forced scan path, cg_test_scan_path, takes the two-kernel form so tests reach it)
    if (n_nars > 0 && n_nars <= ASM_FUSED_MAX && g_scan_path == 0) {
        const B3PlanOut none{};
        hipLaunchKernelGGL(k_assemble_counts, dim3((uint32_t)n_nars), dim3(64), 0, st, d_nar_off, d_cap_base,
                           d_wchunk, d_nar_nchunks, d_nar_first, n_nars, (DescRaw *)d_out, out_cap, d_chunk_abs,
                           b3 ? *b3 : none, host_first);
        *wrote_host_first = host_first != nullptr;
        return b3 != nullptr;
    }
    launch_exclusive_scan_u32(d_nar_nchunks, d_nar_first, n_nars, 0, d_scan_tmp, st);
    if (n_nars == 0) return false;
    hipLaunchKernelGGL(k_assemble, dim3((uint32_t)n_nars), dim3(64), 0, st, d_nar_off, d_cap_base, d_wchunk,
                       d_nar_first, n_nars, (DescRaw *)d_out, out_cap, d_chunk_abs);
    return false;
}

// Host tables (NAR offsets, capacity bases, walk pieces) into HBM: one block per copy,
// dwords read straight from mapped host memory.
__global__ __launch_bounds__(256) void k_stage_in(StageIn c) {
    const uint32_t k = blockIdx.y;
    const uint32_t *src = static_cast<const uint32_t *>(c.src[k]);
    uint32_t *dst = static_cast<uint32_t *>(c.dst[k]);
    const uint64_t n = c.bytes[k] / 4;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
}

void launch_stage_in(const StageIn &c, hipStream_t st) {
    if (!c.n) return;
    const uint64_t mx = std::max<uint64_t>(c.bytes[0], c.n > 1 ? c.bytes[1] : 0) / 4;
    const uint32_t bx = (uint32_t)std::min<uint64_t>((mx + 255) / 256, 256);
    hipLaunchKernelGGL(k_stage_in, dim3(std::max(bx, 1u), (uint32_t)c.n), dim3(256), 0, st, c);
}

// Digest-only entry: spans (offset,length) -> desc/abs arrays + total.
__global__ void k_spans(const uint64_t *__restrict__ off, const uint64_t *__restrict__ len, uint64_t n,
                        uint64_t *__restrict__ abs, DescRaw *__restrict__ desc, uint64_t *__restrict__ total) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g == 0) *total = n;
    if (g >= n) return;
    abs[g] = off[g];
    desc[g].offset = off[g];
    desc[g].length = len[g];
}

void launch_spans_to_desc(const uint64_t *d_off, const uint64_t *d_len, uint64_t n, uint64_t *d_abs, void *d_desc,
                          uint64_t *d_total, hipStream_t st) {
    const uint64_t blocks = n ? (n + 255) / 256 : 1;
    hipLaunchKernelGGL(k_spans, dim3((uint32_t)blocks), dim3(256), 0, st, d_off, d_len, n, d_abs, (DescRaw *)d_desc,
                       d_total);
}

}  // namespace cg
