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
#include "common.h"

namespace cg {

__device__ __forceinline__ uint64_t lower_bound_u64(const uint64_t *__restrict__ a, uint64_t n, uint64_t key) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (a[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(64) void k_walk(const uint8_t *__restrict__ data, const uint64_t *__restrict__ gear_g,
                                             const uint64_t *__restrict__ entries,
                                             const uint64_t *__restrict__ eoff, uint64_t nseg,
                                             const uint64_t *__restrict__ nar_off,
                                             const uint64_t *__restrict__ cap_base, uint64_t n_nars, CdcParams P,
                                             uint64_t *__restrict__ wchunk, uint32_t *__restrict__ nar_nchunks) {
    __shared__ uint64_t gear[256];
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) gear[i] = gear_g[i];
    __syncthreads();

    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_nars) return;
    const uint64_t n_entries = eoff[nseg];
    uint64_t c = nar_off[i];
    const uint64_t end = nar_off[i + 1];
    uint64_t *out = wchunk + 2 * cap_base[i];
    uint32_t k = 0;
    uint64_t ptr = lower_bound_u64(entries, n_entries, ((c / CG_SEG) * CG_SEG) << 2);
    const uint64_t s_off = 2 * (P.min / 2);

    while (c < end) {
        const uint64_t rem = end - c;
        uint64_t len;
        if (rem <= P.min) {
            len = rem;
        } else {
            uint64_t R = rem, center = P.avg;
            if (R > P.max)
                R = P.max;
            else if (R < center)
                center = R;
            const uint64_t s = c + s_off, cs = c + 2 * (center / 2), ce = c + 2 * (R / 2);
            bool found = false;
            uint64_t cut = 0;
            // (1) exact restarted hash over the first 47 tested positions
            const uint64_t wend = s + 47 < ce ? s + 47 : ce;
            uint64_t h = 0;
            for (uint64_t p = s; p < wend; ++p) {
                h = (h << 1) + gear[data[p]];
                const uint64_t m = p < cs ? P.mask_s : P.mask_l;
                if ((h & m) == 0) {
                    cut = p;
                    found = true;
                    break;
                }
            }
            // (2) later positions from the candidate list (windowed hash == chunk hash there)
            if (!found) {
                const uint64_t q0 = wend;
                while (ptr < n_entries) {  // drop entries wholly below q0 (monotone across chunks)
                    const uint64_t e = entries[ptr];
                    const uint64_t hi = (e & 3u) ? (e >> 2) + 1 : (e >> 2) + CG_SEG;
                    if (hi <= q0)
                        ++ptr;
                    else
                        break;
                }
                for (uint64_t sp = ptr; sp < n_entries; ++sp) {
                    const uint64_t e = entries[sp];
                    const uint64_t pos = e >> 2;
                    const uint32_t f = (uint32_t)(e & 3u);
                    if (pos >= ce) break;
                    if (f) {
                        if (f & (pos < cs ? CG_FLAG_S : CG_FLAG_L)) {
                            cut = pos;
                            found = true;
                            break;
                        }
                    } else {  // dense segment: exact windowed rescan of [max(pos,q0), min(pos+SEG,ce))
                        const uint64_t lo = pos > q0 ? pos : q0;
                        const uint64_t hi = pos + CG_SEG < ce ? pos + CG_SEG : ce;
                        if (lo < hi) {
                            uint64_t hh = 0;
                            for (uint64_t p = lo - CG_HALO; p < lo; ++p) hh = (hh << 1) + gear[data[p]];
                            for (uint64_t p = lo; p < hi; ++p) {
                                hh = (hh << 1) + gear[data[p]];
                                if ((hh & (p < cs ? P.mask_s : P.mask_l)) == 0) {
                                    cut = p;
                                    found = true;
                                    break;
                                }
                            }
                            if (found) break;
                        }
                    }
                }
            }
            len = found ? cut - c : R;
        }
        out[2 * k] = c;
        out[2 * k + 1] = len;
        ++k;
        c += len;
    }
    nar_nchunks[i] = k;
}

void launch_walk(const uint8_t *d_data, const uint64_t *d_gear, const uint64_t *d_entries, const uint64_t *d_eoff,
                 uint64_t nseg, const uint64_t *d_nar_off, const uint64_t *d_cap_base, uint64_t n_nars,
                 CdcParams p, uint64_t *d_wchunk, uint32_t *d_nar_nchunks, hipStream_t st) {
    if (n_nars == 0) return;
    hipLaunchKernelGGL(k_walk, dim3((uint32_t)((n_nars + 63) / 64)), dim3(64), 0, st, d_data, d_gear, d_entries,
                       d_eoff, nseg, d_nar_off, d_cap_base, n_nars, p, d_wchunk, d_nar_nchunks);
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

void launch_assemble(const uint64_t *d_nar_off, const uint64_t *d_cap_base, const uint64_t *d_wchunk,
                     const uint64_t *d_nar_first, uint64_t n_nars, void *d_out, uint64_t out_cap,
                     uint64_t *d_chunk_abs, hipStream_t st) {
    if (n_nars == 0) return;
    hipLaunchKernelGGL(k_assemble, dim3((uint32_t)n_nars), dim3(64), 0, st, d_nar_off, d_cap_base, d_wchunk,
                       d_nar_first, n_nars, (DescRaw *)d_out, out_cap, d_chunk_abs);
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
