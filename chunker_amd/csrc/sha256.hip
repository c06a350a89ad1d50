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

// One round: 14 VALU (4 Sigma1, 1 Ch, 4 Sigma0, 1 Maj, 4 adds); renaming by macro
// argument rotation, so no register moves.
#define SHA_RND(a, b, c, d, e, f, g, h, i)                          \
    {                                                               \
        const uint32_t t1 = add3(add3(h, w[(i) & 15], SHA_K[i]), SHA_S1(e), ch(e, f, g)); \
        d += t1;                                                    \
        h = add3(t1, SHA_S0(a), maj(a, b, c));                      \
    }

__device__ __forceinline__ void sha256_compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; i += 8) {
        if (i >= 16) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int t = i + j;
                w[t & 15] = add3(w[t & 15], SHA_s0(w[(t - 15) & 15]), w[(t - 7) & 15]) + SHA_s1(w[(t - 2) & 15]);
            }
        }
        SHA_RND(a, b, c, d, e, f, g, h, i + 0);
        SHA_RND(h, a, b, c, d, e, f, g, i + 1);
        SHA_RND(g, h, a, b, c, d, e, f, i + 2);
        SHA_RND(f, g, h, a, b, c, d, e, i + 3);
        SHA_RND(e, f, g, h, a, b, c, d, i + 4);
        SHA_RND(d, e, f, g, h, a, b, c, i + 5);
        SHA_RND(c, d, e, f, g, h, a, b, i + 6);
        SHA_RND(b, c, d, e, f, g, h, a, i + 7);
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

__global__ __launch_bounds__(64) void k_sha256(const uint8_t *__restrict__ data, const uint64_t *__restrict__ abs,
                                               const DescRaw *__restrict__ desc, const uint64_t *__restrict__ total_p,
                                               uint64_t max_chunks, uint8_t *__restrict__ hash_base,
                                               size_t stride) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t total = *total_p;
    if (total > max_chunks) total = max_chunks;
    if (g >= total) return;
    const uint64_t len = desc[g].length;
    const uint8_t *p = data + abs[g];
    const uint32_t shift = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t *base = reinterpret_cast<const uint32_t *>(p - shift);
    // v_perm selector: big-endian word from bytes shift..shift+3 of {hi:lo}
    const uint32_t sel = (shift << 24) | ((shift + 1) << 16) | ((shift + 2) << 8) | (shift + 3);

    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    const uint64_t nb = len >> 6;
    // software pipeline: block k+1's 17 dwords are in flight while block k compresses
    uint32_t nx[17];
    if (nb) {
#pragma unroll
        for (int i = 0; i < 16; ++i) nx[i] = base[i];
        nx[16] = shift ? base[16] : 0u;
    }
    for (uint64_t blk = 0; blk < nb; ++blk) {
        uint32_t w[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) w[i] = __builtin_amdgcn_perm(nx[i + 1], nx[i], sel);
        if (blk + 1 < nb) {
            const uint32_t *q = base + 16 * (blk + 1);
#pragma unroll
            for (int i = 0; i < 16; ++i) nx[i] = q[i];
            nx[16] = shift ? q[16] : 0u;
        }
        sha256_compress(st, w);
    }
    // final block(s): tail bytes, 0x80, zeros, 64-bit big-endian bit length
    const uint32_t rem = (uint32_t)(len & 63u);
    const uint32_t *q = base + 16 * nb;
    const uint8_t *endp = p + len;
    uint32_t dw[17], w[16];
#pragma unroll
    for (int i = 0; i < 17; ++i) dw[i] = (reinterpret_cast<const uint8_t *>(q + i) < endp) ? q[i] : 0u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t v = __builtin_amdgcn_perm(dw[i + 1], dw[i], sel);
        const int r = (int)rem - 4 * i;  // bytes of this word that are message
        uint32_t o;
        if (r >= 4)
            o = v;
        else if (r < 0)
            o = 0u;
        else
            o = (r ? (v & (0xffffffffu << (32 - 8 * r))) : 0u) | (0x80u << (24 - 8 * r));
        w[i] = o;
    }
    const uint64_t bits = len << 3;
    if (rem < 56) {
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        sha256_compress(st, w);
    } else {
        sha256_compress(st, w);
#pragma unroll
        for (int i = 0; i < 14; ++i) w[i] = 0u;
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        sha256_compress(st, w);
    }
    uint4 *o = reinterpret_cast<uint4 *>(hash_base + g * stride);
    o[0] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                      __builtin_bswap32(st[3]));
    o[1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                      __builtin_bswap32(st[7]));
}

void launch_sha256(const uint8_t *d_data, const uint64_t *d_abs, const void *d_desc, const uint64_t *d_total,
                   uint64_t max_chunks, uint8_t *d_hash_base, size_t hash_stride, hipStream_t st) {
    if (max_chunks == 0) return;
    hipLaunchKernelGGL(k_sha256, dim3((uint32_t)((max_chunks + 63) / 64)), dim3(64), 0, st, d_data, d_abs,
                       (const DescRaw *)d_desc, d_total, max_chunks, d_hash_base, hash_stride);
}

}  // namespace cg
