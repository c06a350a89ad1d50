// microbench.hip -- diagnostic only (not on the product path): cycles per SHA-256
// round for the round code the consumer wave of k_sha256 runs, measured with
// s_memtime on the device.  Exposed as cg_diag_sha_rounds() for DESIGN.md's latency
// model.
#include "common.h"

namespace cg {

static constexpr uint32_t MK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t mrot(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
#define MX3(a, b, c) __builtin_amdgcn_bitop3_b32(a, b, c, 0x96)
#define MS0(a) MX3(mrot(a, 2), mrot(a, 13), mrot(a, 22))
#define MS1(e) MX3(mrot(e, 6), mrot(e, 11), mrot(e, 25))
#define MRND(a, b, c, d, e, f, g, h, i, wv)                                                                  \
    {                                                                                                        \
        const uint32_t t1 = (h + (wv) + MK[i]) + MS1(e) + __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);      \
        d += t1;                                                                                             \
        h = t1 + MS0(a) + __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);                                       \
    }

__global__ void k_diag_sha_rounds(uint32_t iters, uint32_t *out, unsigned long long *cycles) {
    const uint32_t lane = threadIdx.x;
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = lane * 16 + i;
    uint32_t a = lane, b = 1, c = 2, d = 3, e = 4, f = 5, g = 6, h = 7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 64; i += 8) {
            MRND(a, b, c, d, e, f, g, h, i + 0, w[(i + 0) & 15]);
            MRND(h, a, b, c, d, e, f, g, i + 1, w[(i + 1) & 15]);
            MRND(g, h, a, b, c, d, e, f, i + 2, w[(i + 2) & 15]);
            MRND(f, g, h, a, b, c, d, e, i + 3, w[(i + 3) & 15]);
            MRND(e, f, g, h, a, b, c, d, i + 4, w[(i + 4) & 15]);
            MRND(d, e, f, g, h, a, b, c, i + 5, w[(i + 5) & 15]);
            MRND(c, d, e, f, g, h, a, b, i + 6, w[(i + 6) & 15]);
            MRND(b, c, d, e, f, g, h, a, i + 7, w[(i + 7) & 15]);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + lane] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
    if ((lane & 63) == 0) {
        const uint32_t wv = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
        cycles[2 * wv] = t1 - t0;      // shader clocks
        cycles[2 * wv + 1] = r1 - r0;  // 100 MHz ticks
    }
}

// Variant: W read from LDS every block (16 ds_read_b128 + a counter read/write),
// as the consumer wave of k_sha256 does.
__global__ void k_diag_sha_rounds_lds(uint32_t iters, uint32_t *out, unsigned long long *cycles) {
    __shared__ __attribute__((aligned(16))) uint32_t sW[64 * 68];
    __shared__ uint32_t s_ctr;
    const uint32_t lane = threadIdx.x;
    for (int i = 0; i < 68; ++i) sW[lane * 68 + i] = lane * 16 + i;
    if (lane == 0) s_ctr = 0;
    __syncthreads();
    uint32_t a = lane, b = 1, c = 2, d = 3, e = 4, f = 5, g = 6, h = 7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t it = 0; it < iters; ++it) {
        while (__hip_atomic_load(&s_ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < it) __builtin_amdgcn_s_sleep(1);
        uint4 wv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) wv[i] = *reinterpret_cast<const uint4 *>(&sW[lane * 68 + 4 * i]);
#pragma unroll
        for (int i = 0; i < 64; i += 8) {
            const uint4 wa = wv[i / 4], wb = wv[i / 4 + 1];
            MRND(a, b, c, d, e, f, g, h, i + 0, wa.x);
            MRND(h, a, b, c, d, e, f, g, i + 1, wa.y);
            MRND(g, h, a, b, c, d, e, f, i + 2, wa.z);
            MRND(f, g, h, a, b, c, d, e, i + 3, wa.w);
            MRND(e, f, g, h, a, b, c, d, i + 4, wb.x);
            MRND(d, e, f, g, h, a, b, c, i + 5, wb.y);
            MRND(c, d, e, f, g, h, a, b, i + 6, wb.z);
            MRND(b, c, d, e, f, g, h, a, i + 7, wb.w);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        if (lane == 0) __hip_atomic_store(&s_ctr, it + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + lane] = a ^ b ^ c ^ d ^ e ^ f ^ g ^ h;
    if (lane == 0) {
        cycles[2 * blockIdx.x] = t1 - t0;
        cycles[2 * blockIdx.x + 1] = r1 - r0;
    }
}

}  // namespace cg

extern "C" int cg_diag_sha_rounds_lds(uint32_t iters, uint32_t blocks, unsigned long long *h_cycles) {
    uint32_t *d_out = nullptr;
    unsigned long long *d_cyc = nullptr;
    if (hipMalloc(&d_out, (size_t)blocks * 64 * 4) != hipSuccess) return 2;
    if (hipMalloc(&d_cyc, blocks * 16) != hipSuccess) return 2;
    hipLaunchKernelGGL(cg::k_diag_sha_rounds_lds, dim3(blocks), dim3(64), 0, 0, iters, d_out, d_cyc);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(h_cycles, d_cyc, blocks * 16, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    return e == hipSuccess ? 0 : 2;
}

// cycles[2k], cycles[2k+1] = shader clocks, 100 MHz ticks of wave k; blocks x threads_per_block launched (threads multiple of 64)
extern "C" int cg_diag_sha_rounds(uint32_t iters, uint32_t blocks, uint32_t threads, unsigned long long *h_cycles) {
    uint32_t *d_out = nullptr;
    unsigned long long *d_cyc = nullptr;
    const uint32_t waves = blocks * (threads / 64);
    if (hipMalloc(&d_out, (size_t)blocks * threads * 4) != hipSuccess) return 2;
    if (hipMalloc(&d_cyc, waves * 16) != hipSuccess) return 2;
    hipLaunchKernelGGL(cg::k_diag_sha_rounds, dim3(blocks), dim3(threads), 0, 0, iters, d_out, d_cyc);
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(h_cycles, d_cyc, waves * 16, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    return e == hipSuccess ? 0 : 2;
}

namespace cg {
extern unsigned long long *g_sha_diag;
extern uint32_t g_sha_mode;
}
// 0 = product; 1 = producer idle (consumer rounds on stale LDS schedules); 2 = consumer
// also skips its LDS schedule reads.  Digests are garbage in modes 1 and 2.
extern "C" void cg_diag_sha_mode(uint32_t mode) { cg::g_sha_mode = mode; }
namespace cg {
extern uint32_t g_scan_diag;
}
extern "C" void cg_diag_scan_mode(uint32_t mode) { cg::g_scan_diag = mode; }
namespace cg {
extern uint32_t g_scan_variant;
}
// 0 = product; 1 = round-1 quad-transpose kernel; 2 = LDS-staged; 3 = page per wave; 4 = k_scan; 5 = k_scan_flat by mode
extern "C" void cg_diag_scan_variant(uint32_t v) { cg::g_scan_variant = v; }
namespace cg {
extern uint32_t g_scan_spw_max;
}
// k_scan_flat's segments-per-wave cap (a multiple of 4; 0 = the product default)
extern "C" void cg_diag_scan_spw_max(uint32_t v) { cg::g_scan_spw_max = v; }
namespace cg {
extern uint32_t g_b3_diag;
}
// 1 = BLAKE3 leaves compress register words without loading them (digests garbage)
extern "C" void cg_diag_b3_mode(uint32_t mode) { cg::g_b3_diag = mode; }
// Enable (n_wg > 0) / read back / disable (n_wg == 0) per-workgroup SHA producer and
// consumer timing: out[8*wg + {0,1,2,3}] = producer spin, producer total, consumer
// spin, consumer total (shader clocks); + {4,5} consumer start/end (s_memrealtime,
// 100 MHz), {6,7} consumer/producer wave location (HW_ID | XCC_ID << 32).  Diagnostics only.
namespace cg {
extern unsigned long long *g_walk_diag;
}
// Per-NAR k_walk phase clocks (8 u64 per NAR, see walk.hip): n = 0 disarms, out = NULL
// arms a zeroed buffer for n NARs, else copies it out after a device sync.
extern "C" int cg_diag_walk_stats(uint32_t n, unsigned long long *out) {
    static unsigned long long *buf = nullptr;
    static uint32_t cap = 0;
    if (n == 0) {
        cg::g_walk_diag = nullptr;
        return 0;
    }
    if (out == nullptr) {
        if (n > cap) {
            if (buf) (void)hipFree(buf);
            if (hipMalloc(&buf, (size_t)n * 64) != hipSuccess) return 2;
            cap = n;
        }
        (void)hipMemset(buf, 0, (size_t)n * 64);
        cg::g_walk_diag = buf;
        return 0;
    }
    (void)hipDeviceSynchronize();
    return hipMemcpy(out, buf, (size_t)n * 64, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 2;
}

extern "C" int cg_diag_sha_stats(uint32_t n_wg, unsigned long long *out) {
    static unsigned long long *buf = nullptr;
    static uint32_t cap = 0;
    if (n_wg == 0) {
        cg::g_sha_diag = nullptr;
        return 0;
    }
    if (out == nullptr) {  // arm
        if (n_wg > cap) {
            if (buf) (void)hipFree(buf);
            if (hipMalloc(&buf, (size_t)n_wg * 64) != hipSuccess) return 2;
            cap = n_wg;
        }
        (void)hipMemset(buf, 0, (size_t)n_wg * 64);
        cg::g_sha_diag = buf;
        return 0;
    }
    (void)hipDeviceSynchronize();
    return hipMemcpy(out, buf, (size_t)n_wg * 64, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 2;
}

// ---------------------------------------------------------------------------
// HBM read-pattern microbenchmark (diagnostics only): 512 x 512-thread workgroups,
// each wave owns a contiguous 256 KiB region read in 64 rounds of 4 KiB; in a round
// the wave reads 4096/L runs of L contiguous bytes from 4096/L different 4 KiB
// segments (L = 64 is the scan's quad-cooperative pattern, L = 4096 fully
// contiguous).  Two rounds are kept in flight.
// ---------------------------------------------------------------------------
namespace cg {
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int DEPTH, bool NT>
__global__ __launch_bounds__(512) void k_diag_read(const uint8_t *__restrict__ data, uint32_t run_log2,
                                                   uint32_t *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * 8 + (threadIdx.x >> 6);
    const uint8_t *region = data + wave * (256u << 10);
    const uint32_t L = 1u << run_log2, k = 4096u >> run_log2, groups = 64u / k;
    auto addr = [&](uint32_t r, uint32_t i) {
        r = r < 64 ? r : 63;
        const uint32_t g = r % groups, off = (r / groups) * L;
        const uint32_t b = i * 1024u + lane * 16u, run = b >> run_log2, within = b & (L - 1u);
        return reinterpret_cast<const u32x4 *>(region + (uint64_t)(g * k + run) * 4096u + off + within);
    };
    auto ld = [&](const u32x4 *p) { return NT ? __builtin_nontemporal_load(p) : *p; };
    u32x4 buf[DEPTH + 1][4];
    uint32_t acc = 0;
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
        for (int i = 0; i < 4; ++i) buf[d][i] = ld(addr(d, i));
#pragma unroll 1
    for (uint32_t r = 0; r < 64; r += DEPTH + 1) {
#pragma unroll
        for (int u = 0; u < DEPTH + 1; ++u) {
#pragma unroll
            for (int i = 0; i < 4; ++i) buf[(u + DEPTH) % (DEPTH + 1)][i] = ld(addr(r + u + DEPTH, i));
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc ^= buf[u][i].x ^ buf[u][i].y ^ buf[u][i].z ^ buf[u][i].w;
        }
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}
}  // namespace cg

extern "C" float cg_diag_read_pattern(const uint8_t *d_data, uint32_t run_log2, uint32_t *d_out) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    // run_log2 bits 0-7: run length; bit 8: nt loads; bits 12-15: in-flight depth (2 or 4)
    const bool nt = (run_log2 >> 8) & 1u;
    const uint32_t depth = (run_log2 >> 12) & 15u;
    auto k = depth == 4 ? (nt ? cg::k_diag_read<4, true> : cg::k_diag_read<4, false>)
                        : (nt ? cg::k_diag_read<2, true> : cg::k_diag_read<2, false>);
    run_log2 &= 0xffu;
    hipLaunchKernelGGL(k, dim3(512), dim3(512), 0, 0, d_data, run_log2, d_out);
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(k, dim3(512), dim3(512), 0, 0, d_data, run_log2, d_out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return ms;
}

// ---------------------------------------------------------------------------
// Instruction issue-cost microbenchmark (diagnostics only): each wave runs `iters`
// x 16 instructions of one kind over 8 independent register chains (inline asm, so
// the compiler cannot rewrite them); cycles per instruction per wave via s_memtime.
// kind: 0 v_add_u32, 1 v_lshl_add_u64, 2 v_perm_b32, 3 v_add_co_u32+v_addc_co_u32
// pair (counted as 2), 4 v_alignbit_b32, 5 v_bitop3_b32, 6 v_lshlrev_b64,
// 7 v_mov_b32_dpp quad_perm, 8 v_add3_u32, 9 v_cndmask_b32, 10 dependent v_lshl_add_u64
// chain (one chain), 11 dependent v_add_u32 chain (one chain), 12 v_xor_b32_dpp quad_perm,
// 13 v_add_u32_dpp row_shl:4, 14 v_mov_b32_dpp row_shl:4, 15 plain v_mov_b32.
// ---------------------------------------------------------------------------
namespace cg {
template <int KIND>
__device__ __forceinline__ void op16(uint32_t (&r)[16], uint64_t (&q)[8]) {
#pragma unroll
    for (int i = 0; i < 32; ++i) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if constexpr (KIND == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 1) asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(q[c]));
            if constexpr (KIND == 2) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(r[c + 8]), "s"(0x0c0c0001u));
            if constexpr (KIND == 3) {
                if (c & 1) continue;
                asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, %2, %3, vcc"
                             : "+v"(r[c]), "+v"(r[c + 1]) : "v"(r[c + 8]), "v"(r[c + 9]) : "vcc");
            }
            if constexpr (KIND == 4) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[c]));
            if constexpr (KIND == 5) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[c]) : "v"(r[c + 8]), "v"(r[(c + 9) & 15]));
            if constexpr (KIND == 6) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(q[c]));
            if constexpr (KIND == 7) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 8) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(r[c + 8]), "v"(r[(c + 9) & 15]));
            if constexpr (KIND == 9) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 10) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(q[0]) : "v"(q[1 + (c & 1)]));
            if constexpr (KIND == 11) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[0]) : "v"(r[c + 8]));
            if constexpr (KIND == 12)
                asm volatile("v_xor_b32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 13)
                asm volatile("v_add_u32_dpp %0, %1, %0 row_shl:4 row_mask:0xf bank_mask:0xf" : "+v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 14) asm volatile("v_mov_b32_dpp %0, %1 row_shl:4 row_mask:0xf bank_mask:0xf" : "=v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 15) asm volatile("v_mov_b32 %0, %1" : "=v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 16)
                asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 17) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(r[c]) : "v"(r[c + 8]), "v"(r[(c + 9) & 15]));
            if constexpr (KIND == 18) asm volatile("v_and_b32 %0, %0, %1" : "+v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 19) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(r[c]));
            if constexpr (KIND == 20) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 21) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(r[c + 8]), "v"(r[(c + 9) & 15]));
            if constexpr (KIND == 22) asm volatile("v_min_u32 %0, %0, %1" : "+v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 23) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(r[c]));
            if constexpr (KIND == 24) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(r[c]) : "v"(r[c + 8]), "v"(r[(c + 9) & 15]));
            if constexpr (KIND == 25) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(r[c]) : "v"(r[c + 8]) : "vcc");
            if constexpr (KIND == 26) asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(r[c]) : "v"(r[c + 8]));
            if constexpr (KIND == 27) asm volatile("v_cmp_eq_u32_e64 s[40:41], %0, %1" :: "v"(r[c]), "v"(r[c + 8]) : "s40", "s41");
        }
    }
}

template <int KIND>
__global__ void k_diag_ops(uint32_t iters, uint32_t *out, unsigned long long *cycles) {
    uint32_t r[16];
    uint64_t q[8];
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = threadIdx.x * 16 + i;
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = threadIdx.x * 8ull + i;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t it = 0; it < iters; ++it) op16<KIND>(r, q);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) x ^= r[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) cycles[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}
}  // namespace cg

// cycles per wave for `iters` x 16 instructions of `kind`; one workgroup of `threads`
extern "C" int cg_diag_ops(int kind, uint32_t iters, uint32_t threads, unsigned long long *h_cycles) {
    const uint32_t waves = threads / 64;
    uint32_t *d_out = nullptr;
    unsigned long long *d_c = nullptr;
    if (hipMalloc(&d_out, threads * 4) != hipSuccess) return 2;
    if (hipMalloc(&d_c, waves * 8) != hipSuccess) return 2;
    void (*ks[28])(uint32_t, uint32_t *, unsigned long long *) = {
        cg::k_diag_ops<0>,  cg::k_diag_ops<1>,  cg::k_diag_ops<2>,  cg::k_diag_ops<3>, cg::k_diag_ops<4>,  cg::k_diag_ops<5>,
        cg::k_diag_ops<6>,  cg::k_diag_ops<7>,  cg::k_diag_ops<8>,  cg::k_diag_ops<9>, cg::k_diag_ops<10>, cg::k_diag_ops<11>,
        cg::k_diag_ops<12>, cg::k_diag_ops<13>, cg::k_diag_ops<14>, cg::k_diag_ops<15>,
        cg::k_diag_ops<16>, cg::k_diag_ops<17>, cg::k_diag_ops<18>, cg::k_diag_ops<19>, cg::k_diag_ops<20>,
        cg::k_diag_ops<21>, cg::k_diag_ops<22>, cg::k_diag_ops<23>, cg::k_diag_ops<24>, cg::k_diag_ops<25>,
        cg::k_diag_ops<26>, cg::k_diag_ops<27>};
    if (kind < 0 || kind > 27) return 1;
    hipLaunchKernelGGL(ks[kind], dim3(1), dim3(threads), 0, 0, iters, d_out, d_c);
    hipLaunchKernelGGL(ks[kind], dim3(1), dim3(threads), 0, 0, iters, d_out, d_c);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h_cycles, d_c, waves * 8, hipMemcpyDeviceToHost);
    (void)hipFree(d_out);
    (void)hipFree(d_c);
    return 0;
}
