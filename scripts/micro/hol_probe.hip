// hol_probe.hip -- does a launch whose workgroups cannot all be placed hold back another
// queue's small workgroups? (round 6: the digest pipeline's scans stall ~20-26 ms right after
// each merged SHA-256 launch starts, profiles/r06_v22_*)
// Kernel A on stream A: `a_wgs` workgroups of 128 threads, `a_lds` bytes of dynamic LDS each,
// each spinning `a_ms`.  Then kernel B on stream B (a different hardware queue): 256
// workgroups of 256 threads, `b_lds` bytes of LDS, each spinning 0.2 ms.  Prints how long B
// took from its launch to its end.  Every wave leaves after its spin (bounded by construction).
// usage: hol_probe <a_wgs> <a_lds> <a_ms> <b_lds> <b_prio_high>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

// the resource footprints of the real kernels: k_sha256 (128 threads, 130-136 VGPRs, 70 KiB
// LDS) and k_scan_flat32 (512 threads, 128 VGPRs, 18 / 68 KiB LDS)
__global__ __launch_bounds__(128) void k_spin_sha(unsigned long long ticks, unsigned *out) {
    extern __shared__ unsigned s[];
    asm volatile("" ::: "v135");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned x = threadIdx.x;
    if (threadIdx.x == 0) s[0] = x;
    __syncthreads();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) out[threadIdx.x] = x + s[0];
}
__global__ __launch_bounds__(512) void k_spin_scan(unsigned long long ticks, unsigned *out) {
    extern __shared__ unsigned s[];
    asm volatile("" ::: "v127");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned x = threadIdx.x;
    if (threadIdx.x == 0) s[0] = x;
    __syncthreads();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) out[threadIdx.x] = x + s[0];
}

// variants of the scan's shape: 256 threads at 128 VGPRs, 512 threads at 112 VGPRs
__global__ __launch_bounds__(256) void k_spin_scan256(unsigned long long ticks, unsigned *out) {
    extern __shared__ unsigned s[];
    asm volatile("" ::: "v127");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned x = threadIdx.x;
    if (threadIdx.x == 0) s[0] = x;
    __syncthreads();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) out[threadIdx.x] = x + s[0];
}
__global__ __launch_bounds__(512) void k_spin_scan112(unsigned long long ticks, unsigned *out) {
    extern __shared__ unsigned s[];
    asm volatile("" ::: "v111");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned x = threadIdx.x;
    if (threadIdx.x == 0) s[0] = x;
    __syncthreads();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) out[threadIdx.x] = x + s[0];
}

__global__ void k_spin(unsigned long long ticks, unsigned *out) {
    extern __shared__ unsigned s[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned x = threadIdx.x;
    if (threadIdx.x == 0) s[0] = x;
    __syncthreads();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) out[threadIdx.x] = x + s[0];
}

#define CK(e)                                                                        \
    do {                                                                             \
        hipError_t _e = (e);                                                         \
        if (_e != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #e, hipGetErrorString(_e));                  \
            return 1;                                                                \
        }                                                                            \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 6) return 2;
    const int a_wgs = atoi(argv[1]), a_lds = atoi(argv[2]), b_lds = atoi(argv[4]), hi = atoi(argv[5]);
    const int real = argc > 6 ? atoi(argv[6]) : 0;  // 1: the real kernels' footprints (k_spin_sha / k_spin_scan)
    const double a_ms = atof(argv[3]);
    if (a_wgs < 1 || a_wgs > 4096 || a_lds < 4 || a_lds > 160 * 1024 || b_lds < 4 || b_lds > 96 * 1024 || a_ms > 100)
        return 2;
    unsigned *d = nullptr;
    CK(hipMalloc(&d, 4096));
    int lo = 0, hp = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hp));
    hipStream_t sa, sb;
    CK(hipStreamCreateWithPriority(&sa, hipStreamNonBlocking, hp));
    CK(hipStreamCreateWithPriority(&sb, hipStreamNonBlocking, hi ? hp : lo));
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 4, sa, 1000ull, d);
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 4, sb, 1000ull, d);
    CK(hipDeviceSynchronize());
    for (int r = 0; r < 3; ++r) {
        if (real)
            hipLaunchKernelGGL(k_spin_sha, dim3(a_wgs), dim3(128), a_lds, sa, (unsigned long long)(a_ms * 1e5), d);
        else
            hipLaunchKernelGGL(k_spin, dim3(a_wgs), dim3(128), a_lds, sa, (unsigned long long)(a_ms * 1e5), d);
        // let A's first workgroups land
        const auto w0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count() < 2.0) {
        }
        const auto t0 = std::chrono::steady_clock::now();
        if (real == 2)
            hipLaunchKernelGGL(k_spin_scan256, dim3(2048), dim3(256), b_lds, sb, 10000ull, d);
        else if (real == 3)
            hipLaunchKernelGGL(k_spin_scan112, dim3(1024), dim3(512), b_lds, sb, 10000ull, d);
        else if (real)
            hipLaunchKernelGGL(k_spin_scan, dim3(1024), dim3(512), b_lds, sb, 10000ull, d);
        else
            hipLaunchKernelGGL(k_spin, dim3(256), dim3(256), b_lds, sb, 20000ull, d);
        CK(hipStreamSynchronize(sb));
        const double b = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        CK(hipDeviceSynchronize());
        const double all = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
        printf("{\"real\": %d, \"a_wgs\": %d, \"a_lds\": %d, \"a_ms\": %.1f, \"b_lds\": %d, \"b_high\": %d, \"b_ms\": %.2f, \"all_ms\": %.1f}\n",
               real, a_wgs, a_lds, a_ms, b_lds, hi, b, all);
    }
    return 0;
}
