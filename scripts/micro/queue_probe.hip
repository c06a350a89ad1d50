// queue_probe.hip -- which HIP streams get a hardware queue of their own (round 6).
//
// HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues and streams that share a queue
// run their kernels one after another.  The digest pipeline (pipeline.hip) needs its
// boundary stream and its digest lanes on distinct queues whatever other streams the
// process holds.  This probe first creates `fillers` ordinary streams (so the ordinary
// pool is exhausted and shared), then `n` test streams of one kind, launches one
// time-bounded spin kernel (one workgroup, `ms` milliseconds of s_memrealtime) on each,
// and reports the wall time: ~ms = the test streams ran side by side, ~n x ms = they
// shared a queue.
// kinds: 0 ordinary, 1 high priority, 2 low priority, 3 full CU mask.
// usage: queue_probe <kind> <n> <fillers> <ms> [busy]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_spin(unsigned long long ticks, unsigned *out) {
    // s_memrealtime runs at 100 MHz; every wave leaves after `ticks` (bounded by construction)
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned x = threadIdx.x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x = x * 1664525u + 1013904223u;
    if (x == 0x12345678u) out[threadIdx.x] = x;
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
    if (argc < 5) {
        fprintf(stderr, "usage: %s kind n fillers ms\n", argv[0]);
        return 2;
    }
    const int kind = atoi(argv[1]), n = atoi(argv[2]), fillers = atoi(argv[3]);
    const double ms = atof(argv[4]);
    if (n < 1 || n > 16 || fillers < 0 || fillers > 64 || ms <= 0 || ms > 200) return 2;
    unsigned *d = nullptr;
    CK(hipMalloc(&d, 4096));
    std::vector<hipStream_t> fill(fillers), test(n);
    for (auto &s : fill) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    for (auto &s : test) {
        if (kind == 0) {
            CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        } else if (kind == 1) {
            CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi));
        } else if (kind == 2) {
            CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, lo));
        } else {
            hipDeviceProp_t p;
            CK(hipGetDeviceProperties(&p, 0));
            std::vector<uint32_t> mask((p.multiProcessorCount + 31) / 32, 0xffffffffu);
            CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
        }
    }
    // one kernel on each filler (they must be live queues, not idle stream objects)
    for (auto &s : fill) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 1000ull, d);
    CK(hipDeviceSynchronize());
    const unsigned long long ticks = (unsigned long long)(ms * 1e5);
    // busy = 1: every filler runs a spin of the same length at the same time, so a test
    // stream sharing a hardware queue with a filler finishes a spin later
    const int busy = argc > 5 ? atoi(argv[5]) : 0;
    for (int r = 0; r < 3; ++r) {
        if (busy)
            for (auto &s : fill) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, ticks, d);
        const auto t0 = std::chrono::steady_clock::now();
        for (auto &s : test) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, ticks, d);
        for (auto &s : test) CK(hipStreamSynchronize(s));
        const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        CK(hipDeviceSynchronize());
        const double all = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        printf("{\"kind\": %d, \"n\": %d, \"fillers\": %d, \"busy\": %d, \"spin_ms\": %.1f, \"test_ms\": %.2f, "
               "\"ratio\": %.2f, \"all_ms\": %.2f, \"prio_range\": [%d, %d]}\n",
               kind, n, fillers, busy, ms, wall, wall / ms, all, lo, hi);
    }
    return 0;
}
