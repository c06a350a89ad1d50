// issue_rates.hip -- diagnostics only (never linked into the product): VALU issue
// throughput per SIMD on gfx950 for the integer instructions the scan, SHA-256 and
// BLAKE3 kernels are built from, at 1, 2, 4 and 8 waves per SIMD.
//
// Method (round 4; replaces round 2's per-wave s_memtime table, whose per-wave
// durations under-count the SIMD's span when waves of one SIMD do not overlap fully):
//  * every CU gets exactly w waves per SIMD: 256 x w/4... workgroups of 256 threads
//    (one wave per SIMD) with dynamic LDS sized so that at most w fit on a CU;
//  * each wave runs `iters` x 256 instructions of one kind over 8 independent
//    register chains (inline asm: the compiler cannot merge or reorder them);
//  * the kernel's wall time (HIP events, ~10-40 ms per launch) times the clock the
//    waves measured in-kernel (s_memtime / s_memrealtime x 100 MHz, median) gives
//    shader clocks per SIMD; / (w x iters x 256) = clocks per instruction per SIMD.
// Kinds >= 100 are instruction mixes taken from the product kernels (BLAKE3's G
// step as blake3.hip interleaves it; the scan's 32-byte lane-block hash).
//
// Build: make -C scripts/micro   Run: scripts/micro/_bin/issue_rates [kinds] > out.json
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHK(x)                                                                                   \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
            exit(2);                                                                             \
        }                                                                                        \
    } while (0)

struct Kind {
    int id;
    const char *name;
};

// 8 chains: dst r[c], sources r[8 + c], r[8 + ((c + 1) & 7)]
#define OP2(ins) asm volatile(ins " %0, %0, %1" : "+v"(r[c]) : "v"(r[8 + c]))
#define OP3(ins) asm volatile(ins " %0, %0, %1, %2" : "+v"(r[c]) : "v"(r[8 + c]), "v"(r[8 + ((c + 1) & 7)]))

template <int K>
__device__ __forceinline__ void body(uint32_t (&r)[16], uint64_t (&q)[8], float (&f)[16]) {
#pragma unroll
    for (int i = 0; i < 32; ++i) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if constexpr (K == 0) OP2("v_add_u32");
            if constexpr (K == 1) OP2("v_xor_b32");
            if constexpr (K == 2) OP2("v_and_b32");
            if constexpr (K == 3) OP3("v_add3_u32");
            if constexpr (K == 4) OP3("v_xad_u32");
            if constexpr (K == 5) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[c]));
            if constexpr (K == 6) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[c]) : "v"(r[8 + c]), "v"(r[8 + ((c + 1) & 7)]));
            if constexpr (K == 7) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(q[c]) : "v"(q[(c + 1) & 7]));
            if constexpr (K == 8) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(r[c]));
            if constexpr (K == 9) OP3("v_min3_u32");
            if constexpr (K == 10)
                asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 11) OP3("v_perm_b32");
            if constexpr (K == 12)
                asm volatile("v_add_u32_dpp %0, %1, %0 row_shl:4 row_mask:0xf bank_mask:0xf" : "+v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 13) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[c]) : "v"(f[8 + c]));
            if constexpr (K == 14) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(f[8 + c]), "v"(f[8 + ((c + 1) & 7)]));
            if constexpr (K == 15) OP2("v_pk_add_u16");
            if constexpr (K == 16) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(q[c]) : "v"(q[(c + 1) & 7]), "v"(q[(c + 2) & 7]));
            if constexpr (K == 17) OP2("v_mul_u32_u24");
            if constexpr (K == 18) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 19) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 20) OP3("v_or3_b32");
            if constexpr (K == 21) asm volatile("v_alignbyte_b32 %0, %0, %1, 3" : "+v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 22) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(r[c]));
            if constexpr (K == 23) OP3("v_mad_u32_u24");
            if constexpr (K == 24) OP2("v_min_u32");
            if constexpr (K == 25) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 26) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(r[c]) : "v"(r[8 + c]) : "vcc");
            if constexpr (K == 27) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(q[c]));
            if constexpr (K == 28) asm volatile("v_mov_b32 %0, %1" : "=v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 29) OP3("v_bfi_b32");
            if constexpr (K == 30) OP3("v_add_lshl_u32");
            if constexpr (K == 31) OP3("v_and_or_b32");
            if constexpr (K == 32) asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 33) OP2("v_mul_lo_u32");
            if constexpr (K == 34) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 35) asm volatile("v_xor_b32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 36) asm volatile("v_mov_b32_dpp %0, %1 row_ror:1 row_mask:0xf bank_mask:0xf" : "=v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 37) OP2("v_sub_u32");
            if constexpr (K == 38) OP2("v_or_b32");
            if constexpr (K == 39) asm volatile("v_lshl_add_u64 %0, %0, 4, %1" : "+v"(q[c]) : "v"(q[(c + 1) & 7]));
            if constexpr (K == 40) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(q[c]) : "v"(q[(c + 1) & 7]));
            if constexpr (K == 41) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(q[c]) : "v"(r[8 + c]), "v"(r[8 + ((c + 1) & 7)]) : "s40", "s41");
            if constexpr (K == 42) asm volatile("v_add_u32 %0, %0, 1" : "+v"(r[c]));
            if constexpr (K == 43) asm volatile("v_pk_mov_b32 %0, %1, %2 op_sel:[0,1]" : "=v"(q[c]) : "v"(q[(c + 1) & 7]), "v"(q[(c + 2) & 7]));
            if constexpr (K == 44) asm volatile("v_bitop3_b32 %0, %0, %1, 7 bitop3:0x96" : "+v"(r[c]) : "v"(r[8 + c]));
            if constexpr (K == 45) asm volatile("v_lshlrev_b16 %0, 3, %0" : "+v"(r[c]));
            if constexpr (K == 46) OP2("v_pk_lshlrev_b16");
            if constexpr (K == 47) asm volatile("v_lshl_add_u64 %0, %1, 1, %2" : "=v"(q[c]) : "v"(q[(c + 1) & 7]), "v"(q[(c + 2) & 7]));
        }
    }
}


// Mixes (kinds 110..): a 16-instruction pattern repeated 16 times per iteration over the 8
// chains, H = v_add3_u32 (half-rate alone), F = v_add_u32 (full-rate alone), B = v_bitop3_b32,
// L = v_lshl_add_u64, S = SDWA byte move, M = v_min3_u32, R = v_lshrrev_b32.
template <char T>
__device__ __forceinline__ void mix_op(uint32_t (&r)[16], uint64_t (&q)[8], int c) {
    if constexpr (T == 'H') OP3("v_add3_u32");
    if constexpr (T == 'F') OP2("v_add_u32");
    if constexpr (T == 'B') asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[c]) : "v"(r[8 + c]), "v"(r[8 + ((c + 1) & 7)]));
    if constexpr (T == 'L') asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(q[c]) : "v"(q[(c + 1) & 7]));
    if constexpr (T == 'S')
        asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(r[c]) : "v"(r[8 + c]));
    if constexpr (T == 'M') OP3("v_min3_u32");
    if constexpr (T == 'R') asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(r[c]));
    // operand-order probes (kinds 120-123): the accumulated register as src1 (the form the
    // compiler emits for a commutative op: v_add_u32_e32 vD, vS, vD), or a fresh destination
    if constexpr (T == 'f') asm volatile("v_add_u32 %0, %1, %0" : "+v"(r[c]) : "v"(r[8 + c]));
    if constexpr (T == 'x') asm volatile("v_xor_b32 %0, %1, %0" : "+v"(r[c]) : "v"(r[8 + c]));
    if constexpr (T == 'X') asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[c]) : "v"(r[8 + c]));
    if constexpr (T == 'n') asm volatile("v_add_u32 %0, %1, %2" : "=v"(r[c]) : "v"(r[8 + c]), "v"(r[(c + 1) & 7]));
}
template <char... P>
__device__ __forceinline__ void mix_body(uint32_t (&r)[16], uint64_t (&q)[8]) {
    constexpr char pat[] = {P...};
    static_assert(sizeof(pat) == 16, "16-op patterns");
#pragma unroll
    for (int i = 0; i < 16; ++i) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int c = j & 7;
            if (pat[j] == 'H') mix_op<'H'>(r, q, c);
            if (pat[j] == 'F') mix_op<'F'>(r, q, c);
            if (pat[j] == 'B') mix_op<'B'>(r, q, c);
            if (pat[j] == 'L') mix_op<'L'>(r, q, c);
            if (pat[j] == 'S') mix_op<'S'>(r, q, c);
            if (pat[j] == 'M') mix_op<'M'>(r, q, c);
            if (pat[j] == 'R') mix_op<'R'>(r, q, c);
            if (pat[j] == 'f') mix_op<'f'>(r, q, c);
            if (pat[j] == 'x') mix_op<'x'>(r, q, c);
            if (pat[j] == 'X') mix_op<'X'>(r, q, c);
            if (pat[j] == 'n') mix_op<'n'>(r, q, c);
        }
    }
}
#define MIXK(K, ...) if constexpr (KK == K) mix_body<__VA_ARGS__>(r, q);
template <int KK>
__device__ __forceinline__ void mix_kind(uint32_t (&r)[16], uint64_t (&q)[8]) {
    MIXK(110, 'H','F','H','F','H','F','H','F','H','F','H','F','H','F','H','F')
    MIXK(111, 'H','H','H','H','H','H','H','H','F','F','F','F','F','F','F','F')
    MIXK(112, 'H','F','F','F','H','F','F','F','H','F','F','F','H','F','F','F')
    MIXK(113, 'F','F','F','F','F','F','F','F','F','F','F','F','F','F','F','H')
    MIXK(114, 'B','F','B','F','B','F','B','F','B','F','B','F','B','F','B','F')
    MIXK(115, 'L','F','L','F','L','F','L','F','L','F','L','F','L','F','L','F')
    MIXK(116, 'S','B','S','B','S','B','S','B','S','B','S','B','S','B','S','B')
    MIXK(117, 'H','H','H','H','H','H','H','H','H','H','H','H','H','H','H','F')
    MIXK(118, 'R','F','R','F','R','F','R','F','R','F','R','F','R','F','R','F')
    MIXK(119, 'L','L','L','L','F','F','F','F','M','M','F','F','S','S','S','S')
    MIXK(120, 'H','f','H','f','H','f','H','f','H','f','H','f','H','f','H','f')
    MIXK(121, 'f','f','f','f','f','f','f','f','f','f','f','f','f','f','f','f')
    MIXK(122, 'H','x','H','x','H','x','H','x','H','x','H','x','H','x','H','x')
    MIXK(123, 'H','X','H','X','H','X','H','X','H','X','H','X','H','X','H','X')
    MIXK(124, 'H','n','H','n','H','n','H','n','H','n','H','n','H','n','H','n')
}

// Explicit-register variants (VGPR bank hypothesis): v40..v63 written / read by hand.
// bank of vN assumed N mod 4.  One instruction per chain c = 0..7.
template <int K>
__device__ __forceinline__ void body_x() {
#define X8(fmt_same)                                                                               \
    asm volatile(fmt_same ::: "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", \
                 "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61",  \
                 "v62", "v63")
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        if constexpr (K == 60)  // add3, all three sources in one bank
            X8("v_add3_u32 v40, v40, v48, v56\n v_add3_u32 v41, v41, v49, v57\n v_add3_u32 v42, v42, v50, v58\n"
               " v_add3_u32 v43, v43, v51, v59\n v_add3_u32 v44, v44, v52, v60\n v_add3_u32 v45, v45, v53, v61\n"
               " v_add3_u32 v46, v46, v54, v62\n v_add3_u32 v47, v47, v55, v63");
        if constexpr (K == 61)  // add3, sources in three different banks
            X8("v_add3_u32 v40, v40, v49, v58\n v_add3_u32 v41, v41, v50, v59\n v_add3_u32 v42, v42, v51, v56\n"
               " v_add3_u32 v43, v43, v48, v57\n v_add3_u32 v44, v44, v53, v62\n v_add3_u32 v45, v45, v54, v63\n"
               " v_add3_u32 v46, v46, v55, v60\n v_add3_u32 v47, v47, v52, v61");
        if constexpr (K == 62)  // alignbit rotate (same source twice)
            X8("v_alignbit_b32 v40, v40, v40, 7\n v_alignbit_b32 v41, v41, v41, 7\n v_alignbit_b32 v42, v42, v42, 7\n"
               " v_alignbit_b32 v43, v43, v43, 7\n v_alignbit_b32 v44, v44, v44, 7\n v_alignbit_b32 v45, v45, v45, 7\n"
               " v_alignbit_b32 v46, v46, v46, 7\n v_alignbit_b32 v47, v47, v47, 7");
        if constexpr (K == 63)  // alignbit with two different sources, different banks
            X8("v_alignbit_b32 v40, v40, v49, 7\n v_alignbit_b32 v41, v41, v50, 7\n v_alignbit_b32 v42, v42, v51, 7\n"
               " v_alignbit_b32 v43, v43, v48, 7\n v_alignbit_b32 v44, v44, v53, 7\n v_alignbit_b32 v45, v45, v54, 7\n"
               " v_alignbit_b32 v46, v46, v55, 7\n v_alignbit_b32 v47, v47, v52, 7");
        if constexpr (K == 64)  // lshl_add_u64, sources in the same bank pair
            X8("v_lshl_add_u64 v[40:41], v[40:41], 1, v[48:49]\n v_lshl_add_u64 v[42:43], v[42:43], 1, v[50:51]\n"
               " v_lshl_add_u64 v[44:45], v[44:45], 1, v[52:53]\n v_lshl_add_u64 v[46:47], v[46:47], 1, v[54:55]\n"
               " v_lshl_add_u64 v[56:57], v[56:57], 1, v[48:49]\n v_lshl_add_u64 v[58:59], v[58:59], 1, v[50:51]\n"
               " v_lshl_add_u64 v[60:61], v[60:61], 1, v[52:53]\n v_lshl_add_u64 v[62:63], v[62:63], 1, v[54:55]");
        if constexpr (K == 65)  // lshl_add_u64, sources in different bank pairs
            X8("v_lshl_add_u64 v[40:41], v[40:41], 1, v[50:51]\n v_lshl_add_u64 v[42:43], v[42:43], 1, v[48:49]\n"
               " v_lshl_add_u64 v[44:45], v[44:45], 1, v[54:55]\n v_lshl_add_u64 v[46:47], v[46:47], 1, v[52:53]\n"
               " v_lshl_add_u64 v[56:57], v[56:57], 1, v[50:51]\n v_lshl_add_u64 v[58:59], v[58:59], 1, v[48:49]\n"
               " v_lshl_add_u64 v[60:61], v[60:61], 1, v[54:55]\n v_lshl_add_u64 v[62:63], v[62:63], 1, v[52:53]");
        if constexpr (K == 66)  // add_u32, two sources same bank
            X8("v_add_u32 v40, v40, v48\n v_add_u32 v41, v41, v49\n v_add_u32 v42, v42, v50\n v_add_u32 v43, v43, v51\n"
               " v_add_u32 v44, v44, v52\n v_add_u32 v45, v45, v53\n v_add_u32 v46, v46, v54\n v_add_u32 v47, v47, v55");
        if constexpr (K == 67)  // add_u32, two sources different banks
            X8("v_add_u32 v40, v40, v49\n v_add_u32 v41, v41, v50\n v_add_u32 v42, v42, v51\n v_add_u32 v43, v43, v48\n"
               " v_add_u32 v44, v44, v53\n v_add_u32 v45, v45, v54\n v_add_u32 v46, v46, v55\n v_add_u32 v47, v47, v52");
        if constexpr (K == 68)  // add3 where 2 sources share a bank
            X8("v_add3_u32 v40, v40, v48, v57\n v_add3_u32 v41, v41, v49, v58\n v_add3_u32 v42, v42, v50, v59\n"
               " v_add3_u32 v43, v43, v51, v56\n v_add3_u32 v44, v44, v52, v61\n v_add3_u32 v45, v45, v53, v62\n"
               " v_add3_u32 v46, v46, v54, v63\n v_add3_u32 v47, v47, v55, v60");
    }
#undef X8
}

// BLAKE3 G step interleave as blake3.hip's B3_G4 (4 independent G chains, op by op).
__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) { return __builtin_amdgcn_alignbit(x, x, n); }
#define G4(a0, b0, c0, d0, a1, b1, c1, d1, a2, b2, c2, d2, a3, b3, c3, d3, m0, m1)          \
    {                                                                                       \
        v[a0] = v[a0] + v[b0] + m[m0];                                                      \
        v[a1] = v[a1] + v[b1] + m[m0 + 2];                                                  \
        v[a2] = v[a2] + v[b2] + m[m0 + 4];                                                  \
        v[a3] = v[a3] + v[b3] + m[m0 + 6];                                                  \
        v[d0] = rotr(v[d0] ^ v[a0], 16);                                                    \
        v[d1] = rotr(v[d1] ^ v[a1], 16);                                                    \
        v[d2] = rotr(v[d2] ^ v[a2], 16);                                                    \
        v[d3] = rotr(v[d3] ^ v[a3], 16);                                                    \
        v[c0] = v[c0] + v[d0];                                                              \
        v[c1] = v[c1] + v[d1];                                                              \
        v[c2] = v[c2] + v[d2];                                                              \
        v[c3] = v[c3] + v[d3];                                                              \
        v[b0] = rotr(v[b0] ^ v[c0], 12);                                                    \
        v[b1] = rotr(v[b1] ^ v[c1], 12);                                                    \
        v[b2] = rotr(v[b2] ^ v[c2], 12);                                                    \
        v[b3] = rotr(v[b3] ^ v[c3], 12);                                                    \
        v[a0] = v[a0] + v[b0] + m[m1];                                                      \
        v[a1] = v[a1] + v[b1] + m[m1 + 2];                                                  \
        v[a2] = v[a2] + v[b2] + m[m1 + 4];                                                  \
        v[a3] = v[a3] + v[b3] + m[m1 + 6];                                                  \
        v[d0] = rotr(v[d0] ^ v[a0], 8);                                                     \
        v[d1] = rotr(v[d1] ^ v[a1], 8);                                                     \
        v[d2] = rotr(v[d2] ^ v[a2], 8);                                                     \
        v[d3] = rotr(v[d3] ^ v[a3], 8);                                                     \
        v[c0] = v[c0] + v[d0];                                                              \
        v[c1] = v[c1] + v[d1];                                                              \
        v[c2] = v[c2] + v[d2];                                                              \
        v[c3] = v[c3] + v[d3];                                                              \
        v[b0] = rotr(v[b0] ^ v[c0], 7);                                                     \
        v[b1] = rotr(v[b1] ^ v[c1], 7);                                                     \
        v[b2] = rotr(v[b2] ^ v[c2], 7);                                                     \
        v[b3] = rotr(v[b3] ^ v[c3], 7);                                                     \
    }

// kind 100: 7 rounds x (column + diagonal G4) = one compression (672 VALU: 56 G x 12)
// kind 101: the same with the 16-/8-bit rotations as v_perm_b32 (byte permutes)
// kind 102: the same with rotations by 16 as v_pk ... (kept out: see DESIGN)
template <int K>
__device__ __forceinline__ void b3_body(uint32_t (&v)[16], const uint32_t (&m)[16]) {
#pragma unroll
    for (int rr = 0; rr < 7; ++rr) {
        G4(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15, 0, 1);
        G4(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14, 8, 9);
    }
}


// BLAKE3 variants (kinds 101-103): 101 = add3 split into two v_add_u32 (more dual-issuable
// ops, 784 VALU per compression); 102 = two compressions per lane, their G steps interleaved
// (runs of 8 same-kind ops); 103 = both.
template <bool SPLIT>
__device__ __forceinline__ uint32_t add3x(uint32_t a, uint32_t b, uint32_t c) {
    if constexpr (SPLIT) {
        uint32_t t;
        asm volatile("v_add_u32 %0, %1, %2" : "=v"(t) : "v"(a), "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(t) : "v"(c));
        return t;
    } else {
        return a + b + c;
    }
}
// SEP (kinds 107-108): between the op groups 0 = nothing, 1 = an `s_nop 0`, 2 = a
// scheduling barrier (the groups stay in order, no instruction between them)
template <int SEP>
__device__ __forceinline__ void gsep() {
    if constexpr (SEP == 1) asm volatile("s_nop 0");
    if constexpr (SEP == 2) __builtin_amdgcn_sched_barrier(0);
}
template <bool SPLIT, int NS, int SEP = 0>
__device__ __forceinline__ void g4x(uint32_t (*st)[16], const uint32_t (&m)[16], const int (&ix)[4][4], int mo) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) st[s][ix[j][0]] = add3x<SPLIT>(st[s][ix[j][0]], st[s][ix[j][1]], m[(mo + 2 * j) & 15]);
    gsep<SEP>();
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) st[s][ix[j][3]] = rotr(st[s][ix[j][3]] ^ st[s][ix[j][0]], 16);
    gsep<SEP>();
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) st[s][ix[j][2]] = st[s][ix[j][2]] + st[s][ix[j][3]];
    gsep<SEP>();
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) st[s][ix[j][1]] = rotr(st[s][ix[j][1]] ^ st[s][ix[j][2]], 12);
    gsep<SEP>();
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) st[s][ix[j][0]] = add3x<SPLIT>(st[s][ix[j][0]], st[s][ix[j][1]], m[(mo + 2 * j + 1) & 15]);
    gsep<SEP>();
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) st[s][ix[j][3]] = rotr(st[s][ix[j][3]] ^ st[s][ix[j][0]], 8);
    gsep<SEP>();
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) st[s][ix[j][2]] = st[s][ix[j][2]] + st[s][ix[j][3]];
    gsep<SEP>();
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) st[s][ix[j][1]] = rotr(st[s][ix[j][1]] ^ st[s][ix[j][2]], 7);
}
template <bool SPLIT, int NS, int SEP = 0>
__device__ __forceinline__ void b3_var(uint32_t (*st)[16], const uint32_t (&m)[16]) {
    constexpr int col[4][4] = {{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14}, {3, 7, 11, 15}};
    constexpr int dia[4][4] = {{0, 5, 10, 15}, {1, 6, 11, 12}, {2, 7, 8, 13}, {3, 4, 9, 14}};
#pragma unroll
    for (int rr = 0; rr < 7; ++rr) {
        g4x<SPLIT, NS, SEP>(st, m, col, 0);
        g4x<SPLIT, NS, SEP>(st, m, dia, 8);
    }
}

// Kinds 104-106 (round 5): the G4 stream in an order pinned by one
// asm volatile per instruction (the compiler keeps volatile asm in program order), so the
// first-class ops (v_add_u32, v_xor_b32) come in runs between the second-class ones
// (v_alignbit_b32 rotations, v_add3_u32).  104: two compressions interleaved, add3 split into
// two v_add_u32 -- per step of 8 G's: 24 F, 8 H, 16 F, 8 H, 24 F, 8 H, 16 F, 8 H (10 F + 4 H
// per G, 784 VALU per compression); 105: the same with one compression (runs of 12 / 8);
// 106: two compressions, add3 kept (6 F + 6 H per G, 672 VALU per compression).
#define A_ADD(d, x, y) asm volatile("v_add_u32 %0, %1, %2" : "=v"(d) : "v"(x), "v"(y))
#define A_ADD3(d, x, y, z) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(x), "v"(y), "v"(z))
#define A_XOR(d, x, y) asm volatile("v_xor_b32 %0, %1, %2" : "=v"(d) : "v"(x), "v"(y))
#define A_ROT(d, x, n) asm volatile("v_alignbit_b32 %0, %1, %1, " #n : "=v"(d) : "v"(x))
// early-clobber forms: the destination register differs from every source (kinds 109, 125-126)
#define E_ADD(d, x, y) asm volatile("v_add_u32 %0, %1, %2" : "=&v"(d) : "v"(x), "v"(y))
#define E_ADD3(d, x, y, z) asm volatile("v_add3_u32 %0, %1, %2, %3" : "=&v"(d) : "v"(x), "v"(y), "v"(z))
#define E_XOR(d, x, y) asm volatile("v_xor_b32 %0, %1, %2" : "=&v"(d) : "v"(x), "v"(y))
#define E_ROT(d, x, n) asm volatile("v_alignbit_b32 %0, %1, %1, " #n : "=&v"(d) : "v"(x))
#define F_ADD(...) do { if constexpr (FRESH >= 1) E_ADD(__VA_ARGS__); else A_ADD(__VA_ARGS__); } while (0)
#define F_XOR(...) do { if constexpr (FRESH >= 1) E_XOR(__VA_ARGS__); else A_XOR(__VA_ARGS__); } while (0)
#define H_ADD3(...) do { if constexpr (FRESH >= 2) E_ADD3(__VA_ARGS__); else A_ADD3(__VA_ARGS__); } while (0)
#define H_ROT(d, x, n) do { if constexpr (FRESH >= 2) E_ROT(d, x, n); else A_ROT(d, x, n); } while (0)
template <bool SPLIT, int NS, int FRESH = 0>
__device__ __forceinline__ void g4p(uint32_t (*st)[16], const uint32_t (&m)[16], const int (&ix)[4][4], int mo) {
    // a += b + m0
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t &a = st[s][ix[j][0]];
            if constexpr (SPLIT) F_ADD(a, a, st[s][ix[j][1]]);
            else H_ADD3(a, a, st[s][ix[j][1]], m[(mo + 2 * j) & 15]);
        }
    if constexpr (SPLIT) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int j = 0; j < 4; ++j) F_ADD(st[s][ix[j][0]], st[s][ix[j][0]], m[(mo + 2 * j) & 15]);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) F_XOR(st[s][ix[j][3]], st[s][ix[j][3]], st[s][ix[j][0]]);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) H_ROT(st[s][ix[j][3]], st[s][ix[j][3]], 16);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) F_ADD(st[s][ix[j][2]], st[s][ix[j][2]], st[s][ix[j][3]]);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) F_XOR(st[s][ix[j][1]], st[s][ix[j][1]], st[s][ix[j][2]]);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) H_ROT(st[s][ix[j][1]], st[s][ix[j][1]], 12);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t &a = st[s][ix[j][0]];
            if constexpr (SPLIT) F_ADD(a, a, st[s][ix[j][1]]);
            else H_ADD3(a, a, st[s][ix[j][1]], m[(mo + 2 * j + 1) & 15]);
        }
    if constexpr (SPLIT) {
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int j = 0; j < 4; ++j) F_ADD(st[s][ix[j][0]], st[s][ix[j][0]], m[(mo + 2 * j + 1) & 15]);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) F_XOR(st[s][ix[j][3]], st[s][ix[j][3]], st[s][ix[j][0]]);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) H_ROT(st[s][ix[j][3]], st[s][ix[j][3]], 8);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) F_ADD(st[s][ix[j][2]], st[s][ix[j][2]], st[s][ix[j][3]]);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) F_XOR(st[s][ix[j][1]], st[s][ix[j][1]], st[s][ix[j][2]]);
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) H_ROT(st[s][ix[j][1]], st[s][ix[j][1]], 7);
}
template <bool SPLIT, int NS, int FRESH = 0>
__device__ __forceinline__ void b3_pinned(uint32_t (*st)[16], const uint32_t (&m)[16]) {
    constexpr int col[4][4] = {{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14}, {3, 7, 11, 15}};
    constexpr int dia[4][4] = {{0, 5, 10, 15}, {1, 6, 11, 12}, {2, 7, 8, 13}, {3, 4, 9, 14}};
#pragma unroll
    for (int rr = 0; rr < 7; ++rr) {
        g4p<SPLIT, NS, FRESH>(st, m, col, 0);
        g4p<SPLIT, NS, FRESH>(st, m, dia, 8);
    }
}

// Kind 127: each G4 step (48 ops) as ONE asm statement: the compiler pads between asm
// statements with s_nop (its hazard model cannot see inside them), so per-op statements
// (kinds 104-126) carry ~1 s_nop per op group; one statement per step carries 1 per 48 ops.
#define G4ASM_BODY(M0, M1, M2, M3, R) \
    "v_add3_u32 %[a0], %[a0], %[b0], %[" M0 "0]\n v_add3_u32 %[a1], %[a1], %[b1], %[" M0 "1]\n" \
    " v_add3_u32 %[a2], %[a2], %[b2], %[" M0 "2]\n v_add3_u32 %[a3], %[a3], %[b3], %[" M0 "3]\n" \
    " v_xor_b32 %[d0], %[d0], %[a0]\n v_xor_b32 %[d1], %[d1], %[a1]\n v_xor_b32 %[d2], %[d2], %[a2]\n v_xor_b32 %[d3], %[d3], %[a3]\n" \
    " v_alignbit_b32 %[d0], %[d0], %[d0], " M1 "\n v_alignbit_b32 %[d1], %[d1], %[d1], " M1 "\n" \
    " v_alignbit_b32 %[d2], %[d2], %[d2], " M1 "\n v_alignbit_b32 %[d3], %[d3], %[d3], " M1 "\n" \
    " v_add_u32 %[c0], %[c0], %[d0]\n v_add_u32 %[c1], %[c1], %[d1]\n v_add_u32 %[c2], %[c2], %[d2]\n v_add_u32 %[c3], %[c3], %[d3]\n" \
    " v_xor_b32 %[b0], %[b0], %[c0]\n v_xor_b32 %[b1], %[b1], %[c1]\n v_xor_b32 %[b2], %[b2], %[c2]\n v_xor_b32 %[b3], %[b3], %[c3]\n" \
    " v_alignbit_b32 %[b0], %[b0], %[b0], " M2 "\n v_alignbit_b32 %[b1], %[b1], %[b1], " M2 "\n" \
    " v_alignbit_b32 %[b2], %[b2], %[b2], " M2 "\n v_alignbit_b32 %[b3], %[b3], %[b3], " M2 "\n" \
    " v_add3_u32 %[a0], %[a0], %[b0], %[" M3 "0]\n v_add3_u32 %[a1], %[a1], %[b1], %[" M3 "1]\n" \
    " v_add3_u32 %[a2], %[a2], %[b2], %[" M3 "2]\n v_add3_u32 %[a3], %[a3], %[b3], %[" M3 "3]\n" \
    " v_xor_b32 %[d0], %[d0], %[a0]\n v_xor_b32 %[d1], %[d1], %[a1]\n v_xor_b32 %[d2], %[d2], %[a2]\n v_xor_b32 %[d3], %[d3], %[a3]\n" \
    " v_alignbit_b32 %[d0], %[d0], %[d0], 8\n v_alignbit_b32 %[d1], %[d1], %[d1], 8\n" \
    " v_alignbit_b32 %[d2], %[d2], %[d2], 8\n v_alignbit_b32 %[d3], %[d3], %[d3], 8\n" \
    " v_add_u32 %[c0], %[c0], %[d0]\n v_add_u32 %[c1], %[c1], %[d1]\n v_add_u32 %[c2], %[c2], %[d2]\n v_add_u32 %[c3], %[c3], %[d3]\n" \
    " v_xor_b32 %[b0], %[b0], %[c0]\n v_xor_b32 %[b1], %[b1], %[c1]\n v_xor_b32 %[b2], %[b2], %[c2]\n v_xor_b32 %[b3], %[b3], %[c3]\n" \
    " v_alignbit_b32 %[b0], %[b0], %[b0], " R "\n v_alignbit_b32 %[b1], %[b1], %[b1], " R "\n" \
    " v_alignbit_b32 %[b2], %[b2], %[b2], " R "\n v_alignbit_b32 %[b3], %[b3], %[b3], " R
#define G4ASM(A0, B0, C0, D0, A1, B1, C1, D1, A2, B2, C2, D2, A3, B3, C3, D3, MO)                                 \
    asm volatile(G4ASM_BODY("x", "16", "12", "y", "7")                                                          \
                 : [a0] "+v"(v[A0]), [b0] "+v"(v[B0]), [c0] "+v"(v[C0]), [d0] "+v"(v[D0]), [a1] "+v"(v[A1]),     \
                   [b1] "+v"(v[B1]), [c1] "+v"(v[C1]), [d1] "+v"(v[D1]), [a2] "+v"(v[A2]), [b2] "+v"(v[B2]),     \
                   [c2] "+v"(v[C2]), [d2] "+v"(v[D2]), [a3] "+v"(v[A3]), [b3] "+v"(v[B3]), [c3] "+v"(v[C3]),     \
                   [d3] "+v"(v[D3])                                                                              \
                 : [x0] "v"(m[(MO) & 15]), [x1] "v"(m[((MO) + 2) & 15]), [x2] "v"(m[((MO) + 4) & 15]),          \
                   [x3] "v"(m[((MO) + 6) & 15]), [y0] "v"(m[((MO) + 1) & 15]), [y1] "v"(m[((MO) + 3) & 15]),    \
                   [y2] "v"(m[((MO) + 5) & 15]), [y3] "v"(m[((MO) + 7) & 15]))
__device__ __forceinline__ void b3_asm_step(uint32_t (&v)[16], const uint32_t (&m)[16]) {
#pragma unroll
    for (int rr = 0; rr < 7; ++rr) {
        G4ASM(0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15, 0);
        G4ASM(0, 5, 10, 15, 1, 6, 11, 12, 2, 7, 8, 13, 3, 4, 9, 14, 8);
    }
}

template <int K>
__global__ __launch_bounds__(256) void k_issue(uint32_t iters, uint32_t *out, unsigned long long *stamps) {
    extern __shared__ uint32_t lds_pad[];
    const uint32_t tid = blockIdx.x * 256 + threadIdx.x;
    if (K == 255) lds_pad[threadIdx.x] = 0;  // keep the dynamic LDS (occupancy cap) referenced
    unsigned long long t0, t1, rt0, rt1;
    uint32_t x = 0;
    // only the state a kind uses is live (<= 64 VGPRs, so 8 waves fit a SIMD)
    if constexpr (K < 60) {
        uint32_t r[16];
        uint64_t q[8];
        float f[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            r[i] = tid * 16 + i;
            f[i] = 1.0f + 1e-7f * (float)(tid + i);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] = tid * 8ull + i;
        t0 = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t it = 0; it < iters; ++it) body<K>(r, q, f);
        t1 = __builtin_amdgcn_s_memtime();
        rt1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int i = 0; i < 16; ++i) x ^= r[i] ^ __float_as_uint(f[i]);
#pragma unroll
        for (int i = 0; i < 8; ++i) x ^= (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32);
    } else if constexpr (K >= 110 && K < 125) {  // (125-127: BLAKE3 forms below)
        uint32_t r[16];
        uint64_t q[8];
#pragma unroll
        for (int i = 0; i < 16; ++i) r[i] = tid * 16 + i;
#pragma unroll
        for (int i = 0; i < 8; ++i) q[i] = tid * 8ull + i;
        t0 = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t it = 0; it < iters; ++it) mix_kind<K>(r, q);
        t1 = __builtin_amdgcn_s_memtime();
        rt1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int i = 0; i < 16; ++i) x ^= r[i];
#pragma unroll
        for (int i = 0; i < 8; ++i) x ^= (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32);
    } else if constexpr (K < 100) {
        t0 = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t it = 0; it < iters; ++it) body_x<K>();
        t1 = __builtin_amdgcn_s_memtime();
        rt1 = __builtin_amdgcn_s_memrealtime();
    } else if constexpr (K == 127) {
        uint32_t v[16], m[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            v[i] = tid * 0x9E3779B9u + i;
            m[i] = tid ^ (i * 0x01010101u);
        }
        t0 = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t it = 0; it < iters; ++it) b3_asm_step(v, m);
        t1 = __builtin_amdgcn_s_memtime();
        rt1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int i = 0; i < 16; ++i) x ^= v[i];
    } else if constexpr ((K >= 104 && K <= 106) || K == 109 || K == 125 || K == 126) {
        constexpr int NS = K == 105 || K == 125 || K == 126 ? 1 : 2;
        constexpr int FRESH = K == 109 || K == 125 ? 1 : K == 126 ? 2 : 0;
        uint32_t st[NS][16], m[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            m[i] = tid ^ (i * 0x01010101u);
#pragma unroll
            for (int k = 0; k < NS; ++k) st[k][i] = tid * 0x9E3779B9u + i + 77 * k;
        }
        t0 = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t it = 0; it < iters; ++it) b3_pinned<K != 106 && K < 109, NS, FRESH>(st, m);
        t1 = __builtin_amdgcn_s_memtime();
        rt1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int i = 0; i < 16; ++i)
#pragma unroll
            for (int k = 0; k < NS; ++k) x ^= st[k][i];
    } else if constexpr ((K >= 101 && K <= 103) || K == 107 || K == 108) {
        constexpr int NS = K == 101 ? 1 : 2;
        uint32_t st[NS][16], m[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            m[i] = tid ^ (i * 0x01010101u);
#pragma unroll
            for (int k = 0; k < NS; ++k) st[k][i] = tid * 0x9E3779B9u + i + 77 * k;
        }
        t0 = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t it = 0; it < iters; ++it) {
            b3_var<K != 102 && K != 107 && K != 108, NS, K == 107 ? 1 : K == 108 ? 2 : 0>(st, m);
#pragma unroll
            for (int k = 0; k < NS; ++k) asm volatile("" : "+v"(st[k][0]), "+v"(st[k][5]), "+v"(st[k][10]), "+v"(st[k][15]));
        }
        t1 = __builtin_amdgcn_s_memtime();
        rt1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int i = 0; i < 16; ++i)
#pragma unroll
            for (int k = 0; k < NS; ++k) x ^= st[k][i];
    } else {
        uint32_t v[16], m[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            v[i] = tid * 0x9E3779B9u + i;
            m[i] = tid ^ (i * 0x01010101u);
        }
        t0 = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t it = 0; it < iters; ++it) {
            b3_body<K>(v, m);
            asm volatile("" : "+v"(v[0]), "+v"(v[5]), "+v"(v[10]), "+v"(v[15]));
        }
        t1 = __builtin_amdgcn_s_memtime();
        rt1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int i = 0; i < 16; ++i) x ^= v[i];
    }
    out[tid] = x;
    if ((threadIdx.x & 63) == 0) {
        const uint32_t wv = tid >> 6;
        stamps[4 * wv + 0] = t0;
        stamps[4 * wv + 1] = t1;
        stamps[4 * wv + 2] = rt0;
        stamps[4 * wv + 3] = rt1;
    }
}

typedef void (*KFn)(uint32_t, uint32_t *, unsigned long long *);

template <int K>
static void reg(std::vector<std::pair<int, KFn>> &v) {
    v.push_back({K, k_issue<K>});
}

static const char *kind_name(int k) {
    switch (k) {
    case 0: return "v_add_u32";
    case 1: return "v_xor_b32";
    case 2: return "v_and_b32";
    case 3: return "v_add3_u32";
    case 4: return "v_xad_u32";
    case 5: return "v_alignbit_b32 (rotate)";
    case 6: return "v_bitop3_b32";
    case 7: return "v_lshl_add_u64";
    case 8: return "v_lshlrev_b32";
    case 9: return "v_min3_u32";
    case 10: return "v_mov_b32_sdwa BYTE_1 preserve";
    case 11: return "v_perm_b32";
    case 12: return "v_add_u32_dpp row_shl:4";
    case 13: return "v_add_f32";
    case 14: return "v_fma_f32";
    case 15: return "v_pk_add_u16";
    case 16: return "v_pk_fma_f32";
    case 17: return "v_mul_u32_u24";
    case 18: return "v_lshl_or_b32";
    case 19: return "v_add_u32_e64";
    case 20: return "v_or3_b32";
    case 21: return "v_alignbyte_b32";
    case 22: return "v_lshrrev_b32";
    case 23: return "v_mad_u32_u24";
    case 24: return "v_min_u32";
    case 25: return "v_cndmask_b32";
    case 26: return "v_add_co_u32 (vcc)";
    case 27: return "v_lshlrev_b64";
    case 28: return "v_mov_b32";
    case 29: return "v_bfi_b32";
    case 30: return "v_add_lshl_u32";
    case 31: return "v_and_or_b32";
    case 32: return "v_lshl_add_u32";
    case 33: return "v_mul_lo_u32";
    case 34: return "v_add_u32_sdwa WORD_1";
    case 35: return "v_xor_b32_dpp quad_perm";
    case 36: return "v_mov_b32_dpp row_ror:1";
    case 37: return "v_sub_u32";
    case 38: return "v_or_b32";
    case 39: return "v_lshl_add_u64 shift 4";
    case 40: return "v_pk_add_f32";
    case 41: return "v_mad_u64_u32";
    case 42: return "v_add_u32 inline constant";
    case 43: return "v_pk_mov_b32";
    case 44: return "v_bitop3_b32 with constant";
    case 45: return "v_lshlrev_b16";
    case 46: return "v_pk_lshlrev_b16";
    case 47: return "v_lshl_add_u64 fresh dst";
    case 60: return "x v_add3_u32 3 srcs same bank";
    case 61: return "x v_add3_u32 3 srcs distinct banks";
    case 62: return "x v_alignbit_b32 rotate";
    case 63: return "x v_alignbit_b32 2 srcs distinct banks";
    case 64: return "x v_lshl_add_u64 srcs same bank pair";
    case 65: return "x v_lshl_add_u64 srcs distinct bank pairs";
    case 66: return "x v_add_u32 srcs same bank";
    case 67: return "x v_add_u32 srcs distinct banks";
    case 68: return "x v_add3_u32 2 of 3 srcs same bank";
    case 100: return "BLAKE3 compression (B3_G4 interleave, 672 VALU)";
    case 101: return "BLAKE3, add3 as two v_add_u32 (784 VALU)";
    case 102: return "BLAKE3, two compressions interleaved (1344 VALU)";
    case 103: return "BLAKE3, two interleaved + add3 split (1568 VALU)";
    case 104: return "BLAKE3 pinned order, two interleaved + add3 split: F runs of 16-24 (1568 VALU)";
    case 105: return "BLAKE3 pinned order, one compression + add3 split: F runs of 8-12 (784 VALU)";
    case 106: return "BLAKE3 pinned order, two interleaved, add3 kept (1344 VALU)";
    case 107: return "BLAKE3 kind 102 + s_nop 0 between op groups (1344 VALU)";
    case 109: return "BLAKE3 kind 106 with fresh destinations for v_add_u32 / v_xor_b32 (1344 VALU)";
    case 125: return "BLAKE3 pinned, one compression, add3 kept, fresh F destinations (672 VALU)";
    case 126: return "BLAKE3 pinned, one compression, add3 kept, every destination fresh (672 VALU)";
    case 127: return "BLAKE3 one compression, each G4 step one asm statement (672 VALU)";
    case 108: return "BLAKE3 kind 102 + sched_barrier between op groups (1344 VALU)";
    case 110: return "mix HF HF (add3 / add alternating)";
    case 111: return "mix 8H 8F";
    case 112: return "mix H FFF";
    case 113: return "mix 15F 1H";
    case 114: return "mix BF (bitop3 / add)";
    case 115: return "mix LF (lshl_add_u64 / add)";
    case 116: return "mix SB (sdwa / bitop3)";
    case 117: return "mix 15H 1F";
    case 118: return "mix RF (lshrrev / add)";
    case 119: return "mix scan-like 4L 4F 2M 2F 4S";
    case 120: return "mix H f (f = v_add_u32 vD, vS, vD: accumulator as src1)";
    case 121: return "all f (v_add_u32 vD, vS, vD)";
    case 122: return "mix H x (x = v_xor_b32 vD, vS, vD)";
    case 123: return "mix H X (X = v_xor_b32 vD, vD, vS)";
    case 124: return "mix H n (n = v_add_u32 vD, vS, vT, fresh destination)";
    default: return "?";
    }
}

int main(int argc, char **argv) {
    std::vector<std::pair<int, KFn>> ks;
    reg<0>(ks); reg<1>(ks); reg<2>(ks); reg<3>(ks); reg<4>(ks); reg<5>(ks); reg<6>(ks); reg<7>(ks);
    reg<8>(ks); reg<9>(ks); reg<10>(ks); reg<11>(ks); reg<12>(ks); reg<13>(ks); reg<14>(ks); reg<15>(ks);
    reg<16>(ks); reg<17>(ks); reg<18>(ks); reg<19>(ks); reg<20>(ks); reg<21>(ks); reg<22>(ks); reg<23>(ks);
    reg<24>(ks); reg<25>(ks); reg<26>(ks); reg<27>(ks); reg<28>(ks); reg<29>(ks); reg<30>(ks); reg<31>(ks);
    reg<32>(ks); reg<33>(ks); reg<34>(ks); reg<35>(ks); reg<36>(ks); reg<37>(ks); reg<38>(ks); reg<39>(ks);
    reg<40>(ks); reg<41>(ks); reg<42>(ks); reg<43>(ks); reg<44>(ks); reg<45>(ks); reg<46>(ks); reg<47>(ks);
    reg<60>(ks); reg<61>(ks); reg<62>(ks); reg<63>(ks); reg<64>(ks); reg<65>(ks); reg<66>(ks); reg<67>(ks);
    reg<68>(ks); reg<100>(ks); reg<101>(ks); reg<102>(ks); reg<103>(ks); reg<104>(ks); reg<105>(ks); reg<106>(ks); reg<107>(ks); reg<108>(ks); reg<109>(ks); reg<125>(ks); reg<126>(ks); reg<127>(ks);
    reg<110>(ks); reg<111>(ks); reg<112>(ks); reg<113>(ks); reg<114>(ks); reg<115>(ks); reg<116>(ks);
    reg<117>(ks); reg<118>(ks); reg<119>(ks); reg<120>(ks); reg<121>(ks); reg<122>(ks); reg<123>(ks); reg<124>(ks);
    std::vector<int> want;
    if (argc > 1) {
        char *s = strdup(argv[1]);
        for (char *t = strtok(s, ","); t; t = strtok(nullptr, ",")) want.push_back(atoi(t));
    }
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const size_t lds_max = prop.sharedMemPerMultiprocessor ? prop.sharedMemPerMultiprocessor : 160 * 1024;
    uint32_t *d_out;
    unsigned long long *d_st;
    CHK(hipMalloc(&d_out, (size_t)cus * 8 * 256 * 4));
    CHK(hipMalloc(&d_st, (size_t)cus * 8 * 4 * 4 * 8));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    printf("{\"what\": \"clocks per instruction per SIMD (kernel wall time x in-kernel clock / instructions per SIMD); "
           "w = waves per SIMD\", \"cus\": %d, \"lds_per_cu\": %zu, \"rows\": [\n", cus, lds_max);
    bool first = true;
    for (auto &kf : ks) {
        if (!want.empty() && std::find(want.begin(), want.end(), kf.first) == want.end()) continue;
        const int K = kf.first;
        const uint32_t per_iter = K == 100 || K == 125 || K == 126 || K == 127 ? 672u : K == 101 || K == 105 ? 784u
                                : K == 102 || K == 106 || K == 107 || K == 108 || K == 109 ? 1344u
                                : K == 103 || K == 104 ? 1568u : 256u;
        CHK(hipFuncSetAttribute((const void *)kf.second, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max));
        printf("%s{\"kind\": %d, \"name\": \"%s\"", first ? "" : ",\n", K, kind_name(K));
        first = false;
        for (int w : {1, 2, 4, 8}) {
            const uint32_t blocks = (uint32_t)cus * w;
            const size_t lds = (lds_max / w) - 1024;  // at most w workgroups per CU
            // ~20 ms per launch at ~4 clocks per instruction
            const uint32_t iters = (uint32_t)(20e-3 * 2.2e9 / (4.0 * per_iter * w));
            hipLaunchKernelGGL(kf.second, dim3(blocks), dim3(256), lds, 0, 4u, d_out, d_st);
            CHK(hipDeviceSynchronize());
            float best = 1e30f;
            double clk = 0;
            for (int rep = 0; rep < 3; ++rep) {
                CHK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(kf.second, dim3(blocks), dim3(256), lds, 0, iters, d_out, d_st);
                CHK(hipEventRecord(e1, 0));
                CHK(hipEventSynchronize(e1));
                float ms = 0;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) {
                    best = ms;
                    const size_t nw = (size_t)blocks * 4;
                    std::vector<unsigned long long> st(nw * 4);
                    CHK(hipMemcpy(st.data(), d_st, nw * 4 * 8, hipMemcpyDeviceToHost));
                    std::vector<double> f;
                    std::vector<double> span;
                    for (size_t i = 0; i < nw; ++i) {
                        const double dc = (double)(st[4 * i + 1] - st[4 * i]);
                        const double dr = (double)(st[4 * i + 3] - st[4 * i + 2]);
                        if (dr > 0) f.push_back(dc / dr * 100e6);
                    }
                    std::sort(f.begin(), f.end());
                    clk = f.empty() ? 2.4e9 : f[f.size() / 2];
                }
            }
            const double clocks = best * 1e-3 * clk;
            const double per = clocks / ((double)w * iters * per_iter);
            printf(", \"w%d\": {\"cyc\": %.3f, \"ms\": %.3f, \"GHz\": %.3f}", w, per, best, clk / 1e9);
        }
        printf("}");
        fflush(stdout);
    }
    printf("\n]}\n");
    return 0;
}
