// scan_common.h -- device helpers shared by the product candidate scan (scan.hip: k_scan,
// k_scan_flat32) and the diagnostics build's alternative scan kernels (scan_diag.hip).
#pragma once
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
#define QPIECE 64u  // bytes per hashed piece (one 64-bit `hits` bit each)

__device__ __forceinline__ uint64_t lds_gear(const char *base, uint32_t addr) {
    return *reinterpret_cast<const uint64_t *>(base + addr);
}

// ---------------------------------------------------------------------------
// K1 (the product kernel).  One lane per CG_SEG segment of the flat batch buffer, after
// a CG_HALO warm-up, as the round-1 quad-transpose kernel (k_scan_quad, diagnostics build), but:
//  * every lane loads its OWN segment (4 x dwordx4 per 64-B piece, both pieces of a
//    128-B line in one burst, two to three pieces ahead), so no quad transpose
//    (the DPP movs + selects cost ~1 VALU per byte in k_scan);
//  * the hash is kept as H' = H << 16 (mod 2^64) with the LDS table pre-shifted
//    (GEAR[v] << 16): exact for H's bits 0..47, where every FastCDC mask lives, and
//    H's bits 16..47 are H''s high dword -- the prefilter test is one v_and_b32 on it
//    (mask bits 12..15 are left to the exact re-walk), folded two bytes at a time
//    into a running v_min3_u32;
//  * a lookup address (byte << 8 | copy offset) is one SDWA v_mov_b32 writing the
//    byte into bits 8..15 of a register that keeps the lane's copy offset in bits
//    0..7 (v_perm_b32 in k_scan is a half-rate instruction on gfx950).
// Per byte: 1 SDWA mov + 1 ds_read_b64 + 1 v_lshl_add_u64 + 1 v_and_b32 + 1/2 v_min3_u32.
// ---------------------------------------------------------------------------
#define SCAN_SHIFT 16u

template <int B>
__device__ __forceinline__ void sdwa_byte_addr(uint32_t &a, uint32_t w) {
    if constexpr (B == 0)
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(a) : "v"(w));
    else if constexpr (B == 1)
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1" : "+v"(a) : "v"(w));
    else if constexpr (B == 2)
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2" : "+v"(a) : "v"(w));
    else
        asm("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_3" : "+v"(a) : "v"(w));
}

// the 4 lookups of dword w: addresses in a[0..3] (bits 0..7 = this lane's copy offset)
__device__ __forceinline__ void lookup4(const char *gbase, uint32_t (&a)[4], uint32_t w, uint64_t (&g)[4]) {
    sdwa_byte_addr<0>(a[0], w);
    sdwa_byte_addr<1>(a[1], w);
    sdwa_byte_addr<2>(a[2], w);
    sdwa_byte_addr<3>(a[3], w);
#pragma unroll
    for (int b = 0; b < 4; ++b) g[b] = lds_gear(gbase, a[b]);
}

// Lean table (round 6): 8 copies at a 64-byte entry stride -- 16 KiB, 18 KiB with the
// candidate slots -- so a scan workgroup fits on a CU beside two SHA-256 digest workgroups
// (2 x 69.7 KiB) of the digest pipeline's merged launches.  The byte no longer lands on a
// byte boundary of the address, so an address takes two VALU (extract, shift-or) instead of
// the SDWA mov's one, and the 4 lanes sharing a copy (of 32 per ds_read_b64 group) meet on a
// bank pair when their bytes agree mod 4.
#define GEAR_COPIES_LEAN 8u
__device__ __forceinline__ void lookup4_lean(const char *gbase, uint32_t lo, uint32_t w, uint64_t (&g)[4]) {
#pragma unroll
    for (int b = 0; b < 4; ++b) g[b] = lds_gear(gbase, (__builtin_amdgcn_ubfe(w, 8 * b, 8) << 6) | lo);
}
// The table fill of a 512-thread workgroup: two threads per entry, each storing half its copies
// (rotated by the entry so a store group spreads over the banks).
template <uint32_t GC>
__device__ __forceinline__ void gear_fill(uint64_t *s_gear, uint64_t gv, uint32_t ge, uint32_t tid) {
    static_assert(GC == 32 || GC == GEAR_COPIES_LEAN, "32 or 8 copies");
#pragma unroll
    for (uint32_t j = 0; j < GC / 2; ++j) s_gear[ge * GC + (((tid & 1u) * (GC / 2) + j + ge) & (GC - 1))] = gv;
}
template <uint32_t GC>
__device__ __forceinline__ void gear_look(const char *gbase, uint32_t (&a)[4], uint32_t lo, uint32_t w,
                                          uint64_t (&g)[4]) {
    if constexpr (GC == 32)
        lookup4(gbase, a, w, g);
    else
        lookup4_lean(gbase, lo, w, g);
}

__device__ __forceinline__ uint32_t gear_flags64(uint64_t h, uint64_t ms, uint64_t ml) {
    return ((h & ms) == 0 ? CG_FLAG_S : 0u) | ((h & ml) == 0 ? CG_FLAG_L : 0u);
}

#define DPP_WAVE_ROR1 0x13C

__device__ __forceinline__ uint32_t wave_ror1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_WAVE_ROR1, 0xf, 0xf, false);
}
// The same rotation as one v_add_u32_dpp of an opaque zero: a v_mov_b32 (DPP or not)
// issues in ~8 clocks on gfx950, a DPP ALU op in ~4.9 (profiles/r02_v7_diag_ops_mov.json).
__device__ __forceinline__ uint32_t wave_ror1_add(uint32_t v, uint32_t zero) {
    // bound_ctrl set (no lane of a rotation lacks a source) so the DPP combine applies
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_WAVE_ROR1, 0xf, 0xf, true) + zero;
}

// (a << 1) + b as one v_lshl_add_u64 (left to itself the compiler re-associates the
// chain into shift-by-2 pairs: 3 instructions per 2 bytes)
__device__ __forceinline__ uint64_t shl1_add(uint64_t a, uint64_t b) {
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// (a << S) + b, S in 1..4 (the shift range of v_lshl_add_u64)
template <int S>
__device__ __forceinline__ uint64_t shl_add(uint64_t a, uint64_t b) {
    static_assert(S >= 1 && S <= 4, "v_lshl_add_u64 shifts by 1..4");
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "n"(S), "v"(b));
    return r;
}

// Segment flush of the flat scans: the first n of the wave's LDS slots (`slots`, wave-uniform
// base) to `dst` (the segment's row of seg_cand, wave-uniform).  The lane index is made here
// by an opaque v_mbcnt pair, so the slot and store addresses cannot be hoisted out of the
// row loop: left to itself the compiler formed both once per kernel, kept them live across
// the row loop and, at 128 VGPRs, spilled them to scratch -- and each reload's
// `s_waitcnt vmcnt` drained the row ring on every segment holding a candidate.  The store
// takes the uniform base in SGPRs plus a 32-bit lane offset (global_store ... saddr).
__device__ __forceinline__ void flush_slots(uint32_t *__restrict__ dst, const uint32_t *slots, uint32_t n) {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    if (l < n) dst[l] = slots[l];
}

}  // namespace cg
