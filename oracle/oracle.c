/*
 * oracle.c -- CPU restatement of FlakeCache/chunker's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product path (chunker_amd/) never links or calls it.
 *
 * What it restates (all citations are into /root/reference unless noted):
 *   - ChunkingOptions::resolve/validate        src/chunking.rs:173-231
 *   - fastcdc 4.0.1 v2020 FastCDC::new / Iterator / cut_gear (un-vendored crate,
 *     Cargo.lock:530-533; call sites src/chunking.rs:334, :553)  [ext]
 *     restated from the published crate, SURVEY.md Appendix A.
 *   - chunk_descriptors_with_hash              src/chunking.rs:323-374
 *     (serial scan, then per-chunk digest on a thread pool -- rayon's role)
 *   - drain_finalized_chunks / PushChunker     src/chunking.rs:541-673, :753-829
 *   - sha256_hash_raw                          src/hashing.rs:36-44  (FIPS 180-4;
 *     SHA-NI when the host CPU has it, as sha2 0.11 does through cpufeatures)
 *   - blake3::hash                             src/chunking.rs:68-71 (BLAKE3 spec)
 *
 * Parity status: SHA-256 is pinned by hashlib (independent) and the KAT at
 * src/lib.rs:54-69; BLAKE3 by the KAT at src/hashing.rs:173-182 and, for tree mode
 * (multi-leaf inputs), by the published BLAKE3 test vectors for 0..102400 bytes
 * (tests/golden/blake3_vectors.json); FastCDC is table-parametric: with the crate's
 * GEAR table it is pinned by src/chunking.rs:1266-1297, with the placeholder
 * table shipped in tables/ it is "parity unpinned" (see DESIGN.md).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
#endif

/* ------------------------------------------------------------------------- */
/* status codes (mirror ChunkingError variants, src/chunking.rs:33-51)        */
/* ------------------------------------------------------------------------- */
enum {
    OR_OK = 0,
    OR_E_BOUNDS = 1,
    OR_E_IO = 2,
    OR_E_ZERO_LENGTH = 3,
    OR_E_INVALID_OPTIONS = 4,
    OR_E_BUFFER_LIMIT = 5,
    OR_E_CAPACITY = 6,
};

typedef struct {
    uint64_t offset;
    uint64_t length;
    uint8_t hash[32];
} or_desc;

/* fastcdc::v2020 range constants [ext] (pinned by src/chunking.rs:1401-1415,
 * tests/streaming_chunking.rs:167-182) */
#define MINIMUM_MIN 64ull
#define MINIMUM_MAX 1048576ull
#define AVERAGE_MIN 256ull
#define AVERAGE_MAX 4194304ull
#define MAXIMUM_MIN 1024ull
#define MAXIMUM_MAX 16777216ull

static uint64_t g_gear[256];
static uint64_t g_masks[26];

void or_set_tables(const uint64_t *gear, const uint64_t *masks) {
    memcpy(g_gear, gear, sizeof g_gear);
    memcpy(g_masks, masks, sizeof g_masks);
}

/* ChunkingOptions::validate -- src/chunking.rs:190-231; same messages. */
int or_validate(uint64_t mn, uint64_t avg, uint64_t mx, char *msg, size_t cap) {
    char buf[160];
    buf[0] = 0;
    int st = OR_OK;
    if (mn < MINIMUM_MIN || mn > MINIMUM_MAX) {
        snprintf(buf, sizeof buf, "min_size must be in %llu..=%llu, got %llu",
                 MINIMUM_MIN, MINIMUM_MAX, (unsigned long long)mn);
        st = OR_E_INVALID_OPTIONS;
    } else if (avg < AVERAGE_MIN || avg > AVERAGE_MAX) {
        snprintf(buf, sizeof buf, "avg_size must be in %llu..=%llu, got %llu",
                 AVERAGE_MIN, AVERAGE_MAX, (unsigned long long)avg);
        st = OR_E_INVALID_OPTIONS;
    } else if (mx < MAXIMUM_MIN || mx > MAXIMUM_MAX) {
        snprintf(buf, sizeof buf, "max_size must be in %llu..=%llu, got %llu",
                 MAXIMUM_MIN, MAXIMUM_MAX, (unsigned long long)mx);
        st = OR_E_INVALID_OPTIONS;
    } else if (mn > avg) {
        snprintf(buf, sizeof buf, "min_size must be <= avg_size");
        st = OR_E_INVALID_OPTIONS;
    } else if (avg > mx) {
        snprintf(buf, sizeof buf, "avg_size must be <= max_size");
        st = OR_E_INVALID_OPTIONS;
    }
    if (msg && cap) {
        strncpy(msg, buf, cap - 1);
        msg[cap - 1] = 0;
    }
    return st;
}

/* fastcdc v2020 `logarithm2`: f64 log2, rounded half away from zero. [ext] */
static uint32_t logarithm2(uint32_t v) { return (uint32_t)round(log2((double)v)); }

typedef struct {
    uint64_t min, avg, max;
    uint64_t mask_s, mask_l, mask_s_ls, mask_l_ls;
} cdc_params;

/* FastCDC::new -> with_level(.., Normalization::Level1) [ext]: bits+1 / bits-1. */
static void cdc_init(cdc_params *p, uint64_t mn, uint64_t avg, uint64_t mx) {
    uint32_t bits = logarithm2((uint32_t)avg);
    p->min = mn;
    p->avg = avg;
    p->max = mx;
    p->mask_s = g_masks[bits + 1];
    p->mask_l = g_masks[bits - 1];
    p->mask_s_ls = p->mask_s << 1;
    p->mask_l_ls = p->mask_l << 1;
}

/* cut_gear [ext].  `src` = bytes from the chunk start,
 * `len` = bytes remaining in the source.  Returns the chunk length.  Two bytes per
 * iteration through GEAR_LS, exactly as the crate does. */
static uint64_t cut_gear(const cdc_params *p, const uint8_t *src, uint64_t len) {
    uint64_t remaining = len;
    if (remaining <= p->min) return remaining;
    uint64_t center = p->avg;
    if (remaining > p->max)
        remaining = p->max;
    else if (remaining < center)
        center = remaining;
    uint64_t index = p->min / 2;
    uint64_t hash = 0;
    while (index < center / 2) {
        uint64_t a = index * 2;
        hash = (hash << 2) + (g_gear[src[a]] << 1);
        if ((hash & p->mask_s_ls) == 0) return a;
        hash = hash + g_gear[src[a + 1]];
        if ((hash & p->mask_s) == 0) return a + 1;
        index++;
    }
    while (index < remaining / 2) {
        uint64_t a = index * 2;
        hash = (hash << 2) + (g_gear[src[a]] << 1);
        if ((hash & p->mask_l_ls) == 0) return a;
        hash = hash + g_gear[src[a + 1]];
        if ((hash & p->mask_l) == 0) return a + 1;
        index++;
    }
    return remaining;
}

/* FastCDC iterator [ext]: advance until `remaining == 0`.  Writes (offset,len)
 * pairs; returns the count, or SIZE_MAX when `cap` is too small. */
size_t or_fastcdc(const uint8_t *data, uint64_t len, uint64_t mn, uint64_t avg, uint64_t mx,
                  uint64_t *offs, uint64_t *lens, size_t cap) {
    cdc_params p;
    cdc_init(&p, mn, avg, mx);
    uint64_t processed = 0;
    size_t n = 0;
    while (processed < len) {
        uint64_t cut = cut_gear(&p, data + processed, len - processed);
        if (cut == 0) break;
        if (n >= cap) return (size_t)-1;
        offs[n] = processed;
        lens[n] = cut;
        n++;
        processed += cut;
    }
    return n;
}

/* ------------------------------------------------------------------------- */
/* SHA-256 (FIPS 180-4)                                                       */
/* ------------------------------------------------------------------------- */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static const uint32_t H256[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

#define ROR32(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_blocks_scalar(uint32_t st[8], const uint8_t *p, size_t nblk) {
    for (size_t b = 0; b < nblk; b++, p += 64) {
        uint32_t w[64];
        for (int i = 0; i < 16; i++)
            w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) |
                   ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
        for (int i = 16; i < 64; i++) {
            uint32_t s0 = ROR32(w[i - 15], 7) ^ ROR32(w[i - 15], 18) ^ (w[i - 15] >> 3);
            uint32_t s1 = ROR32(w[i - 2], 17) ^ ROR32(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = st[0], bb = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
        for (int i = 0; i < 64; i++) {
            uint32_t t1 = h + (ROR32(e, 6) ^ ROR32(e, 11) ^ ROR32(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
            uint32_t t2 = (ROR32(a, 2) ^ ROR32(a, 13) ^ ROR32(a, 22)) + ((a & bb) ^ (a & c) ^ (bb & c));
            h = g; g = f; f = e; e = d + t1; d = c; c = bb; bb = a; a = t1 + t2;
        }
        st[0] += a; st[1] += bb; st[2] += c; st[3] += d;
        st[4] += e; st[5] += f; st[6] += g; st[7] += h;
    }
}

#if defined(__x86_64__)
/* SHA-NI block function (Intel SHA extensions), used when the host has them. */
__attribute__((target("sha,sse4.1"))) static void sha256_blocks_ni(uint32_t st[8], const uint8_t *p,
                                                                  size_t nblk) {
    const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i TMP = _mm_loadu_si128((const __m128i *)&st[0]);
    __m128i STATE1 = _mm_loadu_si128((const __m128i *)&st[4]);
    TMP = _mm_shuffle_epi32(TMP, 0xB1);          /* CDAB */
    STATE1 = _mm_shuffle_epi32(STATE1, 0x1B);    /* EFGH */
    __m128i STATE0 = _mm_alignr_epi8(TMP, STATE1, 8); /* ABEF */
    STATE1 = _mm_blend_epi16(STATE1, TMP, 0xF0);      /* CDGH */
    for (size_t b = 0; b < nblk; b++, p += 64) {
        __m128i ABEF_SAVE = STATE0, CDGH_SAVE = STATE1, MSG, M0, M1, M2, M3;
        M0 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 0)), MASK);
        M1 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 16)), MASK);
        M2 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 32)), MASK);
        M3 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)(p + 48)), MASK);
        __m128i W[4] = {M0, M1, M2, M3};
        for (int r = 0; r < 16; r++) {
            __m128i k = _mm_loadu_si128((const __m128i *)&K256[4 * r]);
            __m128i cur = W[r & 3];
            MSG = _mm_add_epi32(cur, k);
            STATE1 = _mm_sha256rnds2_epu32(STATE1, STATE0, MSG);
            MSG = _mm_shuffle_epi32(MSG, 0x0E);
            STATE0 = _mm_sha256rnds2_epu32(STATE0, STATE1, MSG);
            if (r < 12) {
                /* W[r+4] = sha256msg2(sha256msg1(W[r], W[r+1]) + alignr(W[r+3], W[r+2], 4), W[r+3]) */
                __m128i t = _mm_sha256msg1_epu32(W[r & 3], W[(r + 1) & 3]);
                t = _mm_add_epi32(t, _mm_alignr_epi8(W[(r + 3) & 3], W[(r + 2) & 3], 4));
                W[r & 3] = _mm_sha256msg2_epu32(t, W[(r + 3) & 3]);
            }
        }
        STATE0 = _mm_add_epi32(STATE0, ABEF_SAVE);
        STATE1 = _mm_add_epi32(STATE1, CDGH_SAVE);
    }
    TMP = _mm_shuffle_epi32(STATE0, 0x1B);       /* FEBA */
    STATE1 = _mm_shuffle_epi32(STATE1, 0xB1);    /* DCHG */
    STATE0 = _mm_blend_epi16(TMP, STATE1, 0xF0); /* DCBA */
    STATE1 = _mm_alignr_epi8(STATE1, TMP, 8);    /* ABEF */
    _mm_storeu_si128((__m128i *)&st[0], STATE0);
    _mm_storeu_si128((__m128i *)&st[4], STATE1);
}

static int g_has_shani = -1;
static int has_shani(void) {
    if (g_has_shani < 0) {
        unsigned a, b, c, d;
        g_has_shani = 0;
        if (__get_cpuid_count(7, 0, &a, &b, &c, &d)) g_has_shani = (b >> 29) & 1;
    }
    return g_has_shani;
}
#endif

static int g_force_scalar = 0;
void or_sha256_force_scalar(int on) { g_force_scalar = on; }
int or_sha256_uses_shani(void) {
#if defined(__x86_64__)
    return !g_force_scalar && has_shani();
#else
    return 0;
#endif
}

static void sha256_blocks(uint32_t st[8], const uint8_t *p, size_t nblk) {
#if defined(__x86_64__)
    if (!g_force_scalar && has_shani()) {
        sha256_blocks_ni(st, p, nblk);
        return;
    }
#endif
    sha256_blocks_scalar(st, p, nblk);
}

void or_sha256(const uint8_t *d, uint64_t n, uint8_t out[32]) {
    uint32_t st[8];
    memcpy(st, H256, sizeof st);
    uint64_t full = n / 64;
    sha256_blocks(st, d, full);
    uint8_t tail[128];
    uint64_t rem = n - full * 64;
    memset(tail, 0, sizeof tail);
    memcpy(tail, d + full * 64, rem);
    tail[rem] = 0x80;
    size_t tb = (rem + 1 + 8 <= 64) ? 1 : 2;
    uint64_t bits = n * 8;
    for (int i = 0; i < 8; i++) tail[tb * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha256_blocks(st, tail, tb);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)st[i];
    }
}

/* ------------------------------------------------------------------------- */
/* BLAKE3 (hash mode, 32-byte output), restated from the BLAKE3 specification */
/* ------------------------------------------------------------------------- */
enum { B3_CHUNK_START = 1, B3_CHUNK_END = 2, B3_PARENT = 4, B3_ROOT = 8 };
static const uint8_t B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

#define B3G(a, b, c, d, x, y)           \
    do {                                \
        s[a] = s[a] + s[b] + (x);       \
        s[d] = ROR32(s[d] ^ s[a], 16);  \
        s[c] = s[c] + s[d];             \
        s[b] = ROR32(s[b] ^ s[c], 12);  \
        s[a] = s[a] + s[b] + (y);       \
        s[d] = ROR32(s[d] ^ s[a], 8);   \
        s[c] = s[c] + s[d];             \
        s[b] = ROR32(s[b] ^ s[c], 7);   \
    } while (0)

static void b3_compress(const uint32_t cv[8], const uint32_t mw[16], uint64_t counter, uint32_t blen,
                        uint32_t flags, uint32_t out[16]) {
    uint32_t s[16], m[16], t[16];
    for (int i = 0; i < 8; i++) s[i] = cv[i];
    for (int i = 0; i < 4; i++) s[8 + i] = H256[i];
    s[12] = (uint32_t)counter;
    s[13] = (uint32_t)(counter >> 32);
    s[14] = blen;
    s[15] = flags;
    memcpy(m, mw, sizeof m);
    for (int r = 0; r < 7; r++) {
        B3G(0, 4, 8, 12, m[0], m[1]);
        B3G(1, 5, 9, 13, m[2], m[3]);
        B3G(2, 6, 10, 14, m[4], m[5]);
        B3G(3, 7, 11, 15, m[6], m[7]);
        B3G(0, 5, 10, 15, m[8], m[9]);
        B3G(1, 6, 11, 12, m[10], m[11]);
        B3G(2, 7, 8, 13, m[12], m[13]);
        B3G(3, 4, 9, 14, m[14], m[15]);
        for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]];
        memcpy(m, t, sizeof m);
    }
    for (int i = 0; i < 8; i++) {
        out[i] = s[i] ^ s[i + 8];
        out[i + 8] = s[i + 8] ^ cv[i];
    }
}

static void b3_words(const uint8_t *p, size_t n, uint32_t w[16]) {
    uint8_t blk[64];
    memset(blk, 0, 64);
    memcpy(blk, p, n);
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)blk[4 * i] | ((uint32_t)blk[4 * i + 1] << 8) | ((uint32_t)blk[4 * i + 2] << 16) |
               ((uint32_t)blk[4 * i + 3] << 24);
}

/* Chaining value of one 1 KiB leaf (`n` <= 1024 bytes) with leaf index `ctr`. */
static void b3_leaf(const uint8_t *p, size_t n, uint64_t ctr, int root, uint32_t cv[8]) {
    uint32_t st[8], w[16], o[16];
    memcpy(st, H256, sizeof st);
    size_t nblk = n ? (n + 63) / 64 : 1;
    for (size_t j = 0; j < nblk; j++) {
        size_t bl = (j + 1 < nblk) ? 64 : n - j * 64;
        uint32_t fl = (j == 0 ? B3_CHUNK_START : 0) | (j + 1 == nblk ? B3_CHUNK_END : 0);
        if (root && j + 1 == nblk) fl |= B3_ROOT;
        b3_words(p + j * 64, bl, w);
        b3_compress(st, w, ctr, (uint32_t)bl, fl, o);
        memcpy(st, o, 32);
    }
    memcpy(cv, st, 32);
}

static void b3_parent(const uint32_t l[8], const uint32_t r[8], int root, uint32_t cv[8]) {
    uint32_t w[16], o[16];
    memcpy(w, l, 32);
    memcpy(w + 8, r, 32);
    b3_compress(H256, w, 0, 64, B3_PARENT | (root ? B3_ROOT : 0), o);
    memcpy(cv, o, 32);
}

/* Recursive left-complete tree: left subtree = largest power of two < n leaves. */
static void b3_subtree(const uint8_t *p, uint64_t n_bytes, uint64_t first_leaf, int root, uint32_t cv[8]) {
    uint64_t leaves = n_bytes ? (n_bytes + 1023) / 1024 : 1;
    if (leaves == 1) {
        b3_leaf(p, (size_t)n_bytes, first_leaf, root, cv);
        return;
    }
    uint64_t left = 1;
    while (left * 2 < leaves) left *= 2;
    uint32_t lcv[8], rcv[8];
    b3_subtree(p, left * 1024, first_leaf, 0, lcv);
    b3_subtree(p + left * 1024, n_bytes - left * 1024, first_leaf + left, 0, rcv);
    b3_parent(lcv, rcv, root, cv);
}

void or_blake3(const uint8_t *d, uint64_t n, uint8_t out[32]) {
    uint32_t cv[8];
    b3_subtree(d, n, 0, 1, cv);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)cv[i];
        out[4 * i + 1] = (uint8_t)(cv[i] >> 8);
        out[4 * i + 2] = (uint8_t)(cv[i] >> 16);
        out[4 * i + 3] = (uint8_t)(cv[i] >> 24);
    }
}

/* Second, structurally different BLAKE3 tree: incremental chaining-value stack
 * (merge while the completed-leaf count has trailing zero bits).  Used only to
 * cross-check the recursive form above on multi-leaf inputs. */
void or_blake3_stack(const uint8_t *d, uint64_t n, uint8_t out[32]) {
    uint64_t leaves = n ? (n + 1023) / 1024 : 1;
    uint32_t stack[64][8];
    int sp = 0;
    uint32_t cv[8];
    for (uint64_t i = 0; i < leaves; i++) {
        uint64_t off = i * 1024;
        size_t len = (size_t)((n - off) < 1024 ? (n - off) : 1024);
        if (i + 1 == leaves) {
            b3_leaf(d + off, len, i, leaves == 1, cv);
            while (sp > 0) {
                sp--;
                b3_parent(stack[sp], cv, sp == 0, cv);
            }
        } else {
            b3_leaf(d + off, len, i, 0, cv);
            uint64_t total = i + 1;
            while ((total & 1) == 0) {
                sp--;
                b3_parent(stack[sp], cv, 0, cv);
                total >>= 1;
            }
            memcpy(stack[sp++], cv, 32);
        }
    }
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)cv[i];
        out[4 * i + 1] = (uint8_t)(cv[i] >> 8);
        out[4 * i + 2] = (uint8_t)(cv[i] >> 16);
        out[4 * i + 3] = (uint8_t)(cv[i] >> 24);
    }
}

/* compute_hash -- src/chunking.rs:65-74 (0 = Blake3, 1 = Sha256 as HashAlgorithm order) */
static void compute_hash(const uint8_t *d, uint64_t n, int algo, uint8_t out[32]) {
    if (algo == 0)
        or_blake3(d, n, out);
    else
        or_sha256(d, n, out);
}

/* ------------------------------------------------------------------------- */
/* chunk_descriptors_with_hash -- src/chunking.rs:323-374                     */
/* ------------------------------------------------------------------------- */
typedef struct {
    const uint8_t *data;
    or_desc *out;
    size_t n;
    int algo;
    size_t next; /* shared work counter (atomic) */
} hash_job;

static void *hash_worker(void *arg) {
    hash_job *j = (hash_job *)arg;
    for (;;) {
        size_t i = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (i >= j->n) break;
        compute_hash(j->data + j->out[i].offset, j->out[i].length, j->algo, j->out[i].hash);
    }
    return NULL;
}

/* Phase 2 of chunk_descriptors_with_hash: digests on a pool of `nthreads` (rayon). */
void or_hash_descs(const uint8_t *data, or_desc *out, size_t n, int algo, int nthreads) {
    hash_job job = {data, out, n, algo, 0};
    if (nthreads <= 1 || n <= 1) {
        hash_worker(&job);
        return;
    }
    pthread_t th[256];
    int nt = nthreads > 256 ? 256 : nthreads;
    for (int t = 0; t < nt; t++) pthread_create(&th[t], NULL, hash_worker, &job);
    for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
}

int or_chunk_descriptors(const uint8_t *data, uint64_t len, uint64_t mn, uint64_t avg, uint64_t mx, int algo,
                         or_desc *out, size_t cap, size_t *n_out, int nthreads) {
    int st = or_validate(mn, avg, mx, NULL, 0);
    if (st) return st;
    cdc_params p;
    cdc_init(&p, mn, avg, mx);
    /* Phase 1: the serial FastCDC pass (src/chunking.rs:334-336). */
    uint64_t processed = 0;
    size_t n = 0;
    while (processed < len) {
        uint64_t cut = cut_gear(&p, data + processed, len - processed);
        if (cut == 0) break;
        if (n >= cap) return OR_E_CAPACITY;
        out[n].offset = processed;
        out[n].length = cut;
        n++;
        processed += cut;
    }
    *n_out = n;
    /* Phase 2: per-chunk digest in parallel (src/chunking.rs:340-368). */
    or_hash_descs(data, out, n, algo, nthreads);
    return OR_OK;
}

/* ------------------------------------------------------------------------- */
/* PushChunker / drain_finalized_chunks -- src/chunking.rs:541-673, :753-829  */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint8_t *buf;
    uint64_t len, cap;
    uint64_t position;
    uint64_t mn, avg, mx;
    int algo;
    int finished;
    int nthreads; /* digest pool when a drain emits > 4 chunks (rayon par_iter, src/chunking.rs:637-641) */
} or_push;

or_push *or_push_new(uint64_t mn, uint64_t avg, uint64_t mx, int algo, int *status) {
    int st = or_validate(mn, avg, mx, NULL, 0);
    if (status) *status = st;
    if (st) return NULL;
    or_push *h = (or_push *)calloc(1, sizeof *h);
    h->mn = mn;
    h->avg = avg;
    h->mx = mx;
    h->algo = algo;
    h->nthreads = 1;
    return h;
}

void or_push_set_threads(or_push *h, int nthreads) { h->nthreads = nthreads > 0 ? nthreads : 1; }

void or_push_free(or_push *h) {
    if (!h) return;
    free(h->buf);
    free(h);
}

uint64_t or_push_bytes_consumed(const or_push *h) { return h->position + h->len; }

static int drain(or_push *h, int eof, or_desc *out, size_t cap, size_t *n_out) {
    size_t n = 0;
    uint64_t total = 0;
    if (h->len > 0 && (h->len >= h->mn || eof)) {
        cdc_params p;
        cdc_init(&p, h->mn, h->avg, h->mx);
        uint64_t processed = 0;
        while (processed < h->len) {
            uint64_t cut = cut_gear(&p, h->buf + processed, h->len - processed);
            if (cut == 0) return OR_E_ZERO_LENGTH;
            int touches_end = processed + cut == h->len;
            if (touches_end && !eof && cut < h->mx) break; /* retained tail (:579-584) */
            if (n >= cap) return OR_E_CAPACITY;
            out[n].offset = h->position + processed;
            out[n].length = cut;
            n++;
            processed += cut;
        }
        total = processed;
    }
    if (n > 4 && h->nthreads > 1) /* offsets are stream offsets: rebase the buffer pointer */
        or_hash_descs(h->buf - h->position, out, n, h->algo, h->nthreads);
    else
        for (size_t i = 0; i < n; i++)
            compute_hash(h->buf + (out[i].offset - h->position), out[i].length, h->algo, out[i].hash);
    memmove(h->buf, h->buf + total, h->len - total);
    h->len -= total;
    h->position += total;
    if (eof && h->len > 0) { /* defensive EOF remainder (:651-670) */
        if (n >= cap) return OR_E_CAPACITY;
        out[n].offset = h->position;
        out[n].length = h->len;
        compute_hash(h->buf, h->len, h->algo, out[n].hash);
        n++;
        h->position += h->len;
        h->len = 0;
    }
    *n_out = n;
    return OR_OK;
}

int or_push_push(or_push *h, const uint8_t *d, uint64_t n, or_desc *out, size_t cap, size_t *n_out) {
    *n_out = 0;
    if (h->finished) return OR_E_INVALID_OPTIONS; /* "push called after finish" (:789-793) */
    if (n == 0) return OR_OK;
    if (h->len + n > h->cap) {
        uint64_t nc = (h->len + n) * 2;
        h->buf = (uint8_t *)realloc(h->buf, nc);
        h->cap = nc;
    }
    memcpy(h->buf + h->len, d, n);
    h->len += n;
    return drain(h, 0, out, cap, n_out);
}

int or_push_finish(or_push *h, or_desc *out, size_t cap, size_t *n_out) {
    h->finished = 1;
    return drain(h, 1, out, cap, n_out);
}
