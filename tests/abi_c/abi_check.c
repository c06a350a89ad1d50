/*
 * abi_check.c -- a native C consumer of include/chunker_gpu.h, linked against
 * libchunker_amd.so the way the Rust shim (rust/chunker-hip) links it.
 * It checks what an `extern "C"` binding relies on and Python ctypes cannot show:
 *
 *  - compile time: cg_desc's size and field offsets (the shim's #[repr(C)] CgDesc), the
 *    status / algorithm / object-kind enum values its match arms use, the ABI version;
 *  - `abi_check nodevice`: every entry point the shim declares links and answers
 *    without a GPU -- option validation with the reference's messages
 *    (src/chunking.rs:190-231), capacities, tables, ChunkingError fields through
 *    cg_last_error_detail, and CG_E_NO_DEVICE (no CPU fallback) from each compute entry;
 *  - `abi_check cases <file>`: on a GPU, every case of the file (written by
 *    tests/test_abi_c.py from tests/golden/cdc_golden.json) through
 *    cg_chunk_descriptors, cg_chunk_batch, the push handle (uneven pushes) and the
 *    stream handle -- each must give the golden (offset, length, hash) list.
 *
 * Test infrastructure only: built by tests/test_abi_c.py with gcc.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "chunker_gpu.h"

_Static_assert(sizeof(cg_desc) == 48, "cg_desc is 48 bytes (CgDesc)");
_Static_assert(offsetof(cg_desc, offset) == 0, "offset at 0");
_Static_assert(offsetof(cg_desc, length) == 8, "length at 8");
_Static_assert(offsetof(cg_desc, hash) == 16, "hash at 16");
_Static_assert(sizeof(((cg_desc *)0)->hash) == 32, "32-byte digest");
_Static_assert(CG_ABI_VERSION == 3u, "ABI version 3");
_Static_assert(CG_OK == 0 && CG_E_BOUNDS == 1 && CG_E_IO == 2 && CG_E_ZERO_LENGTH_CHUNK == 3 &&
                   CG_E_INVALID_OPTIONS == 4 && CG_E_BUFFER_LIMIT == 5 && CG_E_CAPACITY == 6 &&
                   CG_E_NO_DEVICE == 7 && CG_E_TABLES == 8,
               "status codes: 1..5 = ChunkingError variants in declaration order");
_Static_assert(CG_BLAKE3 == 0 && CG_SHA256 == 1, "HashAlgorithm order (src/chunking.rs:53-58)");
_Static_assert(CG_KIND_CHUNK == 1 && CG_KIND_LEVEL1_MANIFEST == 3 && CG_KIND_COMMIT == 7,
               "ObjectKind discriminants (crates/core/cas/src/lib.rs:31-48)");

static int failures = 0;
#define CHECK(cond, ...)                                              \
    do {                                                              \
        if (!(cond)) {                                                \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);      \
            fprintf(stderr, __VA_ARGS__);                             \
            fprintf(stderr, " [last error: %s]\n", cg_last_error_message()); \
            ++failures;                                               \
        }                                                             \
    } while (0)

static int nodevice(void) {
    char msg[256];
    uint64_t d[3];
    CHECK(cg_abi_version() == CG_ABI_VERSION, "abi version %u", cg_abi_version());
    /* ChunkingOptions::resolve/validate: defaults, then each range in order */
    CHECK(cg_validate(0, 0, 0, msg, sizeof msg) == CG_OK && msg[0] == 0, "defaults valid");
    CHECK(cg_last_error_detail(d) == CG_OK && d[0] == 0 && d[1] == 0 && d[2] == 0, "detail cleared");
    CHECK(cg_validate(32, 64, 128, msg, sizeof msg) == CG_E_INVALID_OPTIONS &&
              strcmp(msg, "min_size must be in 64..=1048576, got 32") == 0,
          "min message: %s", msg);
    CHECK(strcmp(cg_last_error_message(), msg) == 0, "thread-local message");
    CHECK(cg_validate(64, 4194305, 16777216, msg, sizeof msg) == CG_E_INVALID_OPTIONS &&
              strstr(msg, "avg_size must be in 256..=4194304") != NULL,
          "avg message: %s", msg);
    CHECK(cg_validate(64, 1024, 16777217, msg, sizeof msg) == CG_E_INVALID_OPTIONS &&
              strstr(msg, "max_size must be in 1024..=16777216") != NULL,
          "max message: %s", msg);
    CHECK(cg_validate(4096, 1024, 8192, msg, sizeof msg) == CG_E_INVALID_OPTIONS &&
              strcmp(msg, "min_size must be <= avg_size") == 0,
          "min<=avg: %s", msg);
    CHECK(cg_validate(64, 8192, 4096, NULL, 0) == CG_E_INVALID_OPTIONS, "avg<=max, NULL msg");
    CHECK(cg_last_error_detail(d) == CG_E_INVALID_OPTIONS, "detail status");
    CHECK(cg_capacity(0, 1024) == 0 && cg_capacity(1, 1024) == 1 && cg_capacity(10u << 20, 256u << 10) == 41,
          "capacity");
    /* tables: readable, placeholder flag, masks above bit 47 refused */
    static uint64_t gear[256], masks[26], bad[26];
    cg_get_cdc_tables(gear, masks);
    uint64_t g2[256];
    cg_get_gear_table(g2);
    CHECK(memcmp(gear, g2, sizeof g2) == 0, "gear table views agree");
    CHECK(cg_gear_is_placeholder() == 0 || cg_gear_is_placeholder() == 1, "placeholder flag");
    memcpy(bad, masks, sizeof bad);
    bad[20] |= 1ull << 48;
    CHECK(cg_set_cdc_tables(gear, bad) == CG_E_INVALID_OPTIONS, "mask bit 48 refused");
    CHECK(cg_set_cdc_tables(gear, masks) == CG_OK, "reinstall tables");
    CHECK(cg_tables_verified() == 0, "not verified without a device");
    /* ChunkingError::Bounds fields: a batch whose offsets do not start at 0 */
    uint64_t offs[3] = {5, 10, 40}, first[3];
    CHECK(cg_chunk_batch_device(NULL, offs, 2, 0, 0, 0, CG_SHA256, NULL, 0, first, NULL) == CG_E_BOUNDS, "bounds");
    CHECK(cg_last_error_detail(d) == CG_E_BOUNDS && d[0] == 40 && d[1] == 5 && d[2] == 0,
          "bounds fields %llu %llu %llu", (unsigned long long)d[0], (unsigned long long)d[1],
          (unsigned long long)d[2]);
    /* unknown object kind: InvalidOptions before any device work */
    uint8_t id[32];
    CHECK(cg_cas_id(NULL, 0, 0, id) == CG_E_INVALID_OPTIONS && strstr(cg_last_error_message(), "object kind"),
          "kind 0");
    /* every compute entry: CG_E_NO_DEVICE, never a CPU result */
    static uint8_t data[300000] __attribute__((aligned(64)));
    cg_desc out[64];
    size_t n = 0;
    int st = -1;
    uint64_t boffs[2] = {0, sizeof data};
    CHECK(cg_chunk_descriptors(data, sizeof data, 0, 0, 0, CG_SHA256, out, 64, &n) == CG_E_NO_DEVICE, "descriptors");
    CHECK(cg_chunk_batch(data, boffs, 1, 0, 0, 0, CG_BLAKE3, out, 64, first) == CG_E_NO_DEVICE, "batch");
    CHECK(cg_hash(data, 100, CG_SHA256, id) == CG_E_NO_DEVICE, "hash");
    CHECK(cg_cas_id(data, 100, CG_KIND_CHUNK, id) == CG_E_NO_DEVICE, "cas id");
    CHECK(cg_node_put(data, sizeof data, 4096, 16384, 65536, out, 64, &n, NULL, id) == CG_E_NO_DEVICE, "node put");
    cg_batch *b = NULL;
    CHECK(cg_chunk_batch_device_async(data, boffs, 1, 0, 0, 0, CG_SHA256, out, 64, NULL, &b) == CG_E_NO_DEVICE &&
              b == NULL,
          "async batch");
    b = NULL;
    CHECK(cg_chunk_batch_device_async_after(data, boffs, 1, 0, 0, 0, CG_SHA256, out, 64, NULL, NULL, &b) ==
                  CG_E_NO_DEVICE &&
              b == NULL,
          "async batch after an event");
    cg_pipeline *pl = (cg_pipeline *)1;
    CHECK(cg_pipeline_create(-1, 16, 2, &pl) == CG_E_NO_DEVICE && pl == NULL, "pipeline create");
    CHECK(cg_pipeline_create(0, 65, 2, &pl) == CG_E_INVALID_OPTIONS, "pipeline group above 64");
    CHECK(cg_pipeline_submit(NULL, data, boffs, 1, 0, 0, 0, CG_SHA256, out, 64, NULL, &b) == CG_E_IO,
          "pipeline submit without a pipeline");
    CHECK(cg_pipeline_flush(NULL) == CG_E_IO, "pipeline flush without a pipeline");
    double ps[6];
    CHECK(cg_pipeline_stats(NULL, ps) == CG_E_IO, "pipeline stats without a pipeline");
    cg_pipeline_destroy(NULL);
    void *ev = NULL;
    CHECK(cg_batch_event(NULL, &ev) == CG_E_IO, "batch event without a batch");
    const int devs[2] = {0, 0};
    cg_multi *mu = (cg_multi *)1;
    CHECK(cg_multi_create(devs, 2, 16, 2, &mu) == CG_E_NO_DEVICE && mu == NULL, "multi create");
    CHECK(cg_multi_create(devs, 0, 16, 2, &mu) == CG_E_IO, "multi create without devices");
    const uint8_t *shard_data[1] = {data};
    const uint64_t *shard_offs[1] = {boffs};
    const size_t shard_n[1] = {1};
    cg_multi_batch *mb = NULL;
    CHECK(cg_multi_submit(NULL, shard_data, shard_offs, shard_n, 0, 0, 0, CG_SHA256, out, 64, NULL, &mb) == CG_E_IO,
          "multi submit without a handle");
    CHECK(cg_multi_wait(NULL, first) == CG_E_IO, "multi wait without a batch");
    CHECK(cg_multi_flush(NULL) == CG_E_IO, "multi flush without a handle");
    cg_multi_destroy(NULL);
    cg_push *p = cg_push_new(0, 0, 0, CG_SHA256, &st);
    if (p) {
        CHECK(cg_push_push(p, data, sizeof data, out, 64, &n) == CG_E_NO_DEVICE, "push");
        cg_push_free(p);
    } else {
        CHECK(st == CG_E_NO_DEVICE, "push_new status %d", st);
    }
    cg_stream *s = cg_stream_new(0, 0, 0, CG_SHA256, 0, 0, &st);
    CHECK(s == NULL && st == CG_E_NO_DEVICE, "stream_new status %d", st);
    CHECK(cg_selftest() == CG_E_NO_DEVICE, "selftest");
    if (!failures) printf("abi_check nodevice: ok\n");
    return failures ? 1 : 0;
}

/* ---- GPU mode ----------------------------------------------------------------------- */

typedef struct {
    uint64_t len, mn, avg, mx;
    uint32_t algo, nchunks;
    uint8_t *data;
    cg_desc *want;
} Case;

static int read_u64(FILE *f, uint64_t *v) { return fread(v, 8, 1, f) == 1; }

static int same(const cg_desc *got, size_t n, const Case *c, const char *what, size_t idx) {
    if (n != c->nchunks) {
        fprintf(stderr, "FAIL case %zu %s: %zu chunks, golden %u\n", idx, what, n, c->nchunks);
        return 0;
    }
    for (size_t k = 0; k < n; ++k)
        if (got[k].offset != c->want[k].offset || got[k].length != c->want[k].length ||
            memcmp(got[k].hash, c->want[k].hash, 32) != 0) {
            fprintf(stderr, "FAIL case %zu %s: chunk %zu (%llu, %llu) vs golden (%llu, %llu)%s\n", idx, what, k,
                    (unsigned long long)got[k].offset, (unsigned long long)got[k].length,
                    (unsigned long long)c->want[k].offset, (unsigned long long)c->want[k].length,
                    memcmp(got[k].hash, c->want[k].hash, 32) ? " (digest differs)" : "");
            return 0;
        }
    return 1;
}

static int run_case(const Case *c, size_t idx) {
    int ok = 1;
    const size_t cap = cg_capacity(c->len, c->mn) + 1;
    cg_desc *out = calloc(cap, sizeof(cg_desc));
    size_t n = 0;
    /* chunk_descriptors_with_hash */
    int st = cg_chunk_descriptors(c->data, c->len, c->mn, c->avg, c->mx, (int)c->algo, out, cap, &n);
    if (st) {
        fprintf(stderr, "FAIL case %zu descriptors: status %d %s\n", idx, st, cg_last_error_message());
        ok = 0;
    } else {
        ok &= same(out, n, c, "cg_chunk_descriptors", idx);
    }
    /* a one-NAR host batch */
    uint64_t offs[2] = {0, c->len}, first[2] = {0, 0};
    memset(out, 0, cap * sizeof(cg_desc));
    st = cg_chunk_batch(c->data, offs, 1, c->mn, c->avg, c->mx, (int)c->algo, out, cap, first);
    ok &= st == CG_OK && first[0] == 0 && same(out, (size_t)first[1], c, "cg_chunk_batch", idx);
    /* PushChunker: uneven pushes, chunks appended as they become final */
    cg_push *p = cg_push_new(c->mn, c->avg, c->mx, (int)c->algo, &st);
    if (!p) {
        fprintf(stderr, "FAIL case %zu push_new: %d\n", idx, st);
        ok = 0;
    } else {
        size_t got = 0;
        uint64_t pos = 0, step = 1;
        while (pos < c->len && ok) {
            const uint64_t take = c->len - pos < step ? c->len - pos : step;
            size_t pc = cg_push_out_capacity(p, take), k = 0;
            cg_desc *tmp = calloc(pc ? pc : 1, sizeof(cg_desc));
            st = cg_push_push(p, c->data + pos, take, tmp, pc, &k);
            if (st || got + k > cap) ok = 0;
            else memcpy(out + got, tmp, k * sizeof(cg_desc));
            got += k;
            free(tmp);
            pos += take;
            step = step * 7 + 4093;
        }
        size_t pc = cg_push_out_capacity(p, 0), k = 0;
        cg_desc *tmp = calloc(pc ? pc : 1, sizeof(cg_desc));
        st = cg_push_finish(p, tmp, pc, &k);
        if (st || got + k > cap) ok = 0;
        else memcpy(out + got, tmp, k * sizeof(cg_desc));
        got += k;
        free(tmp);
        ok &= cg_push_bytes_consumed(p) == c->len;
        ok &= same(out, got, c, "cg_push_*", idx);
        cg_push_free(p);
    }
    /* pipelined stream: pushes of 64 KiB, take until drained */
    cg_stream *s = cg_stream_new(c->mn, c->avg, c->mx, (int)c->algo, 64 << 10, 64u << 20, &st);
    if (!s) {
        fprintf(stderr, "FAIL case %zu stream_new: %d %s\n", idx, st, cg_last_error_message());
        ok = 0;
    } else {
        size_t got = 0, k = 0;
        for (uint64_t pos = 0; pos < c->len && ok; pos += 64 << 10) {
            const uint64_t take = c->len - pos < (64 << 10) ? c->len - pos : (64 << 10);
            if (cg_stream_push(s, c->data + pos, take)) ok = 0;
            if (cg_stream_take(s, out + got, cap - got, &k, 0)) ok = 0;
            got += k;
        }
        if (cg_stream_finish(s)) ok = 0;
        while (ok) {
            if (cg_stream_take(s, out + got, cap - got, &k, 1)) ok = 0;
            got += k;
            if (k == 0 && cg_stream_pending(s) == 0) break;
        }
        ok &= cg_stream_bytes_consumed(s) == c->len;
        ok &= same(out, got, c, "cg_stream_*", idx);
        cg_stream_free(s);
    }
    free(out);
    return ok;
}

static int cases(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) {
        perror(path);
        return 2;
    }
    uint64_t count = 0;
    if (!read_u64(f, &count)) return 2;
    size_t passed = 0;
    for (size_t i = 0; i < count; ++i) {
        Case c;
        uint64_t hdr[2];
        if (!read_u64(f, &c.len) || !read_u64(f, &c.mn) || !read_u64(f, &c.avg) || !read_u64(f, &c.mx) ||
            fread(hdr, 8, 2, f) != 2)
            return 2;
        c.algo = (uint32_t)hdr[0];
        c.nchunks = (uint32_t)hdr[1];
        c.data = malloc(c.len ? c.len : 1);
        c.want = malloc((c.nchunks ? c.nchunks : 1) * sizeof(cg_desc));
        if (fread(c.data, 1, c.len, f) != c.len || fread(c.want, sizeof(cg_desc), c.nchunks, f) != c.nchunks) return 2;
        passed += run_case(&c, i);
        free(c.data);
        free(c.want);
    }
    fclose(f);
    printf("abi_check cases: %zu / %llu passed\n", passed, (unsigned long long)count);
    return passed == count ? 0 : 1;
}

int main(int argc, char **argv) {
    if (argc >= 2 && strcmp(argv[1], "nodevice") == 0) return nodevice();
    if (argc >= 3 && strcmp(argv[1], "cases") == 0) return cases(argv[2]);
    fprintf(stderr, "usage: abi_check nodevice | cases <file>\n");
    return 2;
}
