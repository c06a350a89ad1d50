/*
 * chunker_gpu.h -- C ABI of the MI355X (gfx950) FastCDC + per-chunk digest engine.
 *
 * This is the drop-in boundary for FlakeCache/chunker's hot path.  Each entry point
 * names the reference interface it replaces (paths are into the FlakeCache/chunker
 * tree).  The ABI uses plain pointers and sizes only; no HIP, torch or Rust types.
 * A Rust binding for it is given in INTEGRATION.md (the `chunker-hip` shim crate
 * that `chunker`'s `chunk_descriptors_with_hash` / `PushChunker` dispatch to behind
 * a cargo feature, since the reference crate is `unsafe_code = "forbid"`,
 * Cargo.toml:120).
 *
 * Threading: every entry point is re-entrant.  Device state is initialised once per
 * device, lazily; each call takes a workspace from a per-device pool.  A cg_push
 * handle is single-owner (the NIF already serialises it, src/nif.rs:285-297).
 * No entry point panics or aborts: failures are status codes plus a thread-local
 * message (cg_last_error_message).
 */
#ifndef CHUNKER_GPU_H
#define CHUNKER_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CG_ABI_VERSION 3u

/* Status codes.  1..5 map 1:1 onto ChunkingError (src/chunking.rs:33-51) so the
 * host shim can rebuild the exact Display strings. */
typedef enum {
    CG_OK = 0,
    CG_E_BOUNDS = 1,             /* ChunkingError::Bounds */
    CG_E_IO = 2,                 /* ChunkingError::Io (HIP runtime errors map here) */
    CG_E_ZERO_LENGTH_CHUNK = 3,  /* ChunkingError::ZeroLengthChunk */
    CG_E_INVALID_OPTIONS = 4,    /* ChunkingError::InvalidOptions(msg) */
    CG_E_BUFFER_LIMIT = 5,       /* ChunkingError::BufferLimitExceeded (device OOM) */
    CG_E_CAPACITY = 6,           /* ABI only: caller's output array too small */
    CG_E_NO_DEVICE = 7,          /* ABI only: no gfx950 device; there is no CPU fallback */
    CG_E_TABLES = 8,             /* ABI only: FastCDC tables are the placeholder or failed the selftest
                                    (the shim maps it to ChunkingError::Io with the message) */
} cg_status;

/* HashAlgorithm (src/chunking.rs:53-58), same declaration order. */
typedef enum { CG_BLAKE3 = 0, CG_SHA256 = 1 } cg_hash_algo;

/* ChunkDescriptor (src/chunking.rs:100-110): 48 bytes, offsets relative to the NAR. */
typedef struct {
    uint64_t offset;
    uint64_t length;
    uint8_t hash[32];
} cg_desc;

uint32_t cg_abi_version(void);

/* Thread-local message of the last failing call on this thread ("" if none).  For
 * CG_E_INVALID_OPTIONS it is exactly the InvalidOptions payload of
 * ChunkingOptions::validate (src/chunking.rs:190-231). */
const char *cg_last_error_message(void);

/* Fields of the last failure on this thread, so the shim can rebuild the reference's
 * variants exactly (src/chunking.rs:35-50): CG_E_BOUNDS -> out = {data_len, offset,
 * length} (ChunkingError::Bounds); CG_E_BUFFER_LIMIT -> out = {attempted, limit, 0}
 * (BufferLimitExceeded: bytes of the failed device allocation, device bytes free);
 * zeros otherwise.  Returns that failure's status (CG_OK if the last call succeeded). */
int cg_last_error_detail(uint64_t out[3]);

/* ChunkingOptions::resolve/validate (src/chunking.rs:173-231).  Pass 0 for a size to
 * take the reference default (256 KiB / 1 MiB / 4 MiB, :179-181).  `msg` may be NULL. */
int cg_validate(uint64_t min_size, uint64_t avg_size, uint64_t max_size, char *msg, size_t msg_cap);

/* Upper bound on the descriptors one input of `len` bytes can produce:
 * floor(len / (2*floor(min/2))) + 1 (every non-final cut is >= 2*floor(min/2)). */
size_t cg_capacity(uint64_t len, uint64_t min_size);

/* chunk_descriptors_with_hash (src/chunking.rs:323-374) on one host buffer.
 * Replaces `FastCDC::new(..).collect()` + the rayon `compute_hash` pass.  `data` is
 * borrowed (pageable is fine; the library stages it).  Writes *n_out descriptors. */
int cg_chunk_descriptors(const uint8_t *data, uint64_t len, uint64_t min_size, uint64_t avg_size,
                         uint64_t max_size, int algo, cg_desc *out, size_t out_cap, size_t *n_out);

/* Batch of independent NARs in one host buffer: NAR i is
 * data[nar_offsets[i] .. nar_offsets[i+1]).  Descriptors are written NAR after NAR;
 * nar_first[i] = index of NAR i's first descriptor, nar_first[n_nars] = total.
 * Equivalent to one chunk_descriptors_with_hash call per NAR. */
int cg_chunk_batch(const uint8_t *data, const uint64_t *nar_offsets, size_t n_nars, uint64_t min_size,
                   uint64_t avg_size, uint64_t max_size, int algo, cg_desc *out, size_t out_cap,
                   uint64_t *nar_first);

/* Device-resident batch: `d_data` and `d_out` are device pointers on the current
 * HIP device, `nar_offsets`/`nar_first` are host arrays, `stream` is a hipStream_t
 * (NULL = the null stream).  Returns after the descriptors are in HBM (the call
 * synchronises `stream` once to learn the count).  When more than 8 threads are in this
 * entry at once (SHA-256), their digests may be computed by one shared launch on a
 * library stream that `stream` waits for; the results and the return point are the
 * same as for a lone call. */
int cg_chunk_batch_device(const uint8_t *d_data, const uint64_t *nar_offsets, size_t n_nars,
                          uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo,
                          cg_desc *d_out, size_t out_cap, uint64_t *nar_first, void *stream);

/* The same batch without the wait: the whole pipeline is queued on `stream` and the call
 * returns (its host side -- validation, staging, launches -- overlaps whatever the GPU is
 * still running, so a caller that keeps one batch queued behind another leaves the GPU no
 * idle gap between them).  `nar_offsets` is copied before the call returns; `d_data` and
 * `d_out` must stay valid until cg_batch_wait.  cg_batch_wait(batch, nar_first) waits for
 * the batch, reports its errors (CG_E_CAPACITY, the SHA-256 spin guard, HIP failures),
 * fills nar_first (n_nars + 1, may be NULL) and frees the handle, whatever it returns.
 * Every handle must be waited for exactly once; batches on one stream complete in order. */
typedef struct cg_batch cg_batch;
int cg_chunk_batch_device_async(const uint8_t *d_data, const uint64_t *nar_offsets, size_t n_nars,
                                uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo,
                                cg_desc *d_out, size_t out_cap, void *stream, cg_batch **batch);
int cg_batch_wait(cg_batch *batch, uint64_t *nar_first);

/* The same queued batch ordered after `inputs_ready` -- a hipEvent_t recorded after the
 * last write to d_data and the last use of d_out -- instead of after everything queued on
 * `stream` (NULL = cg_chunk_batch_device_async).  The batch (candidate scan, cut walk,
 * descriptor assembly, digest) runs on a library stream of its workspace and `stream` waits
 * for its end: work queued on `stream` afterwards sees the finished descriptors, and
 * cg_batch_wait waits for this batch alone.  So a caller that keeps two batches queued
 * (double-buffered inputs) has the second batch's boundary stages AND digest run beside the
 * first's digest -- SHA-256's digest is bound by its longest chunk's serial chain and leaves
 * most of the chip idle.  (BLAKE3 batches are queued in `stream` order as by
 * cg_chunk_batch_device_async: their digest fills the chip by itself.)  Replaces the
 * collect-then-hash sequence of
 * chunk_descriptors_with_hash (src/chunking.rs:334-342) across consecutive calls. */
int cg_chunk_batch_device_async_after(const uint8_t *d_data, const uint64_t *nar_offsets, size_t n_nars,
                                      uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo,
                                      cg_desc *d_out, size_t out_cap, void *stream, void *inputs_ready,
                                      cg_batch **batch);

/* Digest pipeline: many device batches in flight from one caller without a HIP stream
 * (hardware queue) per batch.  Replaces, across a caller's consecutive
 * chunk_descriptors_with_hash calls, the collect-then-hash sequence of
 * src/chunking.rs:334-368: every batch's candidate scan, cut walk and descriptor assembly
 * run on the pipeline's boundary stream, each after its own `inputs_ready` event (a
 * hipEvent_t recorded after the last write to d_data and the last use of d_out; NULL = no
 * wait); the SHA-256 digests of up to `group_batches` consecutive batches (0 = 16, at most
 * 64) are then computed by ONE merged launch on one of `lanes` digest streams (0 = 3, at
 * most 8), so the next group's boundary stages and digest run beside it.  A group is
 * launched when it is full, when one of its batches is waited for (cg_batch_wait,
 * cg_batch_event) or by cg_pipeline_flush.  Each batch completes as soon as its own chunks
 * are digested (the digest kernel signals it), not when its whole group does.  BLAKE3
 * batches run whole on a boundary stream (a pipeline whose first batch is BLAKE3 has three,
 * used in turn, so consecutive batches overlap).  The pipeline uses
 * 1 + lanes non-blocking high-priority streams on `device` (-1 = the current device; the
 * caller's current device is left unchanged by every pipeline call), which HIP keeps off
 * the hardware queues of the process's ordinary streams whatever GPU_MAX_HW_QUEUES is (its
 * high-priority pool holds four queues: up to 3 lanes get one each).  The boundary stream's
 * scans use a lean form that fits on a CU beside two digest workgroups.
 * A batch is waited for with cg_batch_wait exactly once, as for
 * cg_chunk_batch_device_async; results, errors and nar_first are the same as those of
 * cg_chunk_batch_device on the same inputs.  A pipeline is single-owner; its batches may
 * be waited for from any thread, also after cg_pipeline_destroy (which launches a still
 * open group and waits for the pipeline's streams). */
typedef struct cg_pipeline cg_pipeline;
int cg_pipeline_create(int device, uint32_t group_batches, uint32_t lanes, cg_pipeline **out);
int cg_pipeline_submit(cg_pipeline *p, const uint8_t *d_data, const uint64_t *nar_offsets, size_t n_nars,
                       uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo, cg_desc *d_out,
                       size_t out_cap, void *inputs_ready, cg_batch **batch);
int cg_pipeline_flush(cg_pipeline *p);
/* out = {groups launched, batches in them, groups timed, their digest-kernel ms (sum), their
 * bytes (sum), the last timed group's ms}; groups are timed while cg_set_profiling is on. */
int cg_pipeline_stats(cg_pipeline *p, double out[6]);
void cg_pipeline_destroy(cg_pipeline *p);
/* A hipEvent_t that completes once the batch's results are in HBM (for a pipeline batch:
 * the end of its group's merged digest), so device work can be ordered after it without a
 * host wait; launches the batch's group if it is still open.  Valid until cg_batch_wait. */
int cg_batch_event(cg_batch *batch, void **event);

/* Multi-device batches: north_star's split of a batch of NARs one-file-per-GPU across the
 * GPUs of one node, with the descriptors gathered to one GPU, for a single host process
 * (the reference's node-bin, crates/node-bin/src/main.rs:1-25, whose Node::put calls
 * chunk_data per PUT, crates/node/src/lib.rs:114-132).  A cg_multi holds one digest
 * pipeline per entry of `devices` (cg_pipeline_create(devices[k], group_batches, lanes));
 * a device may be listed more than once.  cg_multi_submit queues shard k -- n_nars[k] NARs
 * at nar_offsets[k] (host array starting at 0) in d_data[k], device memory on devices[k],
 * after inputs_ready[k] (may be NULL, or hold NULLs) -- on device k's pipeline; there is no
 * exchange on the data path (FastCDC state never crosses files).  cg_multi_wait waits for
 * every shard and gathers their descriptors, shard after shard, into d_out (device memory
 * on devices[0], out_cap descriptors) with peer copies over xGMI, and writes the global NAR
 * index nar_first (sum of n_nars + 1 entries, may be NULL): the same result as one
 * cg_chunk_batch_device call over all shards' NARs in order.  Every handle is waited for
 * exactly once; cg_multi_flush launches every device's open group. */
typedef struct cg_multi cg_multi;
typedef struct cg_multi_batch cg_multi_batch;
int cg_multi_create(const int *devices, size_t n_dev, uint32_t group_batches, uint32_t lanes, cg_multi **out);
int cg_multi_submit(cg_multi *m, const uint8_t *const *d_data, const uint64_t *const *nar_offsets,
                    const size_t *n_nars, uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo,
                    cg_desc *d_out, size_t out_cap, void *const *inputs_ready, cg_multi_batch **batch);
int cg_multi_wait(cg_multi_batch *batch, uint64_t *nar_first);
int cg_multi_flush(cg_multi *m);
void cg_multi_destroy(cg_multi *m);

/* PushChunker (src/chunking.rs:753-829) over drain_finalized_chunks (:541-673).
 * push/finish write the chunks that became final; `out_cap` must be at least
 * cg_push_out_capacity(h, len).  push after finish -> CG_E_INVALID_OPTIONS
 * ("push called after finish"). */
typedef struct cg_push cg_push;
cg_push *cg_push_new(uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo, int *status);
int cg_push_push(cg_push *h, const uint8_t *data, uint64_t len, cg_desc *out, size_t out_cap, size_t *n_out);
int cg_push_finish(cg_push *h, cg_desc *out, size_t out_cap, size_t *n_out);
uint64_t cg_push_bytes_consumed(const cg_push *h); /* PushChunker::bytes_consumed */
size_t cg_push_out_capacity(const cg_push *h, uint64_t next_len);
void cg_push_free(cg_push *h);

/* Pipelined stream: ChunkStream::next (src/chunking.rs:675-740) and ChunkStreamAsync
 * (:835-1017) over drain_finalized_chunks (:541-673) with many read slices in flight.
 * Each push finds the slice's cut points at once (the reference's retain rule,
 * :579-584), but the chunks' digests run asynchronously, grouped over several slices;
 * cg_stream_take returns finished chunks strictly in stream order (offsets are stream
 * offsets), with exactly the (offset, length, hash) ChunkStream / PushChunker /
 * ChunkStreamAsync yields.  Device memory is bounded by `inflight_bytes` (0 = 2 GiB):
 * an arena of slots of max_size + slice_bytes (0 = 8 MiB, the reference's read size,
 * :713-716) bytes, each reused only after the digests reading it completed.  The arena
 * starts at two slots at the first push and grows to that budget only when no slot is
 * free (a short stream holds two slots); at the budget a push waits for the oldest
 * digests.  Digests run on one HIP stream at up to 4 hardware queues (HIP's default) and
 * otherwise on up to one per queue beside the call's own and the null stream's
 * (GPU_MAX_HW_QUEUES - 2, at most 8; the variable as the library was loaded),
 * created as they are needed, each on groups of at most 2048 / lanes chunks' expected
 * bytes (so all lanes' SHA-256 workgroups fit the chip at once).
 * push returns once its bytes are copied: the caller may reuse `data` right away.  take
 * with wait = 0 returns what has completed; wait != 0 blocks until at least one chunk is
 * ready or nothing is pending.  push after finish -> CG_E_INVALID_OPTIONS.  The first
 * failure of push / finish / take poisons the handle: every later push / finish / take
 * returns that status again (message prefixed "stream failed earlier", the failure's
 * cg_last_error_detail fields), since a failed push may have left part of its slice in
 * the engine.  Single owner, like cg_push. */
typedef struct cg_stream cg_stream;
cg_stream *cg_stream_new(uint64_t min_size, uint64_t avg_size, uint64_t max_size, int algo, uint64_t slice_bytes,
                         uint64_t inflight_bytes, int *status);
int cg_stream_push(cg_stream *h, const uint8_t *data, uint64_t len);
int cg_stream_finish(cg_stream *h);
int cg_stream_take(cg_stream *h, cg_desc *out, size_t out_cap, size_t *n_out, int wait);
uint64_t cg_stream_pending(const cg_stream *h);       /* chunks found but not yet taken */
uint64_t cg_stream_bytes_consumed(const cg_stream *h); /* bytes pushed so far */
void cg_stream_free(cg_stream *h);

/* Digest-only entry (sha256_hash_raw src/hashing.rs:36-44 / blake3::hash) over n
 * device-resident spans; d_digests receives n*32 bytes. */
int cg_hash_spans_device(const uint8_t *d_data, const uint64_t *d_offsets, const uint64_t *d_lengths, size_t n,
                         int algo, uint8_t *d_digests, void *stream);

/* Host convenience over the same kernels: digest of one host buffer (sha256_hash_raw /
 * blake3::hash, src/hashing.rs:36-53) into out[32].  len <= 16 MiB for BLAKE3. */
int cg_hash(const uint8_t *data, uint64_t len, int algo, uint8_t out[32]);

/* ---- CAS content ids and Node::put ---------------------- */

/* ObjectKind (crates/core/cas/src/lib.rs:31-48), same discriminants. */
typedef enum {
    CG_KIND_CHUNK = 1,
    CG_KIND_LEVEL0_MANIFEST = 2,
    CG_KIND_LEVEL1_MANIFEST = 3,
    CG_KIND_REFCOUNT = 4,
    CG_KIND_WITNESS = 5,
    CG_KIND_RECIPE = 6,
    CG_KIND_COMMIT = 7
} cg_object_kind;

/* ContentId::compute(kind, payload) (crates/core/cas/src/lib.rs:53-69) over n
 * device-resident spans: SHAKE256-256("flakecache-cas" || 0x00 || kind || u16le(1) ||
 * u64le(len) || payload) (shake256_256, crates/core/crypto/src/hash.rs:34-41).
 * d_ids receives n*32 bytes.  An unknown kind -> CG_E_INVALID_OPTIONS. */
int cg_cas_ids_device(const uint8_t *d_data, const uint64_t *d_offsets, const uint64_t *d_lengths, size_t n,
                      uint32_t kind, uint8_t *d_ids, void *stream);

/* Host convenience: ContentId::compute of one host buffer into out[32]. */
int cg_cas_id(const uint8_t *data, uint64_t len, uint32_t kind, uint8_t out[32]);

/* Node::put (crates/node/src/lib.rs:114-132) over a device-resident batch of NARs:
 * chunk_data with SHA-256 (:115, i.e. cg_chunk_batch_device with CG_SHA256) into
 * d_out/nar_first; ContentId(Chunk, payload) of descriptor g -> d_chunk_ids[32 g]
 * (:118-121); NAR i's manifest id ContentId(Level1Manifest, its chunk ids in order)
 * -> manifest_ids[32 i] (host array, :124-129).  The CAS stage runs on a second
 * stream concurrently with the SHA-256 digest. */
int cg_node_put_batch_device(const uint8_t *d_data, const uint64_t *nar_offsets, size_t n_nars, uint64_t min_size,
                             uint64_t avg_size, uint64_t max_size, cg_desc *d_out, size_t out_cap,
                             uint64_t *nar_first, uint8_t *d_chunk_ids, uint8_t *manifest_ids, void *stream);

/* Node::put on one host buffer: descriptors (out), chunk ids (chunk_ids, out_cap*32
 * bytes) and the manifest id (manifest_id[32], the value Node::put returns). */
int cg_node_put(const uint8_t *data, uint64_t len, uint64_t min_size, uint64_t avg_size, uint64_t max_size,
                cg_desc *out, size_t out_cap, size_t *n_out, uint8_t *chunk_ids, uint8_t manifest_id[32]);

/* FastCDC v2020 tables [ext fastcdc 4.0.1 src/v2020]: GEAR[256] and MASKS[26], used by
 * FastCDC::new at src/chunking.rs:334, :553, :893.  The compiled-in set comes from
 * the tables/ text files; its GEAR is a PLACEHOLDER (the crate is not vendored in the reference),
 * so the engine FAILS CLOSED: every chunking entry point (cg_chunk_*, cg_push_push /
 * _finish, cg_node_put*) returns CG_E_TABLES while the placeholder is installed, and
 * runs any other table set only after it reproduced the reference's golden fixture
 * (src/chunking.rs:1266-1297) on the GPU (cg_selftest, run once per installed set on
 * first use).  CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR=1 in the environment lifts the gate
 * (tests and benchmarks; boundaries are then self-consistent, not the reference's).
 * Digest-only entries (cg_hash*, cg_cas_*) do not use the tables and are never gated.
 *
 * cg_set_cdc_tables installs a set process-wide (all devices) for later calls; masks
 * may be NULL to keep the current MASKS; a mask with bits above 47 -> CG_E_INVALID_OPTIONS
 * (the windowed GPU scan needs every tested bit within 48 bytes of history). */
int cg_set_cdc_tables(const uint64_t gear[256], const uint64_t masks[26]);
void cg_get_cdc_tables(uint64_t gear[256], uint64_t masks[26]);
int cg_set_gear_table(const uint64_t gear[256]); /* = cg_set_cdc_tables(gear, NULL) */
void cg_get_gear_table(uint64_t gear[256]);
int cg_gear_is_placeholder(void);
/* Run the reference fixture through the GPU pipeline (scan, walk, assembly) with the
 * installed tables: CG_OK if it gives fastcdc's 10 boundaries (the set is then marked
 * verified), CG_E_TABLES with the boundaries found otherwise.  Needs a device.
 * COVERAGE: the fixture is the reference's only FastCDC vector.  Its bytes take the
 * values 0..250 and its avg 6000 gives bits = 13, so it exercises GEAR[0..250], MASKS[12]
 * and MASKS[14] only.  A table set that is wrong at GEAR[251..255] or at any other
 * MASKS entry passes this selftest, and then cuts other boundaries than fastcdc for
 * inputs holding those bytes or for other averages.  Install the crate's arrays
 * verbatim (scripts/install_fastcdc_tables.py, or the shim's build.rs reading them
 * from the cargo registry), never a transcription. */
int cg_selftest(void);
int cg_tables_verified(void); /* 1 once the installed set passed cg_selftest */

/* Per-stage device times (ms) of the last batch call on this thread, measured with
 * HIP events on the stream the kernels ran on.  Order: scan, compact, walk,
 * assemble, digest, and for the Node::put entries a sixth: cas (descriptor assembly
 * to the last content id, on the side stream).  Returns the number of stages
 * written; 0 if profiling is off.  cg_set_profiling(1) times every stage;
 * cg_set_profiling(2) records only the two events around the digest stage (the other
 * stages read NaN): each timing event between two kernels holds the second back by
 * ~6 us, which on a 0.8 ms config-3 batch is 4 % for the five boundaries of mode 1. */
void cg_set_profiling(int on);
size_t cg_last_stage_times(double *ms, size_t n);

/* Shape of the last SHA-256 digest launch on this thread (K3 k_sha256 work units):
 * out = {quad workgroups (8 chunks, 8 lanes each), pair workgroups (32 chunks, 2 lanes
 * each), one-lane workgroups (64 chunks), LDS pad bytes (non-zero: one workgroup per
 * CU)}.  The quad tier holds the longest chunks (length order), so the digest stage's
 * latency floor is the longest chunk's blocks x 64 rounds at the quad tier's cycles per
 * round when out[0] > 0.  Returns 1 if this thread has launched a SHA-256 digest. */
int cg_last_sha_tiers(uint32_t out[4]);

/* Synthetic NAR writer: nix-archive-1 framing around an
 * xorshift64 payload (crates/node/src/lib.rs:192-203) with seed
 * 0x9E3779B97F4A7C15 ^ (first_index + i), or zeros.  NAR i is nar_sizes[i] bytes
 * (a multiple of 8, >= 120) written back to back into `out`. */
void cg_synth_nars(uint8_t *out, const uint64_t *nar_sizes, size_t n, int zeros, uint64_t first_index);

#ifdef __cplusplus
}
#endif
#endif
