//! Safe wrapper over `include/chunker_gpu.h` (ABI version 3): the MI355X (gfx950) FastCDC
//! + per-chunk SHA-256 / BLAKE3 engine, `libchunker_amd.so`.
//!
//! The reference crate `chunker` is `unsafe_code = "forbid"` (Cargo.toml:120), so the
//! `extern "C"` block lives in this crate and `chunker` calls the safe functions below
//! behind `features = ["gpu"]`.  Every item names the reference
//! interface it serves.  There is no CPU fallback in the engine: without a gfx950 device
//! every compute entry returns `CgError::NoDevice`, and `available()` is false, so the
//! caller keeps running its own CPU code.
//!
//! The same C ABI is exercised from C by `tests/abi_c/abi_check.c` (struct layout, enum
//! values, every entry declared here) and from Python by `chunker_amd/_lib.py`.
use std::ffi::CStr;
use std::os::raw::{c_char, c_int, c_void};
use std::ptr::NonNull;
use std::sync::OnceLock;

mod tables {
    include!(concat!(env!("OUT_DIR"), "/fastcdc_tables.rs"));
}

/// `cg_desc` = ChunkDescriptor (src/chunking.rs:100-110), 48 bytes, offsets relative to
/// the input.
#[repr(C)]
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub struct CgDesc {
    pub offset: u64,
    pub length: u64,
    pub hash: [u8; 32],
}
const _: () = assert!(std::mem::size_of::<CgDesc>() == 48);

#[repr(C)]
pub struct CgPush {
    _p: [u8; 0],
}
#[repr(C)]
pub struct CgStream {
    _p: [u8; 0],
}
#[repr(C)]
pub struct CgBatch {
    _p: [u8; 0],
}
#[repr(C)]
pub struct CgPipeline {
    _p: [u8; 0],
}
#[repr(C)]
pub struct CgMulti {
    _p: [u8; 0],
}
#[repr(C)]
pub struct CgMultiBatch {
    _p: [u8; 0],
}

extern "C" {
    fn cg_abi_version() -> u32;
    fn cg_last_error_message() -> *const c_char;
    fn cg_last_error_detail(out: *mut [u64; 3]) -> c_int;
    fn cg_set_cdc_tables(gear: *const [u64; 256], masks: *const [u64; 26]) -> c_int;
    fn cg_selftest() -> c_int;
    fn cg_capacity(len: u64, min: u64) -> usize;
    fn cg_chunk_descriptors(data: *const u8, len: u64, min: u64, avg: u64, max: u64, algo: c_int,
                            out: *mut CgDesc, cap: usize, n_out: *mut usize) -> c_int;
    fn cg_chunk_batch(data: *const u8, nar_offsets: *const u64, n: usize, min: u64, avg: u64, max: u64,
                      algo: c_int, out: *mut CgDesc, cap: usize, nar_first: *mut u64) -> c_int;
    fn cg_chunk_batch_device_async(d_data: *const u8, nar_offsets: *const u64, n: usize, min: u64, avg: u64,
                                   max: u64, algo: c_int, d_out: *mut CgDesc, cap: usize, stream: *mut c_void,
                                   batch: *mut *mut CgBatch) -> c_int;
    fn cg_chunk_batch_device_async_after(d_data: *const u8, nar_offsets: *const u64, n: usize, min: u64, avg: u64,
                                         max: u64, algo: c_int, d_out: *mut CgDesc, cap: usize,
                                         stream: *mut c_void, inputs_ready: *mut c_void,
                                         batch: *mut *mut CgBatch) -> c_int;
    fn cg_batch_wait(batch: *mut CgBatch, nar_first: *mut u64) -> c_int;
    fn cg_pipeline_create(device: c_int, group: u32, lanes: u32, out: *mut *mut CgPipeline) -> c_int;
    fn cg_pipeline_submit(p: *mut CgPipeline, d_data: *const u8, nar_offsets: *const u64, n: usize, min: u64,
                          avg: u64, max: u64, algo: c_int, d_out: *mut CgDesc, cap: usize,
                          inputs_ready: *mut c_void, batch: *mut *mut CgBatch) -> c_int;
    fn cg_pipeline_flush(p: *mut CgPipeline) -> c_int;
    fn cg_pipeline_destroy(p: *mut CgPipeline);
    fn cg_multi_create(devices: *const c_int, n_dev: usize, group: u32, lanes: u32, out: *mut *mut CgMulti)
        -> c_int;
    fn cg_multi_submit(m: *mut CgMulti, d_data: *const *const u8, nar_offsets: *const *const u64, n_nars: *const usize,
                       min: u64, avg: u64, max: u64, algo: c_int, d_out: *mut CgDesc, cap: usize,
                       inputs_ready: *const *mut c_void, batch: *mut *mut CgMultiBatch) -> c_int;
    fn cg_multi_wait(batch: *mut CgMultiBatch, nar_first: *mut u64) -> c_int;
    fn cg_multi_flush(m: *mut CgMulti) -> c_int;
    fn cg_multi_destroy(m: *mut CgMulti);
    fn cg_push_new(min: u64, avg: u64, max: u64, algo: c_int, status: *mut c_int) -> *mut CgPush;
    fn cg_push_push(h: *mut CgPush, data: *const u8, len: u64, out: *mut CgDesc, cap: usize,
                    n_out: *mut usize) -> c_int;
    fn cg_push_finish(h: *mut CgPush, out: *mut CgDesc, cap: usize, n_out: *mut usize) -> c_int;
    fn cg_push_bytes_consumed(h: *const CgPush) -> u64;
    fn cg_push_out_capacity(h: *const CgPush, next_len: u64) -> usize;
    fn cg_push_free(h: *mut CgPush);
    fn cg_stream_new(min: u64, avg: u64, max: u64, algo: c_int, slice: u64, inflight: u64,
                     status: *mut c_int) -> *mut CgStream;
    fn cg_stream_push(h: *mut CgStream, data: *const u8, len: u64) -> c_int;
    fn cg_stream_finish(h: *mut CgStream) -> c_int;
    fn cg_stream_take(h: *mut CgStream, out: *mut CgDesc, cap: usize, n_out: *mut usize, wait: c_int) -> c_int;
    fn cg_stream_pending(h: *const CgStream) -> u64;
    fn cg_stream_bytes_consumed(h: *const CgStream) -> u64;
    fn cg_stream_free(h: *mut CgStream);
    fn cg_hash(data: *const u8, len: u64, algo: c_int, out: *mut [u8; 32]) -> c_int;
    fn cg_cas_id(data: *const u8, len: u64, kind: u32, out: *mut [u8; 32]) -> c_int;
    fn cg_node_put(data: *const u8, len: u64, min: u64, avg: u64, max: u64, out: *mut CgDesc, cap: usize,
                   n_out: *mut usize, chunk_ids: *mut u8, manifest: *mut [u8; 32]) -> c_int;
}

/// The engine's failure, with everything needed to rebuild ChunkingError exactly
/// (src/chunking.rs:33-51): statuses 1 and 5 carry their fields (cg_last_error_detail).
#[derive(Debug)]
pub enum CgError {
    Bounds { data_len: usize, offset: usize, length: usize }, // 1
    Io(String),                                               // 2
    ZeroLengthChunk,                                          // 3
    InvalidOptions(String),                                   // 4
    BufferLimitExceeded { attempted: usize, limit: usize },   // 5
    Capacity,                                                 // 6 (ABI only)
    NoDevice(String),                                         // 7 (ABI only)
    Tables(String),                                           // 8 (ABI only)
}

fn last_error() -> String {
    unsafe { CStr::from_ptr(cg_last_error_message()) }.to_string_lossy().into_owned()
}

fn check(st: c_int) -> Result<(), CgError> {
    if st == 0 {
        return Ok(());
    }
    let mut d = [0u64; 3];
    unsafe { cg_last_error_detail(&mut d) };
    Err(match st {
        1 => CgError::Bounds { data_len: d[0] as usize, offset: d[1] as usize, length: d[2] as usize },
        2 => CgError::Io(last_error()),
        3 => CgError::ZeroLengthChunk,
        4 => CgError::InvalidOptions(last_error()),
        5 => CgError::BufferLimitExceeded { attempted: d[0] as usize, limit: d[1] as usize },
        6 => CgError::Capacity,
        8 => CgError::Tables(last_error()),
        _ => CgError::NoDevice(last_error()),
    })
}

/// Install fastcdc 4.0.1's tables and run the reference fixture (src/chunking.rs:1266-1297)
/// on the GPU once per process; the GPU path is used only if both succeed.  The digest
/// pipeline (`Pipeline`, `MultiDevice`) needs no hardware-queue setting: HIP's default
/// `GPU_MAX_HW_QUEUES` (4) is the deployment setting.
static READY: OnceLock<Result<(), String>> = OnceLock::new();
pub fn available() -> bool {
    READY
        .get_or_init(|| unsafe {
            if cg_abi_version() != 3 {
                return Err("chunker_amd ABI version".into());
            }
            check(cg_set_cdc_tables(&tables::GEAR, &tables::MASKS)).map_err(|e| format!("{e:?}"))?;
            check(cg_selftest()).map_err(|e| format!("{e:?}"))
        })
        .is_ok()
}

/// HashAlgorithm order (src/chunking.rs:53-58): Blake3 = 0, Sha256 = 1.
pub const BLAKE3: i32 = 0;
pub const SHA256: i32 = 1;

/// Dispatch rule for single synchronous calls (measured by bench.py's
/// drop_in leg): BLAKE3 pays on the GPU from one 10 MiB call on (24-29 vs 2.0-2.9 GiB/s); a
/// SHA-256 call lasts its longest chunk's
/// serial chain (~30-90 ms), so it pays only for large inputs (1 GiB: 11.3 vs 4.9 GiB/s;
/// 256 MiB: even).  Smaller SHA-256 calls stay on the reference's CPU path.
pub const SHA256_SINGLE_CALL_MIN: usize = 512 << 20;
pub fn pays(algo: i32, len: usize) -> bool {
    algo == BLAKE3 || len >= SHA256_SINGLE_CALL_MIN
}

/// chunk_descriptors_with_hash (src/chunking.rs:323-374) for one input.
pub fn chunk_descriptors(data: &[u8], min: usize, avg: usize, max: usize, algo: i32)
    -> Result<Vec<CgDesc>, CgError> {
    let cap = unsafe { cg_capacity(data.len() as u64, min as u64) }.max(1);
    let mut out = Vec::<CgDesc>::with_capacity(cap);
    let mut n = 0usize;
    check(unsafe {
        cg_chunk_descriptors(data.as_ptr(), data.len() as u64, min as u64, avg as u64, max as u64, algo,
                             out.as_mut_ptr(), cap, &mut n)
    })?;
    unsafe { out.set_len(n) };
    Ok(out)
}

/// Many independent inputs (NARs) back to back in `data`, NAR i = data[offs[i]..offs[i+1]]:
/// one chunk_descriptors_with_hash per NAR in one engine call.  Returns the descriptors
/// and nar_first (NAR i's descriptors are [nar_first[i], nar_first[i+1])).
pub fn chunk_batch(data: &[u8], offs: &[u64], min: usize, avg: usize, max: usize, algo: i32)
    -> Result<(Vec<CgDesc>, Vec<u64>), CgError> {
    let n = offs.len().saturating_sub(1);
    // cg_chunk_batch takes no length: it copies data[offs[0]..offs[n]], so the offsets are
    // checked against `data` here, before any arithmetic on them or the FFI call
    let bounds = |offset: u64, length: u64| CgError::Bounds {
        data_len: data.len(),
        offset: offset as usize,
        length: length as usize,
    };
    for i in 0..n {
        if offs[i + 1] < offs[i] {
            return Err(bounds(offs[i], 0));
        }
    }
    if n > 0 && offs[n] > data.len() as u64 {
        return Err(bounds(offs[0], offs[n] - offs[0]));
    }
    let mut cap = 0usize;
    for i in 0..n {
        let c = unsafe { cg_capacity(offs[i + 1] - offs[i], min as u64) };
        cap = cap.checked_add(c).ok_or(CgError::Capacity)?;
    }
    let cap = cap.max(1);
    let mut out = Vec::<CgDesc>::with_capacity(cap);
    let mut first = vec![0u64; n + 1];
    check(unsafe {
        cg_chunk_batch(data.as_ptr(), offs.as_ptr(), n, min as u64, avg as u64, max as u64, algo, out.as_mut_ptr(),
                       cap, first.as_mut_ptr())
    })?;
    unsafe { out.set_len(first[n] as usize) };
    Ok((out, first))
}

/// A device-resident batch queued on a HIP stream (an ingest worker draining NAR batches
/// that already sit in HBM): `wait` consumes it; Drop waits too, so the engine's
/// workspace always returns to its pool.
pub struct BatchInFlight {
    h: *mut CgBatch,
    n: usize,
}
unsafe impl Send for BatchInFlight {}
impl BatchInFlight {
    /// # Safety
    /// `d_data` (16-byte aligned) and `d_out` are device pointers on the current HIP
    /// device that stay valid until the batch is waited for; `stream` is a hipStream_t.
    pub unsafe fn queue(d_data: *const u8, offs: &[u64], min: usize, avg: usize, max: usize, algo: i32,
                        d_out: *mut CgDesc, cap: usize, stream: *mut c_void) -> Result<Self, CgError> {
        let n = offs.len().saturating_sub(1);
        let mut h = std::ptr::null_mut();
        check(cg_chunk_batch_device_async(d_data, offs.as_ptr(), n, min as u64, avg as u64, max as u64, algo, d_out,
                                          cap, stream, &mut h))?;
        Ok(BatchInFlight { h, n })
    }
    /// The same, with the batch ordered after `inputs_ready` (a hipEvent_t recorded after the
    /// last write to `d_data` and the last use of `d_out`) instead of after everything on
    /// `stream`: a SHA-256 batch runs on a stream of its own beside the batches queued
    /// before it, and `stream` waits for its end.  Each batch in flight holds a HIP stream,
    /// so this path scales only with `GPU_MAX_HW_QUEUES` (round 5); an ingest worker with
    /// many batches in flight uses `Pipeline` instead (one merged digest per group of
    /// batches, 4 hardware queues suffice).
    ///
    /// # Safety
    /// As `queue`; `inputs_ready` is a hipEvent_t (or null).
    pub unsafe fn queue_after(d_data: *const u8, offs: &[u64], min: usize, avg: usize, max: usize, algo: i32,
                              d_out: *mut CgDesc, cap: usize, stream: *mut c_void, inputs_ready: *mut c_void)
        -> Result<Self, CgError> {
        let n = offs.len().saturating_sub(1);
        let mut h = std::ptr::null_mut();
        check(cg_chunk_batch_device_async_after(d_data, offs.as_ptr(), n, min as u64, avg as u64, max as u64, algo,
                                                d_out, cap, stream, inputs_ready, &mut h))?;
        Ok(BatchInFlight { h, n })
    }
    pub fn wait(mut self) -> Result<Vec<u64>, CgError> {
        let mut first = vec![0u64; self.n + 1];
        let h = std::mem::replace(&mut self.h, std::ptr::null_mut());
        check(unsafe { cg_batch_wait(h, first.as_mut_ptr()) }).map(|_| first)
    }
}
impl Drop for BatchInFlight {
    fn drop(&mut self) {
        if !self.h.is_null() {
            unsafe { cg_batch_wait(self.h, std::ptr::null_mut()) };
        }
    }
}

/// The digest pipeline (cg_pipeline_*): one ingest worker's device batches in flight, the
/// SHA-256 digests of `group` consecutive batches merged into one launch on one of `lanes`
/// digest streams, each batch handed back when its own chunks are digested.  Replaces,
/// across the worker's consecutive chunk_descriptors_with_hash calls, the collect-then-hash
/// sequence of src/chunking.rs:334-368.  Measured (DESIGN.md §7 "The digest pipeline"):
/// config 2 (1 GiB batches of 256 x 4 MiB NARs) at group 20, 3 lanes, 80 in flight:
/// 736-864 GiB/s at HIP's default 4 hardware queues.  Keep (lanes + 1) x group batches in
/// flight.  `group` 0 / `lanes` 0 = the engine's defaults (16 / 3).
pub struct Pipeline(NonNull<CgPipeline>);
unsafe impl Send for Pipeline {}
impl Pipeline {
    /// `device` -1 = the current HIP device.
    pub fn new(device: i32, group: u32, lanes: u32) -> Result<Self, CgError> {
        let mut h = std::ptr::null_mut();
        check(unsafe { cg_pipeline_create(device, group, lanes, &mut h) })?;
        Ok(Pipeline(NonNull::new(h).ok_or(CgError::Io("cg_pipeline_create returned null".into()))?))
    }
    /// # Safety
    /// `d_data` (16-byte aligned) and `d_out` are device pointers on the pipeline's device
    /// that stay valid and untouched until the batch is waited for; `inputs_ready` is a
    /// hipEvent_t (or null).
    pub unsafe fn submit(&mut self, d_data: *const u8, offs: &[u64], min: usize, avg: usize, max: usize, algo: i32,
                         d_out: *mut CgDesc, cap: usize, inputs_ready: *mut c_void)
        -> Result<BatchInFlight, CgError> {
        let n = offs.len().saturating_sub(1);
        let mut h = std::ptr::null_mut();
        check(cg_pipeline_submit(self.0.as_ptr(), d_data, offs.as_ptr(), n, min as u64, avg as u64, max as u64, algo,
                                 d_out, cap, inputs_ready, &mut h))?;
        Ok(BatchInFlight { h, n })
    }
    /// Launch the digest of the batches submitted since the last full group.
    pub fn flush(&mut self) -> Result<(), CgError> {
        check(unsafe { cg_pipeline_flush(self.0.as_ptr()) })
    }
}
impl Drop for Pipeline {
    fn drop(&mut self) {
        unsafe { cg_pipeline_destroy(self.0.as_ptr()) }
    }
}

/// One process driving several GPUs (cg_multi_*): north_star's split of a batch of NARs
/// one-file-per-GPU, the descriptors gathered into one array on `devices[0]` over xGMI
/// peer copies -- for the reference's single node-bin process (crates/node-bin/src/main.rs,
/// Node::put per PUT, crates/node/src/lib.rs:114-132).
pub struct MultiDevice(NonNull<CgMulti>);
unsafe impl Send for MultiDevice {}
pub struct MultiBatch {
    h: *mut CgMultiBatch,
    n: usize,
}
unsafe impl Send for MultiBatch {}
impl MultiDevice {
    pub fn new(devices: &[i32], group: u32, lanes: u32) -> Result<Self, CgError> {
        let mut h = std::ptr::null_mut();
        check(unsafe { cg_multi_create(devices.as_ptr(), devices.len(), group, lanes, &mut h) })?;
        Ok(MultiDevice(NonNull::new(h).ok_or(CgError::Io("cg_multi_create returned null".into()))?))
    }
    /// Shard k = (device pointer on devices[k], its NAR offsets starting at 0).
    ///
    /// # Safety
    /// Every shard's bytes and `d_out` (on devices[0]) stay valid until the batch is waited
    /// for; `inputs_ready` holds one hipEvent_t (or null) per shard, or is empty.
    pub unsafe fn submit(&mut self, shards: &[(*const u8, &[u64])], min: usize, avg: usize, max: usize, algo: i32,
                         d_out: *mut CgDesc, cap: usize, inputs_ready: &[*mut c_void])
        -> Result<MultiBatch, CgError> {
        let data: Vec<*const u8> = shards.iter().map(|s| s.0).collect();
        let offs: Vec<*const u64> = shards.iter().map(|s| s.1.as_ptr()).collect();
        let nn: Vec<usize> = shards.iter().map(|s| s.1.len().saturating_sub(1)).collect();
        let ready = if inputs_ready.is_empty() { std::ptr::null() } else { inputs_ready.as_ptr() };
        let mut h = std::ptr::null_mut();
        check(cg_multi_submit(self.0.as_ptr(), data.as_ptr(), offs.as_ptr(), nn.as_ptr(), min as u64, avg as u64,
                              max as u64, algo, d_out, cap, ready, &mut h))?;
        Ok(MultiBatch { h, n: nn.iter().sum() })
    }
    pub fn flush(&mut self) -> Result<(), CgError> {
        check(unsafe { cg_multi_flush(self.0.as_ptr()) })
    }
}
impl MultiBatch {
    /// Waits for every shard and gathers the descriptors; returns the global nar_first.
    pub fn wait(mut self) -> Result<Vec<u64>, CgError> {
        let mut first = vec![0u64; self.n + 1];
        let h = std::mem::replace(&mut self.h, std::ptr::null_mut());
        check(unsafe { cg_multi_wait(h, first.as_mut_ptr()) }).map(|_| first)
    }
}
impl Drop for MultiBatch {
    fn drop(&mut self) {
        if !self.h.is_null() {
            unsafe { cg_multi_wait(self.h, std::ptr::null_mut()) };
        }
    }
}
impl Drop for MultiDevice {
    fn drop(&mut self) {
        unsafe { cg_multi_destroy(self.0.as_ptr()) }
    }
}

/// PushChunker's engine (src/chunking.rs:753-829): synchronous, every push returns its
/// final chunks.
pub struct Push(NonNull<CgPush>);
unsafe impl Send for Push {}
impl Push {
    pub fn new(min: usize, avg: usize, max: usize, algo: i32) -> Result<Self, CgError> {
        let mut st = 0;
        let h = unsafe { cg_push_new(min as u64, avg as u64, max as u64, algo, &mut st) };
        check(st)?;
        Ok(Push(NonNull::new(h).ok_or(CgError::Io("cg_push_new returned null".into()))?))
    }
    pub fn push(&mut self, data: &[u8]) -> Result<Vec<CgDesc>, CgError> {
        let cap = unsafe { cg_push_out_capacity(self.0.as_ptr(), data.len() as u64) }.max(1);
        let mut out = Vec::<CgDesc>::with_capacity(cap);
        let mut n = 0usize;
        check(unsafe {
            cg_push_push(self.0.as_ptr(), data.as_ptr(), data.len() as u64, out.as_mut_ptr(), cap, &mut n)
        })?;
        unsafe { out.set_len(n) };
        Ok(out)
    }
    pub fn finish(&mut self) -> Result<Vec<CgDesc>, CgError> {
        let cap = unsafe { cg_push_out_capacity(self.0.as_ptr(), 0) }.max(1);
        let mut out = Vec::<CgDesc>::with_capacity(cap);
        let mut n = 0usize;
        check(unsafe { cg_push_finish(self.0.as_ptr(), out.as_mut_ptr(), cap, &mut n) })?;
        unsafe { out.set_len(n) };
        Ok(out)
    }
    pub fn bytes_consumed(&self) -> u64 {
        unsafe { cg_push_bytes_consumed(self.0.as_ptr()) }
    }
}
impl Drop for Push {
    fn drop(&mut self) {
        unsafe { cg_push_free(self.0.as_ptr()) }
    }
}

/// ChunkStream / ChunkStreamAsync's engine (src/chunking.rs:675-740, :835-1017):
/// pipelined, chunks come back later, in stream order.
pub struct Stream(NonNull<CgStream>);
unsafe impl Send for Stream {}
impl Stream {
    /// slice = the reader's refill size (src/chunking.rs:713-716); inflight = HBM budget (0 = 2 GiB).
    pub fn new(min: usize, avg: usize, max: usize, algo: i32, slice: usize, inflight: usize)
        -> Result<Self, CgError> {
        let mut st = 0;
        let h = unsafe {
            cg_stream_new(min as u64, avg as u64, max as u64, algo, slice as u64, inflight as u64, &mut st)
        };
        check(st)?;
        Ok(Stream(NonNull::new(h).ok_or(CgError::Io("cg_stream_new returned null".into()))?))
    }
    pub fn push(&mut self, data: &[u8]) -> Result<(), CgError> {
        check(unsafe { cg_stream_push(self.0.as_ptr(), data.as_ptr(), data.len() as u64) })
    }
    pub fn finish(&mut self) -> Result<(), CgError> {
        check(unsafe { cg_stream_finish(self.0.as_ptr()) })
    }
    /// Finished chunks (offsets are stream offsets); `wait` blocks until one is ready.
    pub fn take(&mut self, wait: bool, out: &mut Vec<CgDesc>) -> Result<usize, CgError> {
        out.clear();
        out.reserve(4096);
        let mut n = 0usize;
        check(unsafe { cg_stream_take(self.0.as_ptr(), out.as_mut_ptr(), out.capacity(), &mut n, wait as c_int) })?;
        unsafe { out.set_len(n) };
        Ok(n)
    }
    pub fn pending(&self) -> u64 {
        unsafe { cg_stream_pending(self.0.as_ptr()) }
    }
    pub fn bytes_consumed(&self) -> u64 {
        unsafe { cg_stream_bytes_consumed(self.0.as_ptr()) }
    }
}
impl Drop for Stream {
    fn drop(&mut self) {
        unsafe { cg_stream_free(self.0.as_ptr()) }
    }
}

/// sha256_hash_raw / blake3::hash (src/hashing.rs:36-53) of one buffer on the GPU.
pub fn hash(data: &[u8], algo: i32) -> Result<[u8; 32], CgError> {
    let mut out = [0u8; 32];
    check(unsafe { cg_hash(data.as_ptr(), data.len() as u64, algo, &mut out) })?;
    Ok(out)
}

/// ContentId::compute (crates/core/cas/src/lib.rs:53-69): SHAKE-256 over the framed payload.
pub fn content_id(kind: u8, payload: &[u8]) -> Result<[u8; 32], CgError> {
    let mut out = [0u8; 32];
    check(unsafe { cg_cas_id(payload.as_ptr(), payload.len() as u64, kind as u32, &mut out) })?;
    Ok(out)
}

/// (descriptors, chunk ids, manifest id) of Node::put (crates/node/src/lib.rs:114-132)
/// before its storage writes.
pub fn node_put(data: &[u8], min: usize, avg: usize, max: usize)
    -> Result<(Vec<CgDesc>, Vec<[u8; 32]>, [u8; 32]), CgError> {
    let cap = unsafe { cg_capacity(data.len() as u64, min as u64) }.max(1);
    let mut descs = vec![CgDesc { offset: 0, length: 0, hash: [0; 32] }; cap];
    let mut ids = vec![[0u8; 32]; cap];
    let (mut n, mut man) = (0usize, [0u8; 32]);
    check(unsafe {
        cg_node_put(data.as_ptr(), data.len() as u64, min as u64, avg as u64, max as u64, descs.as_mut_ptr(), cap,
                    &mut n, ids.as_mut_ptr() as *mut u8, &mut man)
    })?;
    descs.truncate(n);
    ids.truncate(n);
    Ok((descs, ids, man))
}

#[cfg(test)]
mod tests {
    use super::*;

    /// The reference's golden fixture (src/chunking.rs:1266-1297) through the engine,
    /// when a device is present (available() ran the same fixture as its selftest).
    #[test]
    fn golden_fixture_boundaries() {
        if !available() {
            return;
        }
        let data: Vec<u8> = (0..65_659u64).map(|i| ((i * 31 + i / 7) % 251) as u8).collect();
        let got = chunk_descriptors(&data, 1024, 6000, 16 * 1024, SHA256).unwrap();
        let cuts: Vec<(u64, u64)> = got.iter().map(|d| (d.offset, d.length)).collect();
        assert_eq!(cuts, vec![(0, 6162), (6162, 7028), (13190, 7028), (20218, 7028), (27246, 7028), (34274, 7028),
                              (41302, 7028), (48330, 7028), (55358, 7028), (62386, 3273)]);
    }

    #[test]
    fn desc_layout() {
        assert_eq!(std::mem::size_of::<CgDesc>(), 48);
        assert_eq!(std::mem::align_of::<CgDesc>(), 8);
    }
}
