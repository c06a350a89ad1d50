"""ctypes front-end of the CPU oracle (oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker or the timed CPU baseline. The
product package (chunker_amd) never imports this module.

Each function names the reference item it restates (file:line into the
FlakeCache/chunker snapshot); the restatements themselves live in oracle.c.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent
LIB_PATH = HERE / "_build" / "liboracle.so"

BLAKE3 = 0  # HashAlgorithm::Blake3 (src/chunking.rs:55-58 declaration order)
SHA256 = 1  # HashAlgorithm::Sha256

DESC_DTYPE = np.dtype([("offset", "<u8"), ("length", "<u8"), ("hash", "u1", (32,))])


def read_table(name: str) -> tuple[np.ndarray, bool]:
    """Parse tables/<name> -> (u64 array, placeholder flag)."""
    vals, placeholder = [], False
    for line in (ROOT / "tables" / name).read_text().splitlines():
        line = line.strip()
        if line.startswith("#"):
            placeholder |= "placeholder = true" in line
            continue
        if line:
            vals.append(int(line, 16))
    return np.array(vals, dtype=np.uint64), placeholder


GEAR, GEAR_IS_PLACEHOLDER = read_table("fastcdc_v2020_gear.txt")
MASKS, _ = read_table("fastcdc_v2020_masks.txt")
assert GEAR.shape == (256,) and MASKS.shape == (26,)


def build(force: bool = False) -> Path:
    src = HERE / "oracle.c"
    if force or not LIB_PATH.exists() or LIB_PATH.stat().st_mtime < src.stat().st_mtime:
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(str(LIB_PATH))
        u64, sz, p = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p
        L.or_set_tables.argtypes = [p, p]
        L.or_validate.argtypes = [u64, u64, u64, ctypes.c_char_p, sz]
        L.or_validate.restype = ctypes.c_int
        L.or_fastcdc.argtypes = [p, u64, u64, u64, u64, p, p, sz]
        L.or_fastcdc.restype = sz
        L.or_sha256.argtypes = [p, u64, p]
        L.or_blake3.argtypes = [p, u64, p]
        L.or_blake3_stack.argtypes = [p, u64, p]
        L.or_sha256_force_scalar.argtypes = [ctypes.c_int]
        L.or_sha256_uses_shani.restype = ctypes.c_int
        L.or_chunk_descriptors.argtypes = [p, u64, u64, u64, u64, ctypes.c_int, p, sz,
                                           ctypes.POINTER(sz), ctypes.c_int]
        L.or_chunk_descriptors.restype = ctypes.c_int
        L.or_hash_descs.argtypes = [p, p, sz, ctypes.c_int, ctypes.c_int]
        L.or_push_new.argtypes = [u64, u64, u64, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.or_push_new.restype = p
        L.or_push_free.argtypes = [p]
        L.or_push_push.argtypes = [p, p, u64, p, sz, ctypes.POINTER(sz)]
        L.or_push_push.restype = ctypes.c_int
        L.or_push_finish.argtypes = [p, p, sz, ctypes.POINTER(sz)]
        L.or_push_finish.restype = ctypes.c_int
        L.or_push_set_threads.argtypes = [p, ctypes.c_int]
        L.or_push_bytes_consumed.argtypes = [p]
        L.or_push_bytes_consumed.restype = u64
        L.or_set_tables(GEAR.ctypes.data, MASKS.ctypes.data)
        _lib = L
    return _lib


def set_tables(gear: np.ndarray, masks: np.ndarray = MASKS) -> None:
    gear = np.ascontiguousarray(gear, dtype=np.uint64)
    masks = np.ascontiguousarray(masks, dtype=np.uint64)
    lib().or_set_tables(gear.ctypes.data, masks.ctypes.data)


def _buf(data) -> np.ndarray:
    return np.frombuffer(memoryview(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data


def validate(mn: int, avg: int, mx: int) -> tuple[int, str]:
    """ChunkingOptions::validate (src/chunking.rs:190-231) -> (status, message)."""
    msg = ctypes.create_string_buffer(256)
    st = lib().or_validate(mn, avg, mx, msg, 256)
    return st, msg.value.decode()


def capacity(n: int, mn: int) -> int:
    """Upper bound on chunk count: every non-final cut is >= 2*floor(min/2)."""
    return n // max(2 * (mn // 2), 1) + 1


def fastcdc(data, mn: int, avg: int, mx: int) -> list[tuple[int, int]]:
    """fastcdc::v2020::FastCDC::new(data,min,avg,max).collect() (src/chunking.rs:334-336) [ext]."""
    a = _buf(data)
    cap = capacity(len(a), mn)
    offs = np.empty(cap, np.uint64)
    lens = np.empty(cap, np.uint64)
    n = lib().or_fastcdc(a.ctypes.data, len(a), mn, avg, mx, offs.ctypes.data, lens.ctypes.data, cap)
    return list(zip(offs[:n].tolist(), lens[:n].tolist()))


def sha256(data) -> bytes:
    """sha256_hash_raw (src/hashing.rs:36-44)."""
    a = _buf(data)
    out = (ctypes.c_uint8 * 32)()
    lib().or_sha256(a.ctypes.data, len(a), out)
    return bytes(out)


def blake3(data) -> bytes:
    """blake3::hash(data).as_bytes() (src/chunking.rs:68-71)."""
    a = _buf(data)
    out = (ctypes.c_uint8 * 32)()
    lib().or_blake3(a.ctypes.data, len(a), out)
    return bytes(out)


def blake3_stack(data) -> bytes:
    a = _buf(data)
    out = (ctypes.c_uint8 * 32)()
    lib().or_blake3_stack(a.ctypes.data, len(a), out)
    return bytes(out)


def chunk_descriptors(data, mn=None, avg=None, mx=None, algo=SHA256, nthreads=None) -> np.ndarray:
    """chunk_descriptors_with_hash (src/chunking.rs:323-374) -> structured array (DESC_DTYPE)."""
    mn = 256 * 1024 if mn is None else mn
    avg = 1024 * 1024 if avg is None else avg
    mx = 4 * 1024 * 1024 if mx is None else mx
    a = _buf(data)
    cap = capacity(len(a), max(mn, 2))
    out = np.zeros(cap, DESC_DTYPE)
    n = ctypes.c_size_t(0)
    nt = nthreads if nthreads is not None else (os.cpu_count() or 1)
    st = lib().or_chunk_descriptors(a.ctypes.data, len(a), mn, avg, mx, algo, out.ctypes.data, cap,
                                    ctypes.byref(n), nt)
    if st:
        raise ValueError(f"oracle status {st}: {validate(mn, avg, mx)[1]}")
    return out[: n.value]


def hash_descs(data, descs: np.ndarray, algo=SHA256, nthreads=1) -> None:
    a = _buf(data)
    lib().or_hash_descs(a.ctypes.data, descs.ctypes.data, len(descs), algo, nthreads)


# ---------------------------------------------------------------------------
# CAS content ids and Node::put.  The Keccak sponge is
# hashlib's SHAKE-256 (OpenSSL), an implementation independent of the GPU kernel,
# pinned by the reference KAT (crates/core/crypto/src/hash.rs:46-57, test_oracle.py).
# ---------------------------------------------------------------------------
CAS_DOMAIN = b"flakecache-cas"  # crates/core/cas/src/lib.rs:23
CAS_FORMAT_VERSION = 1          # crates/core/cas/src/lib.rs:25
KIND_CHUNK = 0x01               # ObjectKind::Chunk, crates/core/cas/src/lib.rs:36
KIND_LEVEL1_MANIFEST = 0x03     # ObjectKind::Level1Manifest, :40


def shake256_256(data) -> bytes:
    """shake256_256 (crates/core/crypto/src/hash.rs:34-41): first 32 bytes of SHAKE-256."""
    return hashlib.shake_256(bytes(data)).digest(32)


def content_id(kind: int, payload) -> bytes:
    """ContentId::compute (crates/core/cas/src/lib.rs:59-69):
    SHAKE256-256(domain || 0x00 || kind || u16le(version) || u64le(len) || payload)."""
    payload = memoryview(_buf(payload))
    h = hashlib.shake_256()
    h.update(CAS_DOMAIN + b"\x00" + bytes([kind]) + CAS_FORMAT_VERSION.to_bytes(2, "little")
             + len(payload).to_bytes(8, "little"))
    h.update(payload)
    return h.digest(32)


def content_ids(data, descs: np.ndarray, kind: int = KIND_CHUNK, nthreads: int = 1) -> list[bytes]:
    """One ContentId per descriptor span, in order (crates/node/src/lib.rs:118-121);
    spans are hashed on a thread pool (hashlib drops the GIL for large updates)."""
    buf = memoryview(_buf(data))
    spans = [(int(d["offset"]), int(d["length"])) for d in descs]
    one = lambda s: content_id(kind, buf[s[0]:s[0] + s[1]])  # noqa: E731
    if nthreads <= 1 or len(spans) <= 1:
        return [one(s) for s in spans]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(nthreads) as ex:
        return list(ex.map(one, spans))


def node_put(data, mn=None, avg=None, mx=None, nthreads: int = 1):
    """Node::put (crates/node/src/lib.rs:114-132) without the storage writes:
    chunk_data (SHA-256) -> per-chunk ContentId(Chunk) -> manifest id
    ContentId(Level1Manifest, concatenated chunk ids).  Returns (descs, ids, manifest)."""
    descs = chunk_descriptors(data, mn, avg, mx, algo=SHA256, nthreads=nthreads)
    ids = content_ids(data, descs, KIND_CHUNK, nthreads)
    return descs, ids, content_id(KIND_LEVEL1_MANIFEST, b"".join(ids))


class Push:
    """PushChunker (src/chunking.rs:753-829) over drain_finalized_chunks (:541-673)."""

    def __init__(self, mn=None, avg=None, mx=None, algo=SHA256, nthreads=1):
        self.mn = 256 * 1024 if mn is None else mn
        self.avg = 1024 * 1024 if avg is None else avg
        self.mx = 4 * 1024 * 1024 if mx is None else mx
        st = ctypes.c_int(0)
        self.h = lib().or_push_new(self.mn, self.avg, self.mx, algo, ctypes.byref(st))
        if not self.h:
            raise ValueError(validate(self.mn, self.avg, self.mx)[1])
        lib().or_push_set_threads(self.h, nthreads)
        self._cap_bytes = 0

    def _out(self, extra: int):
        self._cap_bytes += extra
        cap = capacity(self._cap_bytes + self.mx, self.mn) + 2
        return np.zeros(cap, DESC_DTYPE), cap

    def push(self, data) -> np.ndarray:
        a = _buf(data)
        out, cap = self._out(len(a))
        n = ctypes.c_size_t(0)
        st = lib().or_push_push(self.h, a.ctypes.data if len(a) else None, len(a), out.ctypes.data, cap,
                                ctypes.byref(n))
        if st:
            raise ValueError(f"oracle push status {st}")
        return out[: n.value]

    def finish(self) -> np.ndarray:
        out, cap = self._out(0)
        n = ctypes.c_size_t(0)
        st = lib().or_push_finish(self.h, out.ctypes.data, cap, ctypes.byref(n))
        if st:
            raise ValueError(f"oracle finish status {st}")
        return out[: n.value]

    def bytes_consumed(self) -> int:
        return lib().or_push_bytes_consumed(self.h)

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:  # module globals are gone at interpreter exit
            try:
                lib().or_push_free(self.h)
            except TypeError:
                pass
            self.h = None
