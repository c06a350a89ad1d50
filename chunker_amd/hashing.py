"""Digest helpers mirroring src/hashing.rs (sha256_hash_raw :36-44, sha256_hash :26-34,
blake3_hash :46-53), computed by the engine's gfx950 digest kernels (cg_hash)."""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import lib
from .chunking import HashAlgorithm, _as_u8, _check, _ptr


def _digest(data, algo: HashAlgorithm) -> bytes:
    a = _as_u8(data)
    out = (ctypes.c_uint8 * 32)()
    _check(lib.cg_hash(_ptr(a), len(a), int(algo), out))
    return bytes(out)


def sha256_hash_raw(data) -> bytes:
    return _digest(data, HashAlgorithm.Sha256)


def sha256_hash(data) -> str:
    return sha256_hash_raw(data).hex()


def blake3_hash_raw(data) -> bytes:
    return _digest(data, HashAlgorithm.Blake3)


def blake3_hash(data) -> str:
    return blake3_hash_raw(data).hex()


_lib  # re-exported for callers that need the raw ABI
