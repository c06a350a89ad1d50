"""Regenerate tests/golden/cas_vectors.json: ContentId::compute vectors
(crates/core/cas/src/lib.rs:59-69) from the oracle (hashlib SHAKE-256), each
cross-checked against the pure-Python Keccak restatement in tests/test_oracle.py.

Payloads are described, not stored: xorshift64 streams (crates/node/src/lib.rs:192-203)
of the given length and seed.  Lengths straddle the 136-byte SHAKE-256 rate for the
26-byte framing (payload 109/110/111 ...), every kind 1..7 appears.
"""
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import oracle as O  # noqa: E402


def payload(n: int, seed: int) -> bytes:
    out, s = bytearray(), (seed | 1) & 0xFFFFFFFFFFFFFFFF
    while len(out) < n:
        s ^= (s << 13) & 0xFFFFFFFFFFFFFFFF
        s ^= s >> 7
        s ^= (s << 17) & 0xFFFFFFFFFFFFFFFF
        out += s.to_bytes(8, "little")
    return bytes(out[:n])


LENS = [0, 1, 5, 108, 109, 110, 111, 245, 246, 247, 382, 1000, 4096, 65_537]


def main():
    sys.path.insert(0, str(HERE.parent))
    from test_oracle import _shake256_py

    cases = []
    for i, n in enumerate(LENS):
        kind = 1 + i % 7
        p = payload(n, 100 + i)
        cid = O.content_id(kind, p)
        framed = b"flakecache-cas\x00" + bytes([kind]) + b"\x01\x00" + n.to_bytes(8, "little") + p
        assert cid == _shake256_py(framed)
        cases.append({"kind": kind, "len": n, "seed": 100 + i, "id": cid.hex()})
    (HERE / "cas_vectors.json").write_text(json.dumps({"source": "oracle.content_id (hashlib SHAKE-256)",
                                                       "cases": cases}, indent=1) + "\n")


if __name__ == "__main__":
    main()
