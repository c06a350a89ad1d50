"""Regenerate tests/golden/cdc_golden.json from the CPU oracle.

Inputs are described, not stored: xorshift64 streams (crates/node/src/lib.rs:192-203),
the reference fixture pattern (src/chunking.rs:1269-1272) and constant fills.  Every
SHA-256 digest is cross-checked against hashlib before it is written.  The file
records the SHA-256 of the GEAR table it was made with (placeholder table: see
tables/README.md), so a table change forces regeneration.
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import oracle as O  # noqa: E402


def xorshift(seed, n):
    out = np.empty((n + 7) // 8, np.uint64)
    s = (seed | 1) & 0xFFFFFFFFFFFFFFFF
    for i in range(len(out)):
        s ^= (s << 13) & 0xFFFFFFFFFFFFFFFF
        s ^= s >> 7
        s ^= (s << 17) & 0xFFFFFFFFFFFFFFFF
        out[i] = s
    return out.view(np.uint8)[:n].tobytes()


def make_input(spec):
    kind, n = spec["kind"], spec["len"]
    if kind == "xorshift":
        return xorshift(spec["seed"], n)
    if kind == "fixture":
        return bytes(((i * 31 + i // 7) % 251) for i in range(n))
    if kind == "fill":
        return bytes([spec["byte"]]) * n
    raise ValueError(kind)


INPUTS = [
    {"kind": "xorshift", "seed": 1, "len": 1},
    {"kind": "xorshift", "seed": 2, "len": 63},
    {"kind": "xorshift", "seed": 3, "len": 1023},
    {"kind": "xorshift", "seed": 4, "len": 1025},
    {"kind": "xorshift", "seed": 5, "len": 65_537},
    {"kind": "xorshift", "seed": 6, "len": 300_001},
    {"kind": "fixture", "len": 64 * 1024 + 123},
    {"kind": "fill", "byte": 0, "len": 70_000},
    {"kind": "fill", "byte": 42, "len": 3 * 1024 * 1024 + 321},
]
PARAMS = [(64, 256, 1024), (1024, 6000, 16384), (4097, 10000, 70001), (16384, 32768, 65536)]


def main():
    cases = []
    for spec in INPUTS:
        data = make_input(spec)
        for params in PARAMS:
            if spec["len"] > 400_000 and params[0] < 16384:
                continue
            for algo in (O.SHA256, O.BLAKE3):
                descs = O.chunk_descriptors(data, *params, algo=algo, nthreads=4)
                chunks = [[int(d["offset"]), int(d["length"]), bytes(d["hash"]).hex()] for d in descs]
                if algo == O.SHA256:
                    for off, ln, hx in chunks:
                        assert hashlib.sha256(data[off:off + ln]).hexdigest() == hx
                cases.append({"input": spec, "params": list(params), "algo": algo, "chunks": chunks})
    out = {
        "generator": "tests/golden/make_golden.py (CPU oracle; SHA-256 digests checked by hashlib)",
        "gear_placeholder": bool(O.GEAR_IS_PLACEHOLDER),
        "gear_sha256": hashlib.sha256(O.GEAR.tobytes()).hexdigest(),
        "cases": cases,
    }
    (HERE / "cdc_golden.json").write_text(json.dumps(out, separators=(",", ":")) + "\n")


if __name__ == "__main__":
    main()
