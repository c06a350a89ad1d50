"""Install fastcdc 4.0.1's v2020 GEAR / MASKS tables into this tree, after checking them.

The crate is not vendored in the reference (Cargo.lock:530-533 pins fastcdc 4.0.1 from
crates.io) and this build ships a labelled PLACEHOLDER GEAR (tables/README.md), so the
engine fails closed until the real tables are installed.  On a machine with the crate
(e.g. ~/.cargo/registry/src/*/fastcdc-4.0.1/src/v2020/mod.rs):

    python scripts/install_fastcdc_tables.py path/to/fastcdc-4.0.1/src/v2020/mod.rs

The source's `GEAR: [u64; 256]` and `MASKS: [u64; 26]` array literals are parsed (a
plain text file of 256 hex values is accepted for GEAR alone), then:
  1. every mask must live in bits 0..47 (the windowed GPU scan's premise);
  2. the CPU oracle with these tables must reproduce the reference's golden boundary
     fixture (src/chunking.rs:1266-1297) exactly -- otherwise nothing is written;
  3. tables/fastcdc_v2020_{gear,masks}.txt are rewritten (placeholder = false),
     chunker_amd/csrc/gear_table.h regenerated, tests/golden/cdc_golden.json
     regenerated from the oracle.
Rebuild afterwards (python -c 'import __graft_entry__ as g; g.build()'); the engine then
runs its GPU selftest against the same fixture on first use.
"""
from __future__ import annotations

import argparse
import re
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

REFERENCE_FIXTURE = [(0, 6162), (6162, 7028), (13190, 7028), (20218, 7028), (27246, 7028), (34274, 7028),
                     (41302, 7028), (48330, 7028), (55358, 7028), (62386, 3273)]


def parse_array(text: str, name: str, n: int) -> list[int] | None:
    m = re.search(rf"\b{name}\b[^=]*=\s*\[(.*?)\]", text, flags=re.S)
    if not m:
        return None
    body = re.sub(r"//[^\n]*", "", m.group(1))
    vals = [int(v.replace("_", ""), 0) for v in re.findall(r"0x[0-9a-fA-F_]+|\b\d[\d_]*\b", body)]
    if len(vals) != n:
        raise SystemExit(f"{name}: found {len(vals)} values, expected {n}")
    return vals


def fixture() -> np.ndarray:
    i = np.arange(64 * 1024 + 123, dtype=np.int64)
    return ((i * 31 + i // 7) % 251).astype(np.uint8)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("source", type=Path, help="fastcdc v2020 source (mod.rs) or a text file of 256 hex GEAR values")
    ap.add_argument("--dry-run", action="store_true", help="validate only")
    args = ap.parse_args()
    text = args.source.read_text()
    gear = parse_array(text, "GEAR", 256)
    masks = parse_array(text, "MASKS", 26)
    if gear is None:  # plain list of values
        gear = [int(v, 16) for v in re.findall(r"0x[0-9a-fA-F]+", text)]
        if len(gear) != 256:
            raise SystemExit(f"no GEAR array and {len(gear)} hex values in {args.source}")
    from oracle import oracle as O

    m = np.array(masks, np.uint64) if masks is not None else O.MASKS.copy()
    bad = [i for i in range(26) if int(m[i]) >> 48]
    if bad:
        raise SystemExit(f"MASKS{bad} have bits above 47: the windowed GPU scan cannot run these tables")
    g = np.array(gear, np.uint64)
    O.set_tables(g, m)
    got = O.fastcdc(fixture(), 1024, 6000, 16 * 1024)
    if got != REFERENCE_FIXTURE:
        raise SystemExit(f"REFUSED: these tables give {len(got)} chunks {got[:3]}... on the reference fixture "
                         f"(src/chunking.rs:1266-1297), not {REFERENCE_FIXTURE[:3]}...")
    print("reference fixture reproduced by the oracle with the supplied tables")
    if args.dry_run:
        return 0
    src = args.source.name
    (ROOT / "tables" / "fastcdc_v2020_gear.txt").write_text(
        f"# placeholder = false  (fastcdc 4.0.1 v2020 GEAR, installed from {src} by "
        "scripts/install_fastcdc_tables.py; reference fixture verified)\n"
        + "".join(f"0x{int(v):016x}\n" for v in g))
    (ROOT / "tables" / "fastcdc_v2020_masks.txt").write_text(
        f"# fastcdc 4.0.1 v2020 MASKS[0..26] ({'installed from ' + src if masks is not None else 'unchanged'})\n"
        + "".join(f"0x{int(v):016x}\n" for v in m))
    subprocess.run([sys.executable, str(ROOT / "tables" / "gen_header.py")], check=True)
    subprocess.run([sys.executable, str(ROOT / "tests" / "golden" / "make_golden.py")], check=True)
    print("installed; rebuild with: python -c 'import __graft_entry__ as g; g.build()'")
    return 0


if __name__ == "__main__":
    sys.exit(main())
