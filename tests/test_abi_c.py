"""A native C consumer of the C ABI (tests/abi_c/abi_check.c), compiled with gcc against
include/chunker_gpu.h and linked to libchunker_amd.so as the Rust shim links it
(rust/chunker-hip): struct layout and enum values checked at compile
time, every entry the shim declares called without a GPU (CG_E_NO_DEVICE, no CPU
fallback), and on a GPU the golden FastCDC vectors through the descriptor, batch, push
and stream entries."""
import json
import os
import shutil
import struct
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
LIBDIR = ROOT / "chunker_amd"


@pytest.fixture(scope="module")
def abi_check(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    out = tmp_path_factory.mktemp("abi_c") / "abi_check"
    cmd = ["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", f"-I{ROOT / 'include'}",
           str(ROOT / "tests" / "abi_c" / "abi_check.c"), "-o", str(out), f"-L{LIBDIR}", "-l:libchunker_amd.so",
           f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath-link,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out


def run(exe, *args, timeout=300):
    env = dict(os.environ, CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR="1")
    return subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=timeout, env=env)


def test_c_abi_without_device(abi_check):
    """Layout, enums, validation messages, error fields and CG_E_NO_DEVICE from a C
    translation unit (no GPU in this container)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present: the no-device answers do not apply")
    r = run(abi_check, "nodevice")
    assert r.returncode == 0, r.stderr + r.stdout
    assert "abi_check nodevice: ok" in r.stdout


@pytest.mark.gpu
def test_c_abi_golden_cases(abi_check, tmp_path):
    """Every case of tests/golden/cdc_golden.json through cg_chunk_descriptors,
    cg_chunk_batch, cg_push_* (uneven pushes) and cg_stream_* from C: the golden
    (offset, length, digest) list each time."""
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    from make_golden import make_input

    gold = json.loads((ROOT / "tests" / "golden" / "cdc_golden.json").read_text())
    path = tmp_path / "cases.bin"
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(gold["cases"])))
        for c in gold["cases"]:
            data = make_input(c["input"])
            mn, avg, mx = c["params"]
            f.write(struct.pack("<6Q", len(data), mn, avg, mx, c["algo"], len(c["chunks"])))
            f.write(data)
            for off, ln, h in c["chunks"]:
                f.write(struct.pack("<QQ", off, ln) + bytes.fromhex(h))
    r = run(abi_check, "cases", str(path))
    assert r.returncode == 0, r.stderr[-4000:] + r.stdout
    assert f"{len(gold['cases'])} / {len(gold['cases'])} passed" in r.stdout


def test_rust_shim_declares_only_header_entries():
    """rust/chunker-hip/src/lib.rs (source only: no cargo in this image) binds exactly
    entries that include/chunker_gpu.h declares and the library exports, with the
    header's parameter counts, and its CgDesc mirrors cg_desc's three fields."""
    import re

    from test_abi import declared_symbols

    rs = (ROOT / "rust" / "chunker-hip" / "src" / "lib.rs").read_text()
    block = rs[rs.index('extern "C" {'):]
    block = block[:block.index("\n}\n")]
    rust_fns = dict(re.findall(r"fn (cg_[a-z0-9_]+)\(([^)]*)\)", block, flags=re.S))
    hdr = re.sub(r"/\*.*?\*/", "", (ROOT / "include" / "chunker_gpu.h").read_text(), flags=re.S)
    hdr_fns = dict(re.findall(r"\b(cg_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", hdr, flags=re.S))
    assert set(rust_fns) <= set(declared_symbols())
    assert len(rust_fns) >= 25
    for name, params in rust_fns.items():
        n_rust = len([p for p in params.split(",") if p.strip()])
        n_hdr = len([p for p in hdr_fns[name].split(",") if p.strip() and p.strip() != "void"])
        assert n_rust == n_hdr, f"{name}: {n_rust} parameters in the shim, {n_hdr} in the header"
    assert re.search(r"pub struct CgDesc \{\s*pub offset: u64,\s*pub length: u64,\s*pub hash: \[u8; 32\],", rs)
