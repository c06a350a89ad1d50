"""Build chunker_amd/libchunker_amd.so in-tree with hipcc for gfx950."""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

CSRC = Path(__file__).resolve().parent / "csrc"


def build(jobs: int = 8) -> Path:
    env = dict(os.environ)
    env.setdefault("ARCH", "gfx950")
    # the product library and the diagnostics build (scripts/diag_*.py, the DPP probe test)
    subprocess.run(["make", "-s", "-C", str(CSRC), f"-j{jobs}", "all", "diag"], check=True, env=env)
    return CSRC.parent / "libchunker_amd.so"


if __name__ == "__main__":
    print(build())
