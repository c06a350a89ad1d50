import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

# The engine fails closed while the placeholder GEAR table is installed
# (include/chunker_gpu.h, tables/README.md).  The suite compares the GPU path with the
# oracle under the SAME installed table, so it opts in; tests/test_tables.py checks the
# refusal itself with the variable removed.
os.environ["CHUNKER_AMD_ALLOW_PLACEHOLDER_GEAR"] = "1"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: large inputs")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)
    return torch.device("cuda:0")
