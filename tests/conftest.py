"""pytest configuration: `-m gpu` tests need a real MI355X (run via gpurun); everything else is CPU."""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP kernels); run with -m gpu on the GPU box")


def gpu_available() -> bool:
    import torch

    return torch.cuda.is_available()


@pytest.fixture(scope="session")
def golden():
    import json

    with open(ROOT / "tests" / "golden" / "golden_b2.json") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return torch.device("cuda", 0)
