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


def make_dummy_dataset(root: Path, libver: str = "earliest", hw=(256, 256), seed: int = 0) -> str:
    """The reference tests' dummy dataset (tests/conftest.py:14-57): 10 train / 5 test samples, two
    random RGB PNGs each, poses from the committed h5py-written fixture file (h5py is absent here)."""
    import numpy as np
    from PIL import Image

    d = root / f"ds_{libver}"
    (d / "img").mkdir(parents=True, exist_ok=True)
    src = ROOT / "tests" / "golden" / "h5" / f"ds_{libver}" / f"ds_{libver}.hdf5"
    (d / f"ds_{libver}.hdf5").write_bytes(src.read_bytes())
    rng = np.random.default_rng(seed)
    for i in range(15):
        for s in "ab":
            Image.fromarray(rng.integers(0, 256, (*hw, 3), dtype=np.uint8)).save(d / "img" / f"img{i}_{s}.png")
    return str(d)


@pytest.fixture(scope="session")
def dummy_data_path(tmp_path_factory) -> str:
    return make_dummy_dataset(tmp_path_factory.mktemp("tmp"))
