"""CPU: HDF5 reader against h5py-written fixtures; CameraCubePoseDataset semantics
(reference tests/test_data.py: lengths 10/5, keys, (7,) poses, center crop)."""
import json
from pathlib import Path

import numpy as np
import pytest
import torch

from argus_amd import h5lite

GOLD = Path(__file__).resolve().parent / "golden" / "h5"


@pytest.mark.parametrize("libver", ["earliest", "latest", "vlen_earliest", "vlen_latest"])
def test_h5lite_reads_h5py_files(libver):
    """vlen_*: img_stems written as a plain list of str (argus/data_generation.py:256,264), which
    h5py>=3 stores as variable-length strings (global heap); read back as bytes like h5py's [()]."""
    fx = json.loads((GOLD / "fixtures.json").read_text())
    with h5lite.File(str(GOLD / f"ds_{libver}" / f"ds_{libver}.hdf5")) as f:
        assert {k: int(v) for k, v in f.attrs.items()} == fx["attrs"]
        assert sorted(f.keys()) == ["test", "train"]
        for g in ("train", "test"):
            assert np.array_equal(f[g]["cube_poses"][()], np.array(fx["cube_poses"][g]))
            assert np.array_equal(f[f"{g}/q_leap"][()], np.array(fx["q_leap"][g]))
            assert [s.decode() for s in f[g]["img_stems"][()]] == fx["img_stems"][g]


def _make_dataset(tmp_path, libver="earliest", hw=(256, 256)):
    from conftest import make_dummy_dataset

    return Path(make_dummy_dataset(tmp_path, libver, hw))


def test_dataset_items(tmp_path):
    from argus_amd.data import CameraCubePoseDataset, CameraCubePoseDatasetConfig
    from argus_amd.utils import xyzwxyz_to_xyzxyzw_SE3

    d = _make_dataset(tmp_path)
    fx = json.loads((GOLD / "fixtures.json").read_text())
    cfg = CameraCubePoseDatasetConfig(str(d))
    tr, te = CameraCubePoseDataset(cfg, train=True), CameraCubePoseDataset(cfg, train=False)
    assert len(tr) == 10 and len(te) == 5
    ex = tr[3]
    assert set(ex) == {"images", "cube_pose"}
    assert ex["images"].shape == (6, 256, 256) and ex["images"].dtype == torch.float32
    assert ex["cube_pose"].shape == (7,)
    want = xyzwxyz_to_xyzxyzw_SE3(torch.tensor(fx["cube_poses"]["train"][3])).float()
    assert torch.equal(ex["cube_pose"], want)
    from PIL import Image

    a = np.array(Image.open(d / "img" / "img3_a.png"))
    assert torch.equal(ex["images"][:3], torch.from_numpy(a).permute(2, 0, 1).float() / 255.0)


def test_dataset_reads_datagen_vlen_stems(tmp_path):
    from argus_amd.data import CameraCubePoseDataset, CameraCubePoseDatasetConfig

    d = _make_dataset(tmp_path, "vlen_latest")
    ds = CameraCubePoseDataset(CameraCubePoseDatasetConfig(str(d)), train=False)
    assert ds.img_stems == [f"img/img{i}" for i in range(10, 15)]
    assert ds[4]["images"].shape == (6, 256, 256)


def test_center_crop(tmp_path):
    from argus_amd.data import CameraCubePoseDataset, CameraCubePoseDatasetConfig

    d = _make_dataset(tmp_path, "latest", hw=(376, 672))
    ds = CameraCubePoseDataset(CameraCubePoseDatasetConfig(str(d), center_crop=(256, 256)), train=True)
    x = ds[0]["images"]
    assert x.shape == (6, 256, 256)
    from PIL import Image

    a = np.asarray(Image.open(d / "img" / "img0_a.png"))
    assert torch.equal(x[:3], torch.from_numpy(a[60:316, 208:464]).permute(2, 0, 1).float() / 255.0)
    ds = CameraCubePoseDataset(CameraCubePoseDatasetConfig(str(d), center_crop=(128, 128)), train=False)
    assert ds[0]["images"].shape[-2:] == (128, 128)
