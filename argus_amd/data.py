"""CameraCubePoseDataset — drop-in for argus/data.py (dataset + configs), without h5py/kornia.

On-disk format (argus/data.py:137-188, tests/conftest.py:18-57): a directory D with ``D/<D.stem>.hdf5``
(root attrs n_cams/W/H; groups train/test with cube_poses (n,7) [x,y,z,qw,qx,qy,qz], q_leap, img_stems
bytes like b"img/img3") and ``D/<stem>_a.png``, ``D/<stem>_b.png`` (uint8 RGB) per sample.

``__getitem__`` returns ``{"images": (3*n_cams, H, W) float32 in [0,1], "cube_pose": (7,) float32
[x,y,z,qx,qy,qz,qw]}`` (data.py:206-229) after the reference's center crop (kornia
``center_crop``: integer start ``int(src/2 - dst/2)``, which with align_corners bilinear sampling at
integer offsets is exact slicing). The HDF5 file is read by ``argus_amd.h5lite`` (h5py is not
installed here).

Augmentation: the "spaghetti" occluder arcs (data.py:212-215, utils.py:252-275) are drawn exactly
as the reference does (same PIL calls and np.random draws; train and val). The kornia photometric
augmentations (data.py:41-103: Planckian jitter, ColorJiggle, Gaussian / motion blur, plasma
shadow) run on the device instead, on whole uint8 batches after the H2D copy
(``argus_amd.augment.DeviceAugmentation``; ``argus_amd.train`` applies it to training batches): the
dataset itself returns them unapplied, and says so once when used outside ``argus_amd.train``.
``cfg_aug=None`` works (the reference crashes on it, data.py:213). ``CameraCubePoseDatasetConfig``
resolves ROOT-relative paths without tripping its own ``frozen=True`` (data.py:126-130).
``uint8=True`` keeps images as uint8 (4x less host->device traffic; the engine converts on device).
"""
from __future__ import annotations

import os
import warnings
from dataclasses import dataclass
from pathlib import Path
from typing import Optional, Union

import numpy as np
import torch
from PIL import Image
from torch.utils.data import Dataset

from argus_amd import ROOT
from argus_amd import h5lite
from argus_amd.utils import draw_spaghetti, xyzwxyz_to_xyzxyzw_SE3

# the kornia photometric augmentations of argus/data.py:41-103 (not applied here)
PHOTOMETRIC_FLAGS = ("random_erasing", "planckian_jitter", "color_jiggle", "blur", "motion_blur", "plasma_shadow",
                     "salt_and_pepper")
_warned = False


@dataclass(frozen=True)
class AugmentationConfig:
    """Same fields as argus/data.py:18-39. ``num_spaghetti`` is applied by the dataset; the photometric
    flags (random erasing and salt-and-pepper included, off in the reference's defaults) by
    ``argus_amd.augment.DeviceAugmentation`` on the device."""

    brightness: Union[float, tuple] = (0.8, 1.0)
    contrast: Union[float, tuple] = (0.5, 1.2)
    saturation: Union[float, tuple] = (0.25, 1.2)
    hue: Union[float, tuple] = (-0.1, 0.1)
    num_spaghetti: int = 10
    color_jiggle: bool = True
    planckian_jitter: bool = True
    random_erasing: bool = False
    blur: bool = True
    motion_blur: bool = True
    plasma_shadow: bool = True
    salt_and_pepper: bool = False


@dataclass(frozen=True)
class CameraCubePoseDatasetConfig:
    """argus/data.py:106-142: dataset directory + center crop (H, W)."""

    dataset_path: Optional[str] = None
    center_crop: Optional[tuple] = (256, 256)

    def __post_init__(self) -> None:
        assert isinstance(self.dataset_path, str), "The dataset path must be a str!"
        path = self.dataset_path
        if not os.path.exists(path):
            if os.path.exists(ROOT + "/" + path):
                path = ROOT + "/" + path
                object.__setattr__(self, "dataset_path", path)
            else:
                raise FileNotFoundError(f"The specified path does not exist: {path}!")
        assert not Path(path).suffix, "The dataset path must point to a directory!"
        if Path(path).is_dir():
            assert os.path.exists(path + f"/{Path(path).stem}.hdf5"), (
                f"There must be an hdf5 file with the name {Path(path).stem}.hdf5!"
            )
            assert os.path.exists(path + "/img"), "The dataset must have an `img` directory!"


def center_crop_slices(src_hw: tuple, dst_hw: tuple) -> tuple:
    """kornia center_crop start offsets: int(src/2 - dst/2) per axis."""
    sy = int(src_hw[0] / 2 - dst_hw[0] / 2)
    sx = int(src_hw[1] / 2 - dst_hw[1] / 2)
    return slice(sy, sy + dst_hw[0]), slice(sx, sx + dst_hw[1])


class CameraCubePoseDataset(Dataset):
    """The dataset for N cameras and a cube (argus/data.py:145-229)."""

    def __init__(self, cfg_dataset: CameraCubePoseDatasetConfig, cfg_aug: Optional[AugmentationConfig] = None,
                 train: bool = True, uint8: bool = False, device_augmentation: bool = False) -> None:
        dataset_path = cfg_dataset.dataset_path
        with h5lite.File(dataset_path + f"/{Path(dataset_path).stem}.hdf5") as f:
            ds = f["train"] if train else f["test"]
            self.n_cams = int(f.attrs["n_cams"])
            cube = torch.from_numpy(np.asarray(ds["cube_poses"][()], dtype=np.float64))
            self.cube_poses = xyzwxyz_to_xyzxyzw_SE3(cube)  # (x, y, z, qx, qy, qz, qw)
            self.q_leap = torch.from_numpy(np.asarray(ds["q_leap"][()]))
            self.img_stems = [s.decode("utf-8") for s in ds["img_stems"][()]]
        self.cfg_aug = cfg_aug
        self.augmentation = None  # photometric augmentations: on the device (argus_amd.augment)
        enabled = [k for k in PHOTOMETRIC_FLAGS if cfg_aug is not None and getattr(cfg_aug, k)]
        global _warned
        if enabled and train and not _warned and not device_augmentation:
            _warned = True
            warnings.warn(f"argus_amd: the photometric augmentations {enabled} are applied on the device by "
                          "argus_amd.augment.DeviceAugmentation (argus_amd.train does); this dataset returns "
                          "them unapplied (the spaghetti occluders are drawn here)", stacklevel=2)
        self.dataset_path = dataset_path
        self.center_crop = cfg_dataset.center_crop
        self.uint8 = uint8
        self.train = train

    def __len__(self) -> int:
        return self.cube_poses.shape[0]

    def __getitem__(self, idx: int) -> dict:
        stem = self.img_stems[idx]
        suffixes = "abcdefghijklmnopqrstuvwxyz"[: self.n_cams]
        pil = [Image.open(f"{self.dataset_path}/{stem}_{s}.png").convert("RGB") for s in suffixes]
        if self.cfg_aug is not None and self.cfg_aug.num_spaghetti > 0:  # data.py:212-215, train and val
            pil = [draw_spaghetti(im, self.cfg_aug.num_spaghetti) for im in pil]
        imgs = [np.asarray(im) for im in pil]
        arr = np.concatenate(imgs, axis=-1).transpose(2, 0, 1)  # (3*n_cams, H, W) uint8
        if self.center_crop and tuple(arr.shape[-2:]) != tuple(self.center_crop):
            ys, xs = center_crop_slices(arr.shape[-2:], self.center_crop)
            arr = arr[:, ys, xs]
        images = torch.from_numpy(np.ascontiguousarray(arr))
        if not self.uint8:
            images = images.to(torch.float32) / 255.0
        return {"images": images, "cube_pose": self.cube_poses[idx].to(torch.float32)}
