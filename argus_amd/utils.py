"""Pose-order conversions, inference helper and timing (argus/utils.py:110-189).

- ``xyzwxyz_to_xyzxyzw_SE3`` / ``xyzxyzw_to_xyzwxyz_SE3`` (utils.py:110-145): HDF5 stores
  (x, y, z, qw, qx, qy, qz); pypose / the model use (x, y, z, qx, qy, qz, qw). Pure index plumbing.
- ``get_pose(images, model)`` (utils.py:179-189): ``se3(model(images)).Exp()`` -> (B, 7), with the
  Exp on the HIP kernel (argus_se3_exp).
- ``time_torch_fn`` (utils.py:153-171): HIP-event timing of a callable.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable

import torch

from argus_amd._lib import lib, ptr, stream


def xyzwxyz_to_xyzxyzw_SE3(xyzwxyz: torch.Tensor) -> torch.Tensor:
    """(x, y, z, qw, qx, qy, qz) -> (x, y, z, qx, qy, qz, qw)."""
    return torch.cat((xyzwxyz[..., :3], xyzwxyz[..., -3:], xyzwxyz[..., -4:-3]), dim=-1)


def xyzxyzw_to_xyzwxyz_SE3(xyzxyzw: torch.Tensor) -> torch.Tensor:
    """(x, y, z, qx, qy, qz, qw) -> (x, y, z, qw, qx, qy, qz)."""
    return torch.cat((xyzxyzw[..., :3], xyzxyzw[..., -1:], xyzxyzw[..., -4:-1]), dim=-1)


def se3_exp(xi: torch.Tensor, canonical_w: bool = False) -> torch.Tensor:
    """se(3) (..., 6) [rho, phi] -> SE(3) (..., 7) [t, qx, qy, qz, qw] on the GPU."""
    if xi.device.type != "cuda":
        raise RuntimeError("argus_amd.se3_exp runs on the HIP kernel: cuda tensors only")
    lead = xi.shape[:-1]
    x = xi.reshape(-1, 6).contiguous().float()
    out = torch.empty(x.shape[0], 7, dtype=torch.float32, device=x.device)
    if x.shape[0]:
        lib().se3_exp(x.shape[0], ptr(x), ptr(out), int(canonical_w), stream())
    return out.reshape(*lead, 7)


def get_pose(images: torch.Tensor, model: torch.nn.Module) -> torch.Tensor:
    """Cube pose (B, 7), quaternion (x, y, z, w), from (B, 3*n_cams, H, W) images."""
    return se3_exp(model(images))


def time_torch_fn(fn: Callable[[], torch.Tensor]) -> tuple:
    """(result, seconds) of ``fn`` measured with device events (utils.py:153-171)."""
    start = torch.cuda.Event(enable_timing=True)
    end = torch.cuda.Event(enable_timing=True)
    start.record()
    result = fn()
    end.record()
    torch.cuda.synchronize()
    return result, start.elapsed_time(end) / 1000
