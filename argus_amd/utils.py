"""Pose-order conversions, inference helper and timing (argus/utils.py:110-189).

- ``xyzwxyz_to_xyzxyzw_SE3`` / ``xyzxyzw_to_xyzwxyz_SE3`` (utils.py:110-145): HDF5 stores
  (x, y, z, qw, qx, qy, qz); pypose / the model use (x, y, z, qx, qy, qz, qw). Pure index plumbing.
- ``get_pose(images, model)`` (utils.py:179-189): ``se3(model(images)).Exp()`` -> (B, 7), with the
  Exp on the HIP kernel (argus_se3_exp).
- ``time_torch_fn`` (utils.py:153-171): HIP-event timing of a callable.
- ``draw_spaghetti`` (utils.py:252-275): random black PIL arcs ("spaghetti" occluders) drawn on a
  camera image; the same ``np.random`` draws in the same order as the reference, so a seeded worker
  draws the same arcs.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable

import numpy as np
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


def rotation_angle_error(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """|phi| of Log(Exp(pred) @ target^-1) per sample, in radians: the rotation part of the SE(3)
    geodesic the loss squares (argus/train.py:119; SURVEY.md §8d "rotation-angle component").

    pred (..., 6) se(3), target (..., 7) [t, qx, qy, qz, qw]. The rotation of a product does not
    depend on the translations: q = q_pred (x) conj(q_target), |phi| = 2 atan2(|v|, |w|) (shortest
    angle, sign-invariant like the loss's Log). A reporting metric: elementwise torch on (B, 4)."""
    qp = se3_exp(pred)[..., 3:].double()
    qt = target[..., 3:].to(qp.device).double()
    pv, pw = qp[..., :3], qp[..., 3:]
    tv, tw = -qt[..., :3], qt[..., 3:]
    v = pw * tv + tw * pv + torch.cross(pv, tv, dim=-1)
    w = pw * tw - (pv * tv).sum(-1, keepdim=True)
    return (2.0 * torch.atan2(v.norm(dim=-1), w[..., 0].abs())).float()


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


def draw_spaghetti(img, n_arcs: int = 10, width_range=(1.0, 5.0)):
    """Draw ``n_arcs`` random black arcs on the PIL image ``img`` in place and return it.

    Per arc, in this order: top-left corner (x0 in [0, W), y0 in [0, H)), bottom-right corner
    (x1 in [x0, W), y1 in [y0, H)), start and end angle in [0, 360) degrees, stroke width drawn
    uniformly from ``width_range`` and truncated to int (argus/utils.py:252-275)."""
    from PIL import ImageDraw

    draw = ImageDraw.Draw(img)
    for _ in range(n_arcs):
        x0 = np.random.randint(0, img.width)
        y0 = np.random.randint(0, img.height)
        x1 = np.random.randint(x0, img.width)
        y1 = np.random.randint(y0, img.height)
        a0 = np.random.randint(0, 360)
        a1 = np.random.randint(0, 360)
        w = np.random.uniform(*width_range)
        draw.arc((x0, y0, x1, y1), a0, a1, fill=(0, 0, 0), width=int(w))
    return img
