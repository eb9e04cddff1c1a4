"""SE(3) geodesic pose loss on the MI355X — drop-in for ``geometric_loss_fn`` (argus/train.py:105-119).

``geometric_loss_fn(pred (..., 6) se(3) [rho, phi], target (..., 7) SE(3) [t, qx, qy, qz, qw]) -> (...)``
computes ``sum((Exp(pred) @ target^-1).Log() ** 2, -1)`` in one fused HIP kernel (forward and the
exact gradient, argus_amd/csrc/loss.hip). Unbatched inputs give a 0-d result, batched (B, 6)/(B, 7)
give (B,), as the reference (tests/test_train.py:18-36). ``pred`` / ``target`` may be plain tensors
or pypose LieTensors (anything with ``.tensor()``); there is no CPU implementation — inputs must be
on a cuda device.
"""
from __future__ import annotations

import ctypes as C

import torch

from argus_amd._lib import lib, ptr, stream


def _plain(t) -> torch.Tensor:
    return t.tensor() if hasattr(t, "tensor") and callable(t.tensor) and not isinstance(t, torch.nn.Parameter) \
        and type(t) is not torch.Tensor else t


class _SE3Loss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target):
        B = pred.shape[0]
        p = pred.detach().contiguous().float()
        t = target.detach().contiguous().float()
        loss = torch.empty(B, dtype=torch.float32, device=p.device)
        dpred = torch.empty(B, 6, dtype=torch.float32, device=p.device) if pred.requires_grad else None
        lib().se3_loss(B, ptr(p), ptr(t), ptr(loss), ptr(dpred), C.c_float(1.0), stream())
        ctx.save_for_backward(dpred) if dpred is not None else None
        return loss

    @staticmethod
    def backward(ctx, gout):
        (dpred,) = ctx.saved_tensors
        return dpred * gout[:, None].to(dpred.dtype), None


def geometric_loss_fn(pred, target) -> torch.Tensor:
    """Per-sample squared SE(3) log-distance, argus/train.py:105-119."""
    pred, target = _plain(pred), _plain(target)
    if pred.device.type != "cuda" or target.device.type != "cuda":
        raise RuntimeError("argus_amd.geometric_loss_fn runs on the MI355X HIP kernel: inputs must be cuda tensors")
    if pred.shape[-1] != 6 or target.shape[-1] != 7:
        raise ValueError(f"expected pred (..., 6) and target (..., 7); got {tuple(pred.shape)}, {tuple(target.shape)}")
    lead = torch.broadcast_shapes(pred.shape[:-1], target.shape[:-1])
    p = pred.expand(*lead, 6).reshape(-1, 6)
    t = target.to(pred.device).expand(*lead, 7).reshape(-1, 7)
    if p.shape[0] == 0:
        return pred.new_zeros(lead)
    return _SE3Loss.apply(p, t).reshape(lead)
