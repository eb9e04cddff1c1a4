"""SE(3) geodesic loss restated — TEST INFRASTRUCTURE (oracle), never product code.

Reference: ``geometric_loss_fn`` (``argus/train.py:105-119``)::

    torch.sum((pp.se3(pred).Exp() @ target.Inv()).Log() ** 2, axis=-1)

pypose (``pyproject.toml:24`` ``pypose>=0.6.7``, unpinned, absent from /root/reference and this
image) supplies Exp / Inv / @ / Log. Its published closed forms, in its conventions (se3 = [rho, phi];
SE3 = [t (3), q (xyzw)]), restated here:

    Exp : q = [sin(th/2)/th * phi, cos(th/2)], th=|phi|;  t = J_l(phi) rho
          J_l = I + (1-cos th)/th^2 K + (th - sin th)/th^3 K^2   (Taylor for th -> 0)
    Inv : q^-1 = conj(q); t^-1 = -R(q^-1) t
    Mul : q = q1 (x) q2;  t = t1 + R(q1) t2
    Log : phi = 2 atan(|v|/w)/|v| * v  (sign-invariant, shortest angle; Taylor as |v| -> 0)
          tau = J_l^-1(phi) t,  J_l^-1 = I - K/2 + (1 - (th/2)cot(th/2))/th^2 K^2  (1/12 at th -> 0)
    loss = |tau|^2 + |phi|^2

Everything is plain differentiable torch, so ``torch.autograd`` in fp64 gives the oracle gradient
(the Euclidean gradient of the composite map equals pypose's Lie-Jacobian backward,
2 xi_r^T J_l^-1(xi_r) J_l(pred)).
"""
from __future__ import annotations

import torch

_SMALL = 1e-4  # switch to Taylor series below this angle / norm (value is fp64/fp32-safe)


def _skew(v: torch.Tensor) -> torch.Tensor:
    x, y, z = v.unbind(-1)
    o = torch.zeros_like(x)
    return torch.stack(
        [torch.stack([o, -z, y], -1), torch.stack([z, o, -x], -1), torch.stack([-y, x, o], -1)], -2
    )


def quat_mul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Hamilton product, xyzw."""
    av, aw = a[..., :3], a[..., 3:]
    bv, bw = b[..., :3], b[..., 3:]
    v = aw * bv + bw * av + torch.cross(av, bv, dim=-1)
    w = aw * bw - (av * bv).sum(-1, keepdim=True)
    return torch.cat([v, w], -1)


def quat_rotate(q: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
    v, w = q[..., :3], q[..., 3:]
    t = 2.0 * torch.cross(v, p, dim=-1)
    return p + w * t + torch.cross(v, t, dim=-1)


def so3_jl(phi: torch.Tensor) -> torch.Tensor:
    th = phi.norm(dim=-1, keepdim=True)[..., None]
    K = _skew(phi)
    small = th < _SMALL
    th_s = torch.where(small, torch.ones_like(th), th)
    c1 = torch.where(small, 0.5 - th**2 / 24 + th**4 / 720, (1 - torch.cos(th_s)) / th_s**2)
    c2 = torch.where(small, 1.0 / 6 - th**2 / 120 + th**4 / 5040, (th_s - torch.sin(th_s)) / th_s**3)
    eye = torch.eye(3, dtype=phi.dtype).expand(K.shape)
    return eye + c1 * K + c2 * (K @ K)


def so3_jl_inv(phi: torch.Tensor) -> torch.Tensor:
    th = phi.norm(dim=-1, keepdim=True)[..., None]
    K = _skew(phi)
    small = th < _SMALL
    th_s = torch.where(small, torch.ones_like(th), th)
    half = th_s / 2
    c2 = torch.where(
        small, 1.0 / 12 + th**2 / 720 + th**4 / 30240, (1 - half * torch.cos(half) / torch.sin(half)) / th_s**2
    )
    eye = torch.eye(3, dtype=phi.dtype).expand(K.shape)
    return eye - 0.5 * K + c2 * (K @ K)


def se3_exp(xi: torch.Tensor) -> torch.Tensor:
    rho, phi = xi[..., :3], xi[..., 3:]
    th = phi.norm(dim=-1, keepdim=True)
    small = th < _SMALL
    th_s = torch.where(small, torch.ones_like(th), th)
    imag = torch.where(small, 0.5 - th**2 / 48 + th**4 / 3840, torch.sin(th_s / 2) / th_s)
    real = torch.where(small, 1 - th**2 / 8 + th**4 / 384, torch.cos(th_s / 2))
    q = torch.cat([imag * phi, real], -1)
    t = (so3_jl(phi) @ rho[..., None])[..., 0]
    return torch.cat([t, q], -1)


def se3_inv(T: torch.Tensor) -> torch.Tensor:
    t, q = T[..., :3], T[..., 3:]
    qi = torch.cat([-q[..., :3], q[..., 3:]], -1)
    return torch.cat([-quat_rotate(qi, t), qi], -1)


def se3_mul(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    ta, qa = A[..., :3], A[..., 3:]
    tb, qb = B[..., :3], B[..., 3:]
    return torch.cat([ta + quat_rotate(qa, tb), quat_mul(qa, qb)], -1)


def se3_log(T: torch.Tensor) -> torch.Tensor:
    t, q = T[..., :3], T[..., 3:]
    v, w = q[..., :3], q[..., 3:]
    n = v.norm(dim=-1, keepdim=True)
    small = n < _SMALL
    n_s = torch.where(small, torch.ones_like(n), n)
    w_s = torch.where(w == 0, torch.full_like(w, 1e-30), w)
    factor = torch.where(small, 2.0 / w_s - (2.0 / 3.0) * n**2 / w_s**3, 2.0 * torch.atan(n_s / w_s) / n_s)
    phi = factor * v
    tau = (so3_jl_inv(phi) @ t[..., None])[..., 0]
    return torch.cat([tau, phi], -1)


def geometric_loss(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """Per-sample loss (``argus/train.py:119``): sum((Exp(pred) @ target^-1).Log()**2, -1)."""
    return (se3_log(se3_mul(se3_exp(pred), se3_inv(target))) ** 2).sum(-1)


def loss_and_grad(pred: torch.Tensor, target: torch.Tensor, mean: bool = True):
    """fp64 oracle: per-sample losses and d(mean loss)/d(pred) (or d(sum)/d(pred) if not ``mean``)."""
    p = pred.detach().to(torch.float64).requires_grad_(True)
    losses = geometric_loss(p, target.detach().to(torch.float64))
    total = losses.mean() if mean else losses.sum()
    (g,) = torch.autograd.grad(total, p)
    return losses.detach(), g


def random_targets(n: int, generator: torch.Generator | None = None, sigma: float = 0.5) -> torch.Tensor:
    """SURVEY.md §8d synthetic targets: T = Exp(xi), xi ~ N(0, sigma^2)^6, quaternion w >= 0, fp32."""
    xi = torch.randn(n, 6, generator=generator, dtype=torch.float64) * sigma
    T = se3_exp(xi)
    sign = torch.where(T[..., 6:7] < 0, -1.0, 1.0)
    T = torch.cat([T[..., :3], T[..., 3:] * sign], -1)
    return T.to(torch.float32)
