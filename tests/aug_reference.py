"""Torch / numpy restatement of the device augmentation formulas (csrc/augment.hip) — the checker
for tests/test_gpu_augment.py. Each function follows the formula stated in augment.hip's header
(kornia's published definitions); kornia itself is absent, so this pins the kernels to the stated
formulas, not to kornia."""
import math

import numpy as np
import torch

TP = 2 * math.pi


def rgb2hsv(c):  # c: (3, H, W) float64
    r, g, b = c
    mx, _ = c.max(0)
    mn, _ = c.min(0)
    d = mx - mn
    s = d / (mx + 1e-6)
    h = torch.zeros_like(mx)
    safe = torch.where(d == 0, torch.ones_like(d), d)
    hr = torch.fmod((g - b) / safe, 6.0)
    hg = (b - r) / safe + 2.0
    hb = (r - g) / safe + 4.0
    h = torch.where(mx == r, hr, torch.where(mx == g, hg, hb))
    h = torch.where(d == 0, torch.zeros_like(h), h) * (TP / 6.0)
    h = torch.where(h < 0, h + TP, h)
    return h, s, mx


def hsv2rgb(h, s, v):
    hn = h / TP * 6.0
    hn = hn - 6.0 * torch.floor(hn / 6.0)
    hi = torch.floor(hn)
    f = hn - hi
    p, q, t = v * (1 - s), v * (1 - f * s), v * (1 - (1 - f) * s)
    hi = hi.long().clamp(0, 5)
    r = torch.stack([v, q, p, p, t, v])
    g = torch.stack([t, v, v, q, p, p])
    b = torch.stack([p, p, t, v, v, q])
    pick = lambda x: torch.gather(x, 0, hi[None]).squeeze(0)  # noqa: E731
    return torch.stack([pick(r), pick(g), pick(b)])


def color(img_u8, P):
    """(3, H, W) uint8 -> float64 after Planckian gains and the ColorJiggle ops."""
    c = (img_u8.double() / 255.0 * torch.tensor(P["gain"], dtype=torch.float64)[:, None, None]).clamp(0, 1)
    if P["jiggle"]:
        for o in range(4):
            op = (int(P["order"]) >> (2 * o)) & 3
            if op == 0:
                c = (c + (float(P["bright"]) - 1.0)).clamp(0, 1)
            elif op == 1:
                c = (c * float(P["contrast"])).clamp(0, 1)
            else:
                h, s, v = rgb2hsv(c)
                if op == 2:
                    s = (s * float(P["sat"])).clamp(0, 1)
                else:
                    h = torch.fmod(h + float(P["hue"]) * TP, TP)
                    h = torch.where(h < 0, h + TP, h)
                c = hsv2rgb(h, s, v)
    return c


def reflect_idx(i, n):
    i = np.abs(i)
    i = np.where(i >= n, 2 * n - 2 - i, i)
    return np.clip(i, 0, n - 1)


def blur(c, w5):
    if w5[2] == 0:
        return c
    H, W = c.shape[-2:]
    w5 = torch.tensor(np.asarray(w5, dtype=np.float64))
    xs = np.arange(W)
    t = sum(w5[k] * c[..., reflect_idx(xs + k - 2, W)] for k in range(5))
    ys = np.arange(H)
    return sum(w5[k] * t[..., reflect_idx(ys + k - 2, H), :] for k in range(5))


def motion(c, k9):
    k = torch.tensor(np.asarray(k9, dtype=np.float64)).reshape(1, 1, 3, 3).repeat(3, 1, 1, 1)
    if float(k.abs().sum()) == 0:
        return c
    return torch.nn.functional.conv2d(c[None], k, padding=1, groups=3)[0]


M32 = 0xFFFFFFFF


def lattice(seed, o, gx, gy):
    h = ((seed * 0x9E3779B1) ^ (o * 0x85EBCA77) ^ (gx.astype(np.int64) * 0xC2B2AE3D) ^ (gy.astype(np.int64) * 0x27D4EB2F)) & M32
    h ^= h >> 15
    h = (h * 0x2C1B3C6D) & M32
    h ^= h >> 12
    h = (h * 0x297A2D39) & M32
    h ^= h >> 15
    return (h >> 8).astype(np.float64) / 16777216.0


def plasma(seed, rough, H, W):
    y, x = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    cell, amp, tot, norm = max(H, W) * 0.5, 1.0, 0.0, 0.0
    o = 0
    while o < 6 and cell >= 1.0:
        fy, fx = y / cell, x / cell
        gy, gx = np.floor(fy).astype(np.int64), np.floor(fx).astype(np.int64)
        ty, tx = fy - gy, fx - gx
        v00, v01 = lattice(seed, o, gx, gy), lattice(seed, o, gx + 1, gy)
        v10, v11 = lattice(seed, o, gx, gy + 1), lattice(seed, o, gx + 1, gy + 1)
        v = (v00 * (1 - tx) + v01 * tx) * (1 - ty) + (v10 * (1 - tx) + v11 * tx) * ty
        tot = tot + amp * v
        norm += amp
        amp *= float(np.float32(rough))
        cell *= 0.5
        o += 1
    return torch.tensor(tot / norm)


def augment_image(img_u8, P):
    """Full per-image pipeline of argus_augment_photometric in float64."""
    c = blur(color(img_u8, P), P["blur_w"])
    c = motion(c, P["motion"])
    if float(P["plasma_int"]) != 0:
        n = plasma(int(P["seed"]), P["plasma_rough"], *c.shape[-2:])
        c = torch.where((n < float(P["plasma_q"]))[None], c * (1 + float(P["plasma_int"])), c)
    return c.clamp(0, 1)
