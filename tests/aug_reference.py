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
    """(3, H, W) uint8 -> float64 after random erasing, Planckian gains and the ColorJiggle ops."""
    c = erase(img_u8.double() / 255.0, P)
    c = (c * torch.tensor(P["gain"], dtype=torch.float64)[:, None, None]).clamp(0, 1)
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


def hash_u01(seed, stream, idx):
    """augment.hip hash_u01: uniform in [0, 1) from (seed, stream, index), uint32 arithmetic."""
    idx = np.asarray(idx, dtype=np.uint64)
    h = ((int(seed) * 0x9E3779B1) & M32) ^ ((int(stream) * 0x85EBCA77) & M32) ^ ((idx * 0xC2B2AE3D) & M32)
    h = np.asarray(h, dtype=np.uint64)
    h ^= h >> 15
    h = (h * 0x2C1B3C6D) & M32
    h ^= h >> 12
    h = (h * 0x297A2D39) & M32
    h ^= h >> 15
    return (h >> 8).astype(np.float64) / 16777216.0


def diamond_square(seed, rough, H, W):
    """The plasma map of augment.hip's header: (2^k + 1)^2 grid, corners U[0, 1), per level the
    diamond then the square step with (U - 0.5) * rough^(level + 1) noise; H x W crop, min-max to [0, 1]."""
    k = 1
    while (1 << k) < max(H, W) - 1:
        k += 1
    S = (1 << k) + 1
    g = np.zeros((S, S))
    for y in (0, S - 1):
        for x in (0, S - 1):
            g[y, x] = hash_u01(seed, 0, y * S + x)
    rough = float(np.float32(rough))
    step, level, amp = S - 1, 0, 1.0
    while step >= 2:
        half = step // 2
        amp = amp * rough
        m = (S - 1) // step
        # diamond
        c = np.arange(m) * step + half
        yy, xx = np.meshgrid(c, c, indexing="ij")
        mean = 0.25 * ((g[yy - half, xx - half] + g[yy - half, xx + half]) + (g[yy + half, xx - half] + g[yy + half, xx + half]))
        g[yy, xx] = mean + (hash_u01(seed, 1 + 2 * level, yy * S + xx) - 0.5) * amp
        # square
        ys1, xs1 = np.meshgrid(np.arange(m + 1) * step, np.arange(m) * step + half, indexing="ij")
        ys2, xs2 = np.meshgrid(np.arange(m) * step + half, np.arange(m + 1) * step, indexing="ij")
        ys, xs = np.concatenate([ys1.ravel(), ys2.ravel()]), np.concatenate([xs1.ravel(), xs2.ravel()])
        tot, cnt = np.zeros(len(ys)), np.zeros(len(ys))
        for dy, dx in ((-half, 0), (half, 0), (0, -half), (0, half)):
            ny, nx = ys + dy, xs + dx
            ok = (ny >= 0) & (ny < S) & (nx >= 0) & (nx < S)
            tot[ok] += g[ny[ok], nx[ok]]
            cnt[ok] += 1
        g[ys, xs] = tot / cnt + (hash_u01(seed, 2 + 2 * level, ys * S + xs) - 0.5) * amp
        step, level = half, level + 1
    crop = g[:H, :W]
    lo, hi = crop.min(), crop.max()
    return torch.tensor((crop - lo) / (hi - lo) if hi > lo else np.zeros_like(crop))


def erase(c, P):
    for e in range(2):
        y0, x0, h, w = (int(v) for v in P["erase"][e])
        if h > 0:
            c = c.clone()
            c[:, y0:y0 + h, x0:x0 + w] = float(P["erase_val"][e])
    return c


def salt_pepper(c, P):
    amount = float(np.float32(P["sp_amount"]))
    if amount <= 0:
        return c
    H, W = c.shape[-2:]
    idx = np.arange(H * W)
    noisy = hash_u01(int(P["sp_seed"]), 0, idx) < amount
    salt = hash_u01(int(P["sp_seed"]), 1, idx) < float(np.float32(P["sp_salt"]))
    val = torch.tensor(salt.astype(np.float64)).reshape(H, W)
    return torch.where(torch.tensor(noisy).reshape(H, W)[None], val[None], c)


def augment_image(img_u8, P):
    """Full per-image pipeline of argus_augment_photometric in float64."""
    c = blur(color(img_u8, P), P["blur_w"])
    c = motion(c, P["motion"])
    if float(P["plasma_int"]) != 0:
        n = diamond_square(int(P["seed"]), P["plasma_rough"], *c.shape[-2:])
        c = torch.where((n < float(np.float32(P["plasma_q"])))[None], c + float(np.float32(P["plasma_int"])), c)
    return salt_pepper(c.clamp(0, 1), P)
