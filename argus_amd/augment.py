"""Photometric training augmentations on the device — argus/data.py:41-103 after the H2D copy.

The reference runs a kornia ``AugmentationSequential`` in every CPU data-loader worker on each
sample's two camera images (data.py:222-224): RandomErasing x2 (when ``random_erasing``),
RandomPlanckianJitter("blackbody", p=0.5), ColorJiggle(brightness, contrast, saturation, hue;
same_on_batch: one draw per sample, p=1), RandomGaussianBlur((5, 5), sigma U(3, 8), p=0.5),
RandomMotionBlur(3, angle U(-35, 35), direction U(-0.5, 0.5), p=0.7), RandomPlasmaShadow(roughness
U(0.1, 0.4), intensity U(-0.6, 0), quantity U(0, 0.5), p=1), RandomSaltAndPepperNoise(p=0.7) (when
``salt_and_pepper``). ``DeviceAugmentation`` draws the per-image parameters from a seeded torch
generator on the host and applies them to the uint8 batch on the GPU in one
``argus_augment_photometric`` call (csrc/augment.hip, fp32 out).

Parity: kornia is not installed in this image, so the kernels restate kornia's published
definitions (formulas in augment.hip's header) and are pinned to a float64 restatement of those
same formulas (tests/aug_reference.py, tests/test_gpu_augment.py); equality with kornia itself is
unpinned. Known deviation: the blackbody gains come from Tanner Helland's fit of the Planckian locus
(3000-15000 K in 500 K steps), normalized to green, not from kornia's own coefficient table (not
available offline).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from argus_amd._lib import lib, ptr, stream

# C layout of AugParams (csrc/augment.hip): 40 four-byte fields
PARAMS_DTYPE = np.dtype([("gain", "<f4", 3), ("bright", "<f4"), ("contrast", "<f4"), ("sat", "<f4"),
                         ("hue", "<f4"), ("order", "<i4"), ("jiggle", "<i4"), ("blur_w", "<f4", 5),
                         ("motion", "<f4", 9), ("plasma_int", "<f4"), ("plasma_q", "<f4"),
                         ("plasma_rough", "<f4"), ("seed", "<u4"), ("erase", "<i4", (2, 4)),
                         ("erase_val", "<f4", 2), ("sp_amount", "<f4"), ("sp_salt", "<f4"), ("sp_seed", "<u4")])

# data.py:52-64: the two RandomErasing transforms (p, scale, ratio, value)
ERASERS = ((0.5, (0.02, 0.1), (2.0, 3.0), 0.0), (0.5, (0.02, 0.05), (0.8, 1.2), 1.0))
# kornia RandomSaltAndPepperNoise defaults (amount, salt_vs_pepper); p = 0.7 (data.py:95)
SALT_PEPPER = ((0.01, 0.06), (0.4, 0.6), 0.7)


def blackbody_gains(kelvin: float) -> tuple:
    """RGB white point of a blackbody (Tanner Helland's fit), as channel gains normalized to green."""
    t = kelvin / 100.0
    r = 255.0 if t <= 66 else 329.698727446 * (t - 60) ** -0.1332047592
    g = 99.4708025861 * math.log(t) - 161.1195681661 if t <= 66 else 288.1221695283 * (t - 60) ** -0.0755148492
    b = 255.0 if t >= 66 else (0.0 if t <= 19 else 138.5177312231 * math.log(t - 10) - 305.0447927307)
    r, g, b = (min(max(v, 0.0), 255.0) for v in (r, g, b))
    return r / g, 1.0, b / g


BLACKBODY = [blackbody_gains(k) for k in range(3000, 15001, 500)]


def _range(v) -> tuple:
    return (float(v[0]), float(v[1])) if isinstance(v, (tuple, list)) else (max(0.0, 1 - v), 1 + v)


def motion_kernel3(angle_deg: float, direction: float) -> np.ndarray:
    """kornia get_motion_kernel2d(3, angle, direction) with its default nearest-neighbour resampling
    (RandomMotionBlur's resample="nearest"): a centre-row line with weights linspace(d, 1 - d, 3),
    d = (direction + 1) / 2, rotated by ``angle`` about the centre (each output tap takes the line tap
    nearest to its back-rotated position, rounding half to even as torch's grid_sample does), then
    normalized to sum 1."""
    d = (min(max(direction, -1.0), 1.0) + 1.0) / 2.0
    k = np.zeros((3, 3))
    k[1, :] = np.linspace(d, 1.0 - d, 3)
    a = math.radians(angle_deg)
    ca, sa = math.cos(a), math.sin(a)
    out = np.zeros((3, 3))
    for y in range(3):
        for x in range(3):
            dx, dy = x - 1, y - 1  # rotate the sampling point back by the angle
            sx, sy = int(np.rint(ca * dx + sa * dy + 1)), int(np.rint(-sa * dx + ca * dy + 1))
            if 0 <= sy < 3 and 0 <= sx < 3:
                out[y, x] = k[sy, sx]
    s = out.sum()
    return out / s if s > 0 else k / k.sum()


def erase_rects(u: np.ndarray, h: int, w: int, scale: tuple, ratio: tuple) -> np.ndarray:
    """Rectangles (y0, x0, h, w) from 5 uniforms per image, as kornia's
    random_rectangles_params_generator: area = U(scale) * H * W; aspect ratio U(ratio), drawn from
    (ratio[0], 1) or (1, ratio[1]) with equal odds when the range spans 1; side lengths rounded and
    clamped to [1, H] / [1, W]; the corner uniform over the positions that keep the box inside."""
    area = (scale[0] + (scale[1] - scale[0]) * u[:, 0]) * h * w
    if ratio[0] < 1.0 < ratio[1]:
        lo = np.where(u[:, 1] < 0.5, ratio[0], 1.0)
        hi = np.where(u[:, 1] < 0.5, 1.0, ratio[1])
    else:
        lo, hi = np.full(len(u), ratio[0]), np.full(len(u), ratio[1])
    r = lo + (hi - lo) * u[:, 2]
    eh = np.clip(np.rint(np.sqrt(area * r)), 1, h).astype(np.int64)
    ew = np.clip(np.rint(np.sqrt(area / r)), 1, w).astype(np.int64)
    y0 = np.floor(u[:, 3] * (h - eh + 1)).astype(np.int64)
    x0 = np.floor(u[:, 4] * (w - ew + 1)).astype(np.int64)
    return np.stack([y0, x0, eh, ew], 1)


def gaussian5(sigma: float) -> np.ndarray:
    t = np.arange(-2, 3, dtype=np.float64)
    w = np.exp(-(t * t) / (2 * sigma * sigma))
    return w / w.sum()


class DeviceAugmentation:
    """``aug(images_u8) -> fp32 images`` for a (B, 3*n_cams, H, W) uint8 CUDA batch (data.py:222-224,
    applied to all B samples at once). ``train=False`` or a config with every photometric flag off
    returns the batch unchanged (the model takes uint8 batches directly)."""

    def __init__(self, cfg, train: bool = True, seed: int = 0, n_cams: int = 2):
        self.cfg = cfg
        self.train = train
        self.n_cams = n_cams
        self.gen = torch.Generator().manual_seed(seed)
        self.active = train and cfg is not None and any(
            getattr(cfg, k) for k in ("random_erasing", "planckian_jitter", "color_jiggle", "blur", "motion_blur",
                                      "plasma_shadow", "salt_and_pepper"))
        self._scratch = None

    def _u(self, n, lo, hi) -> np.ndarray:
        return (torch.rand(n, generator=self.gen, dtype=torch.float64) * (hi - lo) + lo).numpy()

    def sample(self, n_samples: int, hw: tuple = (256, 256)) -> np.ndarray:
        """Per-image parameters (n_samples * n_cams records) in the reference's ranges; ``hw`` sizes
        the erasing rectangles."""
        c, nc = self.cfg, self.n_cams
        n = n_samples * nc
        p = np.zeros(n, dtype=PARAMS_DTYPE)
        p["gain"] = 1.0
        p["bright"], p["contrast"], p["sat"] = 1.0, 1.0, 1.0
        if getattr(c, "random_erasing", False):  # RandomErasing x2, per image (same_on_batch=False)
            for e, (prob, scale, ratio, value) in enumerate(ERASERS):
                on = self._u(n, 0, 1) < prob
                rect = erase_rects(self._u(5 * n, 0, 1).reshape(n, 5), hw[0], hw[1], scale, ratio)
                p["erase"][on, e] = rect[on]
                p["erase_val"][:, e] = value
        if c.planckian_jitter:  # RandomPlanckianJitter(mode="blackbody"), p = 0.5, per image
            on = self._u(n, 0, 1) < 0.5
            idx = torch.randint(len(BLACKBODY), (n,), generator=self.gen).numpy()
            p["gain"][on] = np.asarray(BLACKBODY, dtype=np.float32)[idx[on]]
        if c.color_jiggle:  # ColorJiggle, same_on_batch: one draw per sample, shared by its cameras
            br, co, sa = _range(c.brightness), _range(c.contrast), _range(c.saturation)
            hu = c.hue if isinstance(c.hue, (tuple, list)) else (-c.hue, c.hue)
            vals = [self._u(n_samples, *r) for r in (br, co, sa, hu)]
            # kornia ColorJiggle draws a fresh op order on every call: one call per sample (per
            # __getitem__), shared by that sample's cameras like its factors
            order = np.zeros(n_samples, dtype=np.int32)
            for b in range(n_samples):
                for i, op in enumerate(torch.randperm(4, generator=self.gen).tolist()):
                    order[b] |= op << (2 * i)
            for key, v in zip(("bright", "contrast", "sat", "hue"), vals):
                p[key] = np.repeat(v, nc)
            p["order"] = np.repeat(order, nc)
            p["jiggle"] = 1
        if c.blur:  # RandomGaussianBlur((5, 5), (3.0, 8.0), p=0.5)
            on = self._u(n, 0, 1) < 0.5
            sig = self._u(n, 3.0, 8.0)
            for i in np.nonzero(on)[0]:
                p["blur_w"][i] = gaussian5(sig[i])
        if c.motion_blur:  # RandomMotionBlur(3, 35.0, 0.5, p=0.7)
            on = self._u(n, 0, 1) < 0.7
            ang, dirn = self._u(n, -35.0, 35.0), self._u(n, -0.5, 0.5)
            for i in np.nonzero(on)[0]:
                p["motion"][i] = motion_kernel3(ang[i], dirn[i]).reshape(-1)
        if c.plasma_shadow:  # RandomPlasmaShadow(roughness, intensity, quantity), p = 1
            p["plasma_rough"] = self._u(n, 0.1, 0.4)
            p["plasma_int"] = self._u(n, -0.6, 0.0)
            p["plasma_q"] = self._u(n, 0.0, 0.5)
            p["seed"] = torch.randint(0, 2**31 - 1, (n,), generator=self.gen).numpy().astype(np.uint32)
        if getattr(c, "salt_and_pepper", False):  # RandomSaltAndPepperNoise(p=0.7), per image
            (a0, a1), (s0, s1), prob = SALT_PEPPER
            on = self._u(n, 0, 1) < prob
            amt, salt = self._u(n, a0, a1), self._u(n, s0, s1)
            p["sp_amount"] = np.where(on, amt, 0.0)
            p["sp_salt"] = salt
            p["sp_seed"] = torch.randint(0, 2**31 - 1, (n,), generator=self.gen).numpy().astype(np.uint32)
        return p

    def apply(self, images_u8: torch.Tensor, params: np.ndarray) -> torch.Tensor:
        """Run the kernels with explicit per-image ``params`` (tests); returns fp32 images."""
        if images_u8.dtype != torch.uint8 or not images_u8.is_cuda:
            raise TypeError("DeviceAugmentation: expects a uint8 CUDA batch (CameraCubePoseDataset(uint8=True))")
        L = lib()
        assert PARAMS_DTYPE.itemsize == L.dll.argus_augment_params_bytes()
        x = images_u8.contiguous()
        B, C6, H, W = x.shape
        nimg = B * C6 // 3
        assert len(params) == nimg
        out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        nbytes = L.dll.argus_augment_scratch_bytes(nimg, H, W)
        if self._scratch is None or self._scratch.numel() * 4 < nbytes:
            self._scratch = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=x.device)
        dev_p = torch.from_numpy(params.view(np.uint8).copy()).to(x.device)
        L.augment_photometric(nimg, H, W, ptr(x), ptr(out), ptr(dev_p), ptr(self._scratch), stream())
        return out

    def __call__(self, images_u8: torch.Tensor) -> torch.Tensor:
        if not self.active:
            return images_u8
        return self.apply(images_u8, self.sample(images_u8.shape[0], tuple(images_u8.shape[-2:])))
