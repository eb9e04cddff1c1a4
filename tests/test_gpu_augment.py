"""Device photometric augmentations (argus_amd.augment, csrc/augment.hip) against the float64
restatement of the same formulas (tests/aug_reference.py). kornia is absent, so equality with
kornia itself is unpinned; these tests pin the kernels to the formulas augment.hip states."""
import numpy as np
import pytest
import torch

import tests.aug_reference as ref
from argus_amd.augment import DeviceAugmentation, gaussian5, motion_kernel3, PARAMS_DTYPE
from argus_amd.data import AugmentationConfig

pytestmark = pytest.mark.gpu


def _params(n, **kw):
    p = np.zeros(n, dtype=PARAMS_DTYPE)
    p["gain"], p["bright"], p["contrast"], p["sat"] = 1.0, 1.0, 1.0, 1.0
    for k, v in kw.items():
        p[k] = v
    return p


def test_identity_when_every_op_is_off(cuda):
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 256, (2, 6, 13, 17), generator=g, dtype=torch.uint8)
    aug = DeviceAugmentation(AugmentationConfig(), train=True)
    out = aug.apply(x.to(cuda), _params(4))
    assert torch.equal(out.cpu(), x.float() / 255.0)
    assert DeviceAugmentation(AugmentationConfig(), train=False)(x.to(cuda)).dtype == torch.uint8  # val: unchanged


@pytest.mark.parametrize("ops", ["color", "blur", "motion", "all_but_plasma"])
def test_ops_match_restatement(cuda, ops):
    g = torch.Generator().manual_seed(1)
    B, H, W = 2, 24, 31  # ragged sizes: reflect / zero borders on every side
    x = torch.randint(0, 256, (B, 6, H, W), generator=g, dtype=torch.uint8)
    n = 2 * B
    rng = np.random.default_rng(5)
    p = _params(n)
    if ops in ("color", "all_but_plasma"):
        p["gain"] = [(1.2, 1.0, 0.7), (0.9, 1.0, 1.3), (1.0, 1.0, 1.0), (1.1, 1.0, 0.95)]
        p["bright"], p["contrast"] = rng.uniform(0.8, 1.0, n), rng.uniform(0.5, 1.2, n)
        p["sat"], p["hue"] = rng.uniform(0.25, 1.2, n), rng.uniform(-0.1, 0.1, n)
        p["order"] = 2 | (0 << 2) | (3 << 4) | (1 << 6)
        p["jiggle"] = 1
    if ops in ("blur", "all_but_plasma"):
        for i in (0, 3):
            p["blur_w"][i] = gaussian5(rng.uniform(3, 8))
    if ops in ("motion", "all_but_plasma"):
        for i in (1, 3):
            p["motion"][i] = motion_kernel3(rng.uniform(-35, 35), rng.uniform(-0.5, 0.5)).reshape(-1)
    out = DeviceAugmentation(AugmentationConfig()).apply(x.to(cuda), p).cpu().double()
    imgs = x.reshape(n, 3, H, W)
    want = torch.stack([ref.augment_image(imgs[i], p[i]) for i in range(n)]).reshape(B, 6, H, W)
    err = (out - want).abs().max().item()
    assert err < 2e-5, (ops, err)


@pytest.mark.parametrize("hw,cams", [((64, 64), 2), ((37, 70), 2), ((64, 64), 3)])
def test_plasma_shadow_matches_restatement(cuda, hw, cams):
    """Diamond-square plasma map (65 x 65 grid for 64 x 64; 129 x 129 cropped to 37 x 70) and the
    additive shade, against the float64 restatement. Three cameras: an odd image count, so the
    per-image min/max scratch follows an odd number of floats (its 16-byte alignment)."""
    g = torch.Generator().manual_seed(2)
    B, (H, W) = 1, hw
    x = torch.randint(0, 256, (B, 3 * cams, H, W), generator=g, dtype=torch.uint8)
    p = _params(cams, plasma_int=[-0.5, -0.3, -0.4][:cams], plasma_q=[0.4, 0.2, 0.3][:cams],
                plasma_rough=[0.3, 0.15, 0.2][:cams], seed=[12345, 777, 31][:cams])
    out = DeviceAugmentation(AugmentationConfig()).apply(x.to(cuda), p).cpu().double()
    want = torch.stack([ref.augment_image(x.reshape(cams, 3, H, W)[i], p[i]) for i in range(cams)]).reshape(
        B, 3 * cams, H, W)
    bad = ((out - want).abs() > 2e-5).double().mean().item()
    assert bad < 1e-3, bad  # fp32 vs fp64 noise can flip the threshold only at exact ties
    for i, q in ((0, 0.4), (1, 0.2)):
        m = ref.diamond_square(int(p["seed"][i]), p["plasma_rough"][i], H, W)
        assert m.min() == 0 and m.max() == 1
        shaded = (m < q).double().mean().item()
        assert 0.005 < shaded < 0.9, shaded  # a real shadow: some, not all, pixels
        cam = out[0, 3 * i:3 * i + 3]
        src = x[0, 3 * i:3 * i + 3].double() / 255.0
        dark = (cam < src - 1e-6).any(0)
        assert (dark <= (m < q)).all()  # only shaded pixels get darker


def test_erasing_and_salt_pepper_match_restatement(cuda):
    """Two erasing rectangles (values 0 and 1, the second over the first) ahead of the colour ops,
    salt-and-pepper last (after the clamp): against the restatement, bit-exact positions."""
    g = torch.Generator().manual_seed(4)
    B, H, W = 2, 40, 52
    x = torch.randint(0, 256, (B, 6, H, W), generator=g, dtype=torch.uint8)
    n = 2 * B
    p = _params(n)
    p["erase"][0, 0] = (3, 5, 10, 20)
    p["erase"][0, 1] = (8, 15, 12, 9)
    p["erase"][2, 1] = (0, 0, 40, 1)
    p["erase_val"][:, 1] = 1.0
    p["gain"][0] = (1.2, 1.0, 0.7)
    p["sp_amount"] = [0.05, 0.0, 0.2, 0.01]
    p["sp_salt"] = [0.5, 0.5, 0.4, 0.6]
    p["sp_seed"] = [11, 12, 13, 14]
    out = DeviceAugmentation(AugmentationConfig()).apply(x.to(cuda), p).cpu().double()
    imgs = x.reshape(n, 3, H, W)
    want = torch.stack([ref.augment_image(imgs[i], p[i]) for i in range(n)]).reshape(B, 6, H, W)
    err = (out - want).abs().max().item()
    assert err < 2e-5, err
    o = out.reshape(n, 3, H, W)
    assert (o[0, :, 3:8, 5:15] == 0).sum() > 0.8 * 3 * 5 * 10  # erased to 0 (salt may flip a few)
    noisy = ((o[2] == 0) | (o[2] == 1)).all(0).double().mean().item()
    assert 0.15 < noisy < 0.3, noisy


def test_sampled_batch_runs_and_stays_in_range(cuda):
    g = torch.Generator().manual_seed(3)
    x = torch.randint(0, 256, (4, 6, 32, 40), generator=g, dtype=torch.uint8).to(cuda)
    aug = DeviceAugmentation(AugmentationConfig(), train=True, seed=11)
    out = aug(x)
    assert out.dtype == torch.float32 and out.shape == x.shape
    assert float(out.min()) >= 0.0 and float(out.max()) <= 1.0
    assert not torch.equal(out, x.float() / 255.0)
    out2 = DeviceAugmentation(AugmentationConfig(), train=True, seed=11)(x)
    assert torch.equal(out, out2)  # seeded: reproducible
