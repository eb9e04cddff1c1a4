"""Host side of the device augmentations: parameter sampling in the reference's ranges
(argus/data.py:41-103 kornia arguments), kernel construction, record layout (no GPU needed)."""
import numpy as np

from argus_amd.augment import BLACKBODY, PARAMS_DTYPE, DeviceAugmentation, erase_rects, gaussian5, motion_kernel3
from argus_amd.data import AugmentationConfig


def test_record_layout_and_kernels():
    assert PARAMS_DTYPE.itemsize == 40 * 4
    w = gaussian5(3.0)
    assert abs(w.sum() - 1) < 1e-12 and np.allclose(w, w[::-1]) and w[2] == w.max()
    k = motion_kernel3(0.0, 0.0)
    assert np.allclose(k[1], 1 / 3) and np.allclose(k[0], 0) and np.allclose(k[2], 0)
    for ang in (-35.0, 10.0, 35.0):
        for d in (-0.5, 0.3):
            k = motion_kernel3(ang, d)
            assert abs(k.sum() - 1) < 1e-12 and (k >= 0).all()
    # nearest-neighbour rotation: small angles keep the line, 35 degrees moves its end taps diagonally;
    # every nonzero weight is one of the line's own weights (renormalized), no bilinear blending
    assert np.allclose(motion_kernel3(10.0, 0.0), motion_kernel3(0.0, 0.0))
    k35 = motion_kernel3(35.0, 0.0)
    assert np.count_nonzero(k35) == 3 and np.allclose(k35[k35 > 0], 1 / 3) and k35[1, 1] > 0
    r3000, _, b3000 = BLACKBODY[0]
    r15k, _, b15k = BLACKBODY[-1]
    assert r3000 > 1 > b3000 and r15k < 1 < b15k  # warm -> red gain, cold -> blue gain


def test_sampling_ranges_and_sharing():
    aug = DeviceAugmentation(AugmentationConfig(), train=True, seed=7)
    p = aug.sample(2000)
    assert len(p) == 4000
    cj = AugmentationConfig()
    for key, (lo, hi) in (("bright", cj.brightness), ("contrast", cj.contrast), ("sat", cj.saturation),
                          ("hue", cj.hue)):
        v = p[key]
        assert v.min() >= lo and v.max() <= hi
        assert np.array_equal(v[0::2], v[1::2])  # ColorJiggle same_on_batch: the two cameras share it
    for o in p["order"][:64]:
        assert sorted((int(o) >> (2 * i)) & 3 for i in range(4)) == [0, 1, 2, 3]
    assert np.array_equal(p["order"][0::2], p["order"][1::2])  # one order per sample, shared by its cameras
    assert len(set(p["order"][0::2].tolist())) > 12  # drawn per sample (24 permutations)
    blur_on = (p["blur_w"][:, 2] > 0).mean()
    motion_on = (np.abs(p["motion"]).sum(1) > 0).mean()
    planck_on = (np.abs(p["gain"] - 1).sum(1) > 1e-6).mean()
    assert 0.45 < blur_on < 0.55 and 0.65 < motion_on < 0.75 and 0.4 < planck_on < 0.55
    assert (p["plasma_int"] >= -0.6).all() and (p["plasma_int"] <= 0).all()
    assert (p["plasma_q"] >= 0).all() and (p["plasma_q"] <= 0.5).all()
    assert not DeviceAugmentation(AugmentationConfig(), train=False).active
    off = AugmentationConfig(color_jiggle=False, planckian_jitter=False, blur=False, motion_blur=False,
                             plasma_shadow=False)
    assert not DeviceAugmentation(off, train=True).active


def test_erasing_and_salt_pepper_sampling():
    """RandomErasing x2 (data.py:52-64) and RandomSaltAndPepperNoise(p=0.7) (data.py:95): rectangles
    inside the image with the configured area fraction and aspect ratio, per-image on/off odds."""
    rng = np.random.default_rng(0)
    u = rng.random((4000, 5))
    for scale, ratio in (((0.02, 0.1), (2.0, 3.0)), ((0.02, 0.05), (0.8, 1.2))):
        r = erase_rects(u, 256, 200, scale, ratio)
        y0, x0, h, w = r.T
        assert (y0 >= 0).all() and (x0 >= 0).all() and (y0 + h <= 256).all() and (x0 + w <= 200).all()
        frac = h * w / (256 * 200)
        assert frac.min() > scale[0] * 0.8 and frac.max() < scale[1] * 1.2
        ar = h / w
        assert ar.min() > ratio[0] * 0.85 and ar.max() < ratio[1] * 1.15
        if ratio[0] < 1 < ratio[1]:
            assert 0.4 < (ar < 1).mean() < 0.6  # the two sides of 1 with equal odds
    cfg = AugmentationConfig(random_erasing=True, salt_and_pepper=True)
    aug = DeviceAugmentation(cfg, train=True, seed=3)
    p = aug.sample(2000, (256, 256))
    for e, val in ((0, 0.0), (1, 1.0)):
        on = p["erase"][:, e, 2] > 0
        assert 0.45 < on.mean() < 0.55 and (p["erase_val"][:, e] == val).all()
    sp_on = p["sp_amount"] > 0
    assert 0.65 < sp_on.mean() < 0.75
    assert p["sp_amount"][sp_on].min() >= 0.01 and p["sp_amount"].max() <= 0.06
    assert p["sp_salt"].min() >= 0.4 and p["sp_salt"].max() <= 0.6
    off = DeviceAugmentation(AugmentationConfig(), train=True, seed=3).sample(100)
    assert (off["erase"] == 0).all() and (off["sp_amount"] == 0).all()  # reference defaults: both off
