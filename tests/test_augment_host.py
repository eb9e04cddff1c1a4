"""Host side of the device augmentations: parameter sampling in the reference's ranges
(argus/data.py:41-103 kornia arguments), kernel construction, record layout (no GPU needed)."""
import numpy as np

from argus_amd.augment import BLACKBODY, PARAMS_DTYPE, DeviceAugmentation, gaussian5, motion_kernel3
from argus_amd.data import AugmentationConfig


def test_record_layout_and_kernels():
    assert PARAMS_DTYPE.itemsize == 27 * 4
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
