"""CPU: the oracle is pinned by the golden fixtures (reference models.py run with the oracle ResNet
injected; closed-form loss KATs; the reference tests' literal vectors)."""
import math

import torch

from oracle import se3
from oracle.ncamera import build_reference_model


def test_loss_kats(golden):
    for kat in golden["loss_kats"]:
        p = torch.tensor([kat["pred"]], dtype=torch.float64)
        t = torch.tensor([kat["target"]], dtype=torch.float64)
        assert abs(se3.geometric_loss(p, t).item() - kat["loss"]) < 1e-12


def test_loss_identity_and_shapes():
    # tests/test_train.py:18-36: unbatched -> scalar, batched -> (B,), loss(p, Exp(p)) == 0
    assert se3.geometric_loss(torch.randn(6), se3.se3_exp(torch.randn(6))).shape == torch.Size([])
    p = torch.randn(32, 6, dtype=torch.float64)
    assert se3.geometric_loss(p, se3.random_targets(32).double()).shape == (32,)
    assert se3.geometric_loss(p, se3.se3_exp(p)).abs().max().item() < 1e-12


def test_loss_gradient_matches_finite_differences():
    g = torch.Generator().manual_seed(0)
    p = torch.randn(8, 6, generator=g, dtype=torch.float64) * 0.8
    T = se3.random_targets(8, generator=g).double()
    _, grad = se3.loss_and_grad(p, T, mean=False)
    eps = 1e-6
    for i in range(6):
        e = torch.zeros_like(p)
        e[:, i] = eps
        fd = (se3.geometric_loss(p + e, T) - se3.geometric_loss(p - e, T)) / (2 * eps)
        assert (fd - grad[:, i]).abs().max().item() < 1e-7


def test_near_pi_sign_invariance():
    # rotation by 1.5 pi == rotation by -0.5 pi: the shortest-angle Log gives pi^2/4
    p = torch.tensor([[0, 0, 0, 0, 0, 1.5 * math.pi]], dtype=torch.float64)
    assert abs(se3.geometric_loss(p, torch.tensor([[0, 0, 0, 0, 0, 0, 1.0]], dtype=torch.float64)).item()
               - math.pi**2 / 4) < 1e-12


def test_state_dict_schema_and_forward_match_golden(golden):
    m = build_reference_model(42)
    sd = m.state_dict()
    assert [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd.items()] == golden["state_dict"]
    assert sum(v.numel() for k, v in sd.items()
               if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))) == golden["n_params"] == 25885766
    import tests.golden.make_golden as mg

    x = mg.synthetic_images(2, 256, 256, seed=1234)
    assert mg.state_sha256(sd) == golden["state_sha256"]
    m.train()
    with torch.no_grad():
        pt = m(x)
        m.eval()
        pe = m(x)
    assert torch.allclose(pt, torch.tensor(golden["pred_train"]), atol=1e-6)
    assert torch.allclose(pe, torch.tensor(golden["pred_eval"]), atol=1e-6)


def test_pose_order_kats(golden):
    from argus_amd.utils import xyzwxyz_to_xyzxyzw_SE3, xyzxyzw_to_xyzwxyz_SE3

    a = torch.tensor(golden["pose_order_kats"]["xyzwxyz"])
    b = torch.tensor(golden["pose_order_kats"]["xyzxyzw"])
    assert torch.allclose(xyzwxyz_to_xyzxyzw_SE3(a), b)
    assert torch.allclose(xyzxyzw_to_xyzwxyz_SE3(b), a)
    assert torch.allclose(xyzwxyz_to_xyzxyzw_SE3(a[0]), b[0])
    r = torch.randn(2, 7)
    assert torch.allclose(xyzxyzw_to_xyzwxyz_SE3(xyzwxyz_to_xyzxyzw_SE3(r)), r)
