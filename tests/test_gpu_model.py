"""Whole-model parity: argus_amd.NCameraCNN (HIP engine) vs the CPU oracle (reference models.py
semantics, pinned by tests/golden/golden_b2.json) on identical seeded weights and batches.

Tolerances
- fp32 path, forward (north_star): pose 6-vector and per-sample loss within 1e-4 absolute, train
  and eval mode; BN running statistics within 1e-4 relative.
- fp32 path, gradients: the train-mode gradient of this network at batch 2 is ill-conditioned —
  the reference's OWN fp32 gradients differ from its fp64 gradients by up to ~18 % (median ~2 %,
  BatchNorm over 256 values per channel at layer4 + ReLU masks). Parity is therefore stated against
  the fp64 oracle relative to that intrinsic fp32 noise: the global relative error of our gradient
  vector must be <= 3x the reference-fp32 one, and no parameter's error may exceed 3x the
  reference's worst parameter. Kernel exactness at full-model shapes is checked separately by
  re-deriving every backward stage of every block in fp64 from the engine's own saved tensors
  (relative error <= 2e-5).
- bf16 path: pose within 2e-2 absolute of the fp32 reference (stated tolerance).
"""
import pytest
import torch

from oracle import se3
from oracle.ncamera import build_reference_model
from tests.stage_checks import stage_checks

pytestmark = pytest.mark.gpu


def _inputs(golden):
    import tests.golden.make_golden as mg

    x = mg.synthetic_images(2, 256, 256, seed=1234)
    T = torch.tensor(golden["inputs"]["targets"], dtype=torch.float32)
    assert abs(float(x.double().sum()) - golden["inputs"]["images_sum"]) < 1e-3
    return x, T


def _product(cuda, dtype="fp32", seed=42):
    from argus_amd.models import NCameraCNN

    torch.manual_seed(seed)
    return NCameraCNN(compute_dtype=dtype).to(cuda)


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def test_forward_train_eval_matches_golden(cuda, golden):
    x, T = _inputs(golden)
    m = _product(cuda)
    with torch.no_grad():
        m.train()
        pt = m(x.to(cuda)).cpu()
        m.eval()
        pe = m(x.to(cuda)).cpu()
    ref_t = torch.tensor(golden["pred_train"])
    ref_e = torch.tensor(golden["pred_eval"])
    assert (pt - ref_t).abs().max().item() < 1e-4, (pt, ref_t)
    assert (pe - ref_e).abs().max().item() < 1e-4, (pe, ref_e)
    losses = se3.geometric_loss(pt.double(), T.double())
    assert (losses - torch.tensor(golden["loss_train"], dtype=torch.float64)).abs().max().item() < 1e-4


def test_gradients_match_fp64_oracle(cuda, golden):
    from argus_amd.losses import geometric_loss_fn

    x, T = _inputs(golden)
    m = _product(cuda)
    m.train()
    pred = m(x.to(cuda))
    losses = geometric_loss_fn(pred, T.to(cuda))
    losses.mean().backward()
    assert (losses.detach().cpu() - torch.tensor(golden["loss_train"])).abs().max().item() < 1e-4

    grads = {}
    for dt in (torch.float32, torch.float64):
        ref = build_reference_model(42).to(dt)
        ref.train()
        se3.geometric_loss(ref(x.to(dt)), T.to(dt)).mean().backward()
        grads[dt] = {n: p.grad.double() for n, p in ref.named_parameters()}
        if dt == torch.float32:
            sd_ref = ref.state_dict()
    g64, g32 = grads[torch.float64], grads[torch.float32]
    ours = {n: p.grad.double().cpu() for n, p in m.named_parameters()}
    assert list(ours) == list(g64)
    flat = lambda d: torch.cat([v.flatten() for v in d.values()])  # noqa: E731
    e_ours = ((flat(ours) - flat(g64)).norm() / flat(g64).norm()).item()
    e_ref = ((flat(g32) - flat(g64)).norm() / flat(g64).norm()).item()
    per_ours = {n: _rel(ours[n], g64[n]) for n in g64}
    per_ref = {n: _rel(g32[n], g64[n]) for n in g64}
    assert e_ours <= 3 * e_ref + 1e-4, (e_ours, e_ref)
    worst = max(per_ours.items(), key=lambda kv: kv[1])
    assert worst[1] <= 3 * max(per_ref.values()) + 1e-4, (worst, max(per_ref.values()))
    # the head (no BatchNorm behind it) is well conditioned: tight bound
    for n in ("output_mlp.4.weight", "output_mlp.4.bias", "output_mlp.2.weight", "output_mlp.0.weight",
              "resnet.fc.weight", "resnet.fc.bias"):
        assert per_ours[n] < 1e-3, (n, per_ours[n])
    # BN running statistics after one train-mode forward
    sd = m.state_dict()
    for k in sd:
        if k.endswith(("running_mean", "running_var")):
            assert _rel(sd[k], sd_ref[k]) < 1e-4, k
        if k.endswith("num_batches_tracked"):
            assert int(sd[k]) == 1


@pytest.mark.parametrize("shape", ["golden_256", "large_376x672"])
def test_block_backward_stages_exact(cuda, golden, shape):
    """Every backward stage of every Bottleneck, re-derived in fp64 from the engine's own tensors —
    at the golden 256x256 batch and at BASELINE config 4's 376x672 frame (odd feature maps 47x84,
    24x42, 12x21: stride-2 dgrad phases of unequal size, no 64-aligned pixel rows)."""
    from argus_amd.losses import geometric_loss_fn

    if shape == "golden_256":
        x, T = _inputs(golden)
    else:
        g = torch.Generator().manual_seed(77)
        x = torch.randint(0, 256, (1, 6, 376, 672), generator=g, dtype=torch.uint8).float() / 255.0
        T = se3.random_targets(1, generator=g)
    m = _product(cuda)
    eng = m._engine(cuda)
    eng.debug = {}
    m.train()
    geometric_loss_fn(m(x.to(cuda)), T.to(cuda)).mean().backward()
    eng_debug, eng.debug = eng.debug, None
    worst = stage_checks(eng, dict(m.named_parameters()), eng_debug, 2e-5)
    print("fp32 worst max-relative error per stage:", {k: f"{v:.2e}" for k, v in worst.items()})


def test_bf16_forward_tolerance(cuda, golden):
    x, _ = _inputs(golden)
    m = _product(cuda, "bf16")
    with torch.no_grad():
        m.train()
        pt = m(x.to(cuda)).cpu()
    ref_t = torch.tensor(golden["pred_train"])
    assert (pt - ref_t).abs().max().item() < 2e-2, (pt, ref_t)


def test_non_4d_input_asserts(cuda):
    m = _product(cuda)
    with pytest.raises(AssertionError):
        m(torch.randn(6, 64, 64, device=cuda))
    out = m(torch.rand(2, 6, 64, 64, device=cuda))
    assert out.shape == (2, 6)


@pytest.mark.parametrize("dtype,tol", [("fp32", 1e-4), ("bf16", 2e-2)])
def test_forward_large_frame_matches_oracle(cuda, dtype, tol):
    """BASELINE config 4 frame (2 cameras of 376x672): train- and eval-mode prediction vs the oracle
    (reference models.py semantics) on the same seeded weights; fp32 within the north_star 1e-4,
    bf16 within its stated 2e-2."""
    g = torch.Generator().manual_seed(5)
    x = torch.randint(0, 256, (1, 6, 376, 672), generator=g, dtype=torch.uint8).float() / 255.0
    m = _product(cuda, dtype)
    ref = build_reference_model(42)
    with torch.no_grad():
        for train in (True, False):
            m.train(train)
            ref.train(train)
            got = m(x.to(cuda)).cpu()
            want = ref(x)
            assert (got - want).abs().max().item() < tol, (dtype, train, got, want)


@pytest.mark.parametrize("compute_dtype", ["fp32", "bf16"])
def test_uint8_images_give_identical_predictions(cuda, compute_dtype):
    """The model accepts the uint8 batches of CameraCubePoseDataset(uint8=True) and predicts exactly
    what it predicts on the reference's fp32 `/255` batch (argus/data.py:214-215)."""
    from argus_amd.models import NCameraCNN

    g = torch.Generator().manual_seed(11)
    u8 = torch.randint(0, 256, (2, 6, 64, 64), generator=g, dtype=torch.uint8)
    torch.manual_seed(42)
    model = NCameraCNN(compute_dtype=compute_dtype).to(cuda).train()
    with torch.no_grad():
        a = model(u8.to(cuda))
        b = model((u8.to(torch.float32) / 255.0).to(cuda))
    assert torch.equal(a, b)
