"""Generate the committed golden fixtures for the argus hot path (run in the BUILD container only).

    python tests/golden/make_golden.py            # writes tests/golden/*.json / *.pt

What it pins:
1. The reference's own ``argus/models.py`` source (loaded from /root/reference by file path, never
   copied) is executed with ``oracle.resnet`` injected as ``torchvision.models`` (torchvision is not
   installed). Its seeded ``NCameraCNN`` must equal ``oracle.ncamera.NCameraCNN`` bit-for-bit: same
   state_dict keys/shapes/values and identical forward outputs. This pins the oracle's wrapper,
   RNG order and reshape/GELU/MLP semantics to the reference source.
2. Fixture values are then produced by the *reference* model object (train-mode forward, eval-mode
   forward, one reference train step: fwd -> SE(3) loss -> mean -> backward -> clip_grad_norm_(1.0)
   -> Adam(1e-4), ``argus/train.py:298-321``). The SE(3) loss uses ``oracle.se3`` (pypose absent).
3. Loss known answers (closed forms) and the reference tests' literal pose-order
   vectors (``tests/test_utils.py:17-47``) are stored as data.

If /root/reference is absent (the GPU box) the script refuses to run; the committed fixtures are
what travels.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import math
import sys
import types
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[2]
REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

from oracle import ncamera as oracle_ncamera  # noqa: E402
from oracle import resnet as oracle_resnet  # noqa: E402
from oracle import se3 as oracle_se3  # noqa: E402


def load_reference_models():
    """Execute /root/reference/argus/models.py with the oracle ResNet as torchvision.models."""
    tv = types.ModuleType("torchvision")
    tvm = types.ModuleType("torchvision.models")
    tvm.resnet50 = oracle_resnet.resnet50
    tv.models = tvm
    saved = {k: sys.modules.get(k) for k in ("torchvision", "torchvision.models")}
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.models"] = tvm
    try:
        spec = importlib.util.spec_from_file_location("_argus_ref_models", REF / "argus" / "models.py")
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return mod


def state_sha256(sd) -> str:
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(v.detach().contiguous().cpu().numpy().tobytes())
    return h.hexdigest()


def synthetic_images(b: int, h: int, w: int, seed: int) -> torch.Tensor:
    """uint8-uniform pixels /255 (as tests/conftest.py:35-41), fp32 NCHW (B, 6, H, W)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (b, 6, h, w), generator=g, dtype=torch.uint8).to(torch.float32) / 255.0


def synthetic_targets(b: int, seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return oracle_se3.random_targets(b, generator=g)


def damp_residual(model, factor: float = 0.1):
    """Scale every Bottleneck's last BN gamma (``*.bn3.weight``) by ``factor``, in place.

    Why: at seeded init the train-mode gradient of this 16-block network is chaotic — the reference's
    OWN fp32 gradient differs from its fp64 gradient by 2.2 % (global, any batch size tried), and its
    bf16-autocast gradient is uncorrelated with fp64 (cosine 0.13). Damping the residual branches
    gives a well-conditioned point of the SAME function (weights are data: a checkpoint could hold
    them) where the reference's fp32 gradient is within 1e-3 of fp64, so gradient parity can be
    pinned tightly there."""
    with torch.no_grad():
        for n, p in model.named_parameters():
            if n.endswith("bn3.weight"):
                p.mul_(factor)
    return model


DAMPED = {"batch": 8, "hw": [128, 128], "image_seed": 4321, "target_seed": 4000, "damp": 0.1}


def flat_grads(model) -> dict:
    return {n: p.grad.detach().double().clone() for n, p in model.named_parameters()}


def grad_errors(g: dict, ref: dict):
    """Global relative L2 error of the flat gradient vector and per-tensor relative L2 errors."""
    fl = lambda d: torch.cat([v.flatten() for v in d.values()])  # noqa: E731
    e = ((fl(g) - fl(ref)).norm() / fl(ref).norm()).item()
    per = {n: ((g[n] - ref[n]).norm() / ref[n].norm().clamp_min(1e-30)).item() for n in ref}
    return e, per


def ref_train_step(model, x, T, lr=1e-4, max_norm=1.0):
    """argus/train.py:298-321 with amp off: fwd, fp32 loss, mean, zero_grad, backward, clip, Adam."""
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    model.train()
    pred = model(x)
    losses = oracle_se3.geometric_loss(pred.to(torch.float32), T)
    loss = losses.mean()
    opt.zero_grad()
    loss.backward()
    gnorm = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm)
    opt.step()
    return pred.detach(), losses.detach(), gnorm.detach()


def main() -> None:
    if not (REF / "argus" / "models.py").exists():
        raise SystemExit("reference not present: fixtures can only be regenerated in the build container")
    torch.set_num_threads(8)
    ref_models = load_reference_models()

    # 1. bit-for-bit pin of the oracle against the reference source
    torch.manual_seed(42)
    ref = ref_models.NCameraCNN(ref_models.NCameraCNNConfig(n_cams=2))
    orc = oracle_ncamera.build_reference_model(42)
    sd_r, sd_o = ref.state_dict(), orc.state_dict()
    init_sha = state_sha256(sd_r)  # before any train-mode forward mutates the running stats
    assert list(sd_r.keys()) == list(sd_o.keys()), "state_dict keys differ"
    for k in sd_r:
        assert sd_r[k].shape == sd_o[k].shape and torch.equal(sd_r[k], sd_o[k]), k
    x = synthetic_images(2, 256, 256, seed=1234)
    T = synthetic_targets(2, seed=2000)
    with torch.no_grad():
        pr, po = ref(x), orc(x)
    assert torch.equal(pr, po), "oracle forward differs from reference forward"
    with torch.no_grad():
        try:
            ref(torch.zeros(6, 256, 256))
            raise AssertionError("reference did not assert on 3-D input")
        except AssertionError as e:
            if "did not assert" in str(e):
                raise

    golden = {
        "generator": "tests/golden/make_golden.py",
        "pinned_against": "reference argus/models.py executed with oracle.resnet as torchvision.models",
        "seed": 42,
        "n_params": sum(v.numel() for k, v in sd_r.items() if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))),
        "state_dict": [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in sd_r.items()],
        "state_sha256": init_sha,
        "inputs": {"images": "synthetic_images(2,256,256,seed=1234)", "targets": "synthetic_targets(2,seed=2000)",
                   "images_sum": float(x.double().sum()), "targets": T.tolist()},
    }

    # 2. reference-model outputs (fresh seeded model: the pin check above ran a train-mode forward)
    torch.manual_seed(42)
    ref = ref_models.NCameraCNN(ref_models.NCameraCNNConfig(n_cams=2))
    with torch.no_grad():
        ref.train()
        pred_train = ref(x)
        ref.eval()
        pred_eval = ref(x)
    losses, dpred = oracle_se3.loss_and_grad(pred_train, T, mean=True)
    golden["pred_train"] = pred_train.tolist()
    golden["pred_eval"] = pred_eval.tolist()
    golden["loss_train"] = losses.tolist()
    golden["dpred_mean"] = dpred.tolist()

    torch.manual_seed(42)
    ref = ref_models.NCameraCNN(ref_models.NCameraCNNConfig(n_cams=2))
    p0, l0, gnorm = ref_train_step(ref, x, T)
    with torch.no_grad():
        ref.train()
        pred_after = ref(x)
    sd_after = ref.state_dict()
    golden["step"] = {
        "pred": p0.tolist(),
        "loss": l0.tolist(),
        "grad_norm": float(gnorm),
        "pred_after_step_train": pred_after.tolist(),
        "bn_running_sums": {k: [float(v.double().sum()), float(v.double().abs().sum())]
                            for k, v in sd_after.items() if k.endswith(("running_mean", "running_var"))},
        "param_sums": {k: [float(v.double().sum()), float(v.double().abs().sum())]
                       for k, v in sd_after.items() if k.endswith(("weight", "bias"))},
        "num_batches_tracked": int(sd_after["resnet.bn1.num_batches_tracked"]),
    }

    # 3. loss KATs (closed forms) and the reference tests' literal pose-order vectors
    pi = math.pi
    golden["loss_kats"] = [
        {"pred": [0, 0, 0, pi / 2, 0, 0], "target": [0, 0, 0, 0, 0, 0, 1], "loss": pi**2 / 4},
        {"pred": [1, 2, 3, 0, 0, 0], "target": [0, 0, 0, 0, 0, 0, 1], "loss": 14.0},
        {"pred": [0, 0, 0, 0, 0, 0], "target": [1, 0, 0, 0, 0, math.sin(pi / 4), math.cos(pi / 4)],
         "loss": 3 * pi**2 / 8},
        {"pred": [0, 0, 0, 0, 0, 1.5 * pi], "target": [0, 0, 0, 0, 0, 0, 1], "loss": pi**2 / 4},
    ]
    golden["pose_order_kats"] = {
        "xyzwxyz": [[1, 2, 3, 0.5, 0.6, 0.7, 0.8], [4, 5, 6, 0.1, 0.2, 0.3, 0.4]],
        "xyzxyzw": [[1, 2, 3, 0.6, 0.7, 0.8, 0.5], [4, 5, 6, 0.2, 0.3, 0.4, 0.1]],
    }
    with open(OUT / "golden_b2.json", "w") as f:
        json.dump(golden, f, indent=1)
    print("wrote", OUT / "golden_b2.json", "pred_train", pred_train.tolist())
    damped_golden(ref_models)


def damped_golden(ref_models) -> None:
    """golden_b8_damped.json: the reference's train step at a well-conditioned point (damp_residual),
    B=8 at 128x128, with the reference's own fp32 / bf16-autocast gradient errors against fp64."""
    cfg = DAMPED
    B, (H, W) = cfg["batch"], cfg["hw"]
    x = synthetic_images(B, H, W, seed=cfg["image_seed"])
    T = synthetic_targets(B, seed=cfg["target_seed"])

    def fresh(dt=torch.float32):
        torch.manual_seed(42)
        m = ref_models.NCameraCNN(ref_models.NCameraCNNConfig(n_cams=2))
        return damp_residual(m, cfg["damp"]).to(dt).train()

    grads, preds = {}, {}
    for mode in ("fp64", "fp32", "bf16_autocast"):
        dt = torch.float64 if mode == "fp64" else torch.float32
        m = fresh(dt)
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=mode == "bf16_autocast"):
            pred = m(x.to(dt))
        pred = pred.to(dt)
        oracle_se3.geometric_loss(pred, T.to(dt)).mean().backward()
        grads[mode], preds[mode] = flat_grads(m), pred.detach()
    e32, per32 = grad_errors(grads["fp32"], grads["fp64"])
    e16, per16 = grad_errors(grads["bf16_autocast"], grads["fp64"])
    norm = lambda d: torch.cat([v.flatten() for v in d.values()]).norm().item()  # noqa: E731

    m = fresh()
    p0, l0, gnorm = ref_train_step(m, x, T)
    with torch.no_grad():
        pred_after = m(x)
    sd_after = m.state_dict()
    out = {
        "generator": "tests/golden/make_golden.py::damped_golden",
        "pinned_against": "reference argus/models.py executed with oracle.resnet as torchvision.models",
        "config": cfg,
        "images_sum": float(x.double().sum()),
        "targets": T.tolist(),
        "pred_train_fp32": preds["fp32"].tolist(),
        "pred_train_fp64": preds["fp64"].tolist(),
        "grad_norm_fp64": norm(grads["fp64"]),
        "grad_norm_fp32": norm(grads["fp32"]),
        "ref_fp32_vs_fp64": {"global": e32, "per_tensor": per32},
        "ref_bf16_autocast_vs_fp64": {"global": e16, "per_tensor": per16},
        "tensor_grad_norms_fp64": {n: v.norm().item() for n, v in grads["fp64"].items()},
        "step": {
            "loss": l0.tolist(),
            "grad_norm": float(gnorm),
            "pred_after_step_train": pred_after.tolist(),
            "bn_running_sums": {k: [float(v.double().sum()), float(v.double().abs().sum())]
                                for k, v in sd_after.items() if k.endswith(("running_mean", "running_var"))},
            "param_sums": {k: [float(v.double().sum()), float(v.double().abs().sum())]
                           for k, v in sd_after.items() if k.endswith(("weight", "bias"))},
        },
    }
    with open(OUT / "golden_b8_damped.json", "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT / "golden_b8_damped.json", "fp32 vs fp64", e32, "bf16 autocast vs fp64", e16)


def _fresh_damped(ref_models, dt=torch.float32):
    torch.manual_seed(42)
    m = ref_models.NCameraCNN(ref_models.NCameraCNNConfig(n_cams=2))
    return damp_residual(m, DAMPED["damp"]).to(dt).train()


def _sums(sd, suffixes):
    return {k: [float(v.double().sum()), float(v.double().abs().sum())] for k, v in sd.items() if k.endswith(suffixes)}


# DDP with DistributedSampler(shuffle=False) (argus/train.py:155-168,199): rank r takes samples r::world of
# the global batch; BN statistics are per rank (no SyncBatchNorm); DDP averages the per-rank mean-loss
# gradients (all-reduce SUM / world) before clip_grad_norm_ and Adam, which every rank then runs alike.
TWO_RANK = {"world": 2, "shard": "rank r takes samples r::world (DistributedSampler, shuffle=False)"}


def shards(x, T, world=2):
    return [(x[r::world], T[r::world]) for r in range(world)]


def two_rank_golden(ref_models) -> None:
    """golden_b8_damped_2rank.json: the reference's DDP train step with two ranks at the damped point
    (global batch 8 = 4 + 4 at 128x128): per-shard BN, averaged gradient, clip 1.0, Adam 1e-4; with the
    reference's own fp32 error of the averaged gradient against fp64."""
    cfg = DAMPED
    B, (H, W) = cfg["batch"], cfg["hw"]
    x = synthetic_images(B, H, W, seed=cfg["image_seed"])
    T = synthetic_targets(B, seed=cfg["target_seed"])
    sh = shards(x, T, TWO_RANK["world"])
    avg = {}
    for mode, dt in (("fp64", torch.float64), ("fp32", torch.float32)):
        gs = []
        for xs, ts in sh:
            m = _fresh_damped(ref_models, dt)
            oracle_se3.geometric_loss(m(xs.to(dt)), ts.to(dt)).mean().backward()
            gs.append(flat_grads(m))
        avg[mode] = {n: (gs[0][n] + gs[1][n]) / 2 for n in gs[0]}
    e32, per32 = grad_errors(avg["fp32"], avg["fp64"])
    norm = lambda d: torch.cat([v.flatten() for v in d.values()]).norm().item()  # noqa: E731

    # the DDP step itself, fp32: one replica per rank
    reps = [_fresh_damped(ref_models) for _ in sh]
    opts = [torch.optim.Adam(m.parameters(), lr=1e-4) for m in reps]
    losses = []
    for m, o, (xs, ts) in zip(reps, opts, sh):
        o.zero_grad()
        lr_ = oracle_se3.geometric_loss(m(xs).to(torch.float32), ts)
        lr_.mean().backward()
        losses.append(lr_.detach())
    with torch.no_grad():  # DDP: all-reduce SUM, then / world, in fp32
        for ps in zip(*(m.parameters() for m in reps)):
            g = (ps[0].grad + ps[1].grad) / len(ps)
            for p in ps:
                p.grad.copy_(g)
    gnorms = [float(torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)) for m in reps]
    for o in opts:
        o.step()
    for a, b in zip(reps[0].parameters(), reps[1].parameters()):
        assert torch.equal(a, b), "DDP replicas diverged"
    sds = [{k: v.clone() for k, v in m.state_dict().items()} for m in reps]
    with torch.no_grad():
        after = [m(xs) for m, (xs, _) in zip(reps, sh)]
    out = {
        "generator": "tests/golden/make_golden.py::two_rank_golden",
        "pinned_against": "reference argus/models.py executed with oracle.resnet as torchvision.models",
        "config": cfg,
        "ddp": TWO_RANK,
        "images_sum": float(x.double().sum()),
        "targets": T.tolist(),
        "grad_norm_fp64": norm(avg["fp64"]),
        "ref_fp32_vs_fp64": {"global": e32, "per_tensor": per32},
        "tensor_grad_norms_fp64": {n: v.norm().item() for n, v in avg["fp64"].items()},
        "step": {
            "loss": [v.tolist() for v in losses],
            "grad_norm": gnorms[0],
            "pred_after_step_train": [v.tolist() for v in after],
            "param_sums": _sums(sds[0], ("weight", "bias")),
            "bn_running_sums": [_sums(sd, ("running_mean", "running_var")) for sd in sds],
        },
    }
    with open(OUT / "golden_b8_damped_2rank.json", "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT / "golden_b8_damped_2rank.json", "fp32 vs fp64", e32, "losses", out["step"]["loss"])


# Ten reference train steps at the damped point (argus/train.py:295-348 with one batch per "epoch"):
# fresh batch per step, clip 1.0 + Adam 1e-4, then an eval-mode validation batch whose mean loss drives
# ReduceLROnPlateau('min', patience=5, factor=0.5) (train.py:232).
TRAJ = {"batch": 8, "hw": [128, 128], "damp": 0.1, "steps": 10, "lr": 1e-3, "max_grad_norm": 1.0,
        "image_seed0": 7000, "target_seed0": 7100, "val_batch": 8, "val_image_seed": 7200, "val_target_seed": 7201,
        "scheduler": {"patience": 1, "factor": 0.5}}


def trajectory_batches(cfg=TRAJ):
    B, (H, W) = cfg["batch"], cfg["hw"]
    train = [(synthetic_images(B, H, W, seed=cfg["image_seed0"] + t), synthetic_targets(B, seed=cfg["target_seed0"] + t))
             for t in range(cfg["steps"])]
    val = (synthetic_images(cfg["val_batch"], H, W, seed=cfg["val_image_seed"]),
           synthetic_targets(cfg["val_batch"], seed=cfg["val_target_seed"]))
    return train, val


def run_trajectory(ref_models, dt):
    cfg = TRAJ
    train, (xv, Tv) = trajectory_batches(cfg)
    m = _fresh_damped(ref_models, dt)
    opt = torch.optim.Adam(m.parameters(), lr=cfg["lr"])
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, "min", **cfg["scheduler"])
    steps = []
    for x, T in train:
        m.train()
        losses = oracle_se3.geometric_loss(m(x.to(dt)).to(dt), T.to(dt))
        opt.zero_grad()
        losses.mean().backward()
        gn = float(torch.nn.utils.clip_grad_norm_(m.parameters(), cfg["max_grad_norm"]))
        opt.step()
        m.eval()
        with torch.no_grad():
            vl = oracle_se3.geometric_loss(m(xv.to(dt)).to(dt), Tv.to(dt)).mean().item()
        sched.step(vl)
        steps.append({"loss": losses.detach().tolist(), "grad_norm": gn, "val_loss": vl,
                      "lr": opt.param_groups[0]["lr"]})
    sd = m.state_dict()
    return steps, {"param_sums": _sums(sd, ("weight", "bias")),
                   "bn_running_sums": _sums(sd, ("running_mean", "running_var")),
                   "num_batches_tracked": int(sd["resnet.bn1.num_batches_tracked"]),
                   "param_sample": param_sample(m),
                   "bn_running": {k: [float(f"{x:.8g}") for x in v.double().tolist()] for k, v in sd.items()
                                  if k.endswith(("running_mean", "running_var"))}}


def param_sample(model, per_tensor: int = 64) -> dict:
    """Up to ``per_tensor`` evenly spaced elements of every parameter (flattened in its state_dict layout):
    a fixed subsample to compare whole trajectories element by element without storing 100 MB."""
    out = {}
    for n, p in model.named_parameters():
        flat = p.detach().double().flatten()
        idx = torch.linspace(0, flat.numel() - 1, min(flat.numel(), per_tensor)).round().long()
        out[n] = [float(f"{x:.10g}") for x in flat[idx].tolist()]
    return out


def trajectory_golden(ref_models) -> None:
    """golden_b8_damped_traj.json: the reference's 10-step trajectory in fp32 and fp64 (the fp32-vs-fp64
    spread per step is what the GPU test's tolerances are stated against)."""
    s32, end32 = run_trajectory(ref_models, torch.float32)
    s64, end64 = run_trajectory(ref_models, torch.float64)
    init = param_sample(_fresh_damped(ref_models))
    flat = lambda d: torch.tensor([v for k in init for v in d[k]], dtype=torch.float64)  # noqa: E731
    upd = (flat(end64["param_sample"]) - flat(init)).norm()
    e_ref = ((flat(end32["param_sample"]) - flat(end64["param_sample"])).norm() / upd).item()
    rs = lambda d: torch.cat([torch.tensor(d[k], dtype=torch.float64) for k in sorted(d)])  # noqa: E731
    rs0 = torch.cat([torch.zeros(len(v)) if k.endswith("mean") else torch.ones(len(v))
                     for k, v in sorted(end64["bn_running"].items())]).double()
    e_rs = ((rs(end32["bn_running"]) - rs(end64["bn_running"])).norm() / (rs(end64["bn_running"]) - rs0).norm()).item()
    out = {
        "generator": "tests/golden/make_golden.py::trajectory_golden",
        "pinned_against": "reference argus/models.py executed with oracle.resnet as torchvision.models",
        "config": TRAJ,
        "fp32": {"steps": s32, "end": end32},
        "fp64": {"steps": s64, "end": end64},
        "param_sample_init": init,
        # || p32 - p64 || / || p64 - p_init || over the sample: the reference fp32's own update error
        "ref_fp32_update_error": e_ref,
        # the same for the BN running statistics (update from their initial 0 / 1)
        "ref_fp32_running_stats_error": e_rs,
    }
    with open(OUT / "golden_b8_damped_traj.json", "w") as f:
        json.dump(out, f, separators=(",", ":"))
    spread = [max(abs(a - b) for a, b in zip(p["loss"], q["loss"])) for p, q in zip(s32, s64)]
    print("wrote", OUT / "golden_b8_damped_traj.json", "lr", [s["lr"] for s in s32], "val", [s["val_loss"] for s in s32],
          "fp32-fp64 loss spread", spread, "update error", e_ref, "running stats error", e_rs)


if __name__ == "__main__":
    # no argument: every fixture; otherwise only the named ones (two_rank, traj)
    parts = set(sys.argv[1:])
    if not parts:
        main()
    if parts:
        if not (REF / "argus" / "models.py").exists():
            raise SystemExit("reference not present: fixtures can only be regenerated in the build container")
        torch.set_num_threads(8)
        _ref = load_reference_models()
        if "two_rank" in parts:
            two_rank_golden(_ref)
        if "traj" in parts:
            trajectory_golden(_ref)
    else:
        _ref = load_reference_models()
        two_rank_golden(_ref)
        trajectory_golden(_ref)
