"""NCameraCNN on the MI355X HIP engine — drop-in for ``argus/models.py``.

Same public surface as the reference (argus/models.py:13-90):
- ``NCameraCNNConfig(n_cams=2, resnet_output_dim=1024)`` (frozen dataclass, ``models.py:13-23``);
- ``NCameraCNN(cfg=None)`` is an ``nn.Module``; ``forward(x: (B, 3*n_cams, H, W) fp32) -> (B, 6)``
  se(3) vector; non-4-D input raises ``AssertionError`` (``models.py:76``); ``state_dict()`` keys,
  shapes (OIHW conv weights) and dtypes equal the reference's;
  ``train()/eval()`` select batch vs running BN statistics.

The module tree is built from ``torch.nn`` containers in torchvision's construction order, so the
seeded initialisation consumes the RNG exactly as ``models.resnet50()`` + the replaced ``fc`` +
``output_mlp`` do (``models.py:43,56,58-64``); the containers only *hold* parameters — no ATen
conv/BN/linear kernel ever runs. ``forward`` is one autograd Function over the whole network whose
forward and backward are the native schedule in ``argus_amd.engine`` (hand-written HIP kernels).
Pretrained ImageNet weights (``weights="DEFAULT"``) are not downloadable offline: seeded init, or
load a local ``.pth``.

Extension: ``compute_dtype`` ("fp32" — parity path, fp32 activations and exact-fp32 MFMA; "bf16" —
throughput path, bf16 activations/weights with fp32 accumulation, statistics and head; "fp8" — the
bf16 path whose conv forward and data-gradient GEMMs take OCP MX-fp8 operands (e4m3 + E8M0 block
scales, BASELINE configs[4]) where the channel count allows). The reference's ``--amp`` (fp16
autocast) maps to "bf16".
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn

from argus_amd.engine import ResNetEngine, conv_grad_shape


@dataclass(frozen=True)
class NCameraCNNConfig:
    """Configuration for the NCameraCNN model (argus/models.py:13-23)."""

    n_cams: int = 2
    resnet_output_dim: int = 1024


# ---- parameter containers in torchvision's order (RNG consumption = models.resnet50()) ----------
class _Bottleneck(nn.Module):
    def __init__(self, inplanes: int, planes: int, stride: int, downsample: Optional[nn.Module]):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.downsample = downsample


class _ResNet50(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        inplanes = 64
        for L, (planes, n, stride) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)], start=1):
            ds = nn.Sequential(nn.Conv2d(inplanes, planes * 4, 1, stride=stride, bias=False), nn.BatchNorm2d(planes * 4))
            blocks = [_Bottleneck(inplanes, planes, stride, ds)]
            inplanes = planes * 4
            blocks += [_Bottleneck(inplanes, planes, 1, None) for _ in range(1, n)]
            setattr(self, f"layer{L}", nn.Sequential(*blocks))
        self.fc = nn.Linear(2048, 1000)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)


class _NetFn(torch.autograd.Function):
    """Whole-network Function: forward/backward are the native HIP schedule (argus_amd.engine)."""

    @staticmethod
    def forward(ctx, x, model, *params):
        engine = model._engine(x.device)
        P, Bf = model._maps()
        pred = engine.forward(x, P, Bf, model.training).clone()
        engine.fwd_id = getattr(engine, "fwd_id", 0) + 1
        ctx.engine, ctx.model, ctx.fwd_id = engine, model, engine.fwd_id
        return pred

    @staticmethod
    def backward(ctx, dpred):
        engine, model = ctx.engine, ctx.model
        if engine.fwd_id != ctx.fwd_id:
            raise RuntimeError("argus_amd: another forward ran before this backward; the engine keeps one "
                               "set of saved activations per model")
        P, _ = model._maps(forward=False)
        G = {}
        for name, p in model.named_parameters():
            if name.endswith(".weight") and p.dim() == 4:
                G[name] = torch.empty(conv_grad_shape(p.shape), dtype=torch.float32, device=p.device)
            else:
                G[name] = torch.empty_like(p)
        engine.backward(dpred, P, G)
        grads = []
        for name, p in model.named_parameters():
            g = G[name]
            grads.append(g.permute(0, 3, 1, 2) if g.dim() == 4 else g)
        return (None, None, *grads)


def strip_checkpoint_prefixes(state_dict):
    """Remove leading ``module.`` / ``_orig_mod.`` (in any nesting) from every key."""
    out = type(state_dict)() if isinstance(state_dict, dict) else {}
    for k, v in state_dict.items():
        while True:
            for p in ("module.", "_orig_mod."):
                if k.startswith(p):
                    k = k[len(p):]
                    break
            else:
                break
        out[k] = v
    if hasattr(state_dict, "_metadata"):
        out._metadata = {strip_checkpoint_prefixes({m: None}).popitem()[0] if m else m: v
                         for m, v in state_dict._metadata.items()}
    return out


class NCameraCNN(nn.Module):
    """A CNN which assumes N cameras are available in the scene (argus/models.py:26-90)."""

    def __init__(self, cfg: Optional[NCameraCNNConfig] = None, compute_dtype: str = "fp32",
                 kernel_tuning: Optional[dict] = None) -> None:
        super().__init__()
        self.resnet = _ResNet50()
        if cfg is None:
            cfg = NCameraCNNConfig()
        self.num_channels = 3 * cfg.n_cams
        self.resnet_output_dim = cfg.resnet_output_dim
        self.n_cams = cfg.n_cams
        self.resnet.fc = nn.Linear(2048, self.resnet_output_dim)
        self.output_mlp = nn.Sequential(
            nn.Linear(self.n_cams * self.resnet_output_dim, 128),
            nn.GELU(),
            nn.Linear(128, 128),
            nn.GELU(),
            nn.Linear(128, 6),
        )
        self.compute_dtype = compute_dtype
        # optional kernel-selection overrides ({policy key: value}, argus_conv_policy_default) for this
        # model's engines - experiments and the kernel-coverage tests; None = the library defaults
        self.kernel_tuning = dict(kernel_tuning) if kernel_tuning else None
        self._engines: dict = {}

    # ---------------------------------------------------------------- engine plumbing
    def _engine(self, device: torch.device) -> ResNetEngine:
        device = torch.device(device)
        if device.type == "cuda" and device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        tuning = tuple(sorted((self.kernel_tuning or {}).items()))
        key = (str(device), self.compute_dtype, tuning)
        eng = self._engines.get(key)
        if eng is None:
            eng = ResNetEngine(self.n_cams, self.resnet_output_dim, self.compute_dtype, device, dict(tuning))
            self._engines[key] = eng
        return eng

    def _maps(self, forward: bool = True):
        """name -> parameter, name -> buffer (+ per-BN ".eps" / ".momentum"). ``forward``: the maps of a
        forward about to run (a train-mode one advances the momentum=None shadow counts below)."""
        P = dict(self.named_parameters())
        Bf = dict(self.named_buffers())
        cma = [(name, m) for name, m in self.named_modules() if isinstance(m, nn.BatchNorm2d) and m.momentum is None]
        # momentum=None is torch's cumulative moving average: factor 1 / num_batches_tracked after the
        # increment. The counters live on the device and the finalize kernels increment them; the host
        # keeps a shadow count per layer (one read when a counter was last written by torch, e.g. by
        # load_state_dict, detected through the tensor's version counter), so a training step does not
        # synchronise with the device to know it.
        counts = {}
        if cma and self.training:
            shadow = self.__dict__.setdefault("_nbt_shadow", {})
            stale = [(name, m) for name, m in cma
                     if shadow.get(name, (None,))[0] != (m.num_batches_tracked.data_ptr(),
                                                         m.num_batches_tracked._version)]
            if stale:
                vals = torch.stack([m.num_batches_tracked for _, m in stale]).cpu().tolist()
                for (name, m), v in zip(stale, vals):
                    shadow[name] = ((m.num_batches_tracked.data_ptr(), m.num_batches_tracked._version), int(v))
            for name, m in cma:
                key, n = shadow[name]
                counts[name] = n
                if forward:
                    shadow[name] = (key, n + 1)  # the forward's finalize increments the device counter
        for name, m in self.named_modules():
            if isinstance(m, nn.BatchNorm2d):
                Bf[name + ".eps"] = m.eps
                Bf[name + ".momentum"] = m.momentum if m.momentum is not None else 1.0 / (counts.get(name, 0) + 1)
        return P, Bf

    def invalidate_bn_counters(self) -> None:
        """Forget the host shadow of every ``num_batches_tracked`` (momentum=None BN, ``_maps``): the next
        train-mode forward re-reads the device counters. Writes through ``.data`` (e.g.
        ``dist.broadcast(b.data)``) do not bump a tensor's version counter, so whoever writes the counters
        that way calls this (``train.sync_bn_buffers`` and the initial broadcast do)."""
        self.__dict__.pop("_nbt_shadow", None)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """``nn.Module.load_state_dict`` that also takes the reference's wrapped checkpoints: keys
        prefixed ``module.`` (a DDP model's state_dict, argus/train.py:199,358) or ``_orig_mod.``
        (a ``torch.compile``d model, train.py:61) are stripped first."""
        return super().load_state_dict(strip_checkpoint_prefixes(state_dict), strict=strict, assign=assign)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(B, 3*n_cams, H, W) fp32 images in [0, 1] -> (B, 6) se(3) poses.

        Extension: uint8 images in [0, 255] (``CameraCubePoseDataset(uint8=True)``) are accepted too;
        the reference's ``/ 255.0`` (argus/data.py:214-215) then runs on the device, bit-identically."""
        assert len(x.shape) == 4, "The input images must be of shape (B, C, H, W)! If B=1, add a dummy dimension."
        if x.device.type != "cuda":
            raise RuntimeError("argus_amd.NCameraCNN runs only on the MI355X HIP path: move the model and the "
                               "images to a cuda device (there is no CPU fallback)")
        params = [p for _, p in self.named_parameters()]
        if any(p.device != x.device or p.dtype != torch.float32 for p in params):
            raise RuntimeError("argus_amd.NCameraCNN parameters must be fp32 on the input's device")
        return _NetFn.apply(x, self, *params)
