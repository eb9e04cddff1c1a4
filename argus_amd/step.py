"""One fused native training step over flat buffers — the body of argus/train.py:298-320.

Reference step (per batch): autocast forward -> fp32 SE(3) loss -> mean -> zero_grad -> backward
(DDP bucketed NCCL all-reduce inside) -> clip_grad_norm_(max_grad_norm) -> Adam.step.

Here: the model's parameters are re-homed into ONE flat fp32 buffer (conv weights stored OHWI —
the nn.Parameters become channels-last views of it, so state_dict()/load_state_dict() keep the
reference's OIHW shapes), gradients go to a parallel flat buffer written directly by the HIP
wgrad / BN / head kernels (no autograd), and the step is:

    engine.forward (bf16 or fp32 HIP kernels) -> se3_loss kernel (loss + dpred/B)
    -> engine.backward, starting a bucketed RCCL all-reduce (SUM, async, own stream) on each flat
       suffix of >= bucket_mb as soon as backward has finished it (DDP's overlap, without DDP); the
       collective is issued behind the weight-gradient side stream, so the main stream never waits
    -> wait -> global-norm kernel -> fused clip + 1/world + Adam kernel (28 B/param, HBM-bound)

Multi-GPU: one process per GPU; torch.distributed "nccl" is RCCL over xGMI on MI355X. BN statistics
stay per rank (as the reference: no SyncBatchNorm).
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.distributed as dist

from argus_amd._lib import lib, ptr, stream


class FlatParams:
    """Flat fp32 parameter / gradient storage for a module (64-element aligned slots)."""

    ALIGN = 64

    def __init__(self, model: torch.nn.Module):
        params = list(model.named_parameters())
        dev = params[0][1].device
        self.slots = []
        off = 0
        for n, p in params:
            self.slots.append((n, p, off, p.numel()))
            off += (p.numel() + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.total = off
        self.param = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        self.offset = {}
        self.G = {}
        for n, p, o, k in self.slots:
            if p.dtype != torch.float32:
                raise TypeError(f"{n}: fp32 parameters required")
            self.offset[n] = o
            pv, gv = self.param[o:o + k], self.grad[o:o + k]
            if p.dim() == 4:  # conv weight: OHWI storage, OIHW (channels-last) view
                K, Cc, R, S = p.shape
                pv.view(K, R, S, Cc).copy_(p.detach().permute(0, 2, 3, 1))
                p.data = pv.view(K, R, S, Cc).permute(0, 3, 1, 2)
                self.G[n] = gv.view(K, R, S, Cc)
                p.grad = self.G[n].permute(0, 3, 1, 2)
            else:
                pv.view(p.shape).copy_(p.detach())
                p.data = pv.view(p.shape)
                self.G[n] = gv.view(p.shape)
                p.grad = self.G[n]


class GradBucketer:
    """Bucketed async SUM all-reduce of a flat gradient buffer, driven by suffix-ready callbacks."""

    def __init__(self, grad: torch.Tensor, offsets: dict, group=None, bucket_mb: float = 25.0, op=None):
        self.grad = grad
        self.offsets = offsets
        self.group = group
        # SUM (DDP's all-reduce; the 1/world of its average is folded into the Adam kernel). Tests pass
        # a PREMUL_SUM to make a one-rank RCCL all-reduce change the values it reduces.
        self.op = dist.ReduceOp.SUM if op is None else op
        self.bucket = int(bucket_mb * 1024 * 1024 / grad.element_size())
        self.works = []
        self.pending_end = grad.numel()

    def start(self) -> None:
        self.works = []
        self.pending_end = self.grad.numel()

    def ready(self, name: str, comm=None) -> None:
        """Gradients of ``name`` and everything after it are issued; ``comm()`` (optional) is the stream
        context, ordered after the work that writes them, to issue the collective in (the engine's
        side stream after a wait on the main stream: the main stream itself does not wait). Issues a
        bucket when the suffix is big enough."""
        start = self.offsets[name]
        if self.pending_end - start >= self.bucket or start == 0:
            if comm is not None:
                with comm():
                    self._issue(start)
            else:
                self._issue(start)

    def _issue(self, start: int) -> None:
        if self.pending_end > start:
            w = dist.all_reduce(self.grad[start:self.pending_end], op=self.op, group=self.group,
                                async_op=True)
            self.works.append(w)
            self.pending_end = start

    def finish(self) -> None:
        self._issue(0)
        for w in self.works:
            w.wait()
        self.works = []


class FusedTrainer:
    """Native train step for ``argus_amd.models.NCameraCNN`` (see module docstring)."""

    def __init__(self, model, lr: float = 1e-4, max_grad_norm: float = 1.0, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, group=None, bucket_mb: float = 25.0):
        self.model = model
        self.flat = FlatParams(model)
        dev = self.flat.param.device
        self.lr = lr
        self.max_grad_norm = max_grad_norm
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.exp_avg = torch.zeros_like(self.flat.param)
        self.exp_avg_sq = torch.zeros_like(self.flat.param)
        self.step_count = 0
        self.norm = torch.zeros(1, dtype=torch.float32, device=dev)
        L = lib()
        self.norm_ws = torch.empty(L.dll.argus_sumsq_workspace_bytes(self.flat.total), dtype=torch.uint8, device=dev)
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self.world = dist.get_world_size(group) if self.distributed else 1
        self.bucketer = GradBucketer(self.flat.grad, self.flat.offset, group, bucket_mb) if self.distributed else None
        self._loss = None
        self._dpred = None
        # when a list (bench.py): per step, the (start, end) events around the wait for the gradient
        # all-reduce after the backward's own work - the collective tail the overlap did not hide
        self.tail_events: list | None = None

    def step(self, images: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        """One optimisation step on a device-resident batch; returns the per-sample losses (B,)."""
        model = self.model
        if not model.training:
            raise RuntimeError("FusedTrainer.step needs model.train()")
        L = lib()
        s = stream()
        B = images.shape[0]
        eng = model._engine(images.device)
        P, Bf = model._maps()
        targets = targets.contiguous().float()
        pred = eng.forward(images, P, Bf, True)
        if self._loss is None or self._loss.shape[0] != B:
            self._loss = torch.empty(B, dtype=torch.float32, device=images.device)
            self._dpred = torch.empty(B, 6, dtype=torch.float32, device=images.device)
        L.se3_loss(B, ptr(pred), ptr(targets), ptr(self._loss), ptr(self._dpred), C.c_float(1.0 / B), s)
        if self.bucketer is not None:
            self.bucketer.start()
            eng.backward(self._dpred, P, self.flat.G, on_ready=self.bucketer.ready)
            t0 = t1 = None
            if self.tail_events is not None:  # main stream: end of its backward work -> collectives done
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record()
            self.bucketer.finish()
            if t1 is not None:
                t1.record()
                self.tail_events.append((t0, t1))
        else:
            eng.backward(self._dpred, P, self.flat.G)
        self.step_count += 1
        b1, b2 = self.betas
        t = self.step_count
        L.global_norm(self.flat.total, ptr(self.flat.grad), ptr(self.norm), ptr(self.norm_ws), s)
        L.adam_step(self.flat.total, ptr(self.flat.param), ptr(self.flat.grad), ptr(self.exp_avg),
                    ptr(self.exp_avg_sq), ptr(self.norm), C.c_float(1.0 / self.world), C.c_float(self.max_grad_norm),
                    C.c_float(self.lr), C.c_float(b1), C.c_float(b2), C.c_float(self.eps),
                    C.c_float(self.weight_decay), C.c_float(1 - b1**t), C.c_float(1 - b2**t), s)
        return self._loss

    def grad_norm(self) -> torch.Tensor:
        """Total gradient norm of the last step (before clipping, after the 1/world average)."""
        return self.norm / self.world
