"""Native ResNet-50 x N-camera forward/backward schedule over libargus_hip (MI355X / gfx950).

Replaces the implicit ATen/cuDNN work behind ``NCameraCNN.forward`` (argus/models.py:66-90, the
torchvision ResNet-50 at :43) and its autograd backward (argus/train.py:316). The schedule is
fixed for the architecture, so it is written out explicitly instead of being traced:

forward (train mode), per Bottleneck (stride on the 3x3, torchvision v1.5):
    y1 = conv1(h)                      + BN1 stats   (epilogue)        -> finalize -> (sc1, sh1)
    y2 = conv2(relu(bn1(y1)))          + BN2 stats   (BN1+ReLU applied while staging y1)
    y3 = conv3(relu(bn2(y2)))          + BN3 stats
    yd = downsample(h)                 + BNd stats   (first block of a stage)
    out = relu(bn3(y3) + (bnd(yd) | h))                                  (one fused pass)
stem: y0 = conv7x7/2(x) + stats; p0 = maxpool3x3/2(relu(bn1(y0))) (fused, argmax kept)
head (fp32): feat = avgpool(out) -> fc 2048->1024 -> reshape (B, n_cams*1024) -> GELU -> MLP -> (B,6)

Saved for backward: y1, y2, y3, yd, out per block (compute dtype), BN mean/invstd/scale/shift,
stem y0 + maxpool argmax, head pre-activations. ReLU masks and normalised activations are
recomputed from the raw conv outputs (no x_hat tensors are stored).

Eval mode uses running statistics (bn_eval_coeffs) and skips all statistics / running updates.
"""
from __future__ import annotations

import ctypes as C
import collections
import contextlib
from dataclasses import dataclass

import torch

from argus_amd._lib import (BnFwdFin, BF16, F32, FP8, BnBwdEpilogue, BnBwdPrologue, ConvDesc, DeviceEvent, lib, ptr,
                             stream)


@dataclass(frozen=True)
class Block:
    prefix: str  # "resnet.layer{L}.{i}"
    cin: int
    width: int
    cout: int
    stride: int
    has_ds: bool


def resnet50_blocks() -> list[Block]:
    blocks, inplanes = [], 64
    for L, (planes, n, stride) in enumerate([(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)], start=1):
        for i in range(n):
            blocks.append(Block(f"resnet.layer{L}.{i}", inplanes, planes, planes * 4, stride if i == 0 else 1, i == 0))
            inplanes = planes * 4
    return blocks


def _out(h: int, k: int, s: int, p: int) -> int:
    return (h + 2 * p - k) // s + 1


@dataclass
class _Conv:
    name: str
    desc: ConvDesc
    wf: torch.Tensor
    wd: torch.Tensor | None
    stat_rows: int
    stat_tile: int
    tags: tuple  # kernel instantiation per pass (fwd, dgrad, wgrad)
    flops: int  # algorithmic flops of one pass
    so_rows: int  # BN partial rows / tile of a statistics-only forward (y not stored: the fused tail)
    so_tile: int
    part_bytes: int = 0  # stat_part bytes either forward form needs (argus_conv_fwd_stat_part_bytes)


class ResNetEngine:
    """Workspace + launch schedule for one (batch, H, W, dtype) configuration on one device."""

    def __init__(self, n_cams: int, resnet_output_dim: int, dtype: str, device: torch.device,
                 tuning: dict | None = None):
        if dtype not in ("fp32", "bf16", "fp8"):
            raise ValueError(f"compute dtype must be 'fp32', 'bf16' or 'fp8', got {dtype!r}")
        self.L = lib()
        # per-call overrides of the library's kernel-selection policy, attached to every conv descriptor
        # of this engine (argus_conv_desc.tuning; None = the library defaults, the benched selection)
        self.tuning = dict(tuning) if tuning else None
        self.n_cams = n_cams
        self.rdim = resnet_output_dim
        self.dtype = dtype
        # "fp8": the bf16 network (tensors, BN, weight gradients) whose conv forward / data-gradient
        # GEMMs take MX-fp8 operands where the shape allows (ARGUS_FP8, igemm_kernel's kFp8Bit variant)
        low = dtype in ("bf16", "fp8")
        self.dt = BF16 if low else F32
        self.cdt = FP8 if dtype == "fp8" else self.dt  # conv fwd / dgrad entry points
        self.tdt = torch.bfloat16 if low else torch.float32
        self.E = 8 if low else 4  # elements per 16-byte chunk
        # materialize a = relu(bn(y)) of bn1/bn2 once per forward (one extra HBM pass each) so that
        # conv2/conv3 forward and weight gradients run without the BN prologue, on the global->LDS
        # kernels; fp32 (parity path) keeps the fused prologue.
        self.materialize = low
        self.device = torch.device(device)
        self.blocks = resnet50_blocks()
        self.shape = None
        self.saved = False
        self.debug: dict | None = None  # when a dict: clones of block outputs / block-input grads
        # Weight gradients run on a side stream, overlapped with the dgrad -> BN-backward chain of the
        # main stream (they only feed the gradient buffer). Events order them after their dy and
        # before any main-stream overwrite of that dy buffer; each bucket all-reduce is issued on the
        # side stream after both streams' work (on_ready's comm) and backward() joins it at its end.
        # False keeps everything on the caller's stream.
        self.wgrad_overlap = True
        # BN-backward apply (dy = ca*dm + cb*y + cc) staged by the consuming dgrad, which also stores dy for
        # the weight gradient (argus_conv_dgrad_bn with a prologue); False runs the apply pass
        self.fuse_apply = True
        # ... and where that dgrad stages the apply inside its kernel (1x1, register-staged:
        # argus_conv_dgrad_stages_prologue), dy is not stored at all: the side-stream weight gradient
        # stages the same apply from dm and y (argus_conv_wgrad_apply). Moves the dy write off the main
        # stream (one more read on the side stream). False stores dy.
        self.wgrad_apply = True
        # BN-backward finalize (dgamma, dbeta, ca / cb / cc) folded into the dgrad launch that produces
        # its partial sums (argus_conv_dgrad_bn with a workspace; +0.3 % at B=64); False runs
        # the separate bwd_finalize kernels. The forward statistics keep their own
        # finalize launch (folding it into the conv measured neutral).
        self.fold_fin = True
        # the forward BN statistics finalize folded into the producing conv's last workgroups
        # (argus_conv_fwd_fin: bit-identical to argus_conv_fwd + argus_bn_finalize; round 6). Off: the
        # last arrivers' fp64 merges serialise at each producer's tail for about as long as the separate
        # launch, and measured 13.27-13.42 vs 13.12-13.19 ms at B=64 (profiles/r06j_ab_b64_fold_fwd_fin.txt)
        self.fold_fwd_fin = False
        # ... and the stem BN's finalize into the maxpool backward pass (argus_maxpool_bwd_bn_fin)
        self.fold_stem_fin = True
        self._side: torch.cuda.Stream | None = None
        self._pending: dict = {}  # buffer data_ptr -> (seq, event) of the last side-stream wgrad reading it
        self._last_side = None
        # Side-stream work of one bottleneck block is issued together at the block's end: one event
        # record on the main stream per block instead of one per weight gradient (each cross-stream
        # event costs the main stream a dispatch gap; +0.6 % at B=64). A single wait per block for the
        # ring buffers it reuses was measured too (-2.5 %: it waits earlier than the per-buffer guards).
        # False issues every weight gradient as soon as its dy is ready.
        self.side_batch = True
        # a block's deferred weight gradients issued in reverse order (conv1 first; they write separate
        # dW buffers and share one workspace in stream order, so the results are identical)
        self.side_reverse = False
        # cross-stream events with a device-scope release / acquire (argus_event_*, hipEventDisableSystemFence)
        # instead of torch.cuda.Event; the collectives' stream hand-off (_comm) keeps torch's events either
        # way. Off: measured 13.34-13.43 vs 13.28-13.34 ms at B=64 (profiles/r06j_ab_b64_light_events.txt);
        # the ~6 us main-stream gap at each cross-stream event is not the system-scope fence
        self.light_events = False
        self._ev_keep: collections.deque = collections.deque(maxlen=512)  # recent events, destroyed late
        self._deferred: list = []  # (cv, fn, buffer data_ptrs)
        self._side_seq = 0
        self._waited_seq = 0
        # the stem weight gradient (main stream, its own split workspace) is issued before the final
        # join, beside the side stream's last weight gradients (+0.2 %); False: after it
        self._stem_overlap = True
        # the first block's downsample weight gradient runs on the main stream after the stem weight
        # gradient instead of on the side stream: the side stream's last weight gradients otherwise
        # outlast the main stream's stem work (an exposed ~150 us tail before the join; +0.4 % at B=64,
        # two paired runs). An attribute, not an environment switch: test_gpu_train.py::
        # test_side_stream_overlap_is_bit_identical runs both placements.
        self.tail_main = True
        self._tail: list = []
        self.dy_ring = 12  # dy ring buffers (set before the first forward)
        # HIP priority of the side stream (torch convention: lower = higher priority; 0 = the main
        # stream's); set before the first backward
        self.side_priority = 0
        # layer-1 conv3: data and weight gradient in one pass over dm3 / y3 on the main stream
        # (argus_conv_dgrad_wgrad_bn) instead of the dgrad + the side stream's wgrad_apply, which read
        # both 256-channel tensors again; set before the first forward
        self.fuse_dgw = True
        # the 3x3 data gradients (compute-bound: ~500 FLOP/B) run alone: before each one the main stream
        # waits for the weight gradients already issued on the side stream, whose workgroups would
        # otherwise hold the CUs' LDS and registers beside it (the block's own deferred weight gradients
        # are issued after it, at the block's end, as usual)
        self.gate3x3 = False
        # ... only for the blocks of at most this width (64: layer 1, whose halo data gradients run at 76 KB of
        # LDS a workgroup and lose CUs to the side stream's 128-148 KB weight-gradient workgroups); 0 = off
        self.gate3x3_width = 0
        # the bottleneck tail on the bf16 schedule: conv3's forward only reduces bn3's statistics (nothing
        # stored), then one pass recomputes its C tile and applies bn3 + the residual + ReLU there
        # (argus_conv_fwd_bn_out): the bn_apply pass no longer reads y3 back (bit-identical outputs)
        self.fuse_out = True
        # the block-output BN's backward reduction (in the epilogue of the next block's conv1 / downsample
        # data gradient) recomputes bn3's input y3 from a2 and conv3's bf16 weights instead of reading it
        # (argus_bn_bwd_epilogue.y_x; bit-identical): the 4w-channel y3 read becomes a w-channel a2 read.
        # Measured slower (round 5, profiles/r05c_*): the recompute GEMM in the epilogue is load-latency
        # bound, the producing dgrads took 244 / 237 us instead of 191 us (B=64; step 14.75 vs 14.06 ms)
        self.yrec_epi = False
        # ... and where every other reader of y3 recomputes it too (layer 1: the fused conv3 data + weight
        # gradient, argus_conv_dgrad_wgrad_bn with pro->y NULL), y3 is never stored: the forward's fused
        # tail writes only the block output (the debug capture keeps storing it for the stage checks);
        # needs yrec_epi (saves ~0.1 ms at B=64 on its own: not enough to pay for it)
        self.y3_free = False
        # fp8: the 3x3 stride-1 convs whose forward (policy key 37 bit 8) / data gradient (bit 2) take
        # MX-fp8 operands read them as stored MX-fp8 copies (argus_conv_fwd_x8 / argus_conv_dgrad_bn_x8):
        # bn1's apply and bn2's backward apply write the e4m3 + E8M0 copy beside their bf16 output (the
        # weight gradient still reads the bf16 one), and the LDS-halo kernel's F8 variant runs the conv at
        # the fp8 MFMA rate; False: the register-staged fp8 kernel quantizes while staging (set before
        # the first forward)
        self.x8 = True
        # training forward with the fused tail: conv3's statistics pass applies bn2 to y2 while staging its
        # operand and stores a2 itself (argus_conv_fwd_apply_out, bit-identical to the bn_apply pass it
        # replaces: one pass over y2 and one launch fewer per block). First measured 0.5 % slower (round 5,
        # profiles/r05o_ab_a2_in_stats.txt); after the register-staged kernels stopped waiting for their
        # loads inside load(), 0.4 % faster at B=64 (13.79-13.81 vs 13.84-13.85 ms, r05u_ab_a2_in_stats.txt)
        # but 1.5 % slower at B=256 (47.2-47.8 vs 46.7-46.9 ms) and 0.9 % at 376x672 (91.5-92.5 vs
        # 90.6-91.5 ms, r05aa_ab_a2_in_stats_*.txt): off
        self.a2_in_stats = False
        # (the schedule switches above are attributes, not environment variables: tools/engine_ab.py
        # A/B-measures them; test_gpu_train.py runs the overlap / tail placements against each other)

    # ------------------------------------------------------------------ allocation
    def _t(self, *shape, dtype=None):
        return torch.empty(shape, dtype=dtype or self.tdt, device=self.device)

    def _f(self, *shape):
        return torch.empty(shape, dtype=torch.float32, device=self.device)

    def ensure(self, B: int, H: int, W: int) -> None:
        if self.shape == (B, H, W):
            return
        self.shape = (B, H, W)
        N = B * self.n_cams
        self.N = N
        L = self.L
        dt = self.dt
        convs: dict[str, _Conv] = {}

        def add(name, n, h, w, c, k, ks, s, p, stem=False):
            d = ConvDesc(n, h, w, c, k, ks, ks, s, p, _out(h, ks, s, p), _out(w, ks, s, p), int(stem)).with_tuning(
                self.tuning)
            if stem:
                wf = self._t(k, 256)
                wd = None
            else:
                wf = self._t(k, ks * ks * c)
                wd = self._t(c, ks * ks * k)
            rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), self.cdt)
            tile = L.dll.argus_conv_fwd_stat_tile(C.byref(d), dt)
            fl = C.c_int64(0)
            tags = tuple(L.dll.argus_conv_launch_info(C.byref(d), dt, ps, C.byref(fl)) for ps in range(3))
            so = (L.dll.argus_conv_fwd_stats_only_rows(C.byref(d), BF16),
                  L.dll.argus_conv_fwd_stats_only_tile(C.byref(d), BF16))
            pb = max(L.dll.argus_conv_fwd_stat_part_bytes(C.byref(d), self.cdt, 0),
                     L.dll.argus_conv_fwd_stat_part_bytes(C.byref(d), dt, 0),
                     L.dll.argus_conv_fwd_stat_part_bytes(C.byref(d), BF16, 1))
            convs[name] = _Conv(name, d, wf, wd, rows, tile, tags, fl.value, *so, part_bytes=pb)
            return d.ho, d.wo

        H1, W1 = add("resnet.conv1", N, H, W, 3, 64, 7, 2, 3, stem=True)
        H2, W2 = _out(H1, 3, 2, 1), _out(W1, 3, 2, 1)
        self.stem_hw = (H1, W1)
        self.pool_hw = (H2, W2)
        self.x0 = self._t(N, H, W, 4)
        self.y0 = self._t(N, H1, W1, 64)
        self.p0 = self._t(N, H2, W2, 64)
        self.amax = torch.empty((N, H2, W2, 64), dtype=torch.uint8, device=self.device)
        act = []
        h, w = H2, W2
        max_elems = N * H1 * W1 * 64
        for b in self.blocks:
            add(b.prefix + ".conv1", N, h, w, b.cin, b.width, 1, 1, 0)
            ho, wo = add(b.prefix + ".conv2", N, h, w, b.width, b.width, 3, b.stride, 1)
            add(b.prefix + ".conv3", N, ho, wo, b.width, b.cout, 1, 1, 0)
            if b.has_ds:
                add(b.prefix + ".downsample.0", N, h, w, b.cin, b.cout, 1, b.stride, 0)
            a = {
                "hw_in": (h, w), "hw": (ho, wo),
                "y1": self._t(N, h, w, b.width), "y2": self._t(N, ho, wo, b.width),
                "y3": self._t(N, ho, wo, b.cout), "out": self._t(N, ho, wo, b.cout),
                "yd": self._t(N, ho, wo, b.cout) if b.has_ds else None,
                "a1": self._t(N, h, w, b.width) if self.materialize else None,
                "a2": self._t(N, ho, wo, b.width) if self.materialize else None,
                # ReLU mask of `out`, one byte per 16-byte chunk (argus_bn_apply mask_out)
                "bits": torch.empty(N * ho * wo * b.cout // self.E, dtype=torch.uint8, device=self.device),
            }
            max_elems = max(max_elems, N * h * w * b.cin, N * h * w * b.width, N * ho * wo * b.cout)
            act.append(a)
            h, w = ho, wo
        self.act = act
        self.final_hw = (h, w)
        self.convs = convs
        # x8 passes of the 3x3 convs (fwd, dgrad) and one scratch buffer for their MX-fp8 operand (written
        # and read back-to-back on the main stream)
        self.x8_conv = {}
        x8_bytes = 16
        for b in self.blocks:
            n = b.prefix + ".conv2"
            d_ = convs[n].desc
            on = self.x8 and self.cdt == FP8 and self.materialize
            f = on and bool(L.dll.argus_conv_x8_ok(C.byref(d_), 0))
            g = on and bool(L.dll.argus_conv_x8_ok(C.byref(d_), 1))
            self.x8_conv[n] = (f, g)
            if f:
                x8_bytes = max(x8_bytes, d_.n * d_.h * d_.w * d_.c * 33 // 32)
            if g:
                x8_bytes = max(x8_bytes, d_.n * d_.ho * d_.wo * d_.k * 33 // 32)
        self.x8buf = torch.empty(x8_bytes, dtype=torch.uint8, device=self.device)

        # BN state: rows of [mean, invstd, scale, shift] and backward coefficients [ca, cb, cc]
        self.bn_names = ["resnet.bn1"]
        for b in self.blocks:
            self.bn_names += [b.prefix + ".bn1", b.prefix + ".bn2", b.prefix + ".bn3"]
            if b.has_ds:
                self.bn_names.append(b.prefix + ".downsample.1")
        chans = {"resnet.bn1": 64}
        for b in self.blocks:
            chans[b.prefix + ".bn1"] = b.width
            chans[b.prefix + ".bn2"] = b.width
            chans[b.prefix + ".bn3"] = b.cout
            if b.has_ds:
                chans[b.prefix + ".downsample.1"] = b.cout
        self.bn_ch = chans
        self.bn_state = {n: self._f(4, c) for n, c in chans.items()}
        self.bn_coef = {n: self._f(3, c) for n, c in chans.items()}

        # sized by the library (argus_conv_fwd_stat_part_bytes): the float2 partials plus the int32 row counts
        # of a ragged producer (negative stat tile: the stem, the persistent statistics-only forward)
        self.stat_part = self._f((max(cv.part_bytes for cv in convs.values()) + 3) // 4)
        self.bn_ws = torch.zeros(L.dll.argus_bn_workspace_bytes(2048), dtype=torch.uint8, device=self.device)
        # the downsample branch's own statistics workspaces (it runs on the side stream in forward)
        self.stat_part_ds = self._f((max([cv.part_bytes for n, cv in convs.items() if ".downsample." in n] or [8])
                                     + 3) // 4)
        self.bn_ws_ds = torch.zeros(L.dll.argus_bn_workspace_bytes(2048), dtype=torch.uint8, device=self.device)
        max_bwd = 0
        for b, a in zip(self.blocks, act):
            for hw, c in ((a["hw_in"], b.width), (a["hw"], b.width), (a["hw"], b.cout)):
                px = N * hw[0] * hw[1]
                max_bwd = max(max_bwd, L.dll.argus_bn_bwd_rows(px, c) * c)
        max_bwd = max(max_bwd, L.dll.argus_bn_bwd_rows(N * H1 * W1, 64) * 64,
                      L.dll.argus_maxpool_bwd_bn_rows(dt, N, H1, W1, 64) * 64)
        for cv in convs.values():  # BN-backward partials written by dgrad epilogues (rows x C_in)
            if not cv.desc.stem:
                d_ = cv.desc
                max_bwd = max(max_bwd, L.dll.argus_conv_dgrad_bn_rows(C.byref(d_), self.cdt) * d_.c,
                              (4 - (-(d_.n * d_.h * d_.w) // 64)) * d_.c)  # y-recompute epilogues: 64-row tiles per phase
        # convs whose data and weight gradient run fused (argus_conv_dgrad_wgrad_bn)
        # (layer-1 conv3s, and the first block's downsample: the same 64 -> 256 channel 1x1 shape). It is a
        # bf16 kernel: with compute_dtype fp8 it serves these convs too unless the fp8 pass policy (key 37)
        # gives the 1x1 data gradients MX-fp8 operands (their weight copies are then fp8)
        f8_1x1 = (self.tuning or {}).get(37, L.dll.argus_conv_policy_default(37)) & 4
        self.dgw_dt = BF16 if self.cdt == FP8 and not f8_1x1 else self.cdt
        self.dgw = {n for n, cv in convs.items() if self.fuse_dgw and n.endswith((".conv3", ".downsample.0"))
                    and not cv.desc.stem and L.dll.argus_conv_dgrad_wgrad_ok(C.byref(cv.desc), self.dgw_dt)}
        dgws = 16
        for n in self.dgw:
            d_ = C.byref(convs[n].desc)
            max_bwd = max(max_bwd, L.dll.argus_conv_dgrad_wgrad_bn_rows(d_, self.dgw_dt) * convs[n].desc.c)
            dgws = max(dgws, L.dll.argus_conv_dgrad_wgrad_workspace_bytes(d_, self.dgw_dt))
        self.dgw_ws = torch.empty(dgws, dtype=torch.uint8, device=self.device)  # main stream only
        self.bwd_part = self._f(max_bwd * 2)
        self.bwd_part2 = self._f(max_bwd * 2)  # second branch (downsample BN) of a dual reduce
        ws = max(L.dll.argus_conv_wgrad_workspace_bytes(C.byref(cv.desc), dt) for cv in convs.values())
        # zeroed: a folded DMA weight gradient (policy key 50) keeps its counters in the last bytes
        self.wg_ws = torch.zeros(ws, dtype=torch.uint8, device=self.device)
        self.wg_ws_bytes = ws
        wss = L.dll.argus_conv_wgrad_workspace_bytes(C.byref(convs["resnet.conv1"].desc), dt)
        # the stem weight gradient's workspace; also the first block's downsample weight gradient's, which
        # runs after it on the main stream (tail_main)
        ds0 = self.blocks[0].prefix + ".downsample.0"
        if ds0 in convs:
            wss = max(wss, L.dll.argus_conv_wgrad_workspace_bytes(C.byref(convs[ds0].desc), dt))
        self.wg_ws_stem = torch.zeros(wss, dtype=torch.uint8, device=self.device)
        self.stages_pro = {n: bool(L.dll.argus_conv_dgrad_stages_prologue(C.byref(cv.desc), self.cdt))
                           for n, cv in convs.items() if not cv.desc.stem}
        self.gbuf = [self._t(max_elems) for _ in range(3)]  # avgpool dh; dza / dzb (the dz of bn2 / bn1)
        # dy operands of the side-stream weight gradients come from a ring, so the main stream can
        # run ahead of the wgrad stream by several layers before it must wait to reuse a buffer
        # (a reuse waits on the event of the wgrad that last read it; 16 buffers measured no better)
        nring = max(8, self.dy_ring)  # >= 2 blocks of takes
        self.dyring = [self._t(max_elems) for _ in range(nring)]
        self._ring_i = 0

        Fd = 512 * 4
        self.feat = self._f(N, Fd)
        self.h0 = self._f(N, self.rdim)
        self.g0 = self._f(B, self.n_cams * self.rdim)
        self.h1, self.g1 = self._f(B, 128), self._f(B, 128)
        self.h2, self.g2 = self._f(B, 128), self._f(B, 128)
        self.pred = self._f(B, 6)
        self.dh2, self.dh1 = self._f(B, 128), self._f(B, 128)
        self.dh0 = self._f(B, self.n_cams * self.rdim)
        self.dfeat = self._f(N, Fd)
        D = self.n_cams * self.rdim
        shapes = [(N, self.rdim, Fd), (B, 128, D), (B, 128, 128), (B, 6, 128), (6, 128, B), (B, 128, 6),
                  (128, 128, B), (128, D, B), (B, D, 128), (self.rdim, Fd, N), (N, Fd, self.rdim)]
        hws = max(L.dll.argus_gemm_f32_workspace_bytes(*sh) for sh in shapes)
        self.gemm_ws = torch.empty(max(hws, 16), dtype=torch.uint8, device=self.device)
        self.gemm_ws_side = torch.empty(max(hws, 16), dtype=torch.uint8, device=self.device)

    # ------------------------------------------------------------------ helpers
    def _bn_train(self, P, Bf, name, rows, tile, count, part=None, ws=None):
        st = self.bn_state[name]
        mom = Bf.get(name + ".momentum", 0.1)
        part = self.stat_part if part is None else part
        ws = self.bn_ws if ws is None else ws
        self.L.bn_finalize(self.bn_ch[name], rows, tile, ptr(part), count, ptr(P[name + ".weight"]),
                           ptr(P[name + ".bias"]), C.c_float(Bf.get(name + ".eps", 1e-5)), C.c_float(mom),
                           ptr(Bf[name + ".running_mean"]), ptr(Bf[name + ".running_var"]),
                           ptr(Bf[name + ".num_batches_tracked"]), ptr(st[0]), ptr(st[1]), ptr(st[2]), ptr(st[3]),
                           ptr(ws), stream())

    def _bn_eval(self, P, Bf, name):
        st = self.bn_state[name]
        self.L.bn_eval_coeffs(self.bn_ch[name], ptr(P[name + ".weight"]), ptr(P[name + ".bias"]),
                              ptr(Bf[name + ".running_mean"]), ptr(Bf[name + ".running_var"]),
                              C.c_float(Bf.get(name + ".eps", 1e-5)), ptr(st[2]), ptr(st[3]), stream())

    def _fwd_fin(self, P, Bf, name, ws):
        """argus_bn_fwd_fin of BN ``name`` (the arguments _bn_train passes to argus_bn_finalize)."""
        st = self.bn_state[name]
        f = BnFwdFin()
        f.workspace, f.gamma, f.beta = ptr(ws), ptr(P[name + ".weight"]), ptr(P[name + ".bias"])
        f.eps, f.momentum = Bf.get(name + ".eps", 1e-5), Bf.get(name + ".momentum", 0.1)
        f.running_mean, f.running_var = ptr(Bf[name + ".running_mean"]), ptr(Bf[name + ".running_var"])
        f.num_batches_tracked = ptr(Bf[name + ".num_batches_tracked"])
        f.mean, f.invstd, f.scale, f.shift = ptr(st[0]), ptr(st[1]), ptr(st[2]), ptr(st[3])
        return f

    def _conv_bn(self, P, Bf, conv, bn, x, y, pro, training, part=None, ws=None, x8=None, x_out=None):
        """conv (+ BN statistics and finalize when training); ``x8``: the input's MX-fp8 copy
        (argus_conv_fwd_x8 instead of argus_conv_fwd); ``x_out``: where the prologue's applied input is
        stored (argus_conv_fwd_apply_out)."""
        cv = self.convs[conv]
        sc = sh = None
        if pro is not None:
            sc, sh = self.bn_state[pro][2], self.bn_state[pro][3]
        part = self.stat_part if part is None else part
        ws = self.bn_ws if ws is None else ws
        if y is None and not training:  # eval: the fused tail needs no statistics pass
            self._bn_eval(P, Bf, bn)
            return
        cdt = BF16 if y is None else self.cdt  # the statistics-only forward is the bf16 kernel
        if x_out is not None:
            self._launch(cv, 0, lambda: self.L.conv_fwd_apply_out(C.byref(cv.desc), cdt, ptr(x), ptr(cv.wf), ptr(y),
                                                                   ptr(sc), ptr(sh), ptr(part) if training else None,
                                                                   ptr(x_out), stream()))
        elif x8 is not None:
            self._launch(cv, 0, lambda: self.L.conv_fwd_x8(C.byref(cv.desc), ptr(x8), ptr(cv.wf), ptr(y),
                                                            ptr(part) if training else None, stream()))
        elif training and self.fold_fwd_fin:
            fin = self._fwd_fin(P, Bf, bn, ws)
            self._launch(cv, 0, lambda: self.L.conv_fwd_fin(C.byref(cv.desc), cdt, ptr(x), ptr(cv.wf), ptr(y),
                                                             ptr(sc), ptr(sh), ptr(part), C.byref(fin), stream()))
            return
        else:
            self._launch(cv, 0, lambda: self.L.conv_fwd(C.byref(cv.desc), cdt, ptr(x), ptr(cv.wf), ptr(y), ptr(sc),
                                                         ptr(sh), ptr(part) if training else None, stream()))
        if training:
            count = cv.desc.n * cv.desc.ho * cv.desc.wo
            if y is None and sc is None and x_out is None:  # the statistics-only forward's partial layout
                self._bn_train(P, Bf, bn, cv.so_rows, cv.so_tile, count, part, ws)
            else:
                self._bn_train(P, Bf, bn, cv.stat_rows, cv.stat_tile, count, part, ws)
        else:
            self._bn_eval(P, Bf, bn)

    def _fused_tail(self) -> bool:
        """The bottleneck tail runs as argus_conv_fwd(stats only) + argus_conv_fwd_bn_out: the bf16
        schedule (materialised a2), with conv3's forward not on MX-fp8 operands (policy key 37 bit 1)."""
        if not (self.fuse_out and self.materialize):
            return False
        if self.cdt == FP8:
            return not ((self.tuning or {}).get(37, self.L.dll.argus_conv_policy_default(37)) & 1)
        return True

    def _act(self, bn, y, out, px, ch, out8=None):
        """out = relu(y*scale + shift) with the finalized coefficients of BN layer ``bn`` (+ its MX-fp8
        copy in ``out8``)."""
        st = self.bn_state[bn]
        if out8 is not None:
            self.L.bn_apply_x8(px, ch, ptr(y), ptr(st[2]), ptr(st[3]), None, None, None, 1, ptr(out), None, ptr(out8),
                               stream())
            return
        self.L.bn_apply(self.dt, px, ch, ptr(y), ptr(st[2]), ptr(st[3]), None, None, None, 1, ptr(out), None, stream())

    def prepare_weights(self, P) -> None:
        """fp32 master weights -> compute-dtype GEMM copies (w_fwd, w_dgrad) of every conv, one launch
        (argus_conv_weight_prep_batch); the device table is rebuilt only when a weight moves."""
        ws = []
        for name in self.convs:
            w = P[name + ".weight"]
            if w.dtype != torch.float32 or w.device != self.device:
                raise TypeError(f"{name}.weight must be fp32 on {self.device}")
            ws.append(w)
        key = tuple((w.data_ptr(), w.stride(), cv.wf.data_ptr(), cv.wd.data_ptr() if cv.wd is not None else 0)
                    for w, cv in zip(ws, self.convs.values()))
        if getattr(self, "_wp_key", None) != key:
            cvs = list(self.convs.values())
            n = len(cvs)
            descs = (ConvDesc * n)(*[cv.desc for cv in cvs])
            masters = (C.c_void_p * n)(*[w.data_ptr() for w in ws])
            strides = (C.c_int64 * (4 * n))(*[x for w in ws for x in w.stride()])
            wfs = (C.c_void_p * n)(*[cv.wf.data_ptr() for cv in cvs])
            wds = (C.c_void_p * n)(*[cv.wd.data_ptr() if cv.wd is not None else None for cv in cvs])
            nbytes = self.L.dll.argus_conv_weight_prep_table_bytes(n)
            host = (C.c_uint8 * nbytes)()
            nblk = C.c_int(0)
            self.L.conv_weight_prep_table(n, descs, masters, strides, wfs, wds, host, nbytes, C.byref(nblk))
            self._wp_table = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(self.device)
            self._wp_n, self._wp_blocks, self._wp_key = n, nblk.value, key
        # fp8: the pre-quantized MX-fp8 copies of the convs whose passes take fp8 operands (cdt = FP8)
        self.L.conv_weight_prep_batch(self.cdt, self._wp_n, ptr(self._wp_table), self._wp_blocks, stream())

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, P: dict, Bf: dict, training: bool) -> torch.Tensor:
        B, Cn, H, W = x.shape
        if Cn != 3 * self.n_cams:
            raise ValueError(f"expected {3 * self.n_cams} input channels, got {Cn}")
        self.ensure(B, H, W)
        x = x.contiguous()
        L, dt, s = self.L, self.dt, stream()
        N = self.N
        self.prepare_weights(P)
        if x.dtype == torch.uint8:  # CameraCubePoseDataset(uint8=True): /255 happens in the layout kernel
            L.images_u8_to_nhwc4(dt, N, H, W, ptr(x), ptr(self.x0), s)
        else:
            if x.dtype != torch.float32:
                x = x.float()
            L.images_to_nhwc4(dt, N, H, W, ptr(x), ptr(self.x0), s)
        # stem
        self._conv_bn(P, Bf, "resnet.conv1", "resnet.bn1", self.x0, self.y0, None, training)
        st = self.bn_state["resnet.bn1"]
        H1, W1 = self.stem_hw
        L.maxpool_fwd(dt, N, H1, W1, 64, ptr(self.y0), ptr(st[2]), ptr(st[3]), ptr(self.p0), ptr(self.amax), s)
        h = self.p0
        for bi, (b, a) in enumerate(zip(self.blocks, self.act)):
            pf = b.prefix
            ds_done = None
            if b.has_ds and self.wgrad_overlap:
                # downsample conv + its BN statistics on the side stream, beside conv1..conv3 (joined
                # before the block's bn_apply); own partial / ticket workspaces
                ds_done = self._on_side(lambda: self._conv_bn(P, Bf, pf + ".downsample.0", pf + ".downsample.1", h,
                                                              a["yd"], None, training, self.stat_part_ds,
                                                              self.bn_ws_ds))
            self._conv_bn(P, Bf, pf + ".conv1", pf + ".bn1", h, a["y1"], None, training)
            tail = self._fused_tail()
            if self.materialize:
                x8f = self.x8_conv[pf + ".conv2"][0]
                self._act(pf + ".bn1", a["y1"], a["a1"], N * a["hw_in"][0] * a["hw_in"][1], b.width,
                          self.x8buf if x8f else None)
                self._conv_bn(P, Bf, pf + ".conv2", pf + ".bn2", a["a1"], a["y2"], None, training,
                              x8=self.x8buf if x8f else None)
                if tail and training and self.a2_in_stats:
                    self._conv_bn(P, Bf, pf + ".conv3", pf + ".bn3", a["y2"], None, pf + ".bn2", training,
                                  x_out=a["a2"])
                else:
                    self._act(pf + ".bn2", a["y2"], a["a2"], N * a["hw"][0] * a["hw"][1], b.width)
                    self._conv_bn(P, Bf, pf + ".conv3", pf + ".bn3", a["a2"], None if tail else a["y3"], None,
                                  training)
            else:
                self._conv_bn(P, Bf, pf + ".conv2", pf + ".bn2", a["y1"], a["y2"], pf + ".bn1", training)
                self._conv_bn(P, Bf, pf + ".conv3", pf + ".bn3", a["y2"], a["y3"], pf + ".bn2", training)
            s3 = self.bn_state[pf + ".bn3"]
            px = N * a["hw"][0] * a["hw"][1]
            if b.has_ds:
                if ds_done is None:
                    self._conv_bn(P, Bf, pf + ".downsample.0", pf + ".downsample.1", h, a["yd"], None, training)
                else:
                    ds_done.wait(torch.cuda.current_stream())
                sd = self.bn_state[pf + ".downsample.1"]
                res, rsc, rsh = a["yd"], sd[2], sd[3]
            else:
                res, rsc, rsh = h, None, None
            if tail:  # conv3's C tile recomputed: out, its mask (and y3 where the backward reads it) in one pass
                cv3 = self.convs[pf + ".conv3"]
                y3 = a["y3"] if training and not self._y3_free(bi) else None
                self._launch(cv3, 0, lambda: L.conv_fwd_bn_out(
                    C.byref(cv3.desc), BF16, ptr(a["a2"]), ptr(cv3.wf), ptr(s3[2]), ptr(s3[3]), ptr(res), ptr(rsc),
                    ptr(rsh), ptr(a["out"]), ptr(a["bits"]), ptr(y3), s))
            else:
                L.bn_apply(dt, px, b.cout, ptr(a["y3"]), ptr(s3[2]), ptr(s3[3]), ptr(res), ptr(rsc), ptr(rsh), 1,
                           ptr(a["out"]), ptr(a["bits"]), s)
            h = a["out"]
            if self.debug is not None:
                self.debug["fwd." + pf] = a["out"].clone()
        hf, wf = self.final_hw
        L.avgpool_fwd(dt, N, hf * wf, 2048, ptr(h), ptr(self.feat), s)
        # head (fp32)
        fcw, fcb = P["resnet.fc.weight"], P["resnet.fc.bias"]
        L.gemm_f32(N, self.rdim, 2048, ptr(self.feat), 2048, 0, ptr(fcw), 2048, 1, ptr(self.h0), self.rdim,
                   ptr(fcb), 1, None, ptr(self.gemm_ws), self.gemm_ws.numel(), s)
        D = self.n_cams * self.rdim
        L.gelu_f32(B * D, ptr(self.h0), ptr(self.g0), s)
        w0, b0 = P["output_mlp.0.weight"], P["output_mlp.0.bias"]
        w2, b2 = P["output_mlp.2.weight"], P["output_mlp.2.bias"]
        w4, b4 = P["output_mlp.4.weight"], P["output_mlp.4.bias"]
        L.gemm_f32(B, 128, D, ptr(self.g0), D, 0, ptr(w0), D, 1, ptr(self.g1), 128, ptr(b0), 2, ptr(self.h1), ptr(self.gemm_ws), self.gemm_ws.numel(), s)
        L.gemm_f32(B, 128, 128, ptr(self.g1), 128, 0, ptr(w2), 128, 1, ptr(self.g2), 128, ptr(b2), 2, ptr(self.h2), ptr(self.gemm_ws), self.gemm_ws.numel(), s)
        L.gemm_f32(B, 6, 128, ptr(self.g2), 128, 0, ptr(w4), 128, 1, ptr(self.pred), 6, ptr(b4), 1, None, ptr(self.gemm_ws), self.gemm_ws.numel(), s)
        self.saved = training
        return self.pred

    # ------------------------------------------------------------------ backward
    def backward(self, dpred: torch.Tensor, P: dict, G: dict, on_ready=None) -> None:
        """Write every parameter gradient into G[name] (fp32; conv weights OHWI-contiguous).

        ``on_ready(name, comm)`` (optional) is called, in stream order, as soon as the gradients of
        parameter ``name`` and of every parameter registered after it have been issued: after the head
        ("resnet.fc.weight"), after each block ("<block>.conv1.weight"), after the stem
        ("resnet.conv1.weight"). Weight gradients may still be running on the side stream then:
        ``with comm():`` is the context to issue a collective over those gradients in - the stream it
        makes current is ordered after both streams' work so far, and the main stream is not made to
        wait (the trainer issues each bucket's all-reduce in it, so the backward keeps its overlap)."""
        if not self.saved:
            raise RuntimeError("backward without a saved train-mode forward")
        L, dt, s = self.L, self.dt, stream()
        B = self.shape[0]
        N = self.N
        D = self.n_cams * self.rdim
        dpred = dpred.contiguous().float()
        w0, w2, w4 = P["output_mlp.0.weight"], P["output_mlp.2.weight"], P["output_mlp.4.weight"]
        # MLP + fc data path (main stream): dh2 -> dh1 -> dh0 -> dfeat
        ws, wsn = ptr(self.gemm_ws), self.gemm_ws.numel()
        L.gemm_f32(B, 128, 6, ptr(dpred), 6, 0, ptr(w4), 128, 0, ptr(self.dh2), 128, None, 3, ptr(self.h2), ws, wsn, s)
        L.gemm_f32(B, 128, 128, ptr(self.dh2), 128, 0, ptr(w2), 128, 0, ptr(self.dh1), 128, None, 3, ptr(self.h1), ws, wsn, s)
        L.gemm_f32(B, D, 128, ptr(self.dh1), 128, 0, ptr(w0), D, 0, ptr(self.dh0), D, None, 3, ptr(self.h0), ws, wsn, s)
        fcw = P["resnet.fc.weight"]
        R = self.rdim

        def head_wgrads():  # weight / bias gradients of the head: nothing downstream reads them
            ss, w2s, w2n = stream(), ptr(self.gemm_ws_side), self.gemm_ws_side.numel()
            L.gemm_f32(6, 128, B, ptr(dpred), 6, 1, ptr(self.g2), 128, 0, ptr(G["output_mlp.4.weight"]), 128, None, 0,
                       None, w2s, w2n, ss)
            L.colsum_f32(B, 6, ptr(dpred), 6, ptr(G["output_mlp.4.bias"]), ss)
            L.gemm_f32(128, 128, B, ptr(self.dh2), 128, 1, ptr(self.g1), 128, 0, ptr(G["output_mlp.2.weight"]), 128, None,
                       0, None, w2s, w2n, ss)
            L.colsum_f32(B, 128, ptr(self.dh2), 128, ptr(G["output_mlp.2.bias"]), ss)
            L.gemm_f32(128, D, B, ptr(self.dh1), 128, 1, ptr(self.g0), D, 0, ptr(G["output_mlp.0.weight"]), D, None, 0,
                       None, w2s, w2n, ss)
            L.colsum_f32(B, 128, ptr(self.dh1), 128, ptr(G["output_mlp.0.bias"]), ss)
            L.gemm_f32(R, 2048, N, ptr(self.dh0), R, 1, ptr(self.feat), 2048, 0, ptr(G["resnet.fc.weight"]), 2048, None, 0,
                       None, w2s, w2n, ss)
            L.colsum_f32(N, R, ptr(self.dh0), R, ptr(G["resnet.fc.bias"]), ss)

        if self.wgrad_overlap:  # beside the fc data gradient and the last blocks' backward
            self._last_side = self._on_side(head_wgrads)
        else:
            head_wgrads()
        L.gemm_f32(N, 2048, R, ptr(self.dh0), R, 0, ptr(fcw), 2048, 0, ptr(self.dfeat), 2048, None, 0, None, ws, wsn, s)
        hf, wf = self.final_hw
        g = self.gbuf
        dh = g[0]
        L.avgpool_bwd(dt, N, hf * wf, 2048, ptr(self.dfeat), ptr(dh), s)
        if on_ready is not None:
            on_ready("resnet.fc.weight", self._comm)

        # BN backward: the reduction over dz = d(BN output) runs in the epilogue of the dgrad that
        # produces dz (argus_conv_dgrad_bn), which stores the ReLU-masked dm and the partial column
        # sums; only finalize + apply (dy = ca*dm + cb*y + cc) remain as passes. Invariant at the top
        # of each block: dh holds dm3 = relu'(out) * dout (bn3's masked input gradient) and bwd_part
        # (bwd_part2: the downsample BN) its partials, rows3 rows - except for the last block, whose
        # dout comes from the average pool unmasked.
        nb = len(self.blocks)
        rows3 = None
        for idx in range(nb - 1, -1, -1):
            b, a = self.blocks[idx], self.act[idx]
            pf = b.prefix
            h_in = self.act[idx - 1]["out"] if idx > 0 else self.p0
            hi, wi = a["hw_in"]
            ho, wo = a["hw"]
            px_o = N * ho * wo
            px_i = N * hi * wi
            dyd = self._next_dy() if b.has_ds else None
            dbg = self.debug
            ds_dgw = (b.has_ds and idx == 0 and self.fuse_apply and rows3 is not None
                      and pf + ".downsample.0" in self.dgw)
            # weight gradients that stage the BN-backward apply from dm themselves (dy never stored;
            # the debug capture keeps storing it for the stage checks)
            wg3_apply = (rows3 is not None and self.fuse_apply and self.wgrad_apply and a["a2"] is not None
                         and self.stages_pro[pf + ".conv3"])
            wg1_apply = idx > 0 and self.fuse_apply and self.wgrad_apply and self.stages_pro[pf + ".conv1"]
            dy3 = None if wg3_apply and dbg is None else self._next_dy()

            def cap(key, t, n, shape):
                if dbg is not None:
                    dbg[key + "." + pf] = t[:n].view(*shape).clone()

            cap("b_dout", dh, px_o * b.cout, (N, ho, wo, b.cout))
            fuse = self.fuse_apply
            dza, dzb = g[1], g[2]
            # bn3 (+ downsample BN) backward
            if rows3 is None:  # last block: mask + reduce pass over the pooled gradient
                L.bn_bwd_reduce(dt, px_o, b.cout, ptr(dh), 3, ptr(a["bits"]), ptr(a["y3"]), None, None,
                                ptr(self.bn_state[pf + ".bn3"][0]), ptr(self.bn_state[pf + ".bn3"][1]),
                                ptr(self.bwd_part), None, None, None, None, s)
                rows3 = L.dll.argus_bn_bwd_rows(px_o, b.cout)
                self._bn_bwd_fin(P, G, pf + ".bn3", px_o, b.cout, self.bwd_part, rows3)
                cf, st3 = self.bn_coef[pf + ".bn3"], self.bn_state[pf + ".bn3"]
                self._guard(dy3)
                L.bn_bwd_apply(dt, px_o, b.cout, ptr(dh), 3, ptr(a["bits"]), ptr(a["y3"]), None, None, ptr(cf[0]),
                               ptr(cf[1]), ptr(cf[2]), ptr(dy3), ptr(dh), None, None, None, None, None, s)
                pro3 = None  # dy3 materialised above
            else:
                if rows3:  # not folded into the producing dgrad
                    self._bn_bwd_fin(P, G, pf + ".bn3", px_o, b.cout, self.bwd_part, rows3)
                    if b.has_ds:
                        self._bn_bwd_fin(P, G, pf + ".downsample.1", px_o, b.cout, self.bwd_part2, rows3)
                if fuse:  # dy3 (and dyd) are staged by the conv3 (downsample) dgrad from dm3 = dh
                    pro3 = (pf + ".bn3", a["y3"], dy3)
                    # block 0's downsample dgrad is a plain dgrad: materialise dyd, unless its data and
                    # weight gradient run fused (staging dyd from dh; dyd then kept for the debug capture only)
                    if b.has_ds and idx == 0 and (not ds_dgw or dbg is not None):
                        self._bn_apply_bwd(pf + ".downsample.1", px_o, b.cout, dh, a["yd"], dyd)
                else:
                    pro3 = None
                    self._bn_apply_bwd(pf + ".bn3", px_o, b.cout, dh, a["y3"], dy3,
                                       (pf + ".downsample.1", a["yd"], dyd) if b.has_ds else None)
            # conv3 -> bn2
            dgw = wg3_apply and self.fold_fin and pf + ".conv3" in self.dgw
            if dgw:  # data + weight gradient in one pass (dW on the main stream; y3 recomputed when not stored)
                r2 = self._dgrad_wgrad_bn(pf + ".conv3", dh, dza, pf + ".bn2", a["y2"], pf + ".bn3",
                                          None if self._y3_free(idx) else a["y3"], a["a2"], P, G)
                if dy3 is not None:  # debug capture only: the fused kernel never stores dy3
                    self._bn_apply_bwd(pf + ".bn3", px_o, b.cout, dh, a["y3"], dy3)
            else:
                r2 = self._dgrad_bn(pf + ".conv3", dh if pro3 else dy3, dza, None, pf + ".bn2", a["y2"], 2, P=P, G=G,
                                    pro=pro3)
            if dy3 is not None:
                cap("b_dy3", dy3, px_o * b.cout, (N, ho, wo, b.cout))
            cap("b_dz2", dza, px_o * b.width, (N, ho, wo, b.width))
            s2 = self.bn_state[pf + ".bn2"]
            if dgw:
                pass
            elif wg3_apply:  # dh holds dm3 (read by the side stream until its event: dh is not reused)
                self._wgrad_apply(pf + ".conv3", a["a2"], dh, pf + ".bn3", a["y3"], G)
            elif a["a2"] is not None:
                self._wgrad(pf + ".conv3", a["a2"], None, dy3, G)
            else:
                self._wgrad(pf + ".conv3", a["y2"], s2, dy3, G)
            if r2:
                self._bn_bwd_fin(P, G, pf + ".bn2", px_o, b.width, self.bwd_part, r2)
            dy2 = self._next_dy()
            x8d = self.x8_conv[pf + ".conv2"][1]
            if fuse and not x8d:
                pro2 = (pf + ".bn2", a["y2"], dy2)
            else:
                pro2 = None
                self._bn_apply_bwd(pf + ".bn2", px_o, b.width, dza, a["y2"], dy2, dy8=self.x8buf if x8d else None)
            # conv2 -> bn1 (dm1 goes to a ring buffer when the side stream's conv1 wgrad reads it)
            if wg1_apply:
                dzb = self._next_dy()
            if self.gate3x3 or b.width <= self.gate3x3_width:
                self._drain_side()
            r1 = self._dgrad_bn(pf + ".conv2", dza if pro2 else dy2, dzb, None, pf + ".bn1", a["y1"], 2, P=P, G=G,
                                pro=pro2, x8=self.x8buf if x8d else None)
            cap("b_dy2", dy2, px_o * b.width, (N, ho, wo, b.width))
            cap("b_dz1", dzb, px_i * b.width, (N, hi, wi, b.width))
            s1 = self.bn_state[pf + ".bn1"]
            if self.materialize:
                self._wgrad(pf + ".conv2", a["a1"], None, dy2, G)
            else:
                self._wgrad(pf + ".conv2", a["y1"], s1, dy2, G)
            if r1:
                self._bn_bwd_fin(P, G, pf + ".bn1", px_i, b.width, self.bwd_part, r1)
            dy1 = None if wg1_apply and dbg is None else self._next_dy()
            pro1 = None
            if fuse and idx > 0:
                # where the weight gradient stages the same apply (wg1_apply), the dgrad stores no dy1: the
                # debug capture materialises it with the apply pass below instead, so the stage checks run
                # the benched kernels (the persistent conv1 dgrad takes no dy_out)
                pro1 = (pf + ".bn1", a["y1"], None if wg1_apply else dy1)
            else:
                self._bn_apply_bwd(pf + ".bn1", px_i, b.width, dzb, a["y1"], dy1)
            # the block-input gradient goes to a fresh ring buffer (dm3 / dm1 may still be read by the
            # side stream; a buffer held across blocks must never be handed out again while live)
            dx = self._next_dy()
            # conv1 (+ downsample) -> the previous block's bn3 (+ its downsample BN): dm3 of block idx-1
            c1_in = dzb if pro1 else dy1
            if idx > 0:
                pb, pa = self.blocks[idx - 1], self.act[idx - 1]
                second = (pb.prefix + ".downsample.1", pa["yd"]) if pb.has_ds else None
                yrec = self._yrec(pb, pa)
                y3p = None if yrec else pa["y3"]
                if b.has_ds:
                    self._dgrad_plain_or_pro(pf + ".conv1", c1_in, dx, pro1)
                    rows3 = self._dgrad_bn(pf + ".downsample.0", dh if fuse else dyd, dx, dx, pb.prefix + ".bn3",
                                           y3p, 3, pa["bits"], second, P=P, G=G,
                                           pro=(pf + ".downsample.1", a["yd"], dyd) if fuse else None, yrec=yrec)
                else:
                    rows3 = self._dgrad_bn(pf + ".conv1", c1_in, dx, dh, pb.prefix + ".bn3", y3p, 3, pa["bits"],
                                           second, P=P, G=G, pro=pro1, yrec=yrec)
            else:
                self._dgrad(pf + ".conv1", dy1, dx)
                if ds_dgw:  # dx += the downsample dgrad, its dW from the same staged dyd tile
                    self._dgrad_wgrad_bn(pf + ".downsample.0", dh, dx, None, None, pf + ".downsample.1", a["yd"],
                                         h_in, P, G, addend=dx)
                elif b.has_ds:
                    self._dgrad(pf + ".downsample.0", dyd, dx, addend=dx)
            if dy1 is not None:
                if pro1 is not None and pro1[2] is None:  # debug capture only (see pro1)
                    self._bn_apply_bwd(pf + ".bn1", px_i, b.width, dzb, a["y1"], dy1)
                cap("b_dy1", dy1, px_i * b.width, (N, hi, wi, b.width))
            if b.has_ds:
                cap("b_dyd", dyd, px_o * b.cout, (N, ho, wo, b.cout))
            if wg1_apply:
                self._wgrad_apply(pf + ".conv1", h_in, dzb, pf + ".bn1", a["y1"], G)
            else:
                self._wgrad(pf + ".conv1", h_in, None, dy1, G)
            if b.has_ds and not ds_dgw:
                # (single process only: with on_ready a bucket holding this gradient could be reduced first)
                if (idx == 0 and on_ready is None and self.tail_main and self.wgrad_overlap and self._stem_overlap
                        and self.fuse_apply):
                    cvd = self.convs[pf + ".downsample.0"]
                    self._tail.append((cvd, lambda cvd=cvd, x=h_in, dy=dyd: self.L.conv_wgrad(
                        C.byref(cvd.desc), self.dt, ptr(x), None, None, ptr(dy), ptr(G[pf + ".downsample.0.weight"]),
                        ptr(self.wg_ws_stem), self.wg_ws_stem.numel(), stream())))
                else:
                    self._wgrad(pf + ".downsample.0", h_in, None, dyd, G)
            dh = dx
            self._flush_side()
            if on_ready is not None:
                on_ready(pf + ".conv1.weight", self._comm)
            if self.debug is not None:
                n_in = N * hi * wi * b.cin
                self.debug["bwd." + pf] = dh[:n_in].view(N, hi, wi, b.cin).clone()
        # stem: maxpool -> relu/bn1 -> conv1 wgrad
        H1, W1 = self.stem_hw
        dz0, dy0 = g[1], self._next_dy()
        if self.fuse_apply:
            # maxpool backward + the stem BN's backward reduction in one pass (stores dm0), finalize, then
            # the stem weight gradient stages dy0 = ca*dm0 + cb*y0 + cc itself (dy0 is never written)
            st, cf = self.bn_state["resnet.bn1"], self.bn_coef["resnet.bn1"]
            if self.fold_fin and self.fold_stem_fin:  # the finalize folded into the pass's last workgroups
                L.maxpool_bwd_bn_fin(dt, N, H1, W1, 64, ptr(dh), ptr(self.amax), ptr(dz0), ptr(self.y0),
                                     ptr(st[2]), ptr(st[3]), ptr(st[0]), ptr(st[1]), ptr(self.bwd_part),
                                     ptr(P["resnet.bn1.weight"]), ptr(G["resnet.bn1.weight"]),
                                     ptr(G["resnet.bn1.bias"]), ptr(cf[0]), ptr(cf[1]), ptr(cf[2]), ptr(self.bn_ws), s)
            else:
                L.maxpool_bwd_bn(dt, N, H1, W1, 64, ptr(dh), ptr(self.amax), ptr(dz0), ptr(self.y0), ptr(st[2]),
                                 ptr(st[3]), ptr(st[0]), ptr(st[1]), ptr(self.bwd_part), s)
                self._bn_bwd_fin(P, G, "resnet.bn1", N * H1 * W1, 64, self.bwd_part,
                                 L.dll.argus_maxpool_bwd_bn_rows(dt, N, H1, W1, 64))
            cv = self.convs["resnet.conv1"]
            ap = BnBwdPrologue(ptr(self.y0), ptr(cf[0]), ptr(cf[1]), ptr(cf[2]), None)
            fn = lambda: L.conv_wgrad_apply(C.byref(cv.desc), dt, ptr(self.x0), ptr(dz0), C.byref(ap),  # noqa: E731
                                            ptr(G["resnet.conv1.weight"]), ptr(self.wg_ws_stem),
                                            self.wg_ws_stem.numel(), stream())
            # on the main stream: it is the last work of the backward
            if not self._stem_overlap:
                self._join()
            self._launch(cv, 2, fn)
            for cvt, fnt in self._tail:  # after the stem's: they share its workspace (stream order)
                self._launch(cvt, 2, fnt)
            self._tail.clear()
        else:
            L.maxpool_bwd(dt, N, H1, W1, 64, ptr(dh), ptr(self.amax), ptr(dz0), s)
            self._bn_bwd(P, G, "resnet.bn1", N * H1 * W1, 64, dz0, 2, None, self.y0, dy0, None)
            self._wgrad("resnet.conv1", self.x0, None, dy0, G)
        self._join()
        if on_ready is not None:
            on_ready("resnet.conv1.weight", self._comm)

    def _y3_free(self, idx: int) -> bool:
        """Block ``idx``'s bn3 input y3 is never stored: its forward tail is fused, the next block's
        BN-backward epilogue recomputes it, and its conv3 backward is the fused data + weight gradient,
        which recomputes it as well (train mode; the last block's bn3 backward reads y3)."""
        b = self.blocks[idx]
        c3 = b.prefix + ".conv3"
        return (self.y3_free and self._fused_tail() and self.debug is None and idx < len(self.blocks) - 1
                and self.fuse_apply and self.wgrad_apply and self.fold_fin and c3 in self.dgw
                and self.stages_pro[c3] and self._yrec(b, self.act[idx]) is not None)

    def _yrec(self, blk, act):
        """(a2, conv3's bf16 w_fwd, width) when block ``blk``'s y3 is recomputed rather than read by the
        BN-backward epilogue that reduces its bn3 (bf16 schedule; not where the 1x1 data gradients take
        MX-fp8 weights, policy key 37 bit 4), else None."""
        if not (self.yrec_epi and self.materialize and act["a2"] is not None):
            return None
        if self.cdt == FP8 and (self.tuning or {}).get(37, self.L.dll.argus_conv_policy_default(37)) & 4:
            return None
        return act["a2"], self.convs[blk.prefix + ".conv3"].wf, blk.width

    def _dgrad_bn(self, conv, dy, dm, addend, bn, y, mode, bits=None, second=None, P=None, G=None, pro=None,
                  yrec=None, x8=None):
        """dgrad of ``conv`` whose output feeds BN ``bn`` (input ``y``) backward: stores the masked dm
        and writes bwd_part (+ bwd_part2 for ``second`` = (bn name, y) of a downsample BN); returns the
        partial row count. With ``fold_fin`` the BN-backward finalize (dgamma, dbeta, ca/cb/cc) runs in
        the same launch and 0 is returned (nothing left to finalize)."""
        cv = self.convs[conv]
        st = self.bn_state[bn]
        e = BnBwdEpilogue()
        if self.fold_fin:
            cf = self.bn_coef[bn]
            e.workspace, e.gamma, e.dgamma, e.dbeta = ptr(self.bn_ws), ptr(P[bn + ".weight"]), ptr(G[bn + ".weight"]), \
                ptr(G[bn + ".bias"])
            e.ca, e.cb, e.cc = ptr(cf[0]), ptr(cf[1]), ptr(cf[2])
            if second is not None:
                cf2 = self.bn_coef[second[0]]
                e.gamma2, e.dgamma2, e.dbeta2 = ptr(P[second[0] + ".weight"]), ptr(G[second[0] + ".weight"]), \
                    ptr(G[second[0] + ".bias"])
                e.ca2, e.cb2, e.cc2 = ptr(cf2[0]), ptr(cf2[1]), ptr(cf2[2])
        e.y, e.mean, e.invstd, e.mask_mode = ptr(y), ptr(st[0]), ptr(st[1]), mode
        if yrec is not None:  # y recomputed in the epilogue: conv1x1(a2, w_fwd of conv3)
            e.y_x, e.y_w, e.y_k = ptr(yrec[0]), ptr(yrec[1]), yrec[2]
        if mode == 2:
            e.scale, e.shift = ptr(st[2]), ptr(st[3])
        else:
            e.mask_bits = ptr(bits)
        e.part = ptr(self.bwd_part)
        if second is not None:
            st2 = self.bn_state[second[0]]
            e.y2, e.mean2, e.invstd2, e.part2 = ptr(second[1]), ptr(st2[0]), ptr(st2[1]), ptr(self.bwd_part2)
        pp = self._prologue(pro)
        self._guard(dm)
        if x8 is not None:  # dy read as its MX-fp8 copy (argus_conv_dgrad_bn_x8; no addend / prologue)
            self._launch(cv, 1, lambda: self.L.conv_dgrad_bn_x8(C.byref(cv.desc), ptr(x8), ptr(cv.wd), ptr(dm),
                                                                 C.byref(e), stream()))
        else:
            self._launch(cv, 1, lambda: self.L.conv_dgrad_bn(C.byref(cv.desc), self.cdt, ptr(dy), ptr(cv.wd),
                                                              ptr(dm), ptr(addend), C.byref(e), pp, stream()))
        return 0 if self.fold_fin else self.L.dll.argus_conv_dgrad_bn_rows(C.byref(cv.desc), self.cdt)

    def _dgrad_wgrad_bn(self, conv, dm, dx, bn, y, pbn, py, x, P, G, addend=None):
        """Fused data + weight gradient of ``conv`` (argus_conv_dgrad_wgrad_bn): dy = the apply of BN
        ``pbn`` (input ``py``) staged from ``dm``, dx = the masked input gradient of BN ``bn`` (input ``y``,
        mask mode 2, finalize folded) or, with ``bn`` None, the plain dx (+ ``addend``); dW from ``x``;
        returns 0 (nothing left to finalize)."""
        cv = self.convs[conv]
        pc = self.bn_coef[pbn]
        e = None
        if bn is not None:
            st, cf = self.bn_state[bn], self.bn_coef[bn]
            e = BnBwdEpilogue()
            e.workspace, e.gamma, e.dgamma, e.dbeta = ptr(self.bn_ws), ptr(P[bn + ".weight"]), \
                ptr(G[bn + ".weight"]), ptr(G[bn + ".bias"])
            e.ca, e.cb, e.cc = ptr(cf[0]), ptr(cf[1]), ptr(cf[2])
            e.y, e.mean, e.invstd, e.mask_mode, e.scale, e.shift = ptr(y), ptr(st[0]), ptr(st[1]), 2, ptr(st[2]), \
                ptr(st[3])
            e.part = ptr(self.bwd_part)
        pro = BnBwdPrologue(ptr(py), ptr(pc[0]), ptr(pc[1]), ptr(pc[2]), None)
        self._guard(dx)
        self._launch(cv, 1, lambda: self.L.conv_dgrad_wgrad_bn(
            C.byref(cv.desc), self.dgw_dt, ptr(dm), ptr(cv.wd), ptr(x), ptr(dx), ptr(addend),
            C.byref(e) if e is not None else None, C.byref(pro), ptr(G[conv + ".weight"]), ptr(self.dgw_ws),
            self.dgw_ws.numel(), stream()))
        return 0

    def _prologue(self, pro):
        """argus_bn_bwd_prologue for ``pro`` = (bn name, y, dy_out): the dgrad stages dy = ca*dm + cb*y + cc
        from its dm operand and stores dy to dy_out (for the weight gradient)."""
        if pro is None:
            return None
        cf = self.bn_coef[pro[0]]
        self._guard(pro[2])
        return C.byref(BnBwdPrologue(ptr(pro[1]), ptr(cf[0]), ptr(cf[1]), ptr(cf[2]), ptr(pro[2]) if pro[2] is not None
                                     else None))

    def _dgrad_plain_or_pro(self, conv, dy, dx, pro):
        """dgrad without a BN epilogue (the conv1 dgrad of a downsample block, accumulated into by the
        downsample dgrad) - with the apply prologue when ``pro`` is given."""
        if pro is None:
            self._dgrad(conv, dy, dx)
            return
        cv = self.convs[conv]
        pp = self._prologue(pro)
        self._guard(dx)
        self._launch(cv, 1, lambda: self.L.conv_dgrad_bn(C.byref(cv.desc), self.cdt, ptr(dy), ptr(cv.wd), ptr(dx),
                                                          None, None, pp, stream()))

    def _bn_apply_bwd(self, name, px, ch, dm, y, dy_out, second=None, dy8=None):
        """dy = ca*dm + cb*y + cc from an already-masked dm (+ the downsample BN's dy2 from the same dm, or
        dy's MX-fp8 copy in ``dy8``)."""
        cf = self.bn_coef[name]
        self._guard(dy_out)
        if dy8 is not None:
            self.L.bn_bwd_apply_x8(px, ch, ptr(dm), ptr(y), ptr(cf[0]), ptr(cf[1]), ptr(cf[2]), ptr(dy_out), ptr(dy8),
                                   stream())
            return
        y2 = ca2 = cb2 = cc2 = dy2 = None
        if second is not None:
            cf2 = self.bn_coef[second[0]]
            y2, dy2 = second[1], second[2]
            ca2, cb2, cc2 = cf2[0], cf2[1], cf2[2]
            self._guard(dy2)
        self.L.bn_bwd_apply(self.dt, px, ch, ptr(dm), 0, None, ptr(y), None, None, ptr(cf[0]), ptr(cf[1]), ptr(cf[2]),
                            ptr(dy_out), None, ptr(y2), ptr(ca2), ptr(cb2), ptr(cc2), ptr(dy2), stream())

    def _bn_bwd(self, P, G, name, px, ch, dz, mode, mask_src, y, dy_out, dm_out):
        L, dt, s = self.L, self.dt, stream()
        st, cf = self.bn_state[name], self.bn_coef[name]
        L.bn_bwd_reduce(dt, px, ch, ptr(dz), mode, ptr(mask_src), ptr(y), ptr(st[2]), ptr(st[3]), ptr(st[0]),
                        ptr(st[1]), ptr(self.bwd_part), None, None, None, None, s)
        self._bn_bwd_fin(P, G, name, px, ch, self.bwd_part, L.dll.argus_bn_bwd_rows(px, ch))
        self._guard(dy_out)
        L.bn_bwd_apply(dt, px, ch, ptr(dz), mode, ptr(mask_src), ptr(y), ptr(st[2]), ptr(st[3]), ptr(cf[0]),
                       ptr(cf[1]), ptr(cf[2]), ptr(dy_out), ptr(dm_out), None, None, None, None, None, s)

    def _bn_bwd_fin(self, P, G, name, px, ch, part, rows):
        st, cf = self.bn_state[name], self.bn_coef[name]
        self.L.bn_bwd_finalize(ch, rows, ptr(part), px, ptr(P[name + ".weight"]), ptr(st[0]), ptr(st[1]),
                               ptr(G[name + ".weight"]), ptr(G[name + ".bias"]), ptr(cf[0]), ptr(cf[1]), ptr(cf[2]),
                               ptr(self.bn_ws), stream())

    def _wgrad(self, conv, x, pro_state, dy, G):
        cv = self.convs[conv]
        sc = sh = None
        if pro_state is not None:
            sc, sh = pro_state[2], pro_state[3]
        fn = lambda: self.L.conv_wgrad(C.byref(cv.desc), self.dt, ptr(x), ptr(sc), ptr(sh), ptr(dy),  # noqa: E731
                                       ptr(G[conv + ".weight"]), ptr(self.wg_ws), self.wg_ws_bytes, stream())
        if not self.wgrad_overlap:
            self._launch(cv, 2, fn)
            return
        # after dy (and x) are complete on the main stream; all wgrads share the one side stream, so
        # wg_ws is never shared
        self._side_issue(cv, fn, dy)

    def _wgrad_apply(self, conv, x, dm, bn, y, G):
        """Weight gradient of ``conv`` whose dy = ca*dm + cb*y + cc (BN ``bn``'s backward apply) is staged
        by the wgrad kernel from dm (argus_conv_wgrad_apply); same placement as _wgrad."""
        cv = self.convs[conv]
        cf = self.bn_coef[bn]
        ap = BnBwdPrologue(ptr(y), ptr(cf[0]), ptr(cf[1]), ptr(cf[2]), None)
        fn = lambda: self.L.conv_wgrad_apply(C.byref(cv.desc), self.dt, ptr(x), ptr(dm), C.byref(ap),  # noqa: E731
                                             ptr(G[conv + ".weight"]), ptr(self.wg_ws), self.wg_ws_bytes, stream())
        if not self.wgrad_overlap:
            self._launch(cv, 2, fn)
            return
        self._side_issue(cv, fn, dm)

    def _side_issue(self, cv, fn, buf):
        """Weight gradient ``fn`` (reading ``buf``) on the side stream: now, or deferred to the block's
        _flush_side (side_batch)."""
        self._deferred.append((cv, fn, buf.data_ptr()))
        if not self.side_batch:
            self._flush_side()

    def _flush_side(self) -> None:
        """Issue the deferred weight gradients on the side stream after the main stream's work so far
        (one event record on the main stream); their buffers become pending on the completion event."""
        if not self._deferred:
            return
        items, self._deferred = self._deferred, []

        def run():
            for cv, fn, _ in (items[::-1] if self.side_reverse else items):
                self._launch(cv, 2, fn)

        done = self._on_side(run)
        self._side_seq += 1
        for _, _, bp in items:
            self._pending[bp] = (self._side_seq, done)
        self._last_side = done

    def _event(self):
        """A cross-stream event (record(stream) / wait(stream)): device-scope (light_events) or torch's."""
        ev = DeviceEvent() if self.light_events else torch.cuda.Event()
        self._ev_keep.append(ev)
        return ev

    def _on_side(self, fn):
        """Run ``fn``'s launches on the side stream after the main stream's work so far; returns the
        side-stream event that marks their completion."""
        main = torch.cuda.current_stream()
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device, priority=self.side_priority)
        ready = self._event()
        ready.record(main)
        ready.wait(self._side)
        with torch.cuda.stream(self._side):
            fn()
        done = self._event()
        done.record(self._side)
        return done

    def _next_dy(self) -> torch.Tensor:
        buf = self.dyring[self._ring_i % len(self.dyring)]
        self._ring_i += 1
        return buf

    def _guard(self, buf) -> None:
        """Before the main stream overwrites ``buf``: wait for the side-stream wgrad still reading it."""
        if buf is None:
            return
        bp = buf.data_ptr()
        if any(d[2] == bp for d in self._deferred):  # its reader is not issued yet: issue it first
            self._flush_side()
        ev = self._pending.pop(bp, None)
        if ev is not None and ev[0] > self._waited_seq:
            ev[1].wait(torch.cuda.current_stream())
            self._waited_seq = ev[0]

    @contextlib.contextmanager
    def _comm(self):
        """Stream context for a collective over the gradients issued so far: the side stream waits for
        the main stream's work so far (one event) and is made current, so the collective (RCCL's
        stream waits on the current one) follows both streams while the main stream runs on."""
        self._flush_side()
        if self._side is None:
            yield
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self._side.wait_event(ev)
        with torch.cuda.stream(self._side):
            yield

    def _drain_side(self) -> None:
        """Main stream waits for the weight gradients issued on the side stream so far (the deferred ones
        stay deferred): nothing of the side stream is resident during the next main-stream launch."""
        if self._last_side is not None and self._waited_seq < self._side_seq:
            self._last_side.wait(torch.cuda.current_stream())
            self._pending.clear()
            self._waited_seq = self._side_seq

    def _join(self) -> None:
        """Main stream waits for every weight gradient issued so far."""
        self._flush_side()
        if self._last_side is not None:
            self._last_side.wait(torch.cuda.current_stream())
            self._pending.clear()
            self._last_side = None
            self._waited_seq = self._side_seq

    def _dgrad(self, conv, dy, dx, addend=None, mask=None):
        cv = self.convs[conv]
        self._guard(dx)
        self._launch(cv, 1, lambda: self.L.conv_dgrad(C.byref(cv.desc), self.cdt, ptr(dy), ptr(cv.wd), ptr(dx),
                                                       ptr(addend), ptr(mask), stream()))

    @staticmethod
    def _launch(cv, pass_, fn):
        fn()


def conv_grad_shape(shape_oihw) -> tuple:
    """OHWI buffer shape for an OIHW conv weight (the layout conv_wgrad writes)."""
    k, c, r, s = shape_oihw
    return (k, r, s, c)
