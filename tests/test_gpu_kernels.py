"""Per-kernel parity of libargus_hip on the MI355X against torch fp64 CPU references.

Every call goes through the C ABI (argus_amd._lib). fp32 path: relative error <= 2e-5 (exact-f32
MFMA, fp32 accumulation). bf16 path: inputs are rounded to bf16 first and the reference is computed
in fp64 on those rounded inputs; tolerance 1.5e-2 of the reference's max magnitude (one bf16 output
rounding + fp32 accumulation order).
"""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

from argus_amd._lib import BF16, F32, FP8, ConvDesc, lib, ptr, stream

pytestmark = pytest.mark.gpu

TOL = {"fp32": 2e-5, "bf16": 1.5e-2}
TDT = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp8": torch.bfloat16}  # fp8: bf16 tensors
DT = {"fp32": F32, "bf16": BF16, "fp8": FP8}

# (cin, cout, k, stride, input size) — every distinct conv shape of SURVEY.md Appendix B at small
# spatial sizes (odd sizes exercise partial tiles and the 376x672 rounding).
CONV_SHAPES = [
    (64, 64, 1, 1, 12), (64, 64, 3, 1, 12), (64, 256, 1, 1, 12), (256, 64, 1, 1, 12), (256, 128, 1, 1, 12),
    (128, 128, 3, 2, 12), (128, 512, 1, 1, 8), (256, 512, 1, 2, 12), (512, 128, 1, 1, 8), (128, 128, 3, 1, 8),
    (512, 256, 1, 1, 8), (256, 256, 3, 2, 9), (256, 1024, 1, 1, 6), (512, 1024, 1, 2, 9), (1024, 256, 1, 1, 6),
    (256, 256, 3, 1, 6), (1024, 512, 1, 1, 6), (512, 512, 3, 2, 7), (512, 2048, 1, 1, 4), (1024, 2048, 1, 2, 7),
    (2048, 512, 1, 1, 4), (512, 512, 3, 1, 4),
]


def _rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _desc(n, h, w, cin, cout, k, s, stem=False):
    p = 3 if stem else (1 if k == 3 else 0)
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    return ConvDesc(n, h, w, cin, cout, k, k, s, p, ho, wo, int(stem)), p


def _prep(d, dt, w_ohwi, cuda):
    """weight_prep from an fp32 OHWI master; returns (w_fwd, w_dgrad)."""
    k, r, s, c = w_ohwi.shape
    if d.stem:
        wf = torch.empty(k, 256, dtype=TDT[dt], device=cuda)
        wd = None
    else:
        wf = torch.empty(k, r * s * c, dtype=TDT[dt], device=cuda)
        wd = torch.empty(c, r * s * k, dtype=TDT[dt], device=cuda)
    lib().conv_weight_prep(C.byref(d), DT[dt], ptr(w_ohwi), None, ptr(wf), ptr(wd), stream())
    return wf, wd


def _q(t, dt):  # round to the compute dtype (reference inputs)
    return t.to(TDT[dt]).to(torch.float64)


def _merge_stats(part, tile, count, counts=None):
    """Chan-merge per-tile {sum, M2} partials (rows, C, 2) -> per-channel (mean, biased var). tile < 0
    (argus_conv_fwd_stat_tile of a ragged producer): row r holds counts[r] elements (the int32 array
    the producer writes after the partials)."""
    if tile < 0:
        assert counts is not None and counts.shape[0] == part.shape[0]
        assert int(counts.sum()) == count and int(counts.max()) <= -tile and int(counts.min()) >= 0
        n = counts.to(torch.float64).clamp_min(1.0)
    else:
        n = torch.tensor([min(tile, count - t * tile) for t in range(part.shape[0])], dtype=torch.float64)
    mean_t = part[..., 0] / n[:, None]
    mean = part[..., 0].sum(0) / count
    q = (part[..., 1] + part[..., 0] * mean_t).sum(0)  # sum of x^2
    return mean, q / count - mean * mean


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_conv_fwd_dgrad_wgrad_all_shapes(cuda, dt):
    torch.manual_seed(0)
    L = lib()
    for cin, cout, k, s, hin in CONV_SHAPES:
        n = 2
        d, p = _desc(n, hin, hin, cin, cout, k, s)
        x = torch.randn(n, hin, hin, cin)
        w = torch.randn(cout, k, k, cin) * (2.0 / (k * k * cin)) ** 0.5
        dy = torch.randn(n, d.ho, d.wo, cout)
        xd, wd_, dyd = x.to(cuda, TDT[dt]), w.to(cuda), dy.to(cuda, TDT[dt])
        wf, wt = _prep(d, dt, wd_, cuda)
        # forward (+ BN statistics partials)
        y = torch.empty(n, d.ho, d.wo, cout, dtype=TDT[dt], device=cuda)
        rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), DT[dt])
        stats = torch.empty(rows, cout, 2, device=cuda)
        L.conv_fwd(C.byref(d), DT[dt], ptr(xd), ptr(wf), ptr(y), None, None, ptr(stats), stream())
        xr, wr, dyr = _q(x, dt).permute(0, 3, 1, 2), _q(w, dt).permute(0, 3, 1, 2), _q(dy, dt).permute(0, 3, 1, 2)
        ref = F.conv2d(xr, wr, stride=s, padding=p)
        e = _rel(y.permute(0, 3, 1, 2), ref)
        assert e < TOL[dt], f"fwd {cin}->{cout} k{k} s{s} {dt}: {e}"
        tile = L.dll.argus_conv_fwd_stat_tile(C.byref(d), DT[dt])
        mean, var = _merge_stats(stats.double().cpu(), tile, n * d.ho * d.wo)
        yr = y.double().cpu().reshape(-1, cout) if dt == "fp32" else ref.permute(0, 2, 3, 1).reshape(-1, cout)
        assert _rel(mean, yr.mean(0)) < 1e-4 or (mean - yr.mean(0)).abs().max() < 1e-5 * yr.std(0).max()
        assert _rel(var, yr.var(0, unbiased=False)) < (1e-5 if dt == "fp32" else 1e-2), f"stats {cin}->{cout}"
        # dgrad (accumulate onto a non-zero buffer to check both modes)
        dx0 = torch.randn(n, hin, hin, cin)
        dx = dx0.to(cuda, TDT[dt])
        L.conv_dgrad(C.byref(d), DT[dt], ptr(dyd), ptr(wt), ptr(dx), ptr(dx), None, stream())
        refd = torch.nn.grad.conv2d_input(xr.shape, wr, dyr, stride=s, padding=p) + _q(dx0, dt).permute(0, 3, 1, 2)
        e = _rel(dx.permute(0, 3, 1, 2), refd)
        assert e < TOL[dt], f"dgrad {cin}->{cout} k{k} s{s} {dt}: {e}"
        # wgrad
        ws = torch.empty(L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), DT[dt]), dtype=torch.uint8, device=cuda)
        dw = torch.empty(cout, k, k, cin, device=cuda)
        L.conv_wgrad(C.byref(d), DT[dt], ptr(xd), None, None, ptr(dyd), ptr(dw), ptr(ws), ws.numel(), stream())
        refw = torch.nn.grad.conv2d_weight(xr, wr.shape, dyr, stride=s, padding=p)
        e = _rel(dw.permute(0, 3, 1, 2), refw)
        assert e < (TOL[dt] if dt == "fp32" else 2e-3), f"wgrad {cin}->{cout} k{k} s{s} {dt}: {e}"


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_conv_bn_relu_prologue(cuda, dt):
    """conv(relu(x*scale+shift)) with the BN+ReLU applied while staging; padding stays zero."""
    torch.manual_seed(1)
    L = lib()
    for cin, cout, k, s, hin in [(64, 64, 3, 1, 10), (128, 128, 3, 2, 11), (256, 64, 1, 1, 6)]:
        n = 2
        d, p = _desc(n, hin, hin, cin, cout, k, s)
        x = torch.randn(n, hin, hin, cin)
        sc, sh = torch.rand(cin) + 0.5, torch.randn(cin) * 0.5
        w = torch.randn(cout, k, k, cin) * 0.05
        wf, _ = _prep(d, dt, w.to(cuda), cuda)
        y = torch.empty(n, d.ho, d.wo, cout, dtype=TDT[dt], device=cuda)
        scd, shd = sc.to(cuda), sh.to(cuda)
        xg = x.to(cuda, TDT[dt])
        L.conv_fwd(C.byref(d), DT[dt], ptr(xg), ptr(wf), ptr(y), ptr(scd), ptr(shd), None, stream())
        xa = torch.relu(_q(x, dt) * sc.double() + sh.double())
        xa = xa.to(TDT[dt]).double() if dt == "bf16" else xa
        ref = F.conv2d(xa.permute(0, 3, 1, 2), _q(w, dt).permute(0, 3, 1, 2), stride=s, padding=p)
        e = _rel(y.permute(0, 3, 1, 2), ref)
        assert e < TOL[dt] * (2 if dt == "bf16" else 1), f"prologue fwd {cin}->{cout}: {e}"
        # wgrad with the same prologue
        dy = torch.randn(n, d.ho, d.wo, cout)
        ws = torch.empty(L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), DT[dt]), dtype=torch.uint8, device=cuda)
        dw = torch.empty(cout, k, k, cin, device=cuda)
        dyg = dy.to(cuda, TDT[dt])
        L.conv_wgrad(C.byref(d), DT[dt], ptr(xg), ptr(scd), ptr(shd), ptr(dyg), ptr(dw), ptr(ws), ws.numel(), stream())
        refw = torch.nn.grad.conv2d_weight(xa.permute(0, 3, 1, 2), (cout, cin, k, k), _q(dy, dt).permute(0, 3, 1, 2),
                                           stride=s, padding=p)
        e = _rel(dw.permute(0, 3, 1, 2), refw)
        assert e < (TOL[dt] if dt == "fp32" else 3e-3), f"prologue wgrad {cin}->{cout}: {e}"


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_stem_fwd_wgrad(cuda, dt):
    torch.manual_seed(2)
    L = lib()
    for hw in [(32, 32), (38, 30)]:
        n, H, W = 3, *hw
        d, p = _desc(n, H, W, 3, 64, 7, 2, stem=True)
        img = torch.rand(n, 3, H, W)
        x4 = torch.empty(n, H, W, 4, dtype=TDT[dt], device=cuda)
        imgg = img.to(cuda)
        L.images_to_nhwc4(DT[dt], n, H, W, ptr(imgg), ptr(x4), stream())
        assert torch.equal(x4[..., :3].permute(0, 3, 1, 2).cpu().float(), _q(img, dt).float())
        assert (x4[..., 3] == 0).all()
        w = torch.randn(64, 7, 7, 3) * 0.1
        wmaster = w.permute(0, 3, 1, 2).contiguous().to(cuda)  # OIHW nn.Parameter layout
        wf = torch.empty(64, 256, dtype=TDT[dt], device=cuda)
        strides = (C.c_int64 * 4)(*wmaster.stride())
        L.conv_weight_prep(C.byref(d), DT[dt], ptr(wmaster), strides, ptr(wf), None, stream())
        y = torch.empty(n, d.ho, d.wo, 64, dtype=TDT[dt], device=cuda)
        L.conv_fwd(C.byref(d), DT[dt], ptr(x4), ptr(wf), ptr(y), None, None, None, stream())
        ref = F.conv2d(_q(img, dt), _q(w, dt).permute(0, 3, 1, 2), stride=2, padding=3)
        e = _rel(y.permute(0, 3, 1, 2), ref)
        assert e < TOL[dt], f"stem fwd {hw} {dt}: {e}"
        dy = torch.randn(n, d.ho, d.wo, 64)
        ws = torch.empty(L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), DT[dt]), dtype=torch.uint8, device=cuda)
        dw = torch.empty(64, 7, 7, 3, device=cuda)
        dyg = dy.to(cuda, TDT[dt])
        L.conv_wgrad(C.byref(d), DT[dt], ptr(x4), None, None, ptr(dyg), ptr(dw), ptr(ws), ws.numel(), stream())
        refw = torch.nn.grad.conv2d_weight(_q(img, dt), (64, 3, 7, 7), _q(dy, dt).permute(0, 3, 1, 2), stride=2,
                                           padding=3)
        e = _rel(dw.permute(0, 3, 1, 2), refw)
        assert e < (TOL[dt] if dt == "fp32" else 2e-3), f"stem wgrad {hw} {dt}: {e}"


def test_stem_lds_patch_kernel(cuda):
    """bf16 stem forward on the LDS-patch kernel (stem.hip: 8 x 32 output tiles, K = 7 filter rows x 32)
    vs torch (bf16 tolerance) and vs the implicit GEMM it replaces (tuning key 19 = 0): outputs within
    the bf16 tolerance of each other, BN statistics partials (one per 128 pixels) merging to the same
    mean / variance (ragged edge tiles: partial rows merged as full ones, stat tile -128); shapes whose
    8 x 32 tiling is mostly padding (19 x 15) keep the implicit GEMM."""
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(33)
    L = lib()
    # 376 x 672 (188 x 336 output) and 100 x 248 (50 x 124): ragged edge tiles in both dimensions
    for n, H, W, served in ((2, 64, 128, True), (1, 256, 256, True), (3, 38, 30, False), (1, 376, 672, True),
                            (2, 100, 248, True)):
        d, p = _desc(n, H, W, 3, 64, 7, 2, stem=True)
        img = torch.rand(n, 3, H, W)
        x4 = torch.empty(n, H, W, 4, dtype=torch.bfloat16, device=cuda)
        imgg = img.to(cuda)
        L.images_to_nhwc4(BF16, n, H, W, ptr(imgg), ptr(x4), stream())
        w = torch.randn(64, 7, 7, 3) * 0.1
        wmaster = w.permute(0, 3, 1, 2).contiguous().to(cuda)
        wf = torch.empty(64, 256, dtype=torch.bfloat16, device=cuda)
        strides = (C.c_int64 * 4)(*wmaster.stride())
        L.conv_weight_prep(C.byref(d), BF16, ptr(wmaster), strides, ptr(wf), None, stream())
        ref = F.conv2d(_q(img, "bf16"), _q(w, "bf16").permute(0, 3, 1, 2), stride=2, padding=3)
        M = n * d.ho * d.wo
        outs = []
        for key19 in (1, 0):
            dk = d.with_tuning({19: key19})
            rows = L.dll.argus_conv_fwd_stat_rows(C.byref(dk), BF16)
            tile = L.dll.argus_conv_fwd_stat_tile(C.byref(dk), BF16)
            assert tile == (-128 if served and key19 and (d.ho % 8 or d.wo % 32) else 128), (n, H, W, key19, tile)
            y = torch.empty(n, d.ho, d.wo, 64, dtype=torch.bfloat16, device=cuda)
            buf = torch.full((rows * 128 + rows,), float("nan"), device=cuda)  # partials (+ counts if ragged)
            stats = buf[:rows * 128].view(rows, 64, 2)
            with KernelTimer() as t:
                L.conv_fwd(C.byref(dk), BF16, ptr(x4), ptr(wf), ptr(y), None, None, ptr(buf), stream())
            names = list(t.summary())
            assert ("argus::stem_fwd_kernel" in names) == (served and key19 == 1), (n, H, W, key19, names)
            assert _rel(y.permute(0, 3, 1, 2), ref) < TOL["bf16"], ("stem fwd", n, H, W, key19)
            assert torch.isfinite(stats).all()
            counts = buf[rows * 128:].view(torch.int32).cpu() if tile < 0 else None
            mean, var = _merge_stats(stats.double().cpu(), tile, M, counts)
            yr = ref.permute(0, 2, 3, 1).reshape(-1, 64)
            vr = yr.var(0, unbiased=False)
            assert (mean - yr.mean(0)).abs().max() < 2e-2 * yr.std(0).max(), ("stats mean", n, H, W, key19)
            assert _rel(var, vr) < 2e-2, ("stats var", n, H, W, key19, _rel(var, vr))
            # the library's finalize (fp64 merge) on the same partials: mean / invstd of the host merge
            g1, b0 = torch.ones(64, device=cuda), torch.zeros(64, device=cuda)
            mo, io = torch.empty(64, device=cuda), torch.empty(64, device=cuda)
            ws = torch.zeros(L.dll.argus_bn_workspace_bytes(64), dtype=torch.uint8, device=cuda)
            L.bn_finalize(64, rows, tile, ptr(buf), M, ptr(g1), ptr(b0), C.c_float(0.0), C.c_float(0.1), None, None,
                          None, ptr(mo), ptr(io), None, None, ptr(ws), stream())
            assert (mo.double().cpu() - mean).abs().max() < 1e-6 * (1 + mean.abs().max()), ("finalize mean", n, H, W)
            assert _rel(io.double().cpu() ** -2, var) < 1e-4, ("finalize var", n, H, W, key19)
            outs.append((y.float(), mean, var))
        assert _rel(outs[0][0], outs[1][0]) < 1e-2
        assert _rel(outs[0][2], outs[1][2]) < 1e-4 and (outs[0][1] - outs[1][1]).abs().max() < 1e-4


def test_bn_finalize_row_counts_large_mean(cuda):
    """argus_bn_finalize with a ragged producer's layout (stat tile -128: int32 row counts after the
    partials, as stem_fwd_kernel writes them) on rows whose mean is 1e4 standard deviations off zero:
    every row keeps its own {sum, M2 about the row mean}, so the fp64 merge recovers the variance to
    fp32 input rounding (re-centring each ragged row to 128 elements in fp32 lost it)."""
    L = lib()
    g = torch.Generator().manual_seed(5)
    rows, c = 300, 64
    counts = torch.randint(1, 129, (rows,), generator=g, dtype=torch.int32)
    counts[::7] = 128
    counts[5] = 0  # an empty half-tile (the bottom half of a 4-row ragged tile)
    mean_c = 1e4 * (1 + torch.rand(c, generator=g, dtype=torch.float64))
    xs = [mean_c + torch.randn(int(k), c, generator=g, dtype=torch.float64) for k in counts]
    part = torch.zeros(rows, c, 2, dtype=torch.float64)
    for r, x in enumerate(xs):
        if x.shape[0]:
            part[r, :, 0] = x.sum(0)
            part[r, :, 1] = ((x - x.mean(0)) ** 2).sum(0)
    allx = torch.cat(xs)
    M = allx.shape[0]
    buf = torch.cat([part.float().flatten(), counts.view(torch.float32)]).to(cuda)
    g1, b0 = torch.ones(c, device=cuda), torch.zeros(c, device=cuda)
    mo, io = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    ws = torch.zeros(L.dll.argus_bn_workspace_bytes(c), dtype=torch.uint8, device=cuda)
    L.bn_finalize(c, rows, -128, ptr(buf), M, ptr(g1), ptr(b0), C.c_float(0.0), C.c_float(0.1), None, None, None,
                  ptr(mo), ptr(io), None, None, ptr(ws), stream())
    var = allx.var(0, unbiased=False)
    got = io.double().cpu() ** -2
    print("max rel var error", _rel(got, var))
    assert _rel(got, var) < 1e-3
    assert ((mo.double().cpu() - allx.mean(0)).abs() / allx.std(0)).max() < 1e-2
    # the host merge used by the stem test agrees
    hm, hv = _merge_stats(part.float().double(), -128, M, counts)
    assert _rel(hv, var) < 1e-3


def test_stem_wgrad_lds_patch_kernel(cuda):
    """bf16 stem weight gradient on the LDS-patch kernel (stem.hip: dy tile + input patch, both MFMA
    operands read pixel-major with ds_read_b64_tr_b16) vs torch's conv2d_weight and vs wgrad_kernel's
    STEM variant it replaces (tuning key 34 = 0), with dy given and with dy staged through the fused
    BN-backward apply (argus_conv_wgrad_apply). 304 x 1856: 551 tiles -> 2 per split, the last split
    ragged; 38 x 30 does not tile and keeps wgrad_kernel."""
    from argus_amd._lib import BnBwdPrologue
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(34)
    L = lib()
    for n, H, W, served in ((2, 64, 128, True), (1, 304, 1856, True), (3, 38, 30, False), (1, 376, 672, True),
                            (2, 100, 248, True)):
        d, _ = _desc(n, H, W, 3, 64, 7, 2, stem=True)
        img = torch.rand(n, 3, H, W)
        x4 = torch.empty(n, H, W, 4, dtype=torch.bfloat16, device=cuda)
        imgg = img.to(cuda)
        L.images_to_nhwc4(BF16, n, H, W, ptr(imgg), ptr(x4), stream())
        dm = torch.randn(n, d.ho, d.wo, 64, device=cuda).to(torch.bfloat16)
        y0 = torch.randn(n, d.ho, d.wo, 64, device=cuda).to(torch.bfloat16)
        ca, cb, cc = (torch.randn(64, device=cuda) * 0.3 for _ in range(3))
        dy_ap = (ca * dm.float() + (cb * y0.float() + cc)).to(torch.bfloat16)  # fmaf rounding aside
        ws = torch.empty(L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), BF16), dtype=torch.uint8, device=cuda)
        for apply in (False, True):
            dyq = dy_ap if apply else dm
            ref = torch.nn.grad.conv2d_weight(_q(img, "bf16"), (64, 3, 7, 7), dyq.double().cpu().permute(0, 3, 1, 2),
                                              stride=2, padding=3)
            outs = []
            for key34 in (1, 0):
                dw = torch.full((64, 7, 7, 3), float("nan"), device=cuda)
                dk = d.with_tuning({34: key34})
                with KernelTimer() as t:
                    if apply:
                        ap = BnBwdPrologue(ptr(y0), ptr(ca), ptr(cb), ptr(cc), None)
                        L.conv_wgrad_apply(C.byref(dk), BF16, ptr(x4), ptr(dm), C.byref(ap), ptr(dw), ptr(ws),
                                           ws.numel(), stream())
                    else:
                        L.conv_wgrad(C.byref(dk), BF16, ptr(x4), None, None, ptr(dm), ptr(dw), ptr(ws),
                                     ws.numel(), stream())
                names = list(t.summary())
                want = f"argus::stem_wgrad_kernel<{'true' if apply else 'false'}>"
                assert (want in names) == (served and key34 == 1), (n, H, W, apply, key34, names)
                e = _rel(dw.permute(0, 3, 1, 2), ref)
                assert e < 2e-3, ("stem wgrad", n, H, W, apply, key34, e)
                outs.append(dw.clone())
            assert _rel(outs[0], outs[1]) < 2e-3


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_bn_train_forward_backward(cuda, dt):
    """finalize + apply(+residual, relu) + backward reduce/finalize/apply vs autograd BatchNorm2d."""
    torch.manual_seed(3)
    L = lib()
    n, h, w, c = 4, 7, 5, 64
    px = n * h * w
    y = torch.randn(n, h, w, c) * 2 + 0.5
    res = torch.randn(n, h, w, c)
    gamma, beta = torch.rand(c) + 0.5, torch.randn(c)
    yq, resq = _q(y, dt), _q(res, dt)
    # partials: one row per pixel block of 5 pixels
    yy = yq.reshape(px, c).reshape(-1, 5, c)
    part = torch.stack([yy.sum(1), ((yy - yy.mean(1, keepdim=True)) ** 2).sum(1)], -1).float()
    rows = part.shape[0]
    rm, rv = torch.zeros(c, device=cuda), torch.ones(c, device=cuda)
    nbt = torch.zeros((), dtype=torch.int64, device=cuda)
    stt = torch.empty(4, c, device=cuda)
    ws = torch.zeros(L.dll.argus_bn_workspace_bytes(c), dtype=torch.uint8, device=cuda)
    gd, bd = gamma.to(cuda), beta.to(cuda)
    partg = part.to(cuda)
    L.bn_finalize(c, rows, 5, ptr(partg), px, ptr(gd), ptr(bd), C.c_float(1e-5), C.c_float(0.1), ptr(rm), ptr(rv),
                  ptr(nbt), ptr(stt[0]), ptr(stt[1]), ptr(stt[2]), ptr(stt[3]), ptr(ws), stream())
    bn = torch.nn.BatchNorm2d(c).double()
    with torch.no_grad():
        bn.weight.copy_(gamma)
        bn.bias.copy_(beta)
    xin = yq.permute(0, 3, 1, 2).clone().requires_grad_(True)
    z = bn(xin)
    out = torch.relu(z + resq.permute(0, 3, 1, 2))
    assert _rel(rm, bn.running_mean) < 1e-5 and _rel(rv, bn.running_var) < 1e-5 and int(nbt) == 1
    yd = y.to(cuda, TDT[dt])
    o = torch.empty_like(yd)
    resg = res.to(cuda, TDT[dt])
    E = 8 if dt == "bf16" else 4
    bits = torch.empty(px * c // E, dtype=torch.uint8, device=cuda)
    L.bn_apply(DT[dt], px, c, ptr(yd), ptr(stt[2]), ptr(stt[3]), ptr(resg), None, None, 1, ptr(o), ptr(bits),
               stream())
    assert _rel(o.permute(0, 3, 1, 2), out) < TOL[dt]
    want_bits = ((o.reshape(-1, E) > 0).int() << torch.arange(E, device=cuda)).sum(1).to(torch.uint8)
    assert torch.equal(bits, want_bits), "ReLU mask bits"
    # backward: mask from the block output (mode 1), dm_out = masked grad
    dout = torch.randn(n, h, w, c)
    doutq = _q(dout, dt)
    out.backward(doutq.permute(0, 3, 1, 2))
    bpart = torch.empty(L.dll.argus_bn_bwd_rows(px, c), c, 2, device=cuda)
    doutg = dout.to(cuda, TDT[dt])
    L.bn_bwd_reduce(DT[dt], px, c, ptr(doutg), 1, ptr(o), ptr(yd), ptr(stt[2]), ptr(stt[3]),
                    ptr(stt[0]), ptr(stt[1]), ptr(bpart), None, None, None, None, stream())
    dg, db = torch.empty(c, device=cuda), torch.empty(c, device=cuda)
    cf = torch.empty(3, c, device=cuda)
    L.bn_bwd_finalize(c, bpart.shape[0], ptr(bpart), px, ptr(gd), ptr(stt[0]), ptr(stt[1]), ptr(dg), ptr(db),
                      ptr(cf[0]), ptr(cf[1]), ptr(cf[2]), ptr(ws), stream())
    dyo, dmo = torch.empty_like(yd), torch.empty_like(yd)
    L.bn_bwd_apply(DT[dt], px, c, ptr(doutg), 1, ptr(o), ptr(yd), ptr(stt[2]), ptr(stt[3]), ptr(cf[0]),
                   ptr(cf[1]), ptr(cf[2]), ptr(dyo), ptr(dmo), None, None, None, None, None, stream())
    tol = TOL[dt] * (3 if dt == "bf16" else 1)
    assert _rel(dg, bn.weight.grad) < tol, "dgamma"
    assert _rel(db, bn.bias.grad) < tol, "dbeta"
    assert _rel(dyo.permute(0, 3, 1, 2), xin.grad) < tol * 2, "dx"
    # mode 3 (mask bits) gives exactly mode 1's results
    bpart3, dg3, db3, cf3 = torch.empty_like(bpart), torch.empty_like(dg), torch.empty_like(db), torch.empty_like(cf)
    dyo3 = torch.empty_like(yd)
    L.bn_bwd_reduce(DT[dt], px, c, ptr(doutg), 3, ptr(bits), ptr(yd), None, None,
                    ptr(stt[0]), ptr(stt[1]), ptr(bpart3), None, None, None, None, stream())
    L.bn_bwd_finalize(c, bpart.shape[0], ptr(bpart3), px, ptr(gd), ptr(stt[0]), ptr(stt[1]), ptr(dg3), ptr(db3),
                      ptr(cf3[0]), ptr(cf3[1]), ptr(cf3[2]), ptr(ws), stream())
    L.bn_bwd_apply(DT[dt], px, c, ptr(doutg), 3, ptr(bits), ptr(yd), None, None, ptr(cf3[0]),
                   ptr(cf3[1]), ptr(cf3[2]), ptr(dyo3), None, None, None, None, None, None, stream())
    assert torch.equal(bpart3, bpart) and torch.equal(dyo3, dyo), "mode 3 == mode 1"
    # mode 2 (relu mask recomputed from y via scale/shift)
    xin2 = yq.permute(0, 3, 1, 2).clone().requires_grad_(True)
    bn2 = torch.nn.BatchNorm2d(c).double()
    with torch.no_grad():
        bn2.weight.copy_(gamma)
        bn2.bias.copy_(beta)
    torch.relu(bn2(xin2)).backward(doutq.permute(0, 3, 1, 2))
    L.bn_bwd_reduce(DT[dt], px, c, ptr(doutg), 2, None, ptr(yd), ptr(stt[2]), ptr(stt[3]),
                    ptr(stt[0]), ptr(stt[1]), ptr(bpart), None, None, None, None, stream())
    L.bn_bwd_finalize(c, bpart.shape[0], ptr(bpart), px, ptr(gd), ptr(stt[0]), ptr(stt[1]), ptr(dg), ptr(db),
                      ptr(cf[0]), ptr(cf[1]), ptr(cf[2]), ptr(ws), stream())
    L.bn_bwd_apply(DT[dt], px, c, ptr(doutg), 2, None, ptr(yd), ptr(stt[2]), ptr(stt[3]), ptr(cf[0]),
                   ptr(cf[1]), ptr(cf[2]), ptr(dyo), None, None, None, None, None, None, stream())
    assert _rel(dyo.permute(0, 3, 1, 2), xin2.grad) < tol * 2, "dx mode 2"
    assert _rel(dg, bn2.weight.grad) < tol, "dgamma mode 2"


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_bn_dual_branch_backward(cuda, dt):
    """out = relu(bnA(y) + bnB(y2)) (bn3 + downsample BN): one dual reduce/apply pass with mask bits
    vs autograd, and the masked residual addend of conv_dgrad."""
    torch.manual_seed(5)
    L = lib()
    n, h, w, c = 3, 6, 5, 128
    px = n * h * w
    E = 8 if dt == "bf16" else 4
    ya, yb = _q(torch.randn(n, h, w, c) * 1.5 + 0.3, dt), _q(torch.randn(n, h, w, c) - 0.2, dt)
    gA, bA, gB, bB = torch.rand(c) + 0.5, torch.randn(c), torch.rand(c) + 0.5, torch.randn(c)
    ws = torch.zeros(L.dll.argus_bn_workspace_bytes(c), dtype=torch.uint8, device=cuda)

    def finalize(yq, g, b):
        yy = yq.reshape(px, c).reshape(-1, 5, c)
        part = torch.stack([yy.sum(1), ((yy - yy.mean(1, keepdim=True)) ** 2).sum(1)], -1).float().to(cuda)
        stt = torch.empty(4, c, device=cuda)
        L.bn_finalize(c, part.shape[0], 5, ptr(part), px, ptr(g), ptr(b), C.c_float(1e-5), C.c_float(0.1), None,
                      None, None, ptr(stt[0]), ptr(stt[1]), ptr(stt[2]), ptr(stt[3]), ptr(ws), stream())
        return stt

    gAd, bAd, gBd, bBd = gA.to(cuda), bA.to(cuda), gB.to(cuda), bB.to(cuda)
    sA, sB = finalize(ya, gAd, bAd), finalize(yb, gBd, bBd)
    yad, ybd = ya.to(cuda, TDT[dt]), yb.to(cuda, TDT[dt])
    o = torch.empty_like(yad)
    bits = torch.empty(px * c // E, dtype=torch.uint8, device=cuda)
    L.bn_apply(DT[dt], px, c, ptr(yad), ptr(sA[2]), ptr(sA[3]), ptr(ybd), ptr(sB[2]), ptr(sB[3]), 1, ptr(o),
               ptr(bits), stream())
    bnA, bnB = torch.nn.BatchNorm2d(c).double(), torch.nn.BatchNorm2d(c).double()
    with torch.no_grad():
        bnA.weight.copy_(gA); bnA.bias.copy_(bA); bnB.weight.copy_(gB); bnB.bias.copy_(bB)
    xa = ya.permute(0, 3, 1, 2).double().requires_grad_(True)
    xb = yb.permute(0, 3, 1, 2).double().requires_grad_(True)
    out = torch.relu(bnA(xa) + bnB(xb))
    assert _rel(o.permute(0, 3, 1, 2), out) < TOL[dt]
    dout = _q(torch.randn(n, h, w, c), dt)
    out.backward(dout.permute(0, 3, 1, 2).double())
    doutg = dout.to(cuda, TDT[dt])
    rows = L.dll.argus_bn_bwd_rows(px, c)
    pA, pB = torch.empty(rows, c, 2, device=cuda), torch.empty(rows, c, 2, device=cuda)
    L.bn_bwd_reduce(DT[dt], px, c, ptr(doutg), 3, ptr(bits), ptr(yad), None, None, ptr(sA[0]), ptr(sA[1]), ptr(pA),
                    ptr(ybd), ptr(sB[0]), ptr(sB[1]), ptr(pB), stream())
    grads = {}
    for nm, part, g, st in (("A", pA, gAd, sA), ("B", pB, gBd, sB)):
        dg, db, cf = torch.empty(c, device=cuda), torch.empty(c, device=cuda), torch.empty(3, c, device=cuda)
        L.bn_bwd_finalize(c, rows, ptr(part), px, ptr(g), ptr(st[0]), ptr(st[1]), ptr(dg), ptr(db), ptr(cf[0]),
                          ptr(cf[1]), ptr(cf[2]), ptr(ws), stream())
        grads[nm] = (dg, db, cf)
    dya, dyb = torch.empty_like(yad), torch.empty_like(yad)
    cfa, cfb = grads["A"][2], grads["B"][2]
    L.bn_bwd_apply(DT[dt], px, c, ptr(doutg), 3, ptr(bits), ptr(yad), None, None, ptr(cfa[0]), ptr(cfa[1]),
                   ptr(cfa[2]), ptr(dya), None, ptr(ybd), ptr(cfb[0]), ptr(cfb[1]), ptr(cfb[2]), ptr(dyb), stream())
    tol = TOL[dt] * (3 if dt == "bf16" else 1)
    assert _rel(grads["A"][0], bnA.weight.grad) < tol and _rel(grads["A"][1], bnA.bias.grad) < tol
    assert _rel(grads["B"][0], bnB.weight.grad) < tol and _rel(grads["B"][1], bnB.bias.grad) < tol
    assert _rel(dya.permute(0, 3, 1, 2), xa.grad) < tol * 2 and _rel(dyb.permute(0, 3, 1, 2), xb.grad) < tol * 2
    # masked residual addend in the dgrad epilogue: dx = dgrad(dy) + relu'(out) * dout
    d, p = _desc(n, h, w, 64, c, 1, 1)
    wt = torch.randn(c, 1, 1, 64) * 0.1
    wf, wdg = _prep(d, dt, wt.to(cuda), cuda)
    dyc = _q(torch.randn(n, h, w, c), dt)
    dycg = dyc.to(cuda, TDT[dt])
    dx = torch.empty(n, h, w, 64, dtype=TDT[dt], device=cuda)
    res = _q(torch.randn(n, h, w, 64), dt)
    resg = res.to(cuda, TDT[dt])
    keep = res.float() > 0.3  # one fp32 mask for both the bits and the reference
    rbits = ((keep.reshape(-1, E).int() << torch.arange(E)).sum(1)).to(torch.uint8).to(cuda)
    L.conv_dgrad(C.byref(d), DT[dt], ptr(dycg), ptr(wdg), ptr(dx), ptr(resg), ptr(rbits), stream())
    ref = torch.nn.grad.conv2d_input((n, 64, h, w), _q(wt, dt).permute(0, 3, 1, 2), dyc.permute(0, 3, 1, 2))
    ref = ref + (res * keep).permute(0, 3, 1, 2)
    assert _rel(dx.permute(0, 3, 1, 2), ref) < TOL[dt]


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_maxpool_avgpool(cuda, dt):
    torch.manual_seed(4)
    L = lib()
    n, h, w, c = 2, 13, 10, 64
    y = torch.randn(n, h, w, c)
    sc, sh = torch.rand(c) + 0.5, torch.randn(c) * 0.3
    yq = _q(y, dt)
    # the kernel pools the exact fp32 z = relu(y*scale+shift) and rounds only the max
    z = torch.relu(yq.float() * sc + sh).double()
    zin = z.permute(0, 3, 1, 2).clone().requires_grad_(True)
    ref = F.max_pool2d(zin, 3, 2, 1)
    ho, wo = ref.shape[2], ref.shape[3]
    out = torch.empty(n, ho, wo, c, dtype=TDT[dt], device=cuda)
    am = torch.empty(n, ho, wo, c, dtype=torch.uint8, device=cuda)
    yg, scg, shg = y.to(cuda, TDT[dt]), sc.to(cuda), sh.to(cuda)
    L.maxpool_fwd(DT[dt], n, h, w, c, ptr(yg), ptr(scg), ptr(shg), ptr(out), ptr(am), stream())
    assert _rel(out.permute(0, 3, 1, 2), ref) < TOL[dt] / 2
    g = torch.randn(n, ho, wo, c)
    ref.backward(_q(g, dt).permute(0, 3, 1, 2))
    dz = torch.empty(n, h, w, c, dtype=TDT[dt], device=cuda)
    gg = g.to(cuda, TDT[dt])
    L.maxpool_bwd(DT[dt], n, h, w, c, ptr(gg), ptr(am), ptr(dz), stream())
    assert _rel(dz.permute(0, 3, 1, 2), zin.grad) < TOL[dt]
    # global average pool
    x = torch.randn(n, 8, 8, 2048)
    feat = torch.empty(n, 2048, device=cuda)
    xg = x.to(cuda, TDT[dt])
    L.avgpool_fwd(DT[dt], n, 64, 2048, ptr(xg), ptr(feat), stream())
    assert _rel(feat, _q(x, dt).mean((1, 2))) < (1e-5 if dt == "fp32" else 2e-3)
    df = torch.randn(n, 2048)
    dx = torch.empty(n, 8, 8, 2048, dtype=TDT[dt], device=cuda)
    dfg = df.to(cuda)
    L.avgpool_bwd(DT[dt], n, 64, 2048, ptr(dfg), ptr(dx), stream())
    assert _rel(dx, (df / 64)[:, None, None, :].expand(n, 8, 8, 2048)) < TOL[dt] / 2


def test_gemm_f32_epilogues(cuda):
    torch.manual_seed(5)
    L = lib()
    for (m, n, k) in [(128, 1024, 2048), (5, 128, 2048), (6, 128, 7), (1024, 2048, 130), (70, 6, 128)]:
        for ta in (0, 1):
            for tb in (0, 1):
                a = torch.randn(k, m) if ta else torch.randn(m, k)
                b = torch.randn(n, k) if tb else torch.randn(k, n)
                ref = (a.double().T if ta else a.double()) @ (b.double().T if tb else b.double())
                c = torch.empty(m, n, device=cuda)
                ag, bg = a.to(cuda), b.to(cuda)
                ws = torch.empty(max(16, L.dll.argus_gemm_f32_workspace_bytes(m, n, k)), dtype=torch.uint8, device=cuda)
                L.gemm_f32(m, n, k, ptr(ag), a.shape[1], ta, ptr(bg), b.shape[1], tb, ptr(c), n, None, 0, None, ptr(ws),
                           ws.numel(), stream())
                assert _rel(c, ref) < 1e-5, (m, n, k, ta, tb)
    m, n, k = 9, 33, 40
    a, b, bias = torch.randn(m, k), torch.randn(n, k), torch.randn(n)
    aux = torch.empty(m, n, device=cuda)
    c = torch.empty(m, n, device=cuda)
    ag, bg, biasg = a.to(cuda), b.to(cuda), bias.to(cuda)
    L.gemm_f32(m, n, k, ptr(ag), k, 0, ptr(bg), k, 1, ptr(c), n, ptr(biasg), 2, ptr(aux), None, 0, stream())
    pre = a.double() @ b.double().T + bias.double()
    assert _rel(aux, pre) < 1e-5 and _rel(c, F.gelu(pre)) < 1e-5
    g = torch.randn(m, n)
    pre_t = pre.clone().requires_grad_(True)
    F.gelu(pre_t).backward(g.double())
    # epilogue 3: C = (A @ B) * gelu'(aux): use A = g, B = I
    eye = torch.eye(n)
    gg, eyeg = g.to(cuda), eye.to(cuda)
    L.gemm_f32(m, n, n, ptr(gg), n, 0, ptr(eyeg), n, 0, ptr(c), n, None, 3, ptr(aux), None, 0, stream())
    assert _rel(c, pre_t.grad) < 1e-5
    cs = torch.empty(n, device=cuda)
    L.colsum_f32(m, n, ptr(gg), n, ptr(cs), stream())
    assert _rel(cs, g.double().sum(0)) < 1e-6


def test_se3_loss_kernel(cuda, golden):
    from oracle import se3

    L = lib()
    for kat in golden["loss_kats"]:
        p = torch.tensor([kat["pred"]], dtype=torch.float32)
        t = torch.tensor([kat["target"]], dtype=torch.float32)
        loss = torch.empty(1, device=cuda)
        pg, tg = p.to(cuda), t.to(cuda)
        L.se3_loss(1, ptr(pg), ptr(tg), ptr(loss), None, C.c_float(1.0), stream())
        assert abs(loss.item() - kat["loss"]) < 1e-5 * max(1.0, kat["loss"]), kat
    g = torch.Generator().manual_seed(6)
    for B, scale in [(64, 0.3), (257, 1.5), (5, 1e-6)]:
        pred = (torch.randn(B, 6, generator=g) * scale).float()
        T = se3.random_targets(B, generator=g)
        ref_l, ref_g = se3.loss_and_grad(pred, T, mean=True)
        loss = torch.empty(B, device=cuda)
        dpred = torch.empty(B, 6, device=cuda)
        pg, tg = pred.to(cuda), T.to(cuda)
        L.se3_loss(B, ptr(pg), ptr(tg), ptr(loss), ptr(dpred), C.c_float(1.0 / B), stream())
        assert (loss.cpu().double() - ref_l).abs().max() < 1e-5 * max(1.0, ref_l.abs().max().item())
        assert (dpred.cpu().double() - ref_g).abs().max() < 1e-6 + 1e-5 * ref_g.abs().max().item()
    # identity: loss(p, Exp(p)) == 0 (tests/test_train.py:32-36)
    pred = torch.randn(32, 6, generator=g).float()
    T = se3.se3_exp(pred.double()).float()
    loss = torch.empty(32, device=cuda)
    pg, tg = pred.to(cuda), T.to(cuda)
    L.se3_loss(32, ptr(pg), ptr(tg), ptr(loss), None, C.c_float(1.0), stream())
    assert loss.abs().max().item() < 1e-8 + 1e-5


def test_norm_and_adam(cuda):
    torch.manual_seed(7)
    L = lib()
    n = 1_000_003
    p0, g0 = torch.randn(n), torch.randn(n) * 1e-3
    ws = torch.empty(L.dll.argus_sumsq_workspace_bytes(n), dtype=torch.uint8, device=cuda)
    # pad to a 16-byte-aligned length (as the flat buffers are)
    pd, gd = p0.to(cuda), g0.to(cuda)
    norm = torch.empty(1, device=cuda)
    L.global_norm(n, ptr(gd), ptr(norm), ptr(ws), stream())
    assert abs(norm.item() - g0.double().norm().item()) < 1e-6 * g0.double().norm().item()
    m, v = torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    ref_p = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref_p], lr=1e-4)
    for step in range(1, 4):
        gs = g0 * (1.0 + 0.5 * step) * 100  # norm >> 1 -> clipping active
        ref_p.grad = gs.clone()
        torch.nn.utils.clip_grad_norm_([ref_p], 1.0)
        opt.step()
        gd = gs.to(cuda)
        L.global_norm(n, ptr(gd), ptr(norm), ptr(ws), stream())
        L.adam_step(n, ptr(pd), ptr(gd), ptr(m), ptr(v), ptr(norm), C.c_float(1.0), C.c_float(1.0), C.c_float(1e-4),
                    C.c_float(0.9),
                    C.c_float(0.999), C.c_float(1e-8), C.c_float(0.0), C.c_float(1 - 0.9**step),
                    C.c_float(1 - 0.999**step), stream())
    assert (pd.cpu() - ref_p.detach()).abs().max().item() < 2e-6


def test_kernel_timer_records_exact_instantiations(cuda):
    from argus_amd.profiling import KernelTimer

    L = lib()
    d, _ = _desc(4, 32, 32, 64, 128, 3, 1)
    x = torch.randn(4, 32, 32, 64, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(128, 3, 3, 64, device=cuda) * 0.05
    wf, wt = _prep(d, "bf16", w, cuda)
    y = torch.empty(4, 32, 32, 128, device=cuda, dtype=torch.bfloat16)
    with KernelTimer() as t:
        for _ in range(3):
            L.conv_fwd(C.byref(d), BF16, ptr(x), ptr(wf), ptr(y), None, None, None, stream())
    s = t.summary()
    assert len(s) == 1
    (name, v), = s.items()
    fl = C.c_int64()
    tag = L.dll.argus_conv_launch_info(C.byref(d), BF16, 0, C.byref(fl))
    bm, bn = divmod(tag % 1000000, 1000)
    # K = 576: the single-buffer kernel (OCC 4; 3 for the 128x128 tile) when K <= tuning key 7
    occ = (3 if bm == bn == 128 else 4) if 576 <= L.dll.argus_conv_policy_default(7) else 2
    assert name == f"argus::igemm_kernel<__bf16, {bm}, {bn}, false, false, {occ}, 0>"
    assert v["launches"] == 3 and v["flops_per_launch"] == fl.value and v["avg_us"] > 0
    assert v["bytes_per_launch"] == 2 * (4 * 32 * 32 * 64 + 128 * 9 * 64 + 4 * 32 * 32 * 128)
    with KernelTimer("argus::wgrad") as t:  # filtered out: nothing recorded
        L.conv_fwd(C.byref(d), BF16, ptr(x), ptr(wf), ptr(y), None, None, None, stream())
    assert t.summary() == {}
    L.conv_fwd(C.byref(d), BF16, ptr(x), ptr(wf), ptr(y), None, None, None, stream())  # disabled: plain launch
    torch.cuda.synchronize()


GLDS_SHAPES = [  # (cin, cout, k, s, hin, n): M >= 1024 rows so the glds kernel is eligible
    (64, 64, 3, 1, 24, 2), (128, 128, 3, 2, 25, 2), (512, 256, 1, 1, 24, 2), (256, 512, 1, 2, 32, 2),
    (64, 128, 3, 1, 20, 3), (576, 64, 1, 1, 23, 2),
]


def test_conv_glds_kernel_parity(cuda):
    """The bf16 global->LDS implicit-GEMM kernel (forced on with tuning key 8) vs torch: forward with
    BN-statistic partials (M tails, 2 x 128-row halves per 256-row tile), dgrad over stride phases,
    in-place and masked addends; the kernel timer confirms it ran."""
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(11)
    L = lib()
    for cin, cout, k, s, hin, n in GLDS_SHAPES:
        d, p = _desc(n, hin, hin, cin, cout, k, s)
        d = d.with_tuning({8: 64, 9: 1})
        x = torch.randn(n, hin, hin, cin)
        w = torch.randn(cout, k, k, cin) * (2.0 / (k * k * cin)) ** 0.5
        dy = torch.randn(n, d.ho, d.wo, cout)
        xd, dyd = x.to(cuda, torch.bfloat16), dy.to(cuda, torch.bfloat16)
        wf, wt = _prep(d, "bf16", w.to(cuda), cuda)
        y = torch.empty(n, d.ho, d.wo, cout, dtype=torch.bfloat16, device=cuda)
        rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), BF16)
        stats = torch.empty(rows, cout, 2, device=cuda)
        with KernelTimer("argus::igemm_glds_kernel") as t:
            L.conv_fwd(C.byref(d), BF16, ptr(xd), ptr(wf), ptr(y), None, None, ptr(stats), stream())
        M = n * d.ho * d.wo
        if M >= 1024 and k * k * cin >= 64 and cout % 128 == 0:
            assert len(t.summary()) == 1, (cin, cout, k, s, hin)
        xr, wr, dyr = _q(x, "bf16").permute(0, 3, 1, 2), _q(w, "bf16").permute(0, 3, 1, 2), _q(dy, "bf16").permute(0, 3, 1, 2)
        ref = F.conv2d(xr, wr, stride=s, padding=p)
        assert _rel(y.permute(0, 3, 1, 2), ref) < TOL["bf16"], ("fwd", cin, cout, k, s)
        tile = L.dll.argus_conv_fwd_stat_tile(C.byref(d), BF16)
        mean, var = _merge_stats(stats.double().cpu(), tile, M)
        yr = ref.permute(0, 2, 3, 1).reshape(-1, cout)
        assert (mean - yr.mean(0)).abs().max() < 2e-2 * yr.std(0).max(), ("stats mean", cin, cout)
        assert _rel(var, yr.var(0, unbiased=False)) < 2e-2, ("stats var", cin, cout)
        # dgrad: plain, in-place accumulate, masked addend from another buffer
        dx0 = torch.randn(n, hin, hin, cin)
        dx = dx0.to(cuda, torch.bfloat16)
        L.conv_dgrad(C.byref(d), BF16, ptr(dyd), ptr(wt), ptr(dx), ptr(dx), None, stream())
        refd = torch.nn.grad.conv2d_input(xr.shape, wr, dyr, stride=s, padding=p)
        assert _rel(dx.permute(0, 3, 1, 2), refd + _q(dx0, "bf16").permute(0, 3, 1, 2)) < TOL["bf16"], ("dgrad+", cin)
        res = _q(torch.randn(n, hin, hin, cin), "bf16")
        keep = res > 0
        bits = ((keep.reshape(-1, 8).int() << torch.arange(8)).sum(1)).to(torch.uint8).to(cuda)
        resg = res.to(cuda, torch.bfloat16)
        L.conv_dgrad(C.byref(d), BF16, ptr(dyd), ptr(wt), ptr(dx), ptr(resg), ptr(bits), stream())
        assert _rel(dx.permute(0, 3, 1, 2), refd + (res * keep).permute(0, 3, 1, 2)) < TOL["bf16"], ("dgrad mask", cin)


HALO_SHAPES = [  # (cin, cout, hw, n): 256-pixel tiles = 4 rows / 8 rows / 1 image / 4 images
    (64, 64, 64, 1), (128, 128, 32, 1), (64, 128, 16, 2), (256, 256, 16, 1), (128, 64, 8, 4), (512, 512, 8, 4),
]


@pytest.mark.parametrize("deep", [0, 1])
def test_conv3x3_halo_kernel_parity(cuda, deep):
    """3x3 stride-1 LDS-halo kernel vs torch (bf16): forward with BN partials at 64- and 128-row tiles,
    dgrad with in-place and masked addends; the kernel timer confirms the halo kernel served every
    call, and a forward with a BN+ReLU prologue (bf16 inputs are materialised by the benched schedule)
    is served by the register-staged kernel instead. deep = policy key 51 (the four-stage weight ring on
    384-position halo images where the halo fits)."""
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(13)
    L = lib()
    _halo_cases(L, cuda, {13: 1, 51: deep})  # force the halo kernel on every eligible shape


def test_halo_deep_ring_bit_identical(cuda):
    """Policy key 51 (conv_halo.hip: 384-position halo images, four weight stages in the ring) changes
    only how far ahead the weight taps are fetched: the forward's y and BN partials, and the data
    gradient's dm, BN-backward partials and folded finalize outputs are bit-identical to the
    three-stage kernel's, and the deep instantiation ran where the halo fits (<= 384 positions)."""
    from argus_amd._lib import BnBwdEpilogue
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(51)
    L = lib()
    # both passes on 128-column tiles (cin and cout % 128): the deep variant serves both
    for cin, cout, hw, n in [(128, 128, 32, 2), (256, 256, 16, 2), (128, 256, 32, 1), (256, 128, 16, 3)]:
        d0, _ = _desc(n, hw, hw, cin, cout, 3, 1)
        w = torch.randn(cout, 3, 3, cin) * (2.0 / (9 * cin)) ** 0.5
        x = (torch.randn(n, hw, hw, cin) * 1.5 + 0.2).to(cuda, torch.bfloat16)
        dy = torch.randn(n, hw, hw, cout).to(cuda, torch.bfloat16)
        yb = torch.randn(n, hw, hw, cin).to(cuda, torch.bfloat16)
        mean, invstd = torch.randn(cin, device=cuda) * 0.1, torch.rand(cin, device=cuda) + 0.5
        sc, sh = torch.randn(cin, device=cuda), torch.randn(cin, device=cuda)
        gamma = torch.rand(cin, device=cuda) + 0.5
        outs = []
        for key in (0, 1):
            d = d0.with_tuning({13: 1, 51: key})
            wf, wt = _prep(d, "bf16", w.to(cuda), cuda)
            rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), BF16)
            stats = torch.zeros(rows, cout, 2, device=cuda)
            y = torch.empty(n, hw, hw, cout, dtype=torch.bfloat16, device=cuda)
            brows = L.dll.argus_conv_dgrad_bn_rows(C.byref(d), BF16)
            part = torch.zeros(brows, cin, 2, device=cuda)
            ws = torch.zeros(L.dll.argus_bn_workspace_bytes(cin), dtype=torch.uint8, device=cuda)
            fin = torch.full((5, cin), float("nan"), device=cuda)
            dm = torch.empty(n, hw, hw, cin, dtype=torch.bfloat16, device=cuda)
            e = BnBwdEpilogue()
            e.y, e.mean, e.invstd, e.mask_mode, e.scale, e.shift, e.part = ptr(yb), ptr(mean), ptr(invstd), 2, \
                ptr(sc), ptr(sh), ptr(part)
            e.workspace, e.gamma = ptr(ws), ptr(gamma)
            e.dgamma, e.dbeta, e.ca, e.cb, e.cc = (ptr(fin[i]) for i in range(5))
            with KernelTimer("argus::conv3x3_halo_kernel") as t:
                L.conv_fwd(C.byref(d), BF16, ptr(x), ptr(wf), ptr(y), None, None, ptr(stats), stream())
                L.conv_dgrad_bn(C.byref(d), BF16, ptr(dy), ptr(wt), ptr(dm), None, C.byref(e), None, stream())
            torch.cuda.synchronize()
            names = list(t.summary())
            assert len(names) == 2 and all(nm.endswith(", true>" if key else ", false>") for nm in names), names
            outs.append((y.view(torch.int16).cpu(), stats.cpu(), dm.view(torch.int16).cpu(), part.cpu(), fin.cpu()))
        for a, b in zip(*outs):
            assert torch.equal(a, b), (cin, cout, hw, n)


def test_layer1_3x3_on_single_buffer_halo_kernel(cuda):
    """Default kernel policy for the 64 -> 64 channel 3x3 stride-1 layers of layer 1 at a grid the
    policy accepts (>= 256 workgroups): forward and dgrad run on the single-halo-buffer 64-column halo
    kernel and agree with torch (bf16 tolerance) and with the register-staged implicit GEMM it
    replaces (policy key 10 = 0: halo kernel off)."""
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(31)
    L = lib()
    n, hw, c = 16, 64, 64
    d, p = _desc(n, hw, hw, c, c, 3, 1)
    x = torch.randn(n, hw, hw, c)
    w = torch.randn(c, 3, 3, c) * (2.0 / (9 * c)) ** 0.5
    dy = torch.randn(n, hw, hw, c)
    wf, wt = _prep(d, "bf16", w.to(cuda), cuda)
    xd, dyd = x.to(cuda, torch.bfloat16), dy.to(cuda, torch.bfloat16)
    xr, wr = _q(x, "bf16").permute(0, 3, 1, 2), _q(w, "bf16").permute(0, 3, 1, 2)
    ref_y = F.conv2d(xr, wr, padding=1).permute(0, 2, 3, 1)
    ref_dx = torch.nn.grad.conv2d_input(xr.shape, wr, _q(dy, "bf16").permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)
    outs = {}
    for key10, kname in ((1, "conv3x3_halo_kernel<64, 0, 1,"), (0, "igemm_kernel")):
        dk = d.with_tuning({10: key10})
        rows = L.dll.argus_conv_fwd_stat_rows(C.byref(dk), BF16)
        stats = torch.empty(rows, c, 2, device=cuda)
        y = torch.empty(n, hw, hw, c, dtype=torch.bfloat16, device=cuda)
        dx = torch.empty(n, hw, hw, c, dtype=torch.bfloat16, device=cuda)
        with KernelTimer() as t:
            L.conv_fwd(C.byref(dk), BF16, ptr(xd), ptr(wf), ptr(y), None, None, ptr(stats), stream())
            L.conv_dgrad(C.byref(dk), BF16, ptr(dyd), ptr(wt), ptr(dx), None, None, stream())
        torch.cuda.synchronize()
        names = list(t.summary())
        assert any(kname in nm for nm in names), (key10, names)
        if key10:
            assert any("conv3x3_halo_kernel<64, 0, 1," in nm for nm in names) and len(names) == 1, names
        assert _rel(y, ref_y) < TOL["bf16"] and _rel(dx, ref_dx) < TOL["bf16"], key10
        outs[key10] = (y.float(), dx.float())
    assert _rel(outs[1][0], outs[0][0]) < 1e-2 and _rel(outs[1][1], outs[0][1]) < 1e-2


def _halo_cases(L, cuda, tuning):
    from argus_amd.profiling import KernelTimer

    for cin, cout, hw, n in HALO_SHAPES:
        d, p = _desc(n, hw, hw, cin, cout, 3, 1)
        d = d.with_tuning(tuning)
        x = torch.randn(n, hw, hw, cin) * 1.5 + 0.2
        w = torch.randn(cout, 3, 3, cin) * (2.0 / (9 * cin)) ** 0.5
        sc, sh = torch.rand(cin) + 0.5, torch.randn(cin) * 0.5
        xd, scd, shd = x.to(cuda, torch.bfloat16), sc.to(cuda), sh.to(cuda)
        wf, wt = _prep(d, "bf16", w.to(cuda), cuda)
        xr, wr = _q(x, "bf16").permute(0, 3, 1, 2), _q(w, "bf16").permute(0, 3, 1, 2)
        rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), BF16)
        tile = L.dll.argus_conv_fwd_stat_tile(C.byref(d), BF16)
        M = n * hw * hw
        for pro in (False, True):
            y = torch.empty(n, hw, hw, cout, dtype=torch.bfloat16, device=cuda)
            stats = torch.empty(rows, cout, 2, device=cuda)
            with KernelTimer("argus::conv3x3_halo_kernel") as t:
                L.conv_fwd(C.byref(d), BF16, ptr(xd), ptr(wf), ptr(y), ptr(scd) if pro else None,
                           ptr(shd) if pro else None, ptr(stats), stream())
            assert len(t.summary()) == (0 if pro else 1), ("halo kernel use", cin, cout, hw, n, pro)
            xin = torch.relu(xr * sc[None, :, None, None] + sh[None, :, None, None]) if pro else xr
            xin = _q(xin.permute(0, 2, 3, 1), "bf16").permute(0, 3, 1, 2) if pro else xin
            ref = F.conv2d(xin, wr, padding=1)
            assert _rel(y.permute(0, 3, 1, 2), ref) < TOL["bf16"], ("fwd", cin, cout, hw, pro)
            mean, var = _merge_stats(stats.double().cpu(), tile, M)
            yr = ref.permute(0, 2, 3, 1).reshape(-1, cout)
            assert (mean - yr.mean(0)).abs().max() < 2e-2 * yr.std(0).max(), ("stats mean", cin, cout, hw)
            assert _rel(var, yr.var(0, unbiased=False)) < 2e-2, ("stats var", cin, cout, hw)
        dy = torch.randn(n, hw, hw, cout)
        dyd = dy.to(cuda, torch.bfloat16)
        refd = torch.nn.grad.conv2d_input(xr.shape, wr, _q(dy, "bf16").permute(0, 3, 1, 2), padding=1)
        dx0 = _q(torch.randn(n, hw, hw, cin), "bf16")
        dx = dx0.to(cuda, torch.bfloat16)
        with KernelTimer("argus::conv3x3_halo_kernel") as t:
            L.conv_dgrad(C.byref(d), BF16, ptr(dyd), ptr(wt), ptr(dx), ptr(dx), None, stream())
        assert len(t.summary()) == 1, ("halo dgrad not used", cin, cout, hw, n)
        assert _rel(dx.permute(0, 3, 1, 2), refd + dx0.permute(0, 3, 1, 2)) < TOL["bf16"], ("dgrad+", cin, cout, hw)
        keep = dx0 > 0
        bits = ((keep.reshape(-1, 8).int() << torch.arange(8)).sum(1)).to(torch.uint8).to(cuda)
        res = dx0.to(cuda, torch.bfloat16)
        L.conv_dgrad(C.byref(d), BF16, ptr(dyd), ptr(wt), ptr(dx), ptr(res), ptr(bits), stream())
        assert _rel(dx.permute(0, 3, 1, 2), refd + (dx0 * keep).permute(0, 3, 1, 2)) < TOL["bf16"], ("dgrad m", cin)


@pytest.mark.parametrize("dt", ["fp32", "bf16", "fp8"])
def test_weight_prep_batch_matches_single(cuda, dt):
    L = lib()
    torch.manual_seed(17)
    convs = [_desc(2, 16, 16, 3, 64, 7, 2, stem=True)[0], _desc(2, 8, 8, 64, 128, 3, 1)[0],
             _desc(2, 8, 8, 256, 64, 1, 1)[0], _desc(2, 8, 8, 128, 128, 3, 2)[0]]  # fp8: fwd / dgrad / both
    masters, single, batch = [], [], []
    for i, d in enumerate(convs):
        w = torch.randn(d.k, d.c, d.r, d.s, device=cuda)  # OIHW contiguous (strided as OHWI)
        if i == 3:
            w = w.to(memory_format=torch.channels_last)   # OHWI-contiguous storage
        masters.append(w)
        shape_f = (d.k, 256) if d.stem else (d.k, d.r * d.s * d.c)
        pair = []
        for _ in range(2):
            wf = torch.empty(shape_f, dtype=TDT[dt], device=cuda)
            wd = None if d.stem else torch.empty(d.c, d.r * d.s * d.k, dtype=TDT[dt], device=cuda)
            pair.append((wf, wd))
        single.append(pair[0])
        batch.append(pair[1])
        st = (C.c_int64 * 4)(w.stride(0), w.stride(1), w.stride(2), w.stride(3))
        L.conv_weight_prep(C.byref(d), DT[dt], ptr(w), st, ptr(pair[0][0]), ptr(pair[0][1]), stream())
    n = len(convs)
    descs = (ConvDesc * n)(*convs)
    ms = (C.c_void_p * n)(*[w.data_ptr() for w in masters])
    strides = (C.c_int64 * (4 * n))(*[w.stride(j) for w in masters for j in range(4)])
    wfs = (C.c_void_p * n)(*[b[0].data_ptr() for b in batch])
    wds = (C.c_void_p * n)(*[b[1].data_ptr() if b[1] is not None else None for b in batch])
    nbytes = L.dll.argus_conv_weight_prep_table_bytes(n)
    host = (C.c_uint8 * nbytes)()
    nblk = C.c_int(0)
    L.conv_weight_prep_table(n, descs, ms, strides, wfs, wds, host, nbytes, C.byref(nblk))
    table = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(cuda)
    L.conv_weight_prep_batch(DT[dt], n, ptr(table), nblk.value, stream())
    torch.cuda.synchronize()
    for d, (sf, sd), (bf, bd) in zip(convs, single, batch):
        if dt == "fp8":  # bytes in use: e4m3 values + E8M0 scales of the fp8 passes, bf16 otherwise
            def used(t, rows, cols, f8):
                return t.view(torch.uint8).reshape(-1)[: rows * cols + rows * cols // 32] if f8 else t.view(torch.uint8)
            cols_f = 256 if d.stem else d.r * d.s * d.c
            assert torch.equal(used(sf, d.k, cols_f, not d.stem and d.c % 128 == 0),
                               used(bf, d.k, cols_f, not d.stem and d.c % 128 == 0))
            if sd is not None:
                f8d = d.k % 128 == 0
                assert torch.equal(used(sd, d.c, d.r * d.s * d.k, f8d), used(bd, d.c, d.r * d.s * d.k, f8d))
            continue
        assert torch.equal(sf, bf)
        assert (sd is None and bd is None) or torch.equal(sd, bd)


@pytest.mark.parametrize("pro", [False, True])
def test_wgrad3x3_halo_kernel_parity(cuda, pro):
    """3x3 stride-1 weight gradient through the LDS-halo kernel vs torch (bf16 inputs, fp32 dW); with
    a BN+ReLU prologue on the input (not a benched schedule: bf16 inputs are materialised) the
    register-staged kernel serves it. The kernel timer confirms which kernel ran."""
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(19)
    L = lib()
    # every channel-tile count (key 14); the default split target (mostly one tile per split) and a
    # target of 3 workgroups per (k, c) tile (long tile runs: the 3-stage ring's steady state, its
    # drain and ragged run lengths)
    for tg in (L.dll.argus_conv_policy_default(12), 3):
        _wgrad_halo_cases(L, cuda, pro, {14: 1 << 20, 12: tg})


def _wgrad_halo_cases(L, cuda, pro, tuning):
    from argus_amd.profiling import KernelTimer

    # square frames: whole-row tiles / whole images; 84-, 168- and 21-wide frames (the 376 x 672
    # layers' widths): 3 x 42, 2 x 56 and 6 x 21 blocks, ragged last row blocks
    for cin, cout, hw, n in [(64, 64, 64, 1), (128, 128, 32, 1), (64, 128, 16, 2), (128, 64, 8, 4), (256, 128, 16, 1),
                             (64, 64, (10, 84), 1), (128, 128, (7, 168), 1), (64, 64, (12, 21), 2),
                             (128, 128, (47, 84), 1)]:
        hh, ww = hw if isinstance(hw, tuple) else (hw, hw)
        d, p = _desc(n, hh, ww, cin, cout, 3, 1)
        d = d.with_tuning(tuning)
        x = _q(torch.randn(n, hh, ww, cin) * 1.3 + 0.1, "bf16")
        dy = _q(torch.randn(n, hh, ww, cout), "bf16")
        sc, sh = torch.rand(cin) + 0.5, torch.randn(cin) * 0.5
        xg, dyg, scg, shg = x.to(cuda, torch.bfloat16), dy.to(cuda, torch.bfloat16), sc.to(cuda), sh.to(cuda)
        dw = torch.empty(cout, 3, 3, cin, device=cuda)
        wsb = L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), BF16)
        ws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
        with KernelTimer("argus::wgrad3x3_halo_kernel") as t:
            L.conv_wgrad(C.byref(d), BF16, ptr(xg), ptr(scg) if pro else None, ptr(shg) if pro else None, ptr(dyg),
                         ptr(dw), ptr(ws), wsb, stream())
        assert len(t.summary()) == (0 if pro else 1), ("halo wgrad use", cin, cout, hw, n, pro)
        xin = x.permute(0, 3, 1, 2)
        if pro:
            xin = _q(torch.relu(xin * sc[None, :, None, None] + sh[None, :, None, None]).permute(0, 2, 3, 1),
                     "bf16").permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_weight(xin.double(), (cout, cin, 3, 3), dy.permute(0, 3, 1, 2).double(), padding=1)
        assert _rel(dw.permute(0, 3, 1, 2), ref) < 2e-3, ("wgrad", cin, cout, hw, n, pro)


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_conv_large_tile_small_k(cuda, dt):
    """1x1 convs with K <= 128 on 128-row tiles (M >= 16K): the single-buffer small-K kernel, whose
    epilogue stages half a C tile (fp32: 64 x 132 floats) in its LDS array."""
    torch.manual_seed(23)
    L = lib()
    for cin, cout in ((64, 128), (64, 256), (128, 64)):
        n, hw = 4, 64
        d, p = _desc(n, hw, hw, cin, cout, 1, 1)
        x = torch.randn(n, hw, hw, cin)
        w = torch.randn(cout, 1, 1, cin) * (1.0 / cin) ** 0.5
        xd = x.to(cuda, TDT[dt])
        wf, wt = _prep(d, dt, w.to(cuda), cuda)
        y = torch.empty(n, hw, hw, cout, dtype=TDT[dt], device=cuda)
        rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), DT[dt])
        stats = torch.empty(rows, cout, 2, device=cuda)
        L.conv_fwd(C.byref(d), DT[dt], ptr(xd), ptr(wf), ptr(y), None, None, ptr(stats), stream())
        ref = F.conv2d(_q(x, dt).permute(0, 3, 1, 2), _q(w, dt).permute(0, 3, 1, 2))
        assert _rel(y.permute(0, 3, 1, 2), ref) < TOL[dt], (dt, cin, cout)
        tile = L.dll.argus_conv_fwd_stat_tile(C.byref(d), DT[dt])
        mean, var = _merge_stats(stats.double().cpu(), tile, n * hw * hw)
        yr = ref.permute(0, 2, 3, 1).reshape(-1, cout)
        assert _rel(var, yr.var(0, unbiased=False)) < (1e-4 if dt == "fp32" else 2e-2), (dt, cin, cout)


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_images_u8_layout_matches_fp32_path(cuda, dt):
    """uint8 input path (CameraCubePoseDataset(uint8=True)): the device-side /255 equals the
    reference's host `.to(torch.float32) / 255.0` (argus/data.py:214-215) bit for bit, and the NHWC4
    layout (camera fold of argus/models.py:81, zero 4th channel) matches the fp32 entry point."""
    L = lib()
    g = torch.Generator().manual_seed(5)
    B, H, W = 3, 7, 11  # ragged sizes: the grid-stride loop's tail
    u8 = torch.randint(0, 256, (B, 6, H, W), generator=g, dtype=torch.uint8)
    f32 = u8.to(torch.float32) / 255.0
    N = 2 * B
    out_u8 = torch.full((N, H, W, 4), 7.0, dtype=TDT[dt], device=cuda)
    out_f = torch.full((N, H, W, 4), 7.0, dtype=TDT[dt], device=cuda)
    L.images_u8_to_nhwc4(DT[dt], N, H, W, ptr(u8.to(cuda)), ptr(out_u8), stream())
    L.images_to_nhwc4(DT[dt], N, H, W, ptr(f32.to(cuda)), ptr(out_f), stream())
    torch.cuda.synchronize()
    want = torch.zeros(N, H, W, 4, dtype=torch.float32)
    want[..., :3] = f32.reshape(N, 3, H, W).permute(0, 2, 3, 1)
    assert torch.equal(out_u8.cpu(), want.to(TDT[dt]))
    assert torch.equal(out_f.cpu(), want.to(TDT[dt]))


# (cin, cout, k, stride, hin, n, tuning, kernel the dgrad lands on)
DGRAD_BN_CASES = [
    (64, 64, 3, 1, 16, 2, {13: 1}, "conv3x3_halo_kernel<64"),
    (128, 128, 3, 1, 16, 2, {13: 1}, "conv3x3_halo_kernel<128"),
    (128, 256, 1, 1, 32, 2, {8: 64, 9: 1}, "igemm_glds_kernel"),
    (128, 128, 3, 2, 11, 2, {}, "igemm_kernel"),
    (256, 512, 1, 2, 9, 2, {}, "igemm_kernel"),     # stride-2 1x1: three phases with no taps
    (64, 256, 1, 1, 12, 3, {}, "igemm_kernel"),
]


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_conv_dgrad_bn_epilogue(cuda, dt):
    """argus_conv_dgrad_bn: dm = (dgrad + addend) * relu-mask and the BN-backward column partials
    {sum dm, sum dm*xhat} (+ the second, downsample branch) vs fp64 torch, on every kernel family the
    dgrad can land on (halo, glds, register-staged with strided phases and empty phases)."""
    from argus_amd._lib import BnBwdEpilogue
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(5)
    L = lib()
    for cin, cout, k, s, hin, n, tune, kname in DGRAD_BN_CASES:
        if dt == "fp32" and kname != "igemm_kernel":
            continue  # halo / glds are bf16 kernels
        d, p = _desc(n, hin, hin, cin, cout, k, s)
        w = torch.randn(cout, k, k, cin) * (2.0 / (k * k * cin)) ** 0.5
        wf, wt = _prep(d, dt, w.to(cuda), cuda)
        dy = torch.randn(n, d.ho, d.wo, cout)
        y = torch.randn(n, hin, hin, cin) * 2 + 0.3
        y2 = torch.randn(n, hin, hin, cin)
        mean, invstd = torch.randn(cin) * 0.1 + 0.3, torch.rand(cin) + 0.5
        mean2, invstd2 = torch.randn(cin) * 0.1, torch.rand(cin) + 0.5
        sc, sh = torch.randn(cin), torch.randn(cin) * 0.5
        for mode, dual, with_add in ((2, False, False), (3, False, True), (3, True, True)):
            add = torch.randn(n, hin, hin, cin)
            bits_t = torch.randint(0, 256, (n * hin * hin * cin // (8 if dt == "bf16" else 4),), dtype=torch.uint8)
            g = {t: v.to(cuda) for t, v in dict(mean=mean, invstd=invstd, sc=sc, sh=sh, mean2=mean2,
                                                 invstd2=invstd2).items()}
            yg, y2g = y.to(cuda, TDT[dt]), y2.to(cuda, TDT[dt])
            dm = add.to(cuda, TDT[dt]) if with_add else torch.empty(n, hin, hin, cin, dtype=TDT[dt], device=cuda)
            bitsg = bits_t.to(cuda)
            dk = d.with_tuning(tune)  # the row count depends on the kernel the tuning selects
            rows = L.dll.argus_conv_dgrad_bn_rows(C.byref(dk), DT[dt])
            part = torch.full((rows, cin, 2), float("nan"), device=cuda)
            part2 = torch.full((rows, cin, 2), float("nan"), device=cuda)
            e = BnBwdEpilogue()
            e.y, e.mean, e.invstd, e.mask_mode, e.part = ptr(yg), ptr(g["mean"]), ptr(g["invstd"]), mode, ptr(part)
            if mode == 2:
                e.scale, e.shift = ptr(g["sc"]), ptr(g["sh"])
            else:
                e.mask_bits = ptr(bitsg)
            if dual:
                e.y2, e.mean2, e.invstd2, e.part2 = ptr(y2g), ptr(g["mean2"]), ptr(g["invstd2"]), ptr(part2)
            dyg = dy.to(cuda, TDT[dt])
            with KernelTimer() as kt:
                L.conv_dgrad_bn(C.byref(dk), DT[dt], ptr(dyg), ptr(wt), ptr(dm), ptr(dm) if with_add else None,
                                C.byref(e), None, stream())
            torch.cuda.synchronize()
            assert any(kname in nm for nm in kt.summary()), (kname, list(kt.summary()))
            # reference
            v = torch.nn.grad.conv2d_input((n, cin, hin, hin), _q(w, dt).permute(0, 3, 1, 2),
                                           _q(dy, dt).permute(0, 3, 1, 2), stride=s, padding=p).permute(0, 2, 3, 1)
            if with_add:
                v = v + _q(add, dt)
            yq, y2q = _q(y, dt), _q(y2, dt)
            if mode == 2:
                mask = (yq * sc.double() + sh.double()) > 0
            else:
                E = 8 if dt == "bf16" else 4
                bb = bits_t.long().repeat_interleave(E).reshape(n, hin, hin, cin)
                shift = torch.arange(cin) % E
                mask = ((bb >> shift) & 1).bool()
            ref = v * mask
            got = dm.double().cpu()
            err = _rel(got, ref)
            assert err < TOL[dt], (cin, cout, k, s, mode, dt, err)
            # partials, from the stored dm (what the apply pass will read)
            xh = (yq - mean.double()) * invstd.double()
            S, T_ = got.sum((0, 1, 2)), (got * xh).sum((0, 1, 2))
            pc = part.double().cpu().sum(0)
            scale = got.abs().sum((0, 1, 2)).max()
            tol = 1e-5 if dt == "fp32" else 1e-4
            assert (pc[:, 0] - S).abs().max() <= tol * scale and (pc[:, 1] - T_).abs().max() <= tol * scale * 4, \
                (cin, cout, mode, dt)
            if dual:
                xh2 = (y2q - mean2.double()) * invstd2.double()
                pc2 = part2.double().cpu().sum(0)
                assert (pc2[:, 1] - (got * xh2).sum((0, 1, 2))).abs().max() <= tol * scale * 4
                assert (pc2[:, 0] - S).abs().max() <= tol * scale


FOLD_CASES = [  # (cin, cout, k, stride, hin, n, tuning): dgrad kernels igemm / halo / glds / strided phases
    (64, 256, 1, 1, 40, 4, {}),
    (128, 128, 3, 1, 16, 4, {13: 1}),
    (256, 256, 1, 1, 32, 2, {8: 64, 9: 1}),
    (128, 128, 3, 2, 21, 3, {}),
]


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_folded_bn_finalize_matches_separate_kernels(cuda, dt):
    """argus_conv_dgrad_bn(workspace): the BN-backward finalize folded into the producing dgrad launch
    (two-level ticket merge) gives what argus_bn_bwd_finalize gives from the same partials, up to fp64
    summation order (1e-6 relative), and leaves its counters at zero; dgrad kernels igemm / halo /
    glds, strided phases."""
    from argus_amd._lib import BnBwdEpilogue

    torch.manual_seed(9)
    L = lib()
    ws_bytes = L.dll.argus_bn_workspace_bytes(2048)
    for cin, cout, k, s, hin, n, tune in FOLD_CASES:
        if dt == "fp32" and tune:
            continue
        d, p = _desc(n, hin, hin, cin, cout, k, s)
        w = torch.randn(cout, k, k, cin) * (2.0 / (k * k * cin)) ** 0.5
        wf, wt = _prep(d, dt, w.to(cuda), cuda)
        # backward: dgrad_bn with the finalize folded vs bn_bwd_finalize on its partials
        dy = torch.randn(n, d.ho, d.wo, cout, device=cuda).to(TDT[dt])
        yb = torch.randn(n, hin, hin, cin, device=cuda).to(TDT[dt])
        mean, invstd = torch.randn(cin, device=cuda) * 0.1, torch.rand(cin, device=cuda) + 0.5
        sc, sh = torch.randn(cin, device=cuda), torch.randn(cin, device=cuda)
        g_in = torch.rand(cin, device=cuda) + 0.5
        res = []
        dk = d.with_tuning(tune)
        brows = L.dll.argus_conv_dgrad_bn_rows(C.byref(dk), DT[dt])
        for folded in (False, True):
            ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=cuda)
            part = torch.empty(brows, cin, 2, device=cuda)
            dm = torch.empty(n, hin, hin, cin, dtype=TDT[dt], device=cuda)
            co = torch.zeros(5, cin, device=cuda)
            e = BnBwdEpilogue()
            e.y, e.mean, e.invstd, e.mask_mode, e.scale, e.shift, e.part = ptr(yb), ptr(mean), ptr(invstd), 2, \
                ptr(sc), ptr(sh), ptr(part)
            if folded:
                e.workspace, e.gamma, e.dgamma, e.dbeta = ptr(ws), ptr(g_in), ptr(co[3]), ptr(co[4])
                e.ca, e.cb, e.cc = ptr(co[0]), ptr(co[1]), ptr(co[2])
            L.conv_dgrad_bn(C.byref(dk), DT[dt], ptr(dy), ptr(wt), ptr(dm), None, C.byref(e), None, stream())
            if not folded:
                L.bn_bwd_finalize(cin, brows, ptr(part), n * hin * hin, ptr(g_in), ptr(mean), ptr(invstd),
                                  ptr(co[3]), ptr(co[4]), ptr(co[0]), ptr(co[1]), ptr(co[2]), ptr(ws), stream())
            torch.cuda.synchronize()
            assert int(ws[:16384].view(torch.int32).abs().sum()) == 0
            res.append((dm.cpu(), co.cpu()))
        assert torch.equal(res[0][0], res[1][0])
        assert _rel(res[0][1], res[1][1]) < 1e-6, (cin, cout, k, s, dt)



@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_dgrad_apply_prologue_matches_apply_pass(cuda, dt):
    """argus_conv_dgrad_bn with an argus_bn_bwd_prologue (the dgrad stages dy = ca*dm + cb*y + cc from
    dm and stores dy): bit-identical dy and dgrad output to argus_bn_bwd_apply + a plain dgrad, on the
    register-staged kernel (strided phases included) and on the LDS-DMA kernels (library fallback),
    with and without a BN-backward epilogue."""
    from argus_amd._lib import BnBwdEpilogue, BnBwdPrologue

    torch.manual_seed(12)
    L = lib()
    for cin, cout, k, s, hin, n, tune, kname in DGRAD_BN_CASES:
        if dt == "fp32" and kname != "igemm_kernel":
            continue
        d, p = _desc(n, hin, hin, cin, cout, k, s)
        w = torch.randn(cout, k, k, cin) * (2.0 / (k * k * cin)) ** 0.5
        _, wt = _prep(d, dt, w.to(cuda), cuda)
        dm = torch.randn(n, d.ho, d.wo, cout, device=cuda).to(TDT[dt])
        yb = torch.randn(n, d.ho, d.wo, cout, device=cuda).to(TDT[dt])
        ca, cb, cc = (torch.randn(cout, device=cuda) * 0.3 for _ in range(3))
        yin = torch.randn(n, hin, hin, cin, device=cuda).to(TDT[dt])
        mean, invstd = torch.randn(cin, device=cuda) * 0.1, torch.rand(cin, device=cuda) + 0.5
        sc, sh = torch.randn(cin, device=cuda), torch.randn(cin, device=cuda)
        for with_epi in (False, True):
            outs = []
            for fused in (False, True):
                dk = d.with_tuning(tune)
                rows = L.dll.argus_conv_dgrad_bn_rows(C.byref(dk), DT[dt])
                part = torch.zeros(rows, cin, 2, device=cuda)
                e = BnBwdEpilogue()
                e.y, e.mean, e.invstd, e.mask_mode, e.scale, e.shift, e.part = ptr(yin), ptr(mean), ptr(invstd), \
                    2, ptr(sc), ptr(sh), ptr(part)
                dy = torch.zeros(n, d.ho, d.wo, cout, device=cuda, dtype=TDT[dt])
                dx = torch.empty(n, hin, hin, cin, device=cuda, dtype=TDT[dt])
                if fused:
                    pro = BnBwdPrologue(ptr(yb), ptr(ca), ptr(cb), ptr(cc), ptr(dy))
                    L.conv_dgrad_bn(C.byref(dk), DT[dt], ptr(dm), ptr(wt), ptr(dx), None,
                                    C.byref(e) if with_epi else None, C.byref(pro), stream())
                else:
                    L.bn_bwd_apply(DT[dt], n * d.ho * d.wo, cout, ptr(dm), 0, None, ptr(yb), None, None, ptr(ca),
                                   ptr(cb), ptr(cc), ptr(dy), None, None, None, None, None, None, stream())
                    if with_epi:
                        L.conv_dgrad_bn(C.byref(dk), DT[dt], ptr(dy), ptr(wt), ptr(dx), None, C.byref(e), None,
                                        stream())
                    else:
                        L.conv_dgrad(C.byref(dk), DT[dt], ptr(dy), ptr(wt), ptr(dx), None, None, stream())
                torch.cuda.synchronize()
                outs.append((dy.cpu(), dx.cpu(), part.cpu()))
            (y0, x0, p0), (y1, x1, p1) = outs
            assert torch.equal(y0, y1), (cin, cout, k, s, dt, "dy")
            assert torch.equal(x0, x1), (cin, cout, k, s, dt, "dx")
            if with_epi:
                assert torch.equal(p0, p1), (cin, cout, k, s, dt, "partials")


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_unstored_apply_and_wgrad_apply(cuda, dt):
    """1x1 dgrads whose kernel stages the apply prologue (argus_conv_dgrad_stages_prologue == 1) with
    dy_out = NULL: dx and the BN-backward partials bit-identical to the stored-dy form; the weight
    gradient staging the same apply from dm (argus_conv_wgrad_apply, non-stem) bit-identical to
    argus_conv_wgrad of the materialised dy (FAST and ragged pixel indexing, every tile shape).
    dy_out = NULL where the dgrad cannot stage the apply is an argument error."""
    from argus_amd._lib import BnBwdEpilogue, BnBwdPrologue

    torch.manual_seed(14)
    L = lib()
    staged = 0
    for cin, cout, k, s, hin, n in [(256, 64, 1, 1, 16, 2), (64, 256, 1, 1, 13, 3), (512, 128, 1, 1, 8, 4),
                                    (256, 512, 1, 2, 15, 2), (1024, 256, 1, 1, 6, 2), (128, 128, 3, 1, 8, 2)]:
        d, p = _desc(n, hin, hin, cin, cout, k, s)
        st = L.dll.argus_conv_dgrad_stages_prologue(C.byref(d), DT[dt])
        w = torch.randn(cout, k, k, cin) * (2.0 / (k * k * cin)) ** 0.5
        _, wt = _prep(d, dt, w.to(cuda), cuda)
        dm = torch.randn(n, d.ho, d.wo, cout, device=cuda).to(TDT[dt])
        yb = torch.randn(n, d.ho, d.wo, cout, device=cuda).to(TDT[dt])
        ca, cb, cc = (torch.randn(cout, device=cuda) * 0.3 for _ in range(3))
        yin = torch.randn(n, hin, hin, cin, device=cuda).to(TDT[dt])
        mean, invstd = torch.randn(cin, device=cuda) * 0.1, torch.rand(cin, device=cuda) + 0.5
        sc, sh = torch.randn(cin, device=cuda), torch.randn(cin, device=cuda)
        rows = L.dll.argus_conv_dgrad_bn_rows(C.byref(d), DT[dt])
        outs = []
        for store in (True, False):
            part = torch.zeros(rows, cin, 2, device=cuda)
            e = BnBwdEpilogue()
            e.y, e.mean, e.invstd, e.mask_mode, e.scale, e.shift, e.part = ptr(yin), ptr(mean), ptr(invstd), \
                2, ptr(sc), ptr(sh), ptr(part)
            dy = torch.zeros(n, d.ho, d.wo, cout, device=cuda, dtype=TDT[dt])
            dx = torch.empty(n, hin, hin, cin, device=cuda, dtype=TDT[dt])
            pro = BnBwdPrologue(ptr(yb), ptr(ca), ptr(cb), ptr(cc), ptr(dy) if store else None)
            rc = L.dll.argus_conv_dgrad_bn(C.byref(d), DT[dt], ptr(dm), ptr(wt), ptr(dx), None, C.byref(e),
                                           C.byref(pro), stream())
            if not store and not st:
                assert rc != 0  # the library would have to materialise dy: dy_out is required
                break
            assert rc == 0, L.dll.argus_last_error()
            torch.cuda.synchronize()
            outs.append((dy.cpu(), dx.cpu(), part.cpu()))
        if not st:
            continue
        staged += 1
        (y0, x0, p0), (y1, x1, p1) = outs
        assert torch.equal(x0, x1) and torch.equal(p0, p1), (cin, cout, k, s, dt)
        assert int((y1 != 0).sum()) == 0  # nothing stored
        # weight gradient: staged apply vs the materialised dy of the first run
        xw = torch.randn(n, hin, hin, cin, device=cuda).to(TDT[dt])
        ws = torch.empty(L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), DT[dt]), dtype=torch.uint8, device=cuda)
        dw_ref = torch.empty(cout, k, k, cin, device=cuda)
        L.conv_wgrad(C.byref(d), DT[dt], ptr(xw), None, None, ptr(y0.to(cuda)), ptr(dw_ref), ptr(ws), ws.numel(),
                     stream())
        dw = torch.empty_like(dw_ref)
        ap = BnBwdPrologue(ptr(yb), ptr(ca), ptr(cb), ptr(cc), None)
        L.conv_wgrad_apply(C.byref(d), DT[dt], ptr(xw), ptr(dm), C.byref(ap), ptr(dw), ptr(ws), ws.numel(), stream())
        torch.cuda.synchronize()
        assert torch.equal(dw.cpu(), dw_ref.cpu()), (cin, cout, k, s, dt)
    assert staged >= 3


def test_wgrad_dma_kernel_bitwise(cuda):
    """1x1 stride-1 bf16 weight gradients on the LDS-DMA ring kernel (policy key 45, conv_wgdma.hip:
    1 = 128 x 128 tiles, 2 / 3 = 128 x 256 where Cin % 256 == 0 with the apply / always) vs the
    register-staged wgrad_kernel
    (key 45 = 0), plain and with the BN-backward apply staged
    from dm (argus_conv_wgrad_apply): dW bit-identical (same apply formula, same MFMA order over
    32-pixel blocks, same splits). Pixel counts that end mid k-step (ragged last split: zero-page
    rows), split targets from one split per tile to many short ones (ring prologue with fewer
    k-steps than stages), and dW against a float64 torch reference."""
    from argus_amd._lib import BnBwdPrologue
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(45)
    L = lib()
    ran = 0
    for cin, cout, hh, ww, n in [(128, 128, 8, 8, 1), (256, 128, 7, 9, 2), (128, 512, 14, 14, 2),
                                 (512, 256, 5, 3, 1), (256, 256, 56, 56, 2), (1024, 256, 13, 11, 3)]:
        for target in (None, 4, 2048):
            tune = {} if target is None else {6: target}
            x = torch.randn(n, hh, ww, cin, device=cuda).to(torch.bfloat16)
            dm = torch.randn(n, hh, ww, cout, device=cuda).to(torch.bfloat16)
            yb = torch.randn(n, hh, ww, cout, device=cuda).to(torch.bfloat16)
            ca, cb, cc = (torch.randn(cout, device=cuda) * 0.3 for _ in range(3))
            for apply in (False, True):
                outs = []
                # key 48: the ring depth of the 128 x 256 apply form (2..5 stages; same arithmetic); key 50:
                # the split sum folded into the launch (zeroed workspace; run twice: the counters reset)
                for key, extra in ((3, {}), (2, {}), (2, {48: 5}), (2, {48: 3}), (2, {48: 2}), (3, {50: 1}),
                                   (2, {50: 1}), (2, {50: 1, 48: 5}), (1, {50: 1}), (1, {}), (0, {})):
                    d, _ = _desc(n, hh, ww, cin, cout, 1, 1)
                    d = d.with_tuning({**tune, 45: key, **extra})
                    wsb = L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), BF16)
                    ws = torch.zeros(wsb, dtype=torch.uint8, device=cuda)
                    dw = torch.empty(cout, 1, 1, cin, device=cuda)
                    with KernelTimer("argus::wgrad_dma_kernel<%s" % ("true" if apply else "false")) as t:
                        if apply:
                            ap = BnBwdPrologue(ptr(yb), ptr(ca), ptr(cb), ptr(cc), None)
                            rc = L.conv_wgrad_apply(C.byref(d), BF16, ptr(x), ptr(dm), C.byref(ap), ptr(dw), ptr(ws),
                                                    wsb, stream())
                        else:
                            rc = L.conv_wgrad(C.byref(d), BF16, ptr(x), None, None, ptr(dm), ptr(dw), ptr(ws), wsb,
                                              stream())
                    assert rc in (0, None), L.dll.argus_last_error()
                    torch.cuda.synchronize()
                    if extra.get(50):
                        # the counters (last 16 KB) are zero again, no spin timed out; a second launch on the
                        # same workspace gives the same bits
                        assert int(ws[-16384:].count_nonzero()) == 0
                        first = dw.clone()
                        dw.zero_()
                        if apply:
                            L.conv_wgrad_apply(C.byref(d), BF16, ptr(x), ptr(dm), C.byref(ap), ptr(dw), ptr(ws), wsb,
                                               stream())
                        else:
                            L.conv_wgrad(C.byref(d), BF16, ptr(x), None, None, ptr(dm), ptr(dw), ptr(ws), wsb, stream())
                        torch.cuda.synchronize()
                        assert torch.equal(dw, first) and int(ws[-16384:].count_nonzero()) == 0
                    ks = list(t.summary())
                    wide = key == 3 or (key == 2 and apply)
                    want = 0 if not key else (256 if wide and cin % 256 == 0 else 128)
                    nsx = extra.get(48, 0) if want == 256 and apply else 0
                    assert len(ks) == (1 if key else 0) and (not key or ks[0] == "argus::wgrad_dma_kernel<%s, %d, false, %d>"
                                                             % ("true" if apply else "false", want, nsx)), \
                        ("dma kernel use", cin, cout, hh, ww, n, key, ks)
                    outs.append(dw.cpu())
                # key 3 plain on 256-wide tiles plans its splits for two workgroups per CU over half the
                # tiles: another split grouping, so another fp32 summation order (checked against fp64)
                resplit = not apply and cin % 256 == 0
                keys = [k for k, _ in ((3, {}), (2, {}), (2, {48: 5}), (2, {48: 3}), (2, {48: 2}), (3, {50: 1}),
                                       (2, {50: 1}), (2, {50: 1, 48: 5}), (1, {50: 1}), (1, {}), (0, {}))]
                same = [o for o, k in zip(outs, keys) if not (resplit and k == 3)]
                assert all(torch.equal(o, outs[-1]) for o in same), (cin, cout, hh, ww, n, target, apply)
                if resplit:  # the key-3 plan, folded or not: one summation order
                    assert torch.equal(outs[0], outs[5]), (cin, cout, hh, ww, n, target)
                dy = dm.double()
                if apply:
                    dy = (ca.double() * dm.double() + (cb.double() * yb.double() + cc.double()))
                    dy = dy.float().to(torch.bfloat16).double()
                ref = torch.einsum("pk,pc->kc", dy.reshape(-1, cout), x.double().reshape(-1, cin)).cpu()
                tol = 1e-3 if apply else 1e-4  # fp32 accumulation of exact bf16 products (+ the bf16 dy rounding)
                for o in (outs[0], outs[-1]):
                    assert _rel(o.reshape(cout, cin), ref) < tol, (cin, cout, apply)
                ran += 1
    assert ran == 36


def test_wgrad_dma_gather_stride2_bitwise(cuda):
    """Stride-2 bf16 weight gradients (1x1 downsample, 3x3 pad 1) on the gathering LDS-DMA kernel
    (policy key 47) vs the register-staged wgrad_kernel (key 47 = 0): dW bit-identical (same MFMA
    order, same splits; rows outside the image read the zero page where the register-staged kernel
    zeroes them). Odd and ragged frames, split targets 4 / default / 2048, and dW against a float64
    torch reference."""
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(47)
    L = lib()
    ran = 0
    for cin, cout, k, hh, ww, n in [(128, 128, 3, 16, 16, 2), (256, 512, 1, 15, 9, 2), (128, 256, 3, 13, 7, 3),
                                    (512, 128, 3, 8, 8, 1), (1024, 256, 1, 12, 21, 1)]:
        for target in (None, 4, 2048):
            tune = {} if target is None else {6: target}
            d0, _ = _desc(n, hh, ww, cin, cout, k, 2)
            x = torch.randn(n, hh, ww, cin, device=cuda).to(torch.bfloat16)
            dy = torch.randn(n, d0.ho, d0.wo, cout, device=cuda).to(torch.bfloat16)
            outs = []
            for key, fold in ((1, 0), (1, 1), (0, 0)):  # + the split sum folded into the launch (key 50)
                d = d0.with_tuning({**tune, 47: key, 50: fold})
                wsb = L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), BF16)
                ws = torch.zeros(wsb, dtype=torch.uint8, device=cuda)
                dw = torch.empty(cout, k, k, cin, device=cuda)
                with KernelTimer("argus::wgrad_dma_kernel<false, 128, true, 0>") as t:
                    L.conv_wgrad(C.byref(d), BF16, ptr(x), None, None, ptr(dy), ptr(dw), ptr(ws), wsb, stream())
                torch.cuda.synchronize()
                assert len(t.summary()) == key, ("gather kernel use", cin, cout, k, hh, ww, n, key)
                assert int(ws[-16384:].count_nonzero()) == 0  # folded: the counters reset, no spin timed out
                outs.append(dw.cpu())
            assert torch.equal(outs[0], outs[2]) and torch.equal(outs[1], outs[2]), (cin, cout, k, hh, ww, n, target)
            ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).double().cpu(), (cout, cin, k, k),
                                              dy.permute(0, 3, 1, 2).double().cpu(), stride=2, padding=(k - 1) // 2)
            assert _rel(outs[0].permute(0, 3, 1, 2), ref) < 1e-4, (cin, cout, k, hh, ww, n)
            ran += 1
    assert ran == 15
    # the default (key 47 = 131072) serves up to that many output pixels; a cap below the launch's pixel
    # count sends it to the register-staged kernel, with the same bits
    d0, _ = _desc(2, 16, 16, 128, 128, 3, 2)
    x = torch.randn(2, 16, 16, 128, device=cuda).to(torch.bfloat16)
    dy = torch.randn(2, d0.ho, d0.wo, 128, device=cuda).to(torch.bfloat16)
    outs = []
    for tune, used in (({}, 1), ({47: 2 * d0.ho * d0.wo - 1}, 0), ({47: 2 * d0.ho * d0.wo}, 1)):
        d = d0.with_tuning(tune)
        wsb = L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), BF16)
        ws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
        dw = torch.empty(128, 3, 3, 128, device=cuda)
        with KernelTimer("argus::wgrad_dma_kernel<false, 128, true, 0>") as t:
            L.conv_wgrad(C.byref(d), BF16, ptr(x), None, None, ptr(dy), ptr(dw), ptr(ws), wsb, stream())
        torch.cuda.synchronize()
        assert len(t.summary()) == used, (tune, used)
        outs.append(dw.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_stem_backward_fusions(cuda, dt):
    """argus_maxpool_bwd_bn (maxpool backward + the stem BN's backward reduction) against
    argus_maxpool_bwd + argus_bn_bwd_reduce(mode 2), and argus_conv_wgrad_apply (the stem weight
    gradient staging dy = ca*dm + cb*y + cc) against argus_bn_bwd_apply + argus_conv_wgrad: bitwise."""
    from argus_amd._lib import BnBwdPrologue

    torch.manual_seed(21)
    L = lib()
    n, H, W = 4, 34, 30  # odd pooled sizes (17 x 15)
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y0 = torch.randn(n, H, W, 64, device=cuda).to(TDT[dt])
    sc, sh = torch.rand(64, device=cuda) + 0.5, torch.randn(64, device=cuda) * 0.3
    mean, invstd = torch.randn(64, device=cuda) * 0.1, torch.rand(64, device=cuda) + 0.5
    pooled = torch.empty(n, Ho, Wo, 64, device=cuda, dtype=TDT[dt])
    amax = torch.empty(n, Ho, Wo, 64, device=cuda, dtype=torch.uint8)
    L.maxpool_fwd(DT[dt], n, H, W, 64, ptr(y0), ptr(sc), ptr(sh), ptr(pooled), ptr(amax), stream())
    dout = torch.randn(n, Ho, Wo, 64, device=cuda).to(TDT[dt])
    # reference path
    dz = torch.empty(n, H, W, 64, device=cuda, dtype=TDT[dt])
    L.maxpool_bwd(DT[dt], n, H, W, 64, ptr(dout), ptr(amax), ptr(dz), stream())
    rows = L.dll.argus_bn_bwd_rows(n * H * W, 64)
    part_ref = torch.empty(rows, 64, 2, device=cuda)
    L.bn_bwd_reduce(DT[dt], n * H * W, 64, ptr(dz), 2, None, ptr(y0), ptr(sc), ptr(sh), ptr(mean), ptr(invstd),
                    ptr(part_ref), None, None, None, None, stream())
    # fused
    rows2 = L.dll.argus_maxpool_bwd_bn_rows(DT[dt], n, H, W, 64)
    part = torch.empty(rows2, 64, 2, device=cuda)
    dm = torch.empty_like(dz)
    L.maxpool_bwd_bn(DT[dt], n, H, W, 64, ptr(dout), ptr(amax), ptr(dm), ptr(y0), ptr(sc), ptr(sh), ptr(mean),
                     ptr(invstd), ptr(part), stream())
    torch.cuda.synchronize()
    mask = (y0.double() * sc.double() + sh.double()) > 0
    assert torch.equal(dm.cpu(), (dz.double() * mask).to(TDT[dt]).cpu())
    a, b = part.double().sum(0).cpu(), part_ref.double().sum(0).cpu()
    assert ((a - b).abs() <= 1e-5 * b.abs().max()).all()
    # the finalize folded into the pass (argus_maxpool_bwd_bn_fin) vs argus_bn_bwd_finalize on the same rows
    _check_maxpool_fin(L, dt, cuda, n, H, W, dout, amax, y0, sc, sh, mean, invstd, dm, part)
    # stem weight gradient with the apply staged
    ca, cb, cc = (torch.randn(64, device=cuda) * 0.2 for _ in range(3))
    x0 = torch.randn(n, 2 * H, 2 * W, 4, device=cuda).to(TDT[dt])
    x0[..., 3] = 0
    d, _ = _desc(n, 2 * H, 2 * W, 3, 64, 7, 2, stem=True)
    assert (d.ho, d.wo) == (H, W)
    ws = torch.empty(L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), DT[dt]), dtype=torch.uint8, device=cuda)
    dy = torch.empty_like(dm)
    L.bn_bwd_apply(DT[dt], n * H * W, 64, ptr(dm), 0, None, ptr(y0), None, None, ptr(ca), ptr(cb), ptr(cc), ptr(dy),
                   None, None, None, None, None, None, stream())
    dw_ref = torch.empty(64, 7, 7, 3, device=cuda)
    L.conv_wgrad(C.byref(d), DT[dt], ptr(x0), None, None, ptr(dy), ptr(dw_ref), ptr(ws), ws.numel(), stream())
    dw = torch.empty_like(dw_ref)
    ap = BnBwdPrologue(ptr(y0), ptr(ca), ptr(cb), ptr(cc), None)
    L.conv_wgrad_apply(C.byref(d), DT[dt], ptr(x0), ptr(dm), C.byref(ap), ptr(dw), ptr(ws), ws.numel(), stream())
    torch.cuda.synchronize()
    assert torch.equal(dw.cpu(), dw_ref.cpu())


def _check_maxpool_fin(L, dt, cuda, n, H, W, dout, amax, y0, sc, sh, mean, invstd, dm_ref, part_ref):
    rows = L.dll.argus_maxpool_bwd_bn_rows(DT[dt], n, H, W, 64)
    gamma = torch.rand(64, device=cuda) + 0.5
    ws = torch.zeros(L.dll.argus_bn_workspace_bytes(64), dtype=torch.uint8, device=cuda)
    ref = [torch.empty(64, device=cuda) for _ in range(5)]  # dgamma, dbeta, ca, cb, cc
    L.bn_bwd_finalize(64, rows, ptr(part_ref), n * H * W, ptr(gamma), ptr(mean), ptr(invstd), *(ptr(t) for t in ref),
                      ptr(ws), stream())
    outs = []
    for _ in range(2):  # deterministic, and the ticket counters are left zero for the next call
        dm, part = torch.empty_like(dm_ref), torch.empty_like(part_ref)
        o = [torch.full((64,), float("nan"), device=cuda) for _ in range(5)]
        L.maxpool_bwd_bn_fin(DT[dt], n, H, W, 64, ptr(dout), ptr(amax), ptr(dm), ptr(y0), ptr(sc), ptr(sh), ptr(mean),
                             ptr(invstd), ptr(part), ptr(gamma), *(ptr(t) for t in o), ptr(ws), stream())
        torch.cuda.synchronize()
        assert torch.equal(dm.cpu(), dm_ref.cpu()) and torch.equal(part.cpu(), part_ref.cpu())
        outs.append(torch.stack(o).cpu())
    assert torch.equal(outs[0], outs[1])
    assert (ws[:16384] == 0).all()
    r = torch.stack(ref).cpu()
    # both merge the same fp32 rows in fp64 (different grouping), then round to fp32: within 2 ulp
    assert torch.allclose(outs[0], r, rtol=2.5e-7, atol=1e-12), (outs[0] - r).abs().max()


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_maxpool_bwd_folded_finalize_full_grid(cuda, dt):
    """argus_maxpool_bwd_bn_fin at a size that caps the pass grid (2048 workgroups = partial rows):
    dm and the partial rows identical to argus_maxpool_bwd_bn, the folded dgamma/dbeta/ca/cb/cc equal to
    argus_bn_bwd_finalize's on those rows."""
    torch.manual_seed(22)
    L = lib()
    n, H, W = 8, 112, 112
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    y0 = torch.randn(n, H, W, 64, device=cuda).to(TDT[dt])
    sc, sh = torch.rand(64, device=cuda) + 0.5, torch.randn(64, device=cuda) * 0.3
    mean, invstd = torch.randn(64, device=cuda) * 0.1, torch.rand(64, device=cuda) + 0.5
    pooled = torch.empty(n, Ho, Wo, 64, device=cuda, dtype=TDT[dt])
    amax = torch.empty(n, Ho, Wo, 64, device=cuda, dtype=torch.uint8)
    L.maxpool_fwd(DT[dt], n, H, W, 64, ptr(y0), ptr(sc), ptr(sh), ptr(pooled), ptr(amax), stream())
    dout = torch.randn(n, Ho, Wo, 64, device=cuda).to(TDT[dt])
    rows = L.dll.argus_maxpool_bwd_bn_rows(DT[dt], n, H, W, 64)
    assert rows == 2048
    part, dm = torch.empty(rows, 64, 2, device=cuda), torch.empty_like(y0)
    L.maxpool_bwd_bn(DT[dt], n, H, W, 64, ptr(dout), ptr(amax), ptr(dm), ptr(y0), ptr(sc), ptr(sh), ptr(mean),
                     ptr(invstd), ptr(part), stream())
    _check_maxpool_fin(L, dt, cuda, n, H, W, dout, amax, y0, sc, sh, mean, invstd, dm, part)


FP8_CASES = [  # (cin, cout, k, stride, hin, n): reduction channels % 128 == 0 in each pass
    (256, 128, 1, 1, 12, 2), (128, 128, 3, 1, 12, 2), (256, 256, 3, 2, 13, 2), (512, 1024, 1, 2, 9, 2),
    (1024, 256, 1, 1, 6, 3), (512, 512, 3, 1, 5, 2),
]


def test_fp8_mx_conv_fwd_dgrad(cuda):
    """ARGUS_FP8: conv fwd (+ BN statistics) and dgrad (+ BN-backward epilogue) with the A and B
    operands quantized to OCP MX-fp8 (e4m3, E8M0 scale per 32 K-elements) on the scaled MFMA, vs
    the fp64 reference on the bf16 inputs (policy key 37 = 7: every pass in fp8, the weights from the
    fp8 weight prep), and a 1x1 dgrad staging the BN-backward apply before the quantization. Stated fp8
    tolerance: max error <= 6e-2 of the output's max magnitude (e4m3 keeps 3 mantissa bits: 2^-4
    relative per operand element)."""
    from argus_amd._lib import BnBwdEpilogue, BnBwdPrologue
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(17)
    L = lib()
    for cin, cout, k, s, hin, n in FP8_CASES:
        d, p = _desc(n, hin, hin, cin, cout, k, s)
        d = d.with_tuning({37: 7})  # every pass on the fp8 kernel (the default takes the dgrads only)
        x = _q(torch.randn(n, hin, hin, cin), "bf16")
        w = torch.randn(cout, k, k, cin) * (2.0 / (k * k * cin)) ** 0.5
        dy = _q(torch.randn(n, d.ho, d.wo, cout), "bf16")
        wf, wt = _prep(d, "fp8", w.to(cuda), cuda)  # the pre-quantized MX-fp8 weight copies
        _check_fp8_weight_layout(wf, w.reshape(cout, -1), k * k * cin)
        y = torch.empty(n, d.ho, d.wo, cout, dtype=torch.bfloat16, device=cuda)
        rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), FP8)
        stats = torch.empty(rows, cout, 2, device=cuda)
        with KernelTimer("argus::igemm_kernel") as t:
            L.conv_fwd(C.byref(d), FP8, ptr(x.to(cuda, torch.bfloat16)), ptr(wf), ptr(y), None, None, ptr(stats),
                       stream())
        names = list(t.summary())
        assert any(nm.endswith(", 32>") for nm in names), names  # the fp8 variant ran
        wr = _q(w, "bf16").permute(0, 3, 1, 2)
        ref = F.conv2d(x.permute(0, 3, 1, 2), wr, stride=s, padding=p)
        e = _rel(y.permute(0, 3, 1, 2), ref)
        assert e < 6e-2, ("fp8 fwd", cin, cout, k, s, e)
        assert e > 1e-4, ("fp8 fwd: no quantization visible?", e)
        # dgrad with a BN-backward epilogue (mask recomputed from the BN input)
        brows = L.dll.argus_conv_dgrad_bn_rows(C.byref(d), FP8)
        part = torch.zeros(brows, cin, 2, device=cuda)
        yin = torch.randn(n, hin, hin, cin, device=cuda).to(torch.bfloat16)
        mean, invstd = torch.zeros(cin, device=cuda), torch.ones(cin, device=cuda)
        sc, sh = torch.ones(cin, device=cuda), torch.zeros(cin, device=cuda)
        e_ = BnBwdEpilogue()
        e_.y, e_.mean, e_.invstd, e_.mask_mode, e_.scale, e_.shift, e_.part = ptr(yin), ptr(mean), ptr(invstd), 2, \
            ptr(sc), ptr(sh), ptr(part)
        dm = torch.empty(n, hin, hin, cin, device=cuda, dtype=torch.bfloat16)
        L.conv_dgrad_bn(C.byref(d), FP8, ptr(dy.to(cuda, torch.bfloat16)), ptr(wt), ptr(dm), None, C.byref(e_), None,
                        stream())
        refd = torch.nn.grad.conv2d_input(x.permute(0, 3, 1, 2).shape, wr, dy.permute(0, 3, 1, 2), stride=s, padding=p)
        refm = refd * (yin.double().cpu().permute(0, 3, 1, 2) > 0)
        e = _rel(dm.permute(0, 3, 1, 2), refm)
        assert e < 6e-2, ("fp8 dgrad", cin, cout, k, s, e)
        colsum = part.double().sum(0)[:, 0].cpu()
        assert _rel(colsum, dm.double().cpu().reshape(-1, cin).sum(0)) < 1e-3  # partials sum what was stored
        if k == 1:  # the BN-backward apply staged before the quantization (dy never stored)
            dmg = _q(torch.randn(n, d.ho, d.wo, cout), "bf16")
            yb = _q(torch.randn(n, d.ho, d.wo, cout), "bf16")
            ca, cb, cc = (torch.randn(cout) * 0.3 for _ in range(3))
            assert L.dll.argus_conv_dgrad_stages_prologue(C.byref(d), FP8) == 1
            pro = BnBwdPrologue(ptr(ybg := yb.to(cuda, torch.bfloat16)), ptr(cag := ca.to(cuda)), ptr(cbg := cb.to(cuda)),
                                ptr(ccg := cc.to(cuda)), None)
            dx = torch.empty(n, hin, hin, cin, device=cuda, dtype=torch.bfloat16)
            with KernelTimer("argus::igemm_kernel") as t:
                L.conv_dgrad_bn(C.byref(d), FP8, ptr(dmg.to(cuda, torch.bfloat16)), ptr(wt), ptr(dx), None, None,
                                C.byref(pro), stream())
            assert any(nm.endswith(", 48>") for nm in t.summary()), list(t.summary())  # fp8 | apply prologue
            dyr = _q(ca * dmg + (cb * yb + cc), "bf16")
            refa = torch.nn.grad.conv2d_input(x.permute(0, 3, 1, 2).shape, wr, dyr.permute(0, 3, 1, 2), stride=s,
                                              padding=p)
            e = _rel(dx.permute(0, 3, 1, 2), refa)
            assert e < 6e-2, ("fp8 dgrad + apply prologue", cin, cout, k, s, e)


def _check_fp8_weight_layout(buf, w_fp32, cols):
    """argus_conv_weight_prep(ARGUS_FP8) layout of a forward copy: e4m3 rows [K][cols] then E8M0 scales
    [K][cols / 32]; the block scale 2^e is the smallest with amax(bf16 block) * 2^-e < 448 (e4m3 max), and
    dequantized values are the bf16 weights to e4m3's 3-bit mantissa (2^-4 relative, 2^-10 absolute
    under the block scale for subnormals) - the same as torch's float8_e4m3fn rounding of w / 2^e."""
    K = w_fp32.shape[0]
    raw = buf.view(torch.uint8).reshape(-1)[: K * cols + K * cols // 32].cpu()
    vals = raw[: K * cols].view(torch.float8_e4m3fn).float().reshape(K, cols)
    e = raw[K * cols:].to(torch.int32).reshape(K, cols // 32) - 127
    scale = torch.pow(2.0, e.double()).repeat_interleave(32, dim=1)
    wb = w_fp32.to(torch.bfloat16).double()  # OHWI flattening = the kernel's K order
    amax = wb.abs().reshape(K, cols // 32, 32).amax(-1).repeat_interleave(32, dim=1)
    assert (amax / scale < 448).all() and ((amax / scale >= 224) | (amax == 0)).all()  # tightest E8M0 scale
    deq = vals.double() * scale
    assert ((deq - wb).abs() <= wb.abs() * 2.0 ** -4 + scale * 2.0 ** -10).all()
    same = (vals == (wb / scale).float().to(torch.float8_e4m3fn).float()).double().mean().item()
    assert same > 0.999, same  # round-to-nearest-even ties may differ


def _deq_x8(buf, rows, cols):
    """MX-fp8 'x8' tensor (e4m3 [rows][cols] then E8M0 [rows][cols / 32]) -> fp64 values, and the raw
    e4m3 values / exponents."""
    raw = buf.view(torch.uint8).reshape(-1)[: rows * cols + rows * cols // 32].cpu()
    vals = raw[: rows * cols].view(torch.float8_e4m3fn).double().reshape(rows, cols)
    e = raw[rows * cols:].to(torch.int32).reshape(rows, cols // 32) - 127
    scale = torch.pow(2.0, e.double()).repeat_interleave(32, dim=1)
    return vals * scale, vals, scale


def _check_x8_quant(buf, t_bf16):
    """x8 copy written by argus_bn_apply_x8 / argus_bn_bwd_apply_x8 of the bf16 tensor t: the tightest
    E8M0 block scale (amax * 2^-e in [224, 448)) and the e4m3 values torch's float8_e4m3fn rounding of
    t / 2^e gives (round-to-nearest-even ties may differ)."""
    P, Cc = t_bf16.numel() // t_bf16.shape[-1], t_bf16.shape[-1]
    deq, vals, scale = _deq_x8(buf, P, Cc)
    tb = t_bf16.reshape(P, Cc).double().cpu()
    amax = tb.abs().reshape(P, Cc // 32, 32).amax(-1).repeat_interleave(32, dim=1)
    assert (amax / scale < 448).all() and ((amax / scale >= 224) | (amax == 0)).all()
    same = (vals == (tb / scale).float().to(torch.float8_e4m3fn).float().double()).double().mean().item()
    assert same > 0.999, same
    assert ((deq - tb).abs() <= tb.abs() * 2.0 ** -4 + scale * 2.0 ** -9).all()
    return deq


X8_CASES = [  # (n, h, w, c, k): whole-image tiles (H*W < 256), row tiles, a 64-column forward (key 13 = 1:
    # the halo kernel at these small grids)
    (8, 8, 8, 128, 128), (2, 16, 16, 256, 128), (4, 32, 32, 128, 256), (2, 16, 16, 512, 512), (2, 16, 16, 128, 64),
]


def test_conv_x8_halo_fwd_dgrad(cuda):
    """MX-fp8 stored operands (ABI 16): argus_bn_apply_x8 / argus_bn_bwd_apply_x8 write the bf16 output
    bit-identical to argus_bn_apply / argus_bn_bwd_apply plus its x8 copy (checked against torch's e4m3
    rounding under the tightest E8M0 scale); argus_conv_fwd_x8 / argus_conv_dgrad_bn_x8 (the LDS-halo
    kernel's F8 variant) against the fp64 conv of the dequantized operands (tolerance: fp32 accumulation
    + the bf16 output rounding, 2^-8 of the output's max magnitude), against the register-staged
    ARGUS_FP8 kernel that quantizes the same bf16 tensors while staging (same bytes, another fp32
    summation order: 2^-7), the forward BN partials and the dgrad's folded BN-backward finalize."""
    from argus_amd._lib import BnBwdEpilogue
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(23)
    L = lib()
    extra = {13: 1}
    for n, h, w, c, k in X8_CASES:
        d, _ = _desc(n, h, w, c, k, 3, 1)
        d = d.with_tuning({37: 10, **extra})  # bit 8: fp8 forward weights of the 3x3 stride-1 convs
        P = n * h * w
        assert L.dll.argus_conv_x8_ok(C.byref(d), 0) == 1
        assert L.dll.argus_conv_x8_ok(C.byref(d), 1) == (1 if k % 128 == 0 else 0)
        assert L.dll.argus_conv_x8_ok(C.byref(d.with_tuning({37: 2, **extra})), 0) == 0  # no fp8 forward weights
        w_ = torch.randn(k, 3, 3, c) * (2.0 / (9 * c)) ** 0.5
        wf, wd = _prep(d, "fp8", w_.to(cuda), cuda)
        wfd = _deq_x8(wf, k, 9 * c)[0].reshape(k, 3, 3, c).permute(0, 3, 1, 2)
        # forward: a = relu(y*scale+shift) with its x8 copy
        yin = torch.randn(n, h, w, c, device=cuda).to(torch.bfloat16)
        sc, sh = torch.rand(c, device=cuda) + 0.5, torch.randn(c, device=cuda) * 0.3
        a = torch.empty_like(yin)
        a_ref = torch.empty_like(yin)
        a8 = torch.empty(P * c * 33 // 32, dtype=torch.uint8, device=cuda)
        L.bn_apply_x8(P, c, ptr(yin), ptr(sc), ptr(sh), None, None, None, 1, ptr(a), None, ptr(a8), stream())
        L.bn_apply(BF16, P, c, ptr(yin), ptr(sc), ptr(sh), None, None, None, 1, ptr(a_ref), None, stream())
        assert torch.equal(a, a_ref)
        ad = _check_x8_quant(a8, a).reshape(n, h, w, c).permute(0, 3, 1, 2)
        rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), FP8)
        stats = torch.empty(rows, k, 2, device=cuda)
        y = torch.empty(n, h, w, k, dtype=torch.bfloat16, device=cuda)
        with KernelTimer("argus::conv3x3_halo_kernel") as t:
            L.conv_fwd_x8(C.byref(d), ptr(a8), ptr(wf), ptr(y), ptr(stats), stream())
        assert any(nm.endswith(", true, false>") for nm in t.summary()), list(t.summary())
        ref = F.conv2d(ad, wfd, padding=1)
        e = _rel(y.permute(0, 3, 1, 2), ref)
        assert e < 2.0 ** -8, ("x8 fwd", n, h, w, c, k, e)
        y_st = torch.empty_like(y)
        L.conv_fwd(C.byref(d), FP8, ptr(a), ptr(wf), ptr(y_st), None, None, None, stream())
        assert _rel(y, y_st) < 2.0 ** -7
        assert _rel(stats.double().sum(0)[:, 0].cpu(), ref.sum((0, 2, 3))) < 1e-3  # the partials sum y
        if k % 128:
            continue
        # data gradient: dy = ca*dm + cb*y2 + cc with its x8 copy, then the mask-mode-2 BN epilogue
        dmz = torch.randn(n, h, w, k, device=cuda).to(torch.bfloat16)
        y2 = torch.randn(n, h, w, k, device=cuda).to(torch.bfloat16)
        ca, cb, cc = (torch.randn(k, device=cuda) * 0.3 for _ in range(3))
        dy, dy_ref = torch.empty_like(dmz), torch.empty_like(dmz)
        dy8 = torch.empty(P * k * 33 // 32, dtype=torch.uint8, device=cuda)
        L.bn_bwd_apply_x8(P, k, ptr(dmz), ptr(y2), ptr(ca), ptr(cb), ptr(cc), ptr(dy), ptr(dy8), stream())
        L.bn_bwd_apply(BF16, P, k, ptr(dmz), 0, None, ptr(y2), None, None, ptr(ca), ptr(cb), ptr(cc), ptr(dy_ref),
                       None, None, None, None, None, None, stream())
        assert torch.equal(dy, dy_ref)
        dyd = _check_x8_quant(dy8, dy).reshape(n, h, w, k).permute(0, 3, 1, 2)
        wdd = _deq_x8(wd, c, 9 * k)[0].reshape(c, 3, 3, k)  # [c][tap][k]: w_dgrad = the forward weights transposed
        wdd = wdd.permute(3, 0, 1, 2)  # [k][c][r][s] as conv2d weights of the forward conv
        ybn = torch.randn(n, h, w, c, device=cuda).to(torch.bfloat16)
        mean, invstd = torch.randn(c, device=cuda) * 0.1, torch.rand(c, device=cuda) + 0.5
        gamma = torch.rand(c, device=cuda) + 0.5
        ws = torch.zeros(L.dll.argus_bn_workspace_bytes(2048), dtype=torch.uint8, device=cuda)
        outs = {}
        for name in ("x8", "staged"):
            brows = L.dll.argus_conv_dgrad_bn_rows(C.byref(d), FP8)
            part = torch.zeros(brows, c, 2, device=cuda)
            coef = torch.zeros(5, c, device=cuda)
            e_ = BnBwdEpilogue()
            e_.y, e_.mean, e_.invstd, e_.mask_mode, e_.scale, e_.shift, e_.part = ptr(ybn), ptr(mean), ptr(invstd), 2, \
                ptr(sc), ptr(sh), ptr(part)
            e_.workspace, e_.gamma, e_.dgamma, e_.dbeta = ptr(ws), ptr(gamma), ptr(coef[0]), ptr(coef[1])
            e_.ca, e_.cb, e_.cc = ptr(coef[2]), ptr(coef[3]), ptr(coef[4])
            dm = torch.empty(n, h, w, c, device=cuda, dtype=torch.bfloat16)
            if name == "x8":
                with KernelTimer("argus::conv3x3_halo_kernel") as t:
                    L.conv_dgrad_bn_x8(C.byref(d), ptr(dy8), ptr(wd), ptr(dm), C.byref(e_), stream())
                assert any(nm.endswith(", 2, 2, true, false>") for nm in t.summary()), list(t.summary())
            else:
                L.conv_dgrad_bn(C.byref(d), FP8, ptr(dy), ptr(wd), ptr(dm), None, C.byref(e_), None, stream())
            outs[name] = (dm, coef)
        refd = torch.nn.grad.conv2d_input((n, c, h, w), wdd, dyd, padding=1)
        mask = ((ybn.double() * sc.double() + sh.double()) > 0).cpu().permute(0, 3, 1, 2)
        dm = outs["x8"][0]
        e = _rel(dm.permute(0, 3, 1, 2), refd * mask)
        assert e < 2.0 ** -8, ("x8 dgrad", n, h, w, c, k, e)
        assert _rel(dm, outs["staged"][0]) < 2.0 ** -7
        for i in range(5):  # dgamma, dbeta, ca, cb, cc of the folded finalize
            assert _rel(outs["x8"][1][i], outs["staged"][1][i]) < 1e-2, i
        assert int(ws[:16384].count_nonzero()) == 0  # ticket counters left at zero


def test_stats_only_forward_persistent_kernel(cuda):
    """Statistics-only 1x1 forward (argus_conv_fwd, y == NULL) on the persistent kernel (policy key 44):
    one {sum, M2} row per row split plus int32 pixel counts (argus_conv_fwd_stats_only_rows / _tile,
    negative tile), merged mean / biased variance within 1e-5 of the fp64 moments of x w^T on the same
    bf16 operands and within 2e-6 of the register-staged igemm's partials (key 44 = 0: the same
    products, another merge grouping); every input width 64..512, ragged pixel counts, more row splits
    than some workgroups get tiles."""
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(37)
    L = lib()
    for n, h, w, c, k in [(4, 16, 16, 64, 256), (3, 7, 9, 128, 512), (2, 8, 8, 256, 1024), (2, 5, 5, 512, 2048),
                          (64, 64, 64, 64, 256)]:
        d, _ = _desc(n, h, w, c, k, 1, 1)
        P = n * h * w
        rows = L.dll.argus_conv_fwd_stats_only_rows(C.byref(d), BF16)
        tile = L.dll.argus_conv_fwd_stats_only_tile(C.byref(d), BF16)
        assert tile < 0 and rows * -tile >= P
        x = torch.randn(n, h, w, c, device=cuda).to(torch.bfloat16)
        wf, _ = _prep(d, "bf16", (torch.randn(k, 1, 1, c) * c ** -0.5).to(cuda), cuda)
        st = torch.full((rows * k * 2 + rows,), float("nan"), device=cuda)
        with KernelTimer("argus::p1x1_fwd_stats_kernel") as t:
            L.conv_fwd(C.byref(d), BF16, ptr(x), ptr(wf), None, None, None, ptr(st), stream())
        assert len(t.summary()) == 1, list(t.summary())
        part = st[: rows * k * 2].reshape(rows, k, 2).double().cpu()
        counts = st[rows * k * 2:].view(torch.int32).cpu()
        mean, var = _merge_stats(part, tile, P, counts)
        y = x.reshape(P, c).double().cpu() @ wf.double().cpu().reshape(k, c).t()
        assert _rel(mean, y.mean(0)) < 1e-5 and _rel(var, y.var(0, unbiased=False)) < 1e-5, (n, h, w, c, k)
        d0 = d.with_tuning({44: 0})
        r0, t0 = (L.dll.argus_conv_fwd_stats_only_rows(C.byref(d0), BF16),
                  L.dll.argus_conv_fwd_stats_only_tile(C.byref(d0), BF16))
        assert (r0, t0) == (L.dll.argus_conv_fwd_stat_rows(C.byref(d0), BF16), L.dll.argus_conv_fwd_stat_tile(C.byref(d0), BF16))
        st0 = torch.empty(r0, k, 2, device=cuda)
        L.conv_fwd(C.byref(d0), BF16, ptr(x), ptr(wf), None, None, None, ptr(st0), stream())
        m0, v0 = _merge_stats(st0.double().cpu(), t0, P)
        assert _rel(mean, m0) < 2e-6 and _rel(var, v0) < 2e-6, (n, h, w, c, k)


def test_conv_fwd_apply_out_matches_apply_then_conv(cuda):
    """argus_conv_fwd_apply_out (ABI 16): a 1x1 stride-1 forward whose BN+ReLU prologue also stores the
    applied input: x_out bit-identical to argus_bn_apply(relu) of x, and y / the BN statistics partials
    bit-identical to argus_conv_fwd on that stored x' (the same bf16 operands in the same k order), with
    y stored and statistics-only (y NULL); ragged M; refused for 3x3 / strided convs and x_out == x."""
    from argus_amd._lib import ArgusHipError

    torch.manual_seed(29)
    L = lib()
    for n, h, w, c, k in [(2, 16, 16, 64, 256), (3, 7, 9, 128, 512), (1, 32, 32, 256, 64)]:
        d, _ = _desc(n, h, w, c, k, 1, 1)
        P = n * h * w
        x = torch.randn(n, h, w, c, device=cuda).to(torch.bfloat16)
        sc, sh = torch.rand(c, device=cuda) + 0.5, torch.randn(c, device=cuda) * 0.5
        wf, _ = _prep(d, "bf16", (torch.randn(k, 1, 1, c) * c ** -0.5).to(cuda), cuda)
        rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), BF16)
        a_ref = torch.empty_like(x)
        L.bn_apply(BF16, P, c, ptr(x), ptr(sc), ptr(sh), None, None, None, 1, ptr(a_ref), None, stream())
        for store_y in (True, False):
            a = torch.full_like(x, float("nan"))
            y = torch.empty(n, h, w, k, device=cuda, dtype=torch.bfloat16) if store_y else None
            st = torch.empty(rows, k, 2, device=cuda)
            L.conv_fwd_apply_out(C.byref(d), BF16, ptr(x), ptr(wf), ptr(y), ptr(sc), ptr(sh), ptr(st), ptr(a),
                                 stream())
            assert torch.equal(a, a_ref), (n, h, w, c, k)
            y_ref = torch.empty(n, h, w, k, device=cuda, dtype=torch.bfloat16) if store_y else None
            st_ref = torch.empty_like(st)
            # (the statistics-only reference on the igemm too: key 44 would send it to the persistent
            # kernel, whose partial rows group differently)
            L.conv_fwd(C.byref(d.with_tuning({44: 0})), BF16, ptr(a_ref), ptr(wf), ptr(y_ref), None, None, ptr(st_ref),
                       stream())
            assert torch.equal(st, st_ref), (n, h, w, c, k, store_y)
            if store_y:
                assert torch.equal(y, y_ref)
    d3, _ = _desc(2, 8, 8, 64, 64, 3, 1)
    with pytest.raises(ArgusHipError, match="apply_out"):
        L.conv_fwd_apply_out(C.byref(d3), BF16, ptr(x), ptr(wf), None, ptr(sc), ptr(sh), ptr(st), ptr(a), stream())
    with pytest.raises(ArgusHipError, match="apply_out"):
        L.conv_fwd_apply_out(C.byref(d), BF16, ptr(x), ptr(wf), None, ptr(sc), ptr(sh), ptr(st), ptr(x), stream())


def test_fused_dgrad_wgrad_matches_separate_passes(cuda):
    """argus_conv_dgrad_wgrad_bn (layer-1 conv3: one pass over dm3 / y3 for both gradients) against
    argus_conv_dgrad_bn (apply prologue, mask-mode-2 epilogue) + argus_conv_wgrad_apply: dx bitwise
    (same staged dy and the same MFMA k order), the folded bn2 finalize outputs and dW to fp32 / fp64
    summation order (1e-5 relative), dW also against an fp64 torch weight gradient of the staged dy;
    ragged row counts (P not a multiple of the 32-row tile, fewer tiles than the grid cap) and the
    counters left at zero. Other shapes are refused."""
    from argus_amd._lib import BnBwdEpilogue, BnBwdPrologue

    torch.manual_seed(31)
    L = lib()
    cin, cout = 64, 256
    bad, _ = _desc(2, 8, 8, 128, 256, 1, 1)
    assert L.dll.argus_conv_dgrad_wgrad_ok(C.byref(bad), BF16) == 0
    ws_bytes = L.dll.argus_bn_workspace_bytes(2048)
    for n, h, w_ in [(2, 33, 33), (1, 5, 7), (8, 64, 64)]:
        d, _ = _desc(n, h, w_, cin, cout, 1, 1)
        assert L.dll.argus_conv_dgrad_wgrad_ok(C.byref(d), BF16) == 1
        assert L.dll.argus_conv_dgrad_wgrad_ok(C.byref(d), F32) == 0
        P = n * h * w_
        wt_ohwi = torch.randn(cout, 1, 1, cin) * (2.0 / cin) ** 0.5
        _, wt = _prep(d, "bf16", wt_ohwi.to(cuda), cuda)
        dm = torch.randn(P, cout, device=cuda).to(torch.bfloat16)
        y3 = torch.randn(P, cout, device=cuda).to(torch.bfloat16)
        ca, cb, cc = (torch.randn(cout, device=cuda) * 0.3 for _ in range(3))
        a2 = torch.relu(torch.randn(P, cin, device=cuda)).to(torch.bfloat16)
        y2 = torch.randn(P, cin, device=cuda).to(torch.bfloat16)
        mean, invstd = torch.randn(cin, device=cuda) * 0.1, torch.rand(cin, device=cuda) + 0.5
        sc, sh = torch.randn(cin, device=cuda), torch.randn(cin, device=cuda)
        g2 = torch.rand(cin, device=cuda) + 0.5
        res = []
        for fused in (False, True):
            ws = torch.zeros(ws_bytes, dtype=torch.uint8, device=cuda)
            rows = (L.dll.argus_conv_dgrad_wgrad_bn_rows if fused else L.dll.argus_conv_dgrad_bn_rows)(C.byref(d), BF16)
            part = torch.empty(rows, cin, 2, device=cuda)
            co = torch.zeros(5, cin, device=cuda)
            e = BnBwdEpilogue()
            e.y, e.mean, e.invstd, e.mask_mode, e.scale, e.shift, e.part = ptr(y2), ptr(mean), ptr(invstd), 2, \
                ptr(sc), ptr(sh), ptr(part)
            e.workspace, e.gamma, e.dgamma, e.dbeta = ptr(ws), ptr(g2), ptr(co[3]), ptr(co[4])
            e.ca, e.cb, e.cc = ptr(co[0]), ptr(co[1]), ptr(co[2])
            pro = BnBwdPrologue(ptr(y3), ptr(ca), ptr(cb), ptr(cc), None)
            dx = torch.empty(P, cin, dtype=torch.bfloat16, device=cuda)
            dw = torch.empty(cout, 1, 1, cin, device=cuda)
            if fused:
                wsw = torch.empty(L.dll.argus_conv_dgrad_wgrad_workspace_bytes(C.byref(d), BF16), dtype=torch.uint8,
                                  device=cuda)
                rc = L.dll.argus_conv_dgrad_wgrad_bn(C.byref(d), BF16, ptr(dm), ptr(wt), ptr(a2), ptr(dx), None,
                                                     C.byref(e), C.byref(pro), ptr(dw), ptr(wsw), wsw.numel(), stream())
                assert rc == 0, L.dll.argus_last_error()
            else:
                L.conv_dgrad_bn(C.byref(d), BF16, ptr(dm), ptr(wt), ptr(dx), None, C.byref(e), C.byref(pro), stream())
                wsw = torch.empty(L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), BF16), dtype=torch.uint8,
                                  device=cuda)
                L.conv_wgrad_apply(C.byref(d), BF16, ptr(a2), ptr(dm), C.byref(pro), ptr(dw), ptr(wsw), wsw.numel(),
                                   stream())
            torch.cuda.synchronize()
            assert int(ws[:16384].view(torch.int32).abs().sum()) == 0
            res.append((dx.cpu(), dw.cpu(), co.cpu()))
        (x0, w0, c0), (x1, w1, c1) = res
        assert torch.equal(x0, x1), (n, h, w_)
        assert _rel(c1, c0) < 1e-5 and _rel(w1, w0) < 1e-5, (n, h, w_, _rel(c1, c0), _rel(w1, w0))
        dy = (ca.double() * dm.double() + (cb.double() * y3.double() + cc.double())).to(torch.bfloat16).double()
        dw64 = (dy.T @ a2.double()).view(cout, 1, 1, cin)
        assert _rel(w1, dw64.cpu()) < 1e-3, (n, h, w_)
        # the plain epilogue (no BN; dx += addend in place: the first block's downsample) against the
        # materialised dy -> argus_conv_dgrad(addend) + argus_conv_wgrad
        dy_b = torch.empty(P, cout, dtype=torch.bfloat16, device=cuda)
        L.bn_bwd_apply(BF16, P, cout, ptr(dm), 0, None, ptr(y3), None, None, ptr(ca), ptr(cb), ptr(cc), ptr(dy_b),
                       None, None, None, None, None, None, stream())
        base = torch.randn(P, cin, device=cuda).to(torch.bfloat16)
        x_ref, x_fused = base.clone(), base.clone()
        L.conv_dgrad(C.byref(d), BF16, ptr(dy_b), ptr(wt), ptr(x_ref), ptr(x_ref), None, stream())
        wsr = torch.empty(L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), BF16), dtype=torch.uint8, device=cuda)
        dw_ref = torch.empty(cout, 1, 1, cin, device=cuda)
        L.conv_wgrad(C.byref(d), BF16, ptr(a2), None, None, ptr(dy_b), ptr(dw_ref), ptr(wsr), wsr.numel(), stream())
        dw_f = torch.empty_like(dw_ref)
        wsw = torch.empty(L.dll.argus_conv_dgrad_wgrad_workspace_bytes(C.byref(d), BF16), dtype=torch.uint8, device=cuda)
        pro = BnBwdPrologue(ptr(y3), ptr(ca), ptr(cb), ptr(cc), None)
        rc = L.dll.argus_conv_dgrad_wgrad_bn(C.byref(d), BF16, ptr(dm), ptr(wt), ptr(a2), ptr(x_fused), ptr(x_fused),
                                             None, C.byref(pro), ptr(dw_f), ptr(wsw), wsw.numel(), stream())
        assert rc == 0, L.dll.argus_last_error()
        torch.cuda.synchronize()
        assert torch.equal(x_fused.cpu(), x_ref.cpu()), (n, h, w_)
        assert _rel(dw_f, dw_ref) < 1e-5, (n, h, w_)


def test_glds_two_stage_ring_matches_three(cuda):
    """The 96 KB two-stage glds ring (policy key 41 = 2, data gradients only) against the three-stage
    ring: same k order, so dx and the BN-backward partials are bit-identical (plain and BN-epilogue
    dgrads; 1x1 K = 1024 and a 3x3 K = 9 * 128 shape, the size thresholds lowered per call)."""
    from argus_amd._lib import BnBwdEpilogue

    torch.manual_seed(41)
    L = lib()
    for cin, cout, k, hin, n in [(256, 1024, 1, 12, 8), (128, 128, 3, 14, 8)]:
        d0, _ = _desc(n, hin, hin, cin, cout, k, 1)
        w = torch.randn(cout, k, k, cin) * (2.0 / (k * k * cin)) ** 0.5
        _, wt = _prep(d0, "bf16", w.to(cuda), cuda)
        dy = torch.randn(n, d0.ho, d0.wo, cout, device=cuda).to(torch.bfloat16)
        yb = torch.randn(n, hin, hin, cin, device=cuda).to(torch.bfloat16)
        mean, invstd = torch.randn(cin, device=cuda) * 0.1, torch.rand(cin, device=cuda) + 0.5
        sc, sh = torch.randn(cin, device=cuda), torch.randn(cin, device=cuda)
        outs = []
        for stages in (3, 2):
            d = d0.with_tuning({36: 1, 9: 1, 10: 0, 41: stages})  # glds for this small shape, no halo
            assert L.dll.argus_conv_launch_info(C.byref(d), BF16, 1, None) > 0
            rows = L.dll.argus_conv_dgrad_bn_rows(C.byref(d), BF16)
            part = torch.zeros(rows, cin, 2, device=cuda)
            e = BnBwdEpilogue()
            e.y, e.mean, e.invstd, e.mask_mode, e.scale, e.shift, e.part = ptr(yb), ptr(mean), ptr(invstd), 2, \
                ptr(sc), ptr(sh), ptr(part)
            dm = torch.empty(n, hin, hin, cin, dtype=torch.bfloat16, device=cuda)
            dx = torch.empty(n, hin, hin, cin, dtype=torch.bfloat16, device=cuda)
            L.conv_dgrad_bn(C.byref(d), BF16, ptr(dy), ptr(wt), ptr(dm), None, C.byref(e), None, stream())
            L.conv_dgrad(C.byref(d), BF16, ptr(dy), ptr(wt), ptr(dx), None, None, stream())
            torch.cuda.synchronize()
            outs.append((dm.cpu(), part.cpu(), dx.cpu()))
        for a, b in zip(*outs):
            assert torch.equal(a, b), (cin, cout, k)


@pytest.mark.parametrize("cin,cout,hw,ds", [(64, 256, 24, False), (64, 256, 24, True), (128, 512, 12, True),
                                            (512, 2048, 5, False), (256, 1024, 7, True)])
def test_conv_fwd_bn_out_matches_conv_and_apply(cuda, cin, cout, hw, ds):
    """argus_conv_fwd_bn_out (the bottleneck tail: conv3's C tile -> bn3 + residual (+ the downsample
    BN) + ReLU, mask bits) and the register-staged statistics-only forward (argus_conv_fwd with y = NULL,
    policy key 44 = 0) against
    argus_conv_fwd + argus_bn_apply: every output bit-identical (y, out, mask bits, BN partials);
    ragged row tiles (hw = 5, 7) included."""
    torch.manual_seed(77)
    L = lib()
    n = 3
    d, _ = _desc(n, hw, hw, cin, cout, 1, 1)
    x = torch.relu(torch.randn(n, hw, hw, cin, device=cuda)).to(torch.bfloat16)
    w = (torch.randn(cout, 1, 1, cin) * (2.0 / cin) ** 0.5).to(cuda)
    wf, _ = _prep(d, "bf16", w, cuda)
    rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), BF16)
    st_ref = torch.full((rows * cout * 2,), float("nan"), device=cuda)
    st_new = torch.full((rows * cout * 2,), float("nan"), device=cuda)
    y_ref = torch.empty(n, hw, hw, cout, dtype=torch.bfloat16, device=cuda)
    L.conv_fwd(C.byref(d), BF16, ptr(x), ptr(wf), ptr(y_ref), None, None, ptr(st_ref), stream())
    # (the register-staged statistics-only pass: key 44 = 0; the persistent one writes another partial
    # layout, test_stats_only_forward_persistent_kernel)
    L.conv_fwd(C.byref(d.with_tuning({44: 0})), BF16, ptr(x), ptr(wf), None, None, None, ptr(st_new), stream())
    assert torch.equal(st_ref, st_new)
    sc, sh = torch.rand(cout, device=cuda) + 0.5, torch.randn(cout, device=cuda)
    res = torch.randn(n, hw, hw, cout, device=cuda).to(torch.bfloat16)
    rsc = rsh = None
    if ds:
        rsc, rsh = torch.rand(cout, device=cuda) + 0.5, torch.randn(cout, device=cuda)
    px = n * hw * hw
    o_ref = torch.empty_like(y_ref)
    b_ref = torch.zeros(px * cout // 8, dtype=torch.uint8, device=cuda)
    L.bn_apply(BF16, px, cout, ptr(y_ref), ptr(sc), ptr(sh), ptr(res), ptr(rsc), ptr(rsh), 1, ptr(o_ref), ptr(b_ref),
               stream())
    for store_y in (True, False):
        y = torch.zeros_like(y_ref)
        o = torch.empty_like(y_ref)
        b = torch.full_like(b_ref, 0x5A)
        L.conv_fwd_bn_out(C.byref(d), BF16, ptr(x), ptr(wf), ptr(sc), ptr(sh), ptr(res), ptr(rsc), ptr(rsh), ptr(o),
                          ptr(b), ptr(y) if store_y else None, stream())
        torch.cuda.synchronize()
        assert torch.equal(o.view(torch.int16), o_ref.view(torch.int16)), (cin, cout, hw, ds, store_y)
        assert torch.equal(b, b_ref)
        if store_y:
            assert torch.equal(y.view(torch.int16), y_ref.view(torch.int16))
        else:
            assert not y.any()
    # and against torch: relu(conv * sc + sh + res')
    ref = torch.einsum("nhwc,kc->nhwk", x.double(), wf.double()).to(torch.bfloat16).double() * sc.double() + sh.double()
    r = res.double() if rsc is None else res.double() * rsc.double() + rsh.double()
    assert _rel(o_ref, torch.relu(ref + r)) < TOL["bf16"]


@pytest.mark.parametrize("w3,cout,hin,k1,s,dual,with_pro", [(64, 256, 12, 64, 1, False, True), (64, 256, 10, 128, 2, True, True),
                                                            (128, 512, 6, 128, 1, True, False), (128, 512, 8, 256, 2, False, True)])
def test_dgrad_bn_epilogue_y_recompute_bit_identical(cuda, w3, cout, hin, k1, s, dual, with_pro):
    """argus_bn_bwd_epilogue.y_x: the block-output BN's input y (= conv3(a2), a 1x1 conv with w3 input
    channels) recomputed inside the BN-backward epilogue of the next data gradient (a 1x1 conv from `cout`
    to k1 channels, stride s: the next block's conv1 or its strided downsample, strided phases with
    no taps included) instead of being read: dm, the partials (+ the downsample branch) and the folded
    finalize's outputs bit-identical to the same dgrad reading the y that argus_conv_fwd stored."""
    from argus_amd._lib import BnBwdEpilogue, BnBwdPrologue

    torch.manual_seed(91)
    L = lib()
    n = 3
    # conv3 of block b: a2 (w3 channels) -> y3 (cout), as the forward stores it
    d3, _ = _desc(n, hin, hin, w3, cout, 1, 1)
    a2 = torch.relu(torch.randn(n, hin, hin, w3, device=cuda)).to(torch.bfloat16)
    wf3, _ = _prep(d3, "bf16", (torch.randn(cout, 1, 1, w3) * (2.0 / w3) ** 0.5).to(cuda), cuda)
    y3 = torch.empty(n, hin, hin, cout, dtype=torch.bfloat16, device=cuda)
    rows3 = L.dll.argus_conv_fwd_stat_rows(C.byref(d3), BF16)
    st3 = torch.empty(rows3 * cout * 2, device=cuda)
    L.conv_fwd(C.byref(d3), BF16, ptr(a2), ptr(wf3), ptr(y3), None, None, ptr(st3), stream())
    # the data gradient of block b+1's 1x1 conv (cout -> k1, stride s) whose output feeds bn3's backward
    d, _ = _desc(n, hin, hin, cout, k1, 1, s)
    _, wt = _prep(d, "bf16", (torch.randn(k1, 1, 1, cout) * (2.0 / cout) ** 0.5).to(cuda), cuda)
    dm_in = torch.randn(n, d.ho, d.wo, k1, device=cuda).to(torch.bfloat16)
    ycoef = torch.randn(n, d.ho, d.wo, k1, device=cuda).to(torch.bfloat16)
    ca, cb, cc = (torch.randn(k1, device=cuda) * 0.5 for _ in range(3))
    yd = torch.randn(n, hin, hin, cout, device=cuda).to(torch.bfloat16)
    mean, invstd = torch.randn(cout, device=cuda) * 0.1, torch.rand(cout, device=cuda) + 0.5
    mean2, invstd2 = torch.randn(cout, device=cuda) * 0.1, torch.rand(cout, device=cuda) + 0.5
    gamma, gamma2 = torch.rand(cout, device=cuda) + 0.5, torch.rand(cout, device=cuda) + 0.5
    bits = torch.randint(0, 256, (n * hin * hin * cout // 8,), dtype=torch.uint8, device=cuda)
    add = torch.randn(n, hin, hin, cout, device=cuda).to(torch.bfloat16)
    rows = L.dll.argus_conv_dgrad_bn_rows(C.byref(d), BF16) + 8
    outs = []
    for rec in (False, True):
        dm = add.clone()
        part = torch.zeros(rows, cout, 2, device=cuda)
        part2 = torch.zeros(rows, cout, 2, device=cuda)
        ws = torch.zeros(L.dll.argus_bn_workspace_bytes(cout), dtype=torch.uint8, device=cuda)
        fin = [torch.full((cout,), float("nan"), device=cuda) for _ in range(10)]
        e = BnBwdEpilogue()
        e.mean, e.invstd, e.mask_mode, e.mask_bits, e.part = ptr(mean), ptr(invstd), 3, ptr(bits), ptr(part)
        e.workspace, e.gamma, e.dgamma, e.dbeta, e.ca, e.cb, e.cc = ptr(ws), ptr(gamma), *(ptr(t) for t in fin[:5])
        if dual:
            e.y2, e.mean2, e.invstd2, e.part2 = ptr(yd), ptr(mean2), ptr(invstd2), ptr(part2)
            e.gamma2, e.dgamma2, e.dbeta2, e.ca2, e.cb2, e.cc2 = ptr(gamma2), *(ptr(t) for t in fin[5:])
        if rec:
            e.y_x, e.y_w, e.y_k = ptr(a2), ptr(wf3), w3
        else:
            e.y = ptr(y3)
        pro = BnBwdPrologue(ptr(ycoef), ptr(ca), ptr(cb), ptr(cc), None) if with_pro else None
        L.conv_dgrad_bn(C.byref(d), BF16, ptr(dm_in), ptr(wt), ptr(dm), ptr(dm), C.byref(e),
                        C.byref(pro) if pro is not None else None, stream())
        torch.cuda.synchronize()
        outs.append((dm.clone(), part.clone(), part2.clone(), [t.clone() for t in fin]))
    (a, p_, q, f), (b, r_, t_, h) = outs
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    assert torch.equal(p_, r_) and torch.equal(q, t_)
    assert all(torch.equal(x, z) or (torch.isnan(x).all() and torch.isnan(z).all()) for x, z in zip(f, h))
    assert torch.isfinite(f[0]).all()


def test_fused_dgrad_wgrad_y_recompute_bit_identical(cuda):
    """argus_conv_dgrad_wgrad_bn with pro->y == NULL: bn3's input y3 = conv3(a2) recomputed inside the fused
    layer-1 conv3 data + weight gradient (from the staged a2 tile and the W images) instead of read:
    dx, dW and the folded bn2 finalize bit-identical to the same kernel reading the y3 argus_conv_fwd
    stored; with and without the BN epilogue; ragged row counts."""
    from argus_amd._lib import BnBwdEpilogue, BnBwdPrologue

    torch.manual_seed(32)
    L = lib()
    cin, cout = 64, 256
    for n, h, w_ in [(2, 33, 33), (1, 5, 7), (4, 64, 64)]:
        d, _ = _desc(n, h, w_, cin, cout, 1, 1)
        P = n * h * w_
        wt_ohwi = (torch.randn(cout, 1, 1, cin) * (2.0 / cin) ** 0.5).to(cuda)
        wf, wt = _prep(d, "bf16", wt_ohwi, cuda)
        a2 = torch.relu(torch.randn(P, cin, device=cuda)).to(torch.bfloat16)
        y3 = torch.empty(P, cout, dtype=torch.bfloat16, device=cuda)
        st = torch.empty(L.dll.argus_conv_fwd_stat_rows(C.byref(d), BF16) * cout * 2, device=cuda)
        L.conv_fwd(C.byref(d), BF16, ptr(a2), ptr(wf), ptr(y3), None, None, ptr(st), stream())
        dm = torch.randn(P, cout, device=cuda).to(torch.bfloat16)
        ca, cb, cc = (torch.randn(cout, device=cuda) * 0.3 for _ in range(3))
        y2 = torch.randn(P, cin, device=cuda).to(torch.bfloat16)
        mean, invstd = torch.randn(cin, device=cuda) * 0.1, torch.rand(cin, device=cuda) + 0.5
        sc, sh = torch.randn(cin, device=cuda), torch.randn(cin, device=cuda)
        g2 = torch.rand(cin, device=cuda) + 0.5
        base = torch.randn(P, cin, device=cuda).to(torch.bfloat16)
        for with_bn in (True, False):
            res = []
            for rec in (False, True):
                ws = torch.zeros(L.dll.argus_bn_workspace_bytes(2048), dtype=torch.uint8, device=cuda)
                rows = L.dll.argus_conv_dgrad_wgrad_bn_rows(C.byref(d), BF16)
                part = torch.empty(rows, cin, 2, device=cuda)
                co = torch.zeros(5, cin, device=cuda)
                e = BnBwdEpilogue()
                e.y, e.mean, e.invstd, e.mask_mode, e.scale, e.shift, e.part = ptr(y2), ptr(mean), ptr(invstd), 2, \
                    ptr(sc), ptr(sh), ptr(part)
                e.workspace, e.gamma, e.dgamma, e.dbeta = ptr(ws), ptr(g2), ptr(co[3]), ptr(co[4])
                e.ca, e.cb, e.cc = ptr(co[0]), ptr(co[1]), ptr(co[2])
                pro = BnBwdPrologue(None if rec else ptr(y3), ptr(ca), ptr(cb), ptr(cc), None)
                dx = base.clone()
                dw = torch.empty(cout, 1, 1, cin, device=cuda)
                wsw = torch.empty(L.dll.argus_conv_dgrad_wgrad_workspace_bytes(C.byref(d), BF16), dtype=torch.uint8,
                                  device=cuda)
                rc = L.dll.argus_conv_dgrad_wgrad_bn(C.byref(d), BF16, ptr(dm), ptr(wt), ptr(a2), ptr(dx),
                                                     None if with_bn else ptr(dx), C.byref(e) if with_bn else None,
                                                     C.byref(pro), ptr(dw), ptr(wsw), wsw.numel(), stream())
                assert rc == 0, L.dll.argus_last_error()
                torch.cuda.synchronize()
                res.append((dx.view(torch.int16).cpu(), dw.cpu(), co.cpu(), part.cpu()))
            (x0, w0, c0, p0), (x1, w1, c1, p1) = res
            assert torch.equal(x0, x1), (n, h, w_, with_bn)
            assert torch.equal(w0, w1), (n, h, w_, with_bn)
            if with_bn:
                assert torch.equal(c0, c1) and torch.equal(p0, p1), (n, h, w_)


@pytest.mark.parametrize("n4w,w,hw,dual", [(256, 64, 12, False), (256, 64, 9, True), (512, 128, 8, True),
                                           (1024, 256, 5, False), (1024, 256, 7, True)])
def test_persistent_conv1_dgrad_matches_igemm(cuda, n4w, w, hw, dual):
    """The persistent 1x1 data gradient (conv_p1x1.hip, policy key 43: a bottleneck conv1's dgrad with the
    BN-backward apply prologue and the previous block's output-BN backward epilogue, mask bits, optional
    downsample branch, folded finalize) against the register-staged igemm_kernel it replaces (key 43 = 0):
    dm bit-identical (same apply, same MFMA order, same bf16 rounding, addend, mask); the finalize outputs
    (dgamma, dbeta, ca, cb, cc of both branches) to fp32 summation order (their partial rows group
    differently); ragged row counts (hw = 5, 7, 9)."""
    from argus_amd._lib import BnBwdEpilogue, BnBwdPrologue
    from argus_amd.profiling import KernelTimer

    torch.manual_seed(93)
    L = lib()
    n = 5
    d, _ = _desc(n, hw, hw, n4w, w, 1, 1)  # conv1: 4w -> w; its dgrad: w -> 4w channels
    _, wt = _prep(d, "bf16", (torch.randn(w, 1, 1, n4w) * (2.0 / n4w) ** 0.5).to(cuda), cuda)
    P = n * hw * hw
    dm1 = torch.randn(P, w, device=cuda).to(torch.bfloat16)
    y1 = torch.randn(P, w, device=cuda).to(torch.bfloat16)
    ca, cb, cc = (torch.randn(w, device=cuda) * 0.5 for _ in range(3))
    dh = torch.randn(P, n4w, device=cuda).to(torch.bfloat16)
    y3 = torch.randn(P, n4w, device=cuda).to(torch.bfloat16)
    yd = torch.randn(P, n4w, device=cuda).to(torch.bfloat16)
    bits = torch.randint(0, 256, (P * n4w // 8,), dtype=torch.uint8, device=cuda)
    mean, invstd = torch.randn(n4w, device=cuda) * 0.1, torch.rand(n4w, device=cuda) + 0.5
    mean2, invstd2 = torch.randn(n4w, device=cuda) * 0.1, torch.rand(n4w, device=cuda) + 0.5
    gamma, gamma2 = torch.rand(n4w, device=cuda) + 0.5, torch.rand(n4w, device=cuda) + 0.5
    rows = L.dll.argus_conv_dgrad_bn_rows(C.byref(d), BF16)
    outs = []
    for key in (0, 1):
        dk = d.with_tuning({43: key, 49: 0})  # 49 = 0: the prologue staged at every width (4w up to 1024)
        out = torch.empty(P, n4w, dtype=torch.bfloat16, device=cuda)
        part = torch.zeros(rows, n4w, 2, device=cuda)
        part2 = torch.zeros(rows, n4w, 2, device=cuda)
        ws = torch.zeros(L.dll.argus_bn_workspace_bytes(n4w), dtype=torch.uint8, device=cuda)
        fin = [torch.full((n4w,), float("nan"), device=cuda) for _ in range(10)]
        e = BnBwdEpilogue()
        e.y, e.mean, e.invstd, e.mask_mode, e.mask_bits, e.part = ptr(y3), ptr(mean), ptr(invstd), 3, ptr(bits), \
            ptr(part)
        e.workspace, e.gamma, e.dgamma, e.dbeta, e.ca, e.cb, e.cc = ptr(ws), ptr(gamma), *(ptr(t) for t in fin[:5])
        if dual:
            e.y2, e.mean2, e.invstd2, e.part2 = ptr(yd), ptr(mean2), ptr(invstd2), ptr(part2)
            e.gamma2, e.dgamma2, e.dbeta2, e.ca2, e.cb2, e.cc2 = ptr(gamma2), *(ptr(t) for t in fin[5:])
        pro = BnBwdPrologue(ptr(y1), ptr(ca), ptr(cb), ptr(cc), None)
        with KernelTimer() as kt:
            L.conv_dgrad_bn(C.byref(dk), BF16, ptr(dm1), ptr(wt), ptr(out), ptr(dh), C.byref(e), C.byref(pro), stream())
        torch.cuda.synchronize()
        names = list(kt.summary())
        assert any(nm.startswith("argus::p1x1_dgrad_kernel") for nm in names) == bool(key), names
        assert int(ws[:16384].view(torch.int32).abs().sum()) == 0  # finalize counters left at zero
        outs.append((out.view(torch.int16).clone(), [t.clone() for t in fin]))
    (o0, f0), (o1, f1) = outs
    assert torch.equal(o0, o1), (n4w, w, hw, dual)
    for i, (a, b) in enumerate(zip(f0, f1)):
        if not dual and i >= 5:
            continue
        assert torch.isfinite(b).all(), i
        assert _rel(b, a) < 1e-5, (i, _rel(b, a))


# (cin, cout, k, stride, hw, n, dtype, tuning, prologue, store y): one forward producer each —
# igemm 1x1 / strided / 3x3 (fp32 + bf16, with and without the BN+ReLU prologue), glds (key 8),
# halo (key 13, plain and deep ring), the persistent statistics-only 1x1 (y NULL), MX-fp8
FWD_FIN_CASES = [
    (64, 256, 1, 1, 12, 3, "fp32", None, False, True), (64, 256, 1, 1, 12, 3, "bf16", None, True, True),
    (256, 512, 1, 2, 13, 2, "bf16", None, False, True), (128, 128, 3, 2, 12, 2, "bf16", None, False, True),
    (128, 128, 3, 1, 9, 3, "fp32", None, True, True),
    (128, 256, 1, 1, 24, 4, "bf16", {8: 64, 9: 1}, False, True), (256, 256, 3, 2, 20, 4, "bf16", {8: 64, 9: 1}, False, True),
    (64, 64, 3, 1, 64, 1, "bf16", {13: 1}, False, True), (128, 128, 3, 1, 16, 3, "bf16", {13: 1, 51: 1}, False, True),
    (64, 256, 1, 1, 16, 4, "bf16", None, False, False), (128, 512, 1, 1, 9, 3, "bf16", None, False, False),
    (256, 1024, 1, 1, 30, 8, "bf16", None, False, False), (256, 1024, 1, 1, 16, 128, "bf16", None, False, False),
    (128, 128, 3, 1, 16, 4, "fp8", {37: 7}, False, True), (256, 512, 1, 1, 12, 4, "fp8", {37: 7}, False, True),
]


def _fwd_fin_run(L, d, dt, x, wf, y, sc, sh, rows, tile, count, cout, folded, cuda):
    """one training forward + finalize: argus_conv_fwd_fin (folded) or argus_conv_fwd + argus_bn_finalize;
    returns every output, the kernel names launched and the workspace counters."""
    from argus_amd._lib import BnFwdFin
    from argus_amd.profiling import KernelTimer

    ws = torch.zeros(L.dll.argus_bn_workspace_bytes(2048), dtype=torch.uint8, device=cuda)
    st = torch.full((rows * cout * 2 + rows,), float("nan"), device=cuda)
    g = torch.linspace(0.5, 1.5, cout, device=cuda)
    b = torch.linspace(-0.2, 0.3, cout, device=cuda)
    rm, rv = torch.linspace(-1, 1, cout, device=cuda), torch.linspace(0.5, 2, cout, device=cuda)
    nbt = torch.full((1,), 7, dtype=torch.int64, device=cuda)
    outs = torch.full((4, cout), float("nan"), device=cuda)
    with KernelTimer() as t:
        if folded:
            f = BnFwdFin()
            f.workspace, f.gamma, f.beta, f.eps, f.momentum = ptr(ws), ptr(g), ptr(b), 1e-5, 0.1
            f.running_mean, f.running_var, f.num_batches_tracked = ptr(rm), ptr(rv), ptr(nbt)
            f.mean, f.invstd, f.scale, f.shift = ptr(outs[0]), ptr(outs[1]), ptr(outs[2]), ptr(outs[3])
            L.conv_fwd_fin(C.byref(d), DT[dt], ptr(x), ptr(wf), ptr(y), ptr(sc), ptr(sh), ptr(st), C.byref(f), stream())
        else:
            L.conv_fwd(C.byref(d), DT[dt], ptr(x), ptr(wf), ptr(y), ptr(sc), ptr(sh), ptr(st), stream())
            L.bn_finalize(cout, rows, tile, ptr(st), count, ptr(g), ptr(b), C.c_float(1e-5), C.c_float(0.1), ptr(rm),
                          ptr(rv), ptr(nbt), ptr(outs[0]), ptr(outs[1]), ptr(outs[2]), ptr(outs[3]), ptr(ws), stream())
        names = set(t.summary())
    torch.cuda.synchronize()
    ctr = int(ws[:16384].view(torch.int32).abs().sum())
    return [v.cpu() for v in ((y if y is not None else st[:0]), st, outs, rm, rv, nbt)], names, ctr


def test_forward_bn_finalize_folded_bit_identical(cuda):
    """argus_conv_fwd_fin (ABI 18): the forward BN statistics finalize folded into the producing conv's
    last-arriving workgroups (bnfin.h: row lanes merge each workgroup's tiles, one group slot per
    argus_bn_finalize group, the last group's arrival finishes the channel) gives BIT-IDENTICAL y,
    partials, mean / invstd / scale / shift, running mean / var and num_batches_tracked to argus_conv_fwd
    + argus_bn_finalize on the same inputs, launches no stats_finalize_kernel where the producer's tiles
    align with the finalize's groups (igemm, persistent statistics-only, stem) and leaves its ticket
    counters at zero; igemm / glds / halo (plain, deep ring) / statistics-only / MX-fp8 producers, with
    and without a BN+ReLU prologue, ragged M; the stem at 376x672 (ragged int32 row counts)."""
    torch.manual_seed(41)
    L = lib()
    unfolded = []
    for cin, cout, k, s, hw, n, dt, tune, pro, store in FWD_FIN_CASES:
        d, _ = _desc(n, hw, hw, cin, cout, k, s)
        if tune:
            d = d.with_tuning(tune)
        wdt = "bf16" if dt == "fp8" else dt  # argus_conv_fwd_stat_tile of an MX-fp8 forward: the bf16 tile
        x = (torch.randn(n, hw, hw, cin, device=cuda) * 1.3 + 0.1).to(TDT[dt])
        wf, _ = _prep(d, dt, (torch.randn(cout, k, k, cin) * (2.0 / (k * k * cin)) ** 0.5).to(cuda), cuda)
        sc = (torch.rand(cin, device=cuda) + 0.5) if pro else None
        sh = (torch.randn(cin, device=cuda) * 0.3) if pro else None
        so = not store and not pro
        rows = (L.dll.argus_conv_fwd_stats_only_rows if so else L.dll.argus_conv_fwd_stat_rows)(C.byref(d), DT[dt])
        tile = (L.dll.argus_conv_fwd_stats_only_tile if so else L.dll.argus_conv_fwd_stat_tile)(C.byref(d), DT[wdt])
        count = n * d.ho * d.wo
        res = []
        for folded in (False, True):
            y = torch.empty(n, d.ho, d.wo, cout, dtype=TDT[dt], device=cuda) if store else None
            res.append(_fwd_fin_run(L, d, dt, x, wf, y, sc, sh, rows, tile, count, cout, folded, cuda))
        case = (cin, cout, k, s, hw, n, dt, tune, pro, store)
        for a, b in zip(res[0][0], res[1][0]):
            assert torch.equal(a.view(torch.uint8) if a.is_floating_point() else a,
                               b.view(torch.uint8) if b.is_floating_point() else b), case
        assert int(res[1][0][5]) == 8 and res[0][2] == 0 and res[1][2] == 0, case
        assert "argus::stats_finalize_kernel" in res[0][1], case
        if "argus::stats_finalize_kernel" in res[1][1]:
            unfolded.append((case, sorted(res[1][1])))
    # the register-staged igemm (one partial row per tile) and the statistics-only kernel always fold
    assert not [c for c in unfolded if any(k.startswith(("argus::igemm_kernel", "argus::p1x1_fwd_stats"))
                                           for k in c[1])], unfolded
    # the stem: ragged 376x672 (int32 row counts after the partials) and a small odd image; n = 1 at
    # 376x672 gives 528 partial rows in 32 finalize groups of 17 rows, which splits a two-row stem tile,
    # so that case takes the separate finalize (still bit-identical); n = 4 (66-row groups) folds
    for n, H, W, folds in [(1, 376, 672, False), (4, 376, 672, True), (3, 38, 30, True)]:
        for dt in ("fp32", "bf16"):
            d, _ = _desc(n, H, W, 3, 64, 7, 2, stem=True)
            x4 = torch.zeros(n, H, W, 4, device=cuda)
            x4[..., :3] = torch.rand(n, H, W, 3, device=cuda)
            x4 = x4.to(TDT[dt])
            wm = (torch.randn(64, 3, 7, 7) * 0.1).to(cuda)
            wf = torch.empty(64, 256, dtype=TDT[dt], device=cuda)
            L.conv_weight_prep(C.byref(d), DT[dt], ptr(wm), (C.c_int64 * 4)(*wm.stride()), ptr(wf), None, stream())
            rows = L.dll.argus_conv_fwd_stat_rows(C.byref(d), DT[dt])
            tile = L.dll.argus_conv_fwd_stat_tile(C.byref(d), DT[dt])
            res = [_fwd_fin_run(L, d, dt, x4, wf, torch.empty(n, d.ho, d.wo, 64, dtype=TDT[dt], device=cuda), None,
                                None, rows, tile, n * d.ho * d.wo, 64, folded, cuda) for folded in (False, True)]
            for a, b in zip(res[0][0], res[1][0]):
                assert torch.equal(a.view(torch.uint8) if a.is_floating_point() else a,
                                   b.view(torch.uint8) if b.is_floating_point() else b), ("stem", n, H, W, dt)
            assert res[1][2] == 0, ("stem", n, H, W, dt)
            if folds or dt == "fp32":  # fp32: the register-staged STEM igemm (one partial row a tile)
                assert "argus::stats_finalize_kernel" not in res[1][1], ("stem", n, H, W, dt, res[1][1])
