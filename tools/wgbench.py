"""1x1 weight-gradient microbenchmark (dev tool, GPU): every distinct 1x1 stride-1 ResNet-50 conv at a
given batch, plain (argus_conv_wgrad) and with the BN-backward apply staged (argus_conv_wgrad_apply),
under policy key 45 = 3 / 2 / 1 (LDS-DMA ring kernel; 3: 256-wide tiles for both forms, 2: for the
apply form, 1: 128-wide) and 0 (register-staged wgrad_kernel), timed in
isolation with HIP events. python tools/wgbench.py [--batch 64] [--hw 256 256]"""
import argparse
import ctypes as C
import sys

import torch

sys.path.insert(0, ".")
from argus_amd._lib import BF16, BnBwdPrologue, lib, ptr, stream  # noqa: E402
from argus_amd.engine import ResNetEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hw", type=int, nargs=2, default=(256, 256))
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = ResNetEngine(2, 1024, "bf16", dev, {})
    eng.ensure(a.batch, *a.hw)
    L = lib()
    seen = set()
    tot = {}
    for name, cv in eng.convs.items():
        d0 = cv.desc
        key = (d0.h, d0.w, d0.c, d0.k)
        if d0.stem or d0.r != 1 or d0.stride != 1 or key in seen:
            continue
        seen.add(key)
        x = torch.randn(d0.n, d0.h, d0.w, d0.c, device=dev).to(torch.bfloat16)
        dm = torch.randn(d0.n, d0.ho, d0.wo, d0.k, device=dev).to(torch.bfloat16)
        yb = torch.randn_like(dm)
        ca, cb, cc = (torch.randn(d0.k, device=dev) for _ in range(3))
        pro = BnBwdPrologue(ptr(yb), ptr(ca), ptr(cb), ptr(cc), None)
        dw = torch.empty(d0.k * d0.c, device=dev)
        cols = []
        for apply in (False, True):
            for k45 in (3, 2, 1, 0):
                d = d0.with_tuning({45: k45})
                wsb = L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), BF16)
                ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
                if apply:
                    fn = lambda: L.conv_wgrad_apply(C.byref(d), BF16, ptr(x), ptr(dm), C.byref(pro), ptr(dw), ptr(ws),
                                                    wsb, stream())
                else:
                    fn = lambda: L.conv_wgrad(C.byref(d), BF16, ptr(x), None, None, ptr(dm), ptr(dw), ptr(ws), wsb,
                                              stream())
                fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.reps):
                    fn()
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) * 1e3 / a.reps
                tot[(apply, k45)] = tot.get((apply, k45), 0.0) + us
                cols.append(f"{'ap' if apply else 'pl'}{k45}:{us:7.1f}")
        print(f"{name:28s} {d0.h:3d}x{d0.w:<3d} {d0.c:4d}->{d0.k:4d}  " + "  ".join(cols))
    print("total us: " + "  ".join(f"{'ap' if k[0] else 'pl'}{k[1]}:{v:8.1f}" for k, v in sorted(tot.items())))


if __name__ == "__main__":
    main()
