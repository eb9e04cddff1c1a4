"""Per-layer conv microbenchmark (dev tool, GPU): fwd / dgrad / wgrad time, TFLOP/s and fraction of
the per-launch roofline max(flops / 2.5 PF, algorithmic bytes / 8 TB/s) for every ResNet-50 conv at a
given batch, through the C ABI.  python tools/convbench.py [--batch 64] [--dtype bf16]"""
import argparse
import ctypes as C
import sys

import torch

sys.path.insert(0, ".")
from argus_amd._lib import BF16, F32, lib, ptr, stream  # noqa: E402
from argus_amd.engine import ResNetEngine  # noqa: E402
from argus_amd.profiling import KernelTimer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hw", type=int, nargs=2, default=(256, 256))
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--filter", default="")
    ap.add_argument("--tune", nargs="*", default=[], help="kernel-selection overrides key=value")
    a = ap.parse_args()
    tuning = {int(k): int(v) for k, v in (kv.split("=") for kv in a.tune)}
    dev = torch.device("cuda", 0)
    eng = ResNetEngine(2, 1024, a.dtype, dev, tuning)
    eng.ensure(a.batch, *a.hw)
    L = lib()
    dt = eng.dt
    tdt = eng.tdt
    tot = {0: 0.0, 1: 0.0, 2: 0.0}
    totf = 0
    seen = {}
    for name, cv in eng.convs.items():
        d = cv.desc
        key = (d.h, d.w, d.c, d.k, d.r, d.stride, d.stem)
        if a.filter and a.filter not in name:
            continue
        x = torch.randn(d.n, d.h, d.w, 4 if d.stem else d.c, device=dev).to(tdt)
        y = torch.empty(d.n, d.ho, d.wo, d.k, device=dev, dtype=tdt)
        dy = torch.randn(d.n, d.ho, d.wo, d.k, device=dev).to(tdt)
        dx = torch.empty(d.n, d.h, d.w, d.c, device=dev, dtype=tdt)
        dw = torch.empty(d.k * d.r * d.s * d.c, device=dev)
        st = torch.empty(cv.stat_rows * d.k * 2 + cv.stat_rows, device=dev)  # + ragged row counts
        ws = torch.empty(L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), dt), dtype=torch.uint8, device=dev)
        wf = cv.wf.normal_() if tdt == torch.float32 else cv.wf.copy_(torch.randn_like(cv.wf, dtype=torch.float32))
        wd = cv.wd if cv.wd is not None else None
        fns = {
            0: lambda: L.conv_fwd(C.byref(d), eng.cdt, ptr(x), ptr(cv.wf), ptr(y), None, None, ptr(st), stream()),
            2: lambda: L.conv_wgrad(C.byref(d), dt, ptr(x), None, None, ptr(dy), ptr(dw), ptr(ws), ws.numel(), stream()),
        }
        if not d.stem:
            fns[1] = lambda: L.conv_dgrad(C.byref(d), eng.cdt, ptr(dy), ptr(wd), ptr(dx), None, None, stream())
        row = [name]
        for ps, fn in fns.items():
            with KernelTimer() as kt:
                fn()
            ksum = kt.summary()
            kname = max(ksum, key=lambda n: ksum[n]["total_ms"])
            main_k = ksum[kname]
            roof_us = max(main_k["flops_per_launch"] / 2.5e15, main_k["bytes_per_launch"] / 8e12) * 1e6
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.reps):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1e3 / a.reps
            tot[ps] += us
            short = kname.replace("argus::", "").replace("_kernel", "").replace("__bf16, ", "").replace("false", "f").replace("true", "t")
            row.append(f"p{ps}:{us:7.1f}us {cv.flops / us / 1e6:6.1f}TF {roof_us / us:4.0%} {short:24s}")
        totf += cv.flops * (2 if d.stem else 3)
        print(f"{name:32s} {d.h:3d}x{d.w:<3d} {d.c:4d}->{d.k:4d} k{d.r} s{d.stride}  " + "  ".join(row[1:]))
    allus = sum(tot.values())
    print(f"total fwd {tot[0]/1e3:.2f} ms dgrad {tot[1]/1e3:.2f} ms wgrad {tot[2]/1e3:.2f} ms = {allus/1e3:.2f} ms, "
          f"{totf / allus / 1e6:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
