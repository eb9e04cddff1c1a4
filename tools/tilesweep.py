"""Sweep conv tile configs per layer/pass (dev tool, GPU) via per-call kernel-selection overrides (ConvDesc.with_tuning).
python tools/tilesweep.py [--batch 64]"""
import argparse
import ctypes as C
import itertools
import sys

import torch

sys.path.insert(0, ".")
from argus_amd._lib import lib, ptr, stream  # noqa: E402
from argus_amd.engine import ResNetEngine  # noqa: E402


def timeit(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dtype", default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = ResNetEngine(2, 1024, a.dtype, dev)
    eng.ensure(a.batch, 256, 256)
    L = lib()
    dt, tdt = eng.dt, eng.tdt
    seen = {}
    best_total = {0: 0.0, 1: 0.0, 2: 0.0}
    base_total = {0: 0.0, 1: 0.0, 2: 0.0}
    for name, cv in eng.convs.items():
        d = cv.desc
        key = (d.h, d.c, d.k, d.r, d.stride, d.stem)
        x = torch.randn(d.n, d.h, d.w, 4 if d.stem else d.c, device=dev).to(tdt)
        y = torch.empty(d.n, d.ho, d.wo, d.k, device=dev, dtype=tdt)
        dy = torch.randn(d.n, d.ho, d.wo, d.k, device=dev).to(tdt)
        dx = torch.empty(d.n, d.h, d.w, d.c, device=dev, dtype=tdt)
        dw = torch.empty(d.k * d.r * d.s * d.c, device=dev)
        st = torch.empty((d.n * d.ho * d.wo // 64 + 1) * d.k * 2, device=dev)
        cv.wf.normal_()
        res = seen.get(key)
        if res is None:
            res = {}
            for ps in (0, 1, 2):
                if ps == 1 and d.stem:
                    continue
                opts = {}
                cfgs = list(itertools.product((64, 128), (64, 128)))
                if ps == 2:
                    cfgs = [(bm, bn, tb) for bm, bn in cfgs for tb in (256, 512, 1024, 2048)]
                d0 = d
                for cfg in cfgs:
                    tun = {ps: cfg[0], 3 + ps: cfg[1]}
                    if ps == 2:
                        tun[6] = cfg[2]
                    d = d0.with_tuning(tun)
                    if d.stem and ps == 0 and cfg != (128, 64):
                        continue
                    if ps == 0:
                        fn = lambda: L.conv_fwd(C.byref(d), dt, ptr(x), ptr(cv.wf), ptr(y), None, None, ptr(st), stream())
                    elif ps == 1:
                        fn = lambda: L.conv_dgrad(C.byref(d), dt, ptr(dy), ptr(cv.wd), ptr(dx), None, None, stream())
                    else:
                        wsb = L.dll.argus_conv_wgrad_workspace_bytes(C.byref(d), dt)
                        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
                        fn = lambda: L.conv_wgrad(C.byref(d), dt, ptr(x), None, None, ptr(dy), ptr(dw), ptr(ws), wsb,
                                                  stream())
                    opts[cfg] = timeit(fn)
                d = d0
                res[ps] = opts
            seen[key] = res
        line = f"{name:30s} {d.h:3d} {d.c:4d}->{d.k:4d} k{d.r}s{d.stride} "
        for ps, opts in res.items():
            b = min(opts, key=opts.get)
            base = [v for c, v in opts.items() if c[:2] == tuple(opts and (128 if True else 64) for _ in range(0))] or [0]
            best_total[ps] += opts[b]
            line += f" p{ps} best {b} {opts[b]:7.1f}us |"
        print(line, flush=True)
    print("best totals (ms):", {k: round(v / 1e3, 3) for k, v in best_total.items()}, sum(best_total.values()) / 1e3)
    for key, res in seen.items():
        print("RAW", key, {ps: {str(c): round(v, 1) for c, v in o.items()} for ps, o in res.items()})


if __name__ == "__main__":
    main()
