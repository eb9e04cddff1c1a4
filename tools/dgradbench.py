"""BN-fused dgrad microbenchmark (dev tool, GPU): for every bottleneck block at a given batch, time the
conv1 dgrad (mask-bit epilogue of the previous bn3 + residual addend, apply prologue of bn1, folded
finalize: the benched schedule), the conv3 dgrad, and with --convs conv2 the 3x3 one (bn1's recomputed-
mask epilogue; its apply prologue is the materialising apply pass), and their stripped variants,
through the C ABI.
python tools/dgradbench.py [--batch 64] [--filter layer3] [--convs conv1,conv3,conv2] [--tune k=v ...]"""
import argparse
import ctypes as C
import sys

import torch

sys.path.insert(0, ".")
from argus_amd._lib import BnBwdEpilogue, BnBwdPrologue, lib, ptr, stream  # noqa: E402
from argus_amd.engine import ResNetEngine  # noqa: E402


def timeit(fn, reps):
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
    ap.add_argument("--hw", type=int, nargs=2, default=(256, 256))
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--filter", default="")
    ap.add_argument("--tune", nargs="*", default=[])
    ap.add_argument("--convs", default="conv1,conv3")
    a = ap.parse_args()
    L = lib()
    tuning = {int(k): int(v) for k, v in (kv.split("=") for kv in a.tune)}
    dev = torch.device("cuda", 0)
    eng = ResNetEngine(2, 1024, "bf16", dev, tuning)
    eng.ensure(a.batch, *a.hw)
    bf = torch.bfloat16
    ws = torch.zeros(L.dll.argus_bn_workspace_bytes(2048), dtype=torch.uint8, device=dev)
    tot = {}
    seen = set()
    for idx, b in enumerate(eng.blocks):
        for which in a.convs.split(","):
            name = f"{b.prefix}.{which}"
            if a.filter and a.filter not in name:
                continue
            cv = eng.convs[name]
            d = cv.desc
            key = (which, d.h, d.w, d.c, d.k, idx == 0 or b.has_ds)
            if key in seen:
                continue
            seen.add(key)
            if which == "conv1" and idx == 0:
                continue  # block 0's conv1 dgrad has no BN epilogue (the stem's maxpool follows)
            px_o, px_i = d.n * d.ho * d.wo, d.n * d.h * d.w
            dm_in = torch.randn(px_o * d.k, device=dev).to(bf)
            y_in = torch.randn(px_o * d.k, device=dev).to(bf)
            out = torch.empty(px_i * d.c, device=dev, dtype=bf)
            add = torch.randn(px_i * d.c, device=dev).to(bf)
            yb = torch.randn(px_i * d.c, device=dev).to(bf)
            bits = torch.randint(0, 256, (px_i * d.c // 8,), dtype=torch.uint8, device=dev)
            ck = lambda n: torch.rand(n, device=dev) + 0.5  # noqa: E731
            cin = {k: ck(d.k) for k in ("ca", "cb", "cc")}
            cout = {k: ck(d.c) for k in ("mean", "invstd", "sc", "sh", "gamma", "dg", "db", "ca", "cb", "cc")}
            rows = L.dll.argus_conv_dgrad_bn_rows(C.byref(d), 1)
            part = torch.empty(rows * d.c * 2, device=dev)
            mode = 3 if which == "conv1" else 2

            def epi(fin):
                e = BnBwdEpilogue()
                e.y, e.mean, e.invstd, e.mask_mode = ptr(yb), ptr(cout["mean"]), ptr(cout["invstd"]), mode
                if mode == 2:
                    e.scale, e.shift = ptr(cout["sc"]), ptr(cout["sh"])
                else:
                    e.mask_bits = ptr(bits)
                e.part = ptr(part)
                if fin:
                    e.workspace, e.gamma, e.dgamma, e.dbeta = ptr(ws), ptr(cout["gamma"]), ptr(cout["dg"]), ptr(cout["db"])
                    e.ca, e.cb, e.cc = ptr(cout["ca"]), ptr(cout["cb"]), ptr(cout["cc"])
                return e

            staged = bool(L.dll.argus_conv_dgrad_stages_prologue(C.byref(d), 1))
            dyo = None if staged else torch.empty(px_o * d.k, device=dev, dtype=bf)
            pro = BnBwdPrologue(ptr(y_in), ptr(cin["ca"]), ptr(cin["cb"]), ptr(cin["cc"]), ptr(dyo) if dyo is not None else None)
            addend = ptr(add) if mode == 3 else None
            variants = {
                "plain": lambda: L.conv_dgrad(C.byref(d), 1, ptr(dm_in), ptr(cv.wd), ptr(out), None, None, stream()),
                "epi": lambda: L.conv_dgrad_bn(C.byref(d), 1, ptr(dm_in), ptr(cv.wd), ptr(out), addend,
                                               C.byref(epi(False)), None, stream()),
                "epi+fin": lambda: L.conv_dgrad_bn(C.byref(d), 1, ptr(dm_in), ptr(cv.wd), ptr(out), addend,
                                                   C.byref(epi(True)), None, stream()),
                "pro": lambda: L.conv_dgrad_bn(C.byref(d), 1, ptr(dm_in), ptr(cv.wd), ptr(out), None, None,
                                               C.byref(pro), stream()),
                "full": lambda: L.conv_dgrad_bn(C.byref(d), 1, ptr(dm_in), ptr(cv.wd), ptr(out), addend,
                                                C.byref(epi(True)), C.byref(pro), stream()),
            }
            E = 2.0
            full_bytes = E * (2 * px_o * d.k + px_i * d.c * (2 + (1 if mode == 3 else 0)) + d.k * d.c) + \
                (px_i * d.c / 8 if mode == 3 else 0)
            row = []
            for vn, fn in variants.items():
                us = timeit(fn, a.reps)
                tot[vn] = tot.get(vn, 0.0) + us
                row.append(f"{vn} {us:7.1f}")
            print(f"{name:26s} {d.h:3d}x{d.w:<3d} {d.k:4d}->{d.c:4d} rows {rows:5d}  " + "  ".join(row) +
                  f"   full {full_bytes / 1e6:7.1f} MB {full_bytes / (us * 1e-6) / 1e12:5.2f} TB/s", flush=True)
    print("totals (distinct shapes):", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
