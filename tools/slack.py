"""Per-kernel slack of one fused train step (dev tool, GPU): every instantiation's measured time next to
the lower bound its algorithmic work allows, per stream.

    python tools/slack.py [--batch 64] [--hw 256 256] [--dtype bf16] [--steps 3] [--pmc profiles/r04d_pmc_traffic.json]

bound_us = max(algorithmic bytes / HBM_ACH, flops / MFMA_ACH) with the achievable rates of
MI355X_MICROARCH.md (a float4 copy reaches ~6.3 TB/s; the dense bf16 MFMA loop ~2.3 PF/s); slack =
measured - bound, summed per step. With --pmc, the measured HBM bytes per launch of that PMC summary
(same workload) are joined by instantiation name: traffic / algorithmic is the re-read factor.
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from bench import synthetic_batch  # noqa: E402

HBM_ACH = 6.3e12
MFMA_ACH = {"bf16": 2.3e15, "fp8": 2.3e15, "fp32": 0.15e15}


def table(summ, nsteps, dtype, pmc):
    rows = []
    for k, v in summ.items():
        n = v["launches"] / nsteps
        t = v["total_ms"] / nsteps
        bound = max(v["bytes_per_launch"] / HBM_ACH, v["flops_per_launch"] / MFMA_ACH[dtype]) * 1e3 * n
        tr = pmc.get(k)
        rows.append((t - bound, t, bound, n, v, k, tr))
    rows.sort(reverse=True)
    tot_t = sum(r[1] for r in rows)
    tot_b = sum(r[2] for r in rows)
    out = [f"{'slack ms':>8} {'meas ms':>8} {'bound ms':>8} {'n/step':>6} {'avg us':>8} {'alg MB':>8} {'GFLOP':>7} "
           f"{'TB/s':>5} {'TF/s':>6} {'pmc/alg':>7}  kernel"]
    for sl, t, b, n, v, k, tr in rows:
        ratio = f"{tr / v['bytes_per_launch']:.2f}" if tr and v["bytes_per_launch"] else "-"
        out.append(f"{sl:8.3f} {t:8.3f} {b:8.3f} {n:6.1f} {v['avg_us']:8.1f} {v['bytes_per_launch'] / 1e6:8.1f} "
                   f"{v['flops_per_launch'] / 1e9:7.2f} {v['bytes_per_launch'] / v['avg_us'] / 1e6:5.2f} "
                   f"{v['flops_per_launch'] / v['avg_us'] / 1e6:6.0f} {ratio:>7}  {k}")
    out.append(f"{tot_t - tot_b:8.3f} {tot_t:8.3f} {tot_b:8.3f}  total (timed kernels only)")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hw", type=int, nargs=2, default=(256, 256))
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pmc", default=None)
    ap.add_argument("--cfg", default="", help="engine attributes attr=value and tune:key=value policy overrides, "
                    "comma-separated (as tools/engine_ab.py)")
    ap.add_argument("--streams", default="main,all", help="which tables: main, all")
    a = ap.parse_args()
    from argus_amd.models import NCameraCNN
    from argus_amd.profiling import KernelTimer
    from argus_amd.step import FusedTrainer

    pmc = {}
    if a.pmc:
        d = json.load(open(a.pmc))
        pmc = {k: v["traffic_bytes_per_launch"] for k, v in d["kernels"].items()}
    dev = torch.device("cuda", 0)
    images, targets = synthetic_batch(a.batch, *a.hw, 1000, dev)
    torch.manual_seed(42)
    tune, attrs = {}, {}
    for kv in filter(None, a.cfg.split(",")):
        k, v = kv.split("=")
        if k.startswith("tune:"):  # a kernel-selection policy override (argus_conv_policy_default key)
            tune[int(k[5:])] = int(v)
        else:
            attrs[k] = v
    m = NCameraCNN(compute_dtype=a.dtype, kernel_tuning=tune or None).to(dev).train()
    eng = m._engine(dev)
    for k, v in attrs.items():
        cur = getattr(eng, k)
        setattr(eng, k, v == "1" if isinstance(cur, bool) else type(cur)(int(v)))
    tr = FusedTrainer(m, lr=1e-4, max_grad_norm=1.0)
    for _ in range(3):
        tr.step(images, targets)
    torch.cuda.synchronize()
    main_stream = torch.cuda.current_stream().cuda_stream
    want = a.streams.split(",")
    for label, st in (("main stream", main_stream), ("all streams", None)):
        if label.split()[0] not in want:
            continue
        t = KernelTimer(stream=st)
        t.start()
        for _ in range(a.steps):
            tr.step(images, targets)
        s = t.summary()
        t.stop()
        print(f"== {label}: B={a.batch} {a.hw[0]}x{a.hw[1]} {a.dtype} [{a.cfg or 'defaults'}], per step (mean of {a.steps})")
        print(table(s, a.steps, a.dtype, pmc), flush=True)


if __name__ == "__main__":
    main()
