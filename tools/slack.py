"""Per-kernel slack over one training step (dev tool, GPU): time vs roofline time
max(flops / 2.5 PF, algorithmic bytes / 8 TB/s) for every timed kernel instantiation (conv GEMMs and
BN passes; the rest of the step is reported as 'untimed').   python tools/slack.py [--batch 64]"""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from argus_amd.models import NCameraCNN  # noqa: E402
from argus_amd.profiling import KernelTimer  # noqa: E402
from argus_amd.step import FusedTrainer  # noqa: E402
from bench import synthetic_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    m = NCameraCNN(compute_dtype="bf16").to(dev).train()
    tr = FusedTrainer(m, lr=1e-4, max_grad_norm=1.0)
    x, t = synthetic_batch(a.batch, 256, 256, 1000, dev)
    for _ in range(3):
        tr.step(x, t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        tr.step(x, t)
    torch.cuda.synchronize()
    step_ms = (time.perf_counter() - t0) / 5 * 1e3
    with KernelTimer() as kt:
        tr.step(x, t)
    s = kt.summary()
    rows = []
    for name, v in s.items():
        roof_ms = max(v["flops_per_launch"] / 2.5e15, v["bytes_per_launch"] / 8e12) * 1e3 * v["launches"]
        rows.append((v["total_ms"] - roof_ms, v["total_ms"], roof_ms, v["launches"], name))
    rows.sort(reverse=True)
    timed = sum(r[1] for r in rows)
    print(f"step {step_ms:.2f} ms; timed kernels {timed:.2f} ms (roof {sum(r[2] for r in rows):.2f} ms); "
          f"untimed {step_ms - timed:.2f} ms")
    print(f"{'slack':>7} {'time':>7} {'roof':>7} {'n':>4}  kernel")
    for sl, tm, rf, n, name in rows:
        print(f"{sl:7.3f} {tm:7.3f} {rf:7.3f} {n:4d}  {name}")


if __name__ == "__main__":
    main()
