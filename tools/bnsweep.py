"""Sweep the BN elementwise-kernel geometry (argus_conv_tuning keys 20-23) over full train steps
(dev tool, GPU). python tools/bnsweep.py [--batch 64]"""
import argparse
import gc
import sys
import time

import torch

sys.path.insert(0, ".")
from argus_amd._lib import lib  # noqa: E402
from argus_amd.models import NCameraCNN  # noqa: E402
from argus_amd.profiling import KernelTimer  # noqa: E402
from argus_amd.step import FusedTrainer  # noqa: E402
from bench import synthetic_batch  # noqa: E402

CONFIGS = [  # (bwd_min_px, bwd_max_rows, ew_target, ew_min_ppt)
    (64, 1024, 512, 16), (32, 2048, 512, 16), (32, 4096, 512, 16), (16, 4096, 512, 16), (64, 2048, 512, 16),
    (64, 1024, 256, 16), (64, 1024, 512, 32), (64, 1024, 1024, 32), (64, 1024, 256, 64), (64, 1024, 768, 8),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    L = lib()
    dev = torch.device("cuda", 0)
    images, targets = synthetic_batch(a.batch, 256, 256, 1000, dev)
    for cfg in CONFIGS:
        for k, v in zip((20, 21, 22, 23), cfg):
            assert L.dll.argus_conv_tuning(k, v) == 0
        torch.manual_seed(42)
        m = NCameraCNN(compute_dtype="bf16").to(dev)
        tr = FusedTrainer(m)
        for _ in range(2):
            tr.step(images, targets)
        torch.cuda.synchronize()
        with KernelTimer() as kt:
            for _ in range(3):
                tr.step(images, targets)
        s = kt.summary()
        bn = {k: v["total_ms"] / 3 for k, v in s.items() if k.startswith("argus::bn_")}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            tr.step(images, targets)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        parts = " ".join(f"{k.split('::')[1].split('<')[0].replace('_kernel', '')}={v:.3f}" for k, v in sorted(bn.items()))
        print(f"{cfg} step {ms:.3f} ms  bn {sum(bn.values()):.3f} ms  {parts}", flush=True)
        del tr, m
        gc.collect()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
