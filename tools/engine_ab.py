"""A/B of engine schedule attributes on full bf16 train steps (dev tool, GPU): configurations run
interleaved (A B A B ...) on one box so drift between them cancels.

    python tools/engine_ab.py --batch 64 --cfg "" --cfg "side_priority=-1" --cfg "tune:6=256" [--rounds 3]

Each configuration is rebuilt (same seed) for every round and freed before the next, so only one
model is resident at a time; the peak device memory of each configuration is printed. Model
instances differ by about 1 % on their own (allocation placement): repeat a configuration (e.g.
defaults first and last) to see that spread.
"""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from bench import synthetic_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--hw", type=int, nargs=2, default=(256, 256))
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--cfg", action="append", default=[],
                    help="attr=value[,attr=value] (\"\" = defaults; tune:key=value a policy override, dtype=bf16|fp8)")
    a = ap.parse_args()
    from argus_amd.models import NCameraCNN
    from argus_amd.step import FusedTrainer

    dev = torch.device("cuda", 0)
    images, targets = synthetic_batch(a.batch, *a.hw, 1000, dev)

    def parse(cfg):
        tune, attrs = {}, {}
        for kv in filter(None, cfg.split(",")):
            k, v = kv.split("=")
            if k.startswith("tune:"):  # a kernel-selection policy override (argus_conv_policy_default key)
                tune[int(k[5:])] = int(v)
            else:
                attrs[k] = v
        return tune, attrs

    def run(cfg):
        """One configuration: build (seeded), 3 warm-up steps, the timed steps, then free everything
        before the next configuration (only one model is resident at a time; r04 kept them all and
        ran out of memory at 376x672 B=128). Returns (ms/step, peak device GiB of this configuration)."""
        tune, attrs = parse(cfg)
        dtype = attrs.pop("dtype", a.dtype)  # a per-configuration compute dtype (e.g. fp8 vs bf16)
        # main_priority=-1: the whole step (the engine's main chain) on a high-priority stream, the side
        # stream at its own side_priority
        mp = int(attrs.pop("main_priority", 0))
        ms_ = torch.cuda.Stream(device=dev, priority=mp) if mp else torch.cuda.current_stream(dev)
        with torch.cuda.stream(ms_):
            return run_on(tune, attrs, dtype)

    def run_on(tune, attrs, dtype):
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(dev)
        torch.manual_seed(42)
        m = NCameraCNN(compute_dtype=dtype, kernel_tuning=tune or None).to(dev).train()
        eng = m._engine(dev)
        for k, v in attrs.items():
            cur = getattr(eng, k)
            setattr(eng, k, v == "1" if isinstance(cur, bool) else type(cur)(int(v)))
        tr = FusedTrainer(m, lr=1e-4, max_grad_norm=1.0)
        for _ in range(3):
            tr.step(images, targets)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            tr.step(images, targets)
        torch.cuda.synchronize()
        ms = 1e3 * (time.perf_counter() - t0) / a.steps
        peak = torch.cuda.max_memory_allocated(dev) / 2**30
        del tr, eng, m
        return ms, peak

    cfgs = a.cfg or [""]
    res = [[] for _ in cfgs]
    peaks = [0.0 for _ in cfgs]
    for _ in range(a.rounds):  # interleaved A B A B ... so drift between configurations cancels
        for i, c in enumerate(cfgs):
            ms, pk = run(c)
            res[i].append(ms)
            peaks[i] = max(peaks[i], pk)
    for c, r, pk in zip(cfgs, res, peaks):
        print(f"{c or 'defaults':40s} ms/step " + " ".join(f"{x:7.3f}" for x in r) +
              f"   img/s best {2 * a.batch / min(r) * 1e3:8.1f}   peak {pk:.2f} GiB", flush=True)

if __name__ == "__main__":
    main()
