"""Live kernel timing with HIP events (torch.cuda.Event records on the launching stream)."""
from __future__ import annotations

import torch


def tag_name(tag: int) -> str:
    """Kernel symbol family for an argus_conv_launch_info tag (matches rocprof's kernel names)."""
    kind, rest = divmod(tag, 10000000)
    dt, rest = divmod(rest, 1000000)
    bm, bn = divmod(rest, 1000)
    t = "__bf16" if dt == 1 else "float"
    k = "igemm_kernel" if kind == 1 else "wgrad_kernel"
    return f"argus::{k}<{t}, {bm}, {bn}>"


class KernelTimer:
    """Records (start, end) events around every launch whose instantiation tag is in ``tags``
    (None = record per tag for all)."""

    def __init__(self, tags=None):
        self.tags = None if tags is None else set(tags)
        self.enabled = False
        self.events: dict[int, list] = {}
        self.flops: dict[int, int] = {}

    def wrap(self, tag: int, flops: int, fn) -> None:
        if not self.enabled or (self.tags is not None and tag not in self.tags):
            fn()
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        self.events.setdefault(tag, []).append((s, e))
        self.flops[tag] = self.flops.get(tag, 0) + flops

    def reset(self) -> None:
        self.events.clear()
        self.flops.clear()

    def summary(self) -> dict:
        """tag -> {launches, total_ms, avg_us, flops_per_launch, tflops}."""
        torch.cuda.synchronize()
        out = {}
        for tag, evs in self.events.items():
            ms = sum(s.elapsed_time(e) for s, e in evs)
            n = len(evs)
            fl = self.flops[tag]
            out[tag] = {"name": tag_name(tag), "launches": n, "total_ms": ms, "avg_us": 1e3 * ms / n,
                        "flops_per_launch": fl / n, "tflops": fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0}
        return out
