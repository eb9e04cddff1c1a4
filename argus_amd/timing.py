"""Forward-latency benchmark — the MI355X counterpart of the reference's ``scripts/timing.py``.

    python -m argus_amd.timing [--trials 100] [--batch 2] [--hw 256 256] [--dtype fp32|bf16]
                               [--eval] [--no-graph]

Reference semantics (scripts/timing.py:10-48): ``NCameraCNN(n_cams=2)`` in fp32 on the GPU, left in
its default (train) mode — BatchNorm uses batch statistics — a fresh ``torch.rand((2, 6, 256, 256))``
batch per trial, ``torch.no_grad()``, 100 timed trials after one untimed first call, each trial timed
with device events by ``time_torch_fn`` (argus/utils.py:153-171).

The reference compiles the model with ``torch.compile(mode="reduce-overhead")``, i.e. it replays a
captured device graph. The equivalent here is a hipGraph of the whole native forward (every HIP
launch of ``ResNetEngine.forward`` on one captured stream), replayed per trial after the new batch is
copied into the graph's static input buffer; ``--no-graph`` times eager launches instead.

One deliberate difference: the reference prints ``np.mean(runtime)`` — the last trial only
(scripts/timing.py:48); this prints the mean (and median, min) over all timed trials.
"""
from __future__ import annotations

import argparse
import json
import statistics

import torch

from argus_amd.models import NCameraCNN, NCameraCNNConfig
from argus_amd.utils import time_torch_fn


def forward_latency(trials: int = 100, batch: int = 2, hw=(256, 256), dtype: str = "fp32", train_mode: bool = True,
                    graph: bool = True, device: str = "cuda") -> dict:
    """Mean / median / min seconds of one NCameraCNN forward (no_grad) over ``trials`` timed trials."""
    torch.manual_seed(0)
    cfg = NCameraCNNConfig(n_cams=2)
    model = NCameraCNN(cfg, compute_dtype=dtype).to(device)
    model.train(train_mode)
    H, W = hw
    static_x = torch.rand((batch, cfg.n_cams * 3, H, W), device=device)
    first = None
    if graph:
        # untimed warm-up (workspaces, weight-prep table), then capture on a side stream
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.no_grad():
            for _ in range(2):
                model(static_x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(g):
            static_out = model(static_x)

        def run(x):
            static_x.copy_(x)
            g.replay()
            return static_out
    else:
        def run(x):
            with torch.no_grad():
                return model(x)

    times = []
    for i in range(trials + 1):
        x = torch.rand((batch, cfg.n_cams * 3, H, W), device=device)
        out, t = time_torch_fn(lambda: run(x))
        if i == 0:
            first = t
        else:
            times.append(t)
    assert torch.isfinite(out).all()
    return {"mean_s": statistics.fmean(times), "median_s": statistics.median(times), "min_s": min(times),
            "first_call_s": first, "trials": trials, "batch": batch, "hw": list(hw), "dtype": dtype,
            "mode": "train" if train_mode else "eval", "graph": graph}


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--trials", type=int, default=100)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--hw", type=int, nargs=2, default=(256, 256))
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--eval", action="store_true", help="eval-mode BN (running statistics)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of a replayed hipGraph")
    a = ap.parse_args()
    r = forward_latency(a.trials, a.batch, tuple(a.hw), a.dtype, not a.eval, not a.no_graph)
    print(f"Forward pass took {r['mean_s']} seconds on average.")
    print(json.dumps(r))


if __name__ == "__main__":
    main()
