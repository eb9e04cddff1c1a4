"""Per-stream critical-path breakdown of a bench run from a rocprofv3 kernel trace (dev tool).

    python tools/timeline.py OUT/run_kernel_trace.csv [--steps K]

Steps are delimited by the optimizer kernel (adam_kernel): one step = from the end of one Adam to the
end of the next. Trace a bench run with --no-isolated (tools/prof_timeline.sh does): otherwise the
last steps are bench.py's two untimed no-overlap steps. For the last K steps it reports the step wall time, each HIP stream's busy time
(union of its kernel intervals) and idle gaps, and the main stream's (the one running Adam) busy time
per kernel family — i.e. what the critical path is made of and how much the side stream overlaps.
"""
import argparse
import csv
import re
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import demangle as _dm  # noqa: E402
from collections import defaultdict


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    return {n: (_dm(n) if n.startswith("_ZN5argus") else o) for n, o in zip(names, out)}


def family(name: str) -> str:
    n = re.sub(r"^argus::", "", name)
    for key, fam in (("wgrad", "wgrad"), ("bn_bwd_apply", "bn_bwd_apply"), ("bn_bwd_reduce", "bn_bwd_reduce"),
                     ("bwd_finalize", "bn_finalize"), ("stats_finalize", "bn_finalize"), ("bn_apply", "bn_apply"),
                     ("igemm", "conv fwd/dgrad"), ("conv3x3_halo", "conv fwd/dgrad"), ("maxpool", "pool"),
                     ("avgpool", "pool"), ("gemm_f32", "head"), ("gelu", "head"), ("colsum", "head"),
                     ("adam", "optimizer"), ("sumsq", "optimizer"), ("norm_finalize", "optimizer"),
                     ("weight_prep", "weight_prep"), ("se3_loss", "loss"), ("images_", "input")):
        if key in n:
            return fam
    return "other"


def union(iv):
    iv = sorted(iv)
    tot, cur = 0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        tot += cur[1] - cur[0]
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--first", type=int, default=None,
                    help="index (0-based, in Adam launches) of the first step to report; default: the last --steps "
                         "steps. bench.py runs warmup + 2 x 3 probe steps before its timed region and 5 critical-path "
                         "timer steps after it, whose per-launch events perturb the main stream")
    ap.add_argument("--list", action="store_true", help="also list the last step's main-stream kernels in order "
                                                        "(start offset, gap before, duration)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    skey = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    names = demangle(sorted({r["Kernel_Name"] for r in rows}))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[skey], names[r["Kernel_Name"]]) for r in rows]
    ks.sort()
    adam = [k for k in ks if "adam_kernel" in k[3]]
    main_stream = adam[-1][2]
    ends = [k[1] for k in adam]
    if a.first is None:
        bounds = ends[-(a.steps + 1):]
    else:
        bounds = ends[a.first - 1:a.first + a.steps]
    per_stream = defaultdict(list)
    fam_main = defaultdict(float)
    fam_side = defaultdict(float)
    n = len(bounds) - 1
    for t0, t1 in zip(bounds[:-1], bounds[1:]):
        sel = [k for k in ks if k[0] >= t0 and k[1] <= t1]
        streams = defaultdict(list)
        for s, e, st, nm in sel:
            streams[st].append((s, e))
            (fam_main if st == main_stream else fam_side)[family(nm)] += (e - s) / 1e6 / n
        for st, iv in streams.items():
            per_stream[st].append((union(iv), t1 - t0, len(iv)))
    wall = sum(t1 - t0 for t0, t1 in zip(bounds[:-1], bounds[1:])) / n / 1e6
    print(f"steps {n}, wall {wall:.3f} ms/step; main stream = {main_stream}")
    for st, v in per_stream.items():
        busy = sum(x[0] for x in v) / len(v) / 1e6
        launches = sum(x[2] for x in v) / len(v)
        tag = "main" if st == main_stream else "side"
        print(f"  stream {st} ({tag}): busy {busy:.3f} ms/step ({busy / wall:.0%}), idle {wall - busy:.3f} ms, "
              f"{launches:.0f} kernels/step")
    if a.list:
        t0, t1 = bounds[-2], bounds[-1]
        sel = [k for k in ks if k[0] >= t0 and k[1] <= t1 and k[2] == main_stream]
        prev = t0
        print("last step, main stream: offset_us gap_us dur_us kernel")
        for st_, en, _, nm in sel:
            print(f"  {(st_ - t0) / 1e3:9.1f} {(st_ - prev) / 1e3:7.1f} {(en - st_) / 1e3:8.1f}  {nm[:110]}")
            prev = en
    for title, fam in (("main-stream kernel time by family (ms/step)", fam_main),
                       ("other-stream kernel time by family (ms/step)", fam_side)):
        print(title)
        for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
            print(f"  {v:7.3f}  {k}")


if __name__ == "__main__":
    main()
