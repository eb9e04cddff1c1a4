"""Summarise a rocprofv3 kernel_stats.csv: per-step ms per kernel (demangled names).

    python tools/profsum.py run_kernel_stats.csv [TOP]

The step count is derived from the trace itself: the optimizer's adam_kernel runs exactly once per
fused train step, so steps = its call count (a caller-supplied count inflated every per-step figure
when the profiled process ran more steps than assumed: probe, timed and critical-path steps).
"""
import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import demangle  # noqa: E402

STEP_MARKER = "adam_kernel"


def main() -> None:
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    rows = list(csv.DictReader(open(path)))
    marks = [r for r in rows if STEP_MARKER in r["Name"]]
    if not marks:
        raise SystemExit(f"{path}: no {STEP_MARKER} launches: cannot derive the step count")
    steps = float(sum(int(r["Calls"]) for r in marks))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"steps = {steps:g} ({STEP_MARKER} calls in the trace)")
    print(f"{'ms/step':>8} {'%':>6} {'calls/step':>10} {'avg us':>9}  kernel")
    for r in rows[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} {float(r['Percentage']):6.2f} "
              f"{int(r['Calls']) / steps:10.1f} {float(r['AverageNs']) / 1e3:9.2f}  {demangle(r['Name'])}")
    print(f"total kernel time {tot / 1e6 / steps:.3f} ms per step (both streams; they overlap, so this can "
          f"exceed the step's wall time)")


if __name__ == "__main__":
    main()
