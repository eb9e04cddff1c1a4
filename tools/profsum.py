"""Summarise a rocprofv3 kernel_stats.csv: per-step ms per kernel (demangled names).

    python tools/profsum.py run_kernel_stats.csv STEPS [TOP]
"""
import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import demangle  # noqa: E402


def main() -> None:
    path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'ms/step':>8} {'%':>6} {'calls/step':>10} {'avg us':>9}  kernel")
    for r in rows[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} {float(r['Percentage']):6.2f} "
              f"{int(r['Calls']) / steps:10.1f} {float(r['AverageNs']) / 1e3:9.2f}  {demangle(r['Name'])}")
    print(f"total {tot / 1e6 / steps:.3f} ms per step-equivalent ({steps:g} steps)")


if __name__ == "__main__":
    main()
