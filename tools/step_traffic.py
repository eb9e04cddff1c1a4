"""HBM traffic per step from a PMC traffic summary (tools/pmc_traffic.py) joined with a kernel-stats
summary (tools/profsum.py: calls per step), per kernel and in total (dev tool, CPU).

    python tools/step_traffic.py profiles/TAG_pmc_traffic.json profiles/TAG_kernel_summary.txt [top]
"""
import json
import re
import sys


def main():
    traffic = json.load(open(sys.argv[1]))["kernels"]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    calls = {}
    for line in open(sys.argv[2]):
        m = re.match(r"\s*([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+(.*\S)", line)
        if m:
            name = re.sub(r"^void ", "", m.group(5))
            name = re.sub(r"\(.*$", "", name).replace(", false>", ">") if "(" in name else name
            calls[name] = float(m.group(3))
    rows, total = [], 0.0
    for k, v in traffic.items():
        per = v.get("traffic_bytes_per_launch")
        n = calls.get(k)
        if n is None:  # kernel-stats names carry the default template arguments the PMC names omit
            n = next((c for nm, c in calls.items() if nm.startswith(k.rstrip(">"))), None)
        if per is None or n is None:
            continue
        rows.append((per * n, n, per, k))
        total += per * n
    rows.sort(reverse=True)
    print(f"{'GB/step':>8} {'calls':>6} {'MB/launch':>10}  kernel")
    for t, n, per, k in rows[:top]:
        print(f"{t / 1e9:8.3f} {n:6.1f} {per / 1e6:10.2f}  {k}")
    print(f"{total / 1e9:8.3f}  total HBM traffic per step (PMC FETCH_SIZE + WRITE_SIZE, gfx950-corrected)")


if __name__ == "__main__":
    main()
