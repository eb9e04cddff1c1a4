"""Per-kernel PMC summary from several rocprofv3 --pmc passes (dev tool; MI355X_MICROARCH.md §PMC).

    python tools/pmc_summary.py OUT.json DIR1 [DIR2 ...] [--top 25]

Every DIR holds one pass's counter_collection.csv. Counters are averaged per dispatch of each
demangled kernel instantiation, then derived:
  mfma_busy   = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMD x 256 CU x GRBM_GUI_ACTIVE / 8)
                (MFMA-pipe busy fraction of every SIMD of the chip over the kernel; GRBM_GUI_ACTIVE
                is summed over the 8 XCDs, hence / 8 = kernel cycles)
  mfma_flops  = 1024 x SQ_VALU_MFMA_BUSY_CYCLES for the 16x16x32 bf16 MFMA (16 SIMD cycles, 16384
                FLOP each) - cross-check against the algorithmic flops
  wait / issue-stall / active = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS cycles per LDS-array cycle)
  valu_per_mfma = SQ_INSTS_VALU / SQ_INSTS_MFMA (vector-ALU instructions issued per MFMA: index math,
                staging transforms and epilogue work competing with the MFMAs for issue)
  clock_ghz   = GRBM_GUI_ACTIVE / 8 / kernel time (when a duration is present in the CSV)
"""
import argparse
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_traffic import demangle  # noqa: E402


def load(dirs):
    vals = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in sorted(Path(d).rglob("*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                vals[demangle(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--workload", nargs=4, default=["64", "256", "256", "bf16"],
                    help="B H W dtype of the bench run (bench.py looks the summary up by it)")
    a = ap.parse_args()
    vals = load(a.dirs)
    res = {}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        d = {"dispatches": n, "counters_per_dispatch": m}
        g = m.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            d["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * g / 8)
            d["mfma_flops_per_dispatch"] = 1024 * m["SQ_VALU_MFMA_BUSY_CYCLES"]
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for key, c in (("wait_frac", "SQ_WAIT_ANY"), ("issue_stall_frac", "SQ_WAIT_INST_ANY"),
                           ("active_frac", "SQ_ACTIVE_INST_ANY"), ("lds_stall_frac", "SQ_WAIT_INST_LDS")):
                if c in m:
                    d[key] = m[c] / wc
        if m.get("SQ_INSTS_MFMA"):
            d["valu_per_mfma"] = m.get("SQ_INSTS_VALU", 0.0) / m["SQ_INSTS_MFMA"]
        if m.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"]
        if g:
            d["gpu_cycles"] = g / 8
        res[k] = d
    meta = {"workload": [int(a.workload[0]), int(a.workload[1]), int(a.workload[2]), a.workload[3]],
            "derived_from": a.dirs}
    Path(a.out).write_text(json.dumps({"meta": meta, "kernels": res}, indent=1))
    order = sorted(res.items(), key=lambda kv: -kv[1].get("gpu_cycles", 0) * kv[1]["dispatches"])
    print(f"{'cyc/disp':>9} {'n':>4} {'mfma':>5} {'wait':>5} {'stall':>5} {'act':>5} {'ldsc':>5} {'v/mf':>6}  kernel")
    for k, d in order[:a.top]:
        f = lambda x: f"{d[x]:5.2f}" if x in d else "    -"  # noqa: E731
        print(f"{d.get('gpu_cycles', 0):9.0f} {d['dispatches']:4d} {f('mfma_busy')} {f('wait_frac')} "
              f"{f('issue_stall_frac')} {f('active_frac')} {f('lds_conflict')} "
              f"{d['valu_per_mfma'] if 'valu_per_mfma' in d else float('nan'):6.1f}  {k[:100]}")


if __name__ == "__main__":
    main()
