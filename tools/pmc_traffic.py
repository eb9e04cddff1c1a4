"""Per-launch HBM traffic from rocprofv3 PMC passes (MI355X_MICROARCH.md §HBM):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -- python bench.py ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_pmc_traffic.json [B H W dtype]

FETCH_SIZE / WRITE_SIZE are KiB (counter_defs.yaml). gfx950 correction: FETCH_SIZE reports 1/2 of the
bytes of a 16-B/lane streaming read (every global load in the conv kernels is a 16-B ld16), so
fetch bytes = 2 * 1024 * FETCH_SIZE; write bytes = 1024 * WRITE_SIZE (exact for 16-B stores).
Output: kernel name -> launches and mean corrected bytes per launch.
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


def demangle(name: str) -> str:
    """rocprof kernel name -> "argus::igemm_kernel<__bf16, 128, 128, false, false>" (no return type or
    argument list). Our template kernels are demangled here (binutils' c++filt predates DF16b);
    names rocprof already prints demangled are cut at their argument list."""
    if name.startswith("void "):
        name = name[5:]
    m = re.match(r"_ZN5argus(\d+)", name)
    if m:
        n = int(m.group(1))
        p = m.end()
        base = name[p:p + n]
        p += n
        if name[p:p + 1] != "I":
            return f"argus::{base}"
        args = []
        p += 1
        while name[p] != "E":
            for pat, fn in ((r"DF16b", lambda g: "__bf16"), (r"f", lambda g: "float"),
                            (r"Li(-?\d+)E", lambda g: g.group(1)), (r"Lb([01])E", lambda g: "true" if g.group(1) == "1" else "false")):
                mm = re.match(pat, name[p:])
                if mm:
                    args.append(fn(mm))
                    p += mm.end()
                    break
            else:
                return name
        return f"argus::{base}<{', '.join(args)}>"
    depth = 0
    for i, ch in enumerate(name):
        depth += ch == "<"
        depth -= ch == ">"
        if ch == "(" and depth == 0:
            return name[:i]
    return name


def per_kernel(d: str, counter: str) -> dict:
    files = sorted(Path(d).rglob("*counter_collection.csv"))
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            acc[demangle(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return acc


def main() -> None:
    fetch, write, out = sys.argv[1], sys.argv[2], sys.argv[3]
    workload = [int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]), sys.argv[7]] if len(sys.argv) > 7 else [64, 256, 256, "bf16"]
    f, w = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fb = 2 * 1024 * sum(f[k]) / len(f[k]) if f.get(k) else None
        wb = 1024 * sum(w[k]) / len(w[k]) if w.get(k) else None
        res[k] = {"launches_fetch_pass": len(f.get(k, [])), "launches_write_pass": len(w.get(k, [])),
                  "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                  "traffic_bytes_per_launch": (fb or 0) + (wb or 0)}
    meta = {"workload": workload, "source": [fetch, write], "correction": "fetch = 2*1024*FETCH_SIZE (gfx950 half-count), write = 1024*WRITE_SIZE"}
    Path(out).write_text(json.dumps({"meta": meta, "kernels": res}, indent=1))
    top = sorted(res.items(), key=lambda kv: -kv[1]["traffic_bytes_per_launch"] * max(kv[1]["launches_fetch_pass"], 1))
    for k, v in top[:15]:
        print(f"{v['traffic_bytes_per_launch'] / 1e6:10.2f} MB/launch  n={v['launches_fetch_pass']:5d}  {k[:90]}")


if __name__ == "__main__":
    main()
