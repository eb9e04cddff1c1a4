"""Static instruction mix of a kernel's innermost loops vs the rest (dev tool, CPU: hipcc cross-compiles
gfx950). Used for the 32x32x16 MFMA question: how many VALU instructions per MFMA sit
in the k-loop (what an MFMA shape change could touch) vs in the prologue / epilogue.

    python tools/isa_loopmix.py conv.hip "igemm_kernel<__bf16, 64, 128, false, false, 4, 19>" [...]

A loop = the instructions between a label and a later backward branch to it (s_cbranch_* / s_branch).
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def functions(asm):
    fns, cur, name = {}, None, None
    for raw in asm.splitlines():
        line = raw.split(";")[0].rstrip()
        s = line.strip()
        if not s:
            continue
        if s.endswith(":") and not s.startswith(".") and not raw.startswith((" ", "\t")):
            name, cur = s[:-1], []
            fns[name] = cur
            continue
        if cur is None:
            continue
        if s.startswith(".Lfunc_end"):
            cur, name = None, None
            continue
        cur.append(s)
    return fns


def loop_mix(body):
    labels = {s[:-1]: i for i, s in enumerate(body) if s.endswith(":")}
    in_loop = [False] * len(body)
    loops = []
    for i, s in enumerate(body):
        m = re.match(r"s_(?:cbranch_\w+|branch)\s+(\.L\w+)", s)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            lo = labels[m.group(1)]
            loops.append((lo, i))
            for j in range(lo, i + 1):
                in_loop[j] = True
    tot = {"loop": {}, "rest": {}}
    for i, s in enumerate(body):
        if s.endswith(":") or s.startswith("."):
            continue
        c = classify(s.split()[0])
        d = tot["loop" if in_loop[i] else "rest"]
        d[c] = d.get(c, 0) + 1
    return loops, tot


def main():
    from argus_amd.build import CSRC, FLAGS, HIPCC

    src, names = sys.argv[1], sys.argv[2:]
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "k.s"
        subprocess.run([HIPCC, *[f for f in FLAGS if f != "-fPIC"], "--cuda-device-only", "-S", str(CSRC / src),
                        "-o", str(out)], check=True)
        asm = out.read_text()
    fns = functions(asm)
    demangled = {}
    cp = subprocess.run(["c++filt"], input="\n".join(f.replace("DF16b", "u6__bf16") for f in fns), capture_output=True, text=True)
    for mangled, dem in zip(fns, cp.stdout.splitlines()):
        demangled[mangled] = dem
    for want in names:
        hits = [m for m, d in demangled.items() if want in d]
        for m in hits:
            loops, tot = loop_mix(fns[m])
            lp, rs = tot["loop"], tot["rest"]
            mf = lp.get("mfma", 0)
            print(f"{demangled[m]}")
            print(f"  loops {len(loops)} (lines {[b - a for a, b in loops]})")
            print(f"  in loops : " + " ".join(f"{k}={v}" for k, v in sorted(lp.items())) +
                  (f"   valu/mfma {lp.get('valu', 0) / mf:.2f}" if mf else ""))
            print(f"  outside  : " + " ".join(f"{k}={v}" for k, v in sorted(rs.items())))
            # innermost MFMA loops (the k-loops): loops with MFMAs that contain no other MFMA loop
            body = fns[m]
            mix = []
            for lo, hi in loops:
                d = {}
                for s in body[lo:hi + 1]:
                    if not (s.endswith(":") or s.startswith(".")):
                        c = classify(s.split()[0])
                        d[c] = d.get(c, 0) + 1
                mix.append((lo, hi, d))
            mf_loops = [x for x in mix if x[2].get("mfma")]
            for lo, hi, d in mf_loops:
                if any(l2 >= lo and h2 <= hi and (l2, h2) != (lo, hi) for l2, h2, _ in mf_loops):
                    continue
                print(f"  k-loop [{lo}:{hi}]: " + " ".join(f"{k}={v}" for k, v in sorted(d.items())) +
                      f"   valu/mfma {d.get('valu', 0) / d['mfma']:.2f}")


if __name__ == "__main__":
    main()
