"""Build-time ISA check of the inline-asm transposed LDS reads (CPU: hipcc cross-compiles gfx950).

conv_halo.hip's and conv_wgdma.hip's weight-gradient kernels issue their ds_read_b64_tr_b16 reads as inline asm (the builtin
made the compiler drain the global->LDS ring before every k-step) and waits for their
data with a separate ``s_waitcnt lgkmcnt(0)`` asm statement. The compiler's waitcnt pass does not see
those reads, so nothing but register allocation keeps an instruction from touching a destination
register before its data has landed (e.g. a v_mov assembling a 128-bit operand from two 64-bit reads).
This test compiles the file to gfx950 assembly and walks every function: from each asm
ds_read_b64_tr_b16 until an lgkmcnt wait retires it (LDS returns in order, so lgkmcnt(N) retires all
but the last N outstanding LDS operations), no instruction may read or write its destination VGPRs.
"""
import re
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

ASM_SOURCES = ["conv_halo.hip", "conv_wgdma.hip"]  # the sources with inline-asm LDS reads


def _vregs(text):
    regs = set()
    for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", text):
        regs.update(range(int(a), int(b) + 1))
    for a in re.findall(r"\bv(\d+)\b", text):
        regs.add(int(a))
    return regs


def check_asm_lds_reads(asm: str):
    """Violations (function, line, instruction, registers) of the rule in the module docstring."""
    bad = []
    fn = None
    pending = []  # outstanding LDS ops in issue order: set of registers (empty for compiler-tracked ones)
    in_asm = False
    for ln, raw in enumerate(asm.splitlines(), 1):
        line = raw.split(";")[0].strip() if not raw.strip().startswith(";;#ASM") else raw.strip()
        if raw.strip().startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if raw.strip().startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not line or line.startswith("."):
            if line.endswith(":") and not line.startswith(".L"):
                fn, pending = line[:-1], []
            continue
        if line.endswith(":"):
            if not line.startswith(".L"):
                fn, pending = line[:-1], []
            continue
        op = line.split()[0]
        m = re.match(r"s_waitcnt\b.*lgkmcnt\((\d+)\)", line)
        if m:
            keep = int(m.group(1))
            pending = pending[len(pending) - keep:] if keep < len(pending) else pending
            if keep == 0:
                pending = []
            continue
        live = set().union(*pending) if pending else set()
        if op.startswith("ds_"):
            regs = _vregs(line)
            if in_asm and op == "ds_read_b64_tr_b16":
                dst = line.split(None, 1)[1].split(",")[0]
                src = _vregs(line.split(",", 1)[1])
                if live & src or live & _vregs(dst):
                    bad.append((fn, ln, line, sorted(live & regs)))
                pending.append(_vregs(dst))
            else:
                if live & regs:
                    bad.append((fn, ln, line, sorted(live & regs)))
                pending.append(set())
            continue
        if live:
            hit = live & _vregs(line)
            if hit:
                bad.append((fn, ln, line, sorted(hit)))
    return bad


def test_check_catches_an_early_use():
    asm = """kern:
\t;;#ASMSTART
\tds_read_b64_tr_b16 v[10:11], v2
\t;;#ASMEND
\tv_mov_b32_e32 v20, v10
\t;;#ASMSTART
\ts_waitcnt lgkmcnt(0)
\t;;#ASMEND
\tv_mov_b32_e32 v21, v11
"""
    bad = check_asm_lds_reads(asm)
    assert len(bad) == 1 and bad[0][3] == [10]
    ok = asm.replace("\tv_mov_b32_e32 v20, v10\n", "")
    assert check_asm_lds_reads(ok) == []


@pytest.mark.parametrize("src", ASM_SOURCES)
def test_inline_asm_lds_reads_are_waited_for(tmp_path, src):
    from argus_amd.build import ARCH, CSRC, FLAGS, HIPCC

    out = tmp_path / (src + ".s")
    cmd = [HIPCC, *[f for f in FLAGS if f != "-fPIC"], "--cuda-device-only", "-S", str(CSRC / src), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    asm = out.read_text()
    assert f"amdgcn-amd-amdhsa--{ARCH}" in asm
    n_reads = sum(1 for _ in re.finditer(r"ds_read_b64_tr_b16", asm))
    assert n_reads > 0, "no transposed LDS reads found: the check would be vacuous"
    bad = check_asm_lds_reads(asm)
    assert not bad, "\n".join(f"{f}:{ln}: {ins}  (registers {regs})" for f, ln, ins, regs in bad[:20])


# ---- batched loads in the small cross-workgroup reductions (common.h kLoadBatch) ------------------
# kernel (mangled-name fragment) -> source; each is a reduction over a runtime-length loop of loads
REDUCTIONS = {
    "stats_finalize_kernel": "bn.hip",
    "bwd_finalize_kernel": "bn.hip",
    "wgrad_reduce_kernel": "reduce.hip",
    "gemm_reduce_kernel": "head.hip",
    "colsum_kernel": "head.hip",
    "avgpool_fwd_kernel": "bn.hip",
    # the folded BN-backward finalize's group merges (bnfin.h) inside a BN-epilogue dgrad
    "igemm_glds_kernelILi256ELi128ELi2E": "conv_glds.hip",
}


def _function_bodies(asm):
    """name -> instruction lines; a loop header label keeps the compiler's "Loop Header" marker as a
    trailing " LOOP" (the compiler's own loop analysis, not a guess from branch directions)."""
    fns, cur = {}, None
    for raw in asm.splitlines():
        s = raw.split(";")[0].rstrip()
        if s and not raw.startswith((" ", "\t")) and s.endswith(":") and not s.startswith("."):
            cur = fns.setdefault(s[:-1], [])
            continue
        if cur is not None and s.strip():
            cur.append(s.strip() + (" LOOP" if "Loop Header" in raw else ""))
    return fns


def loop_load_runs(body):
    """For each loop (a "Loop Header" label .. the last backward branch to it) holding global loads: the
    most loads a trip has in flight at once (each load adds one, s_waitcnt vmcnt(N) leaves N)."""
    labels = {s[:-6]: i for i, s in enumerate(body) if s.endswith(": LOOP")}
    ends = {}
    for i, s in enumerate(body):
        m = re.match(r"s_(?:cbranch_\w+|branch)\s+(\.L\w+)", s)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            ends[m.group(1)] = i
    runs = []
    for lab, i in ends.items():
        seg = body[labels[lab]:i + 1]
        out = most = 0  # loads outstanding (vmcnt(N) leaves at most N), and their maximum in a trip
        for ins in seg:
            if ins.startswith(("global_load", "buffer_load")):
                out += 1
                most = max(most, out)
            else:
                w = re.match(r"s_waitcnt\b.*vmcnt\((\d+)\)", ins)
                if w:
                    out = min(out, int(w.group(1)))
        if any(ins.startswith(("global_load", "buffer_load")) for ins in seg):
            runs.append(most)
    return runs


def test_loop_load_runs_self_test():
    serial = ["x:", ".LBB0_1: LOOP", "global_load_dwordx2 v[0:1], v[2:3], off", "s_waitcnt vmcnt(0)",
              "v_add_f64 v[4:5], v[4:5], v[0:1]", "s_cbranch_scc1 .LBB0_1"]
    batched = ["x:", ".LBB0_1: LOOP"] + [f"global_load_dwordx2 v[{2*i}:{2*i+1}], v[20:21], off" for i in range(8)] + \
        ["s_waitcnt vmcnt(7)", "s_waitcnt vmcnt(0)", "s_cbranch_scc1 .LBB0_1"]
    assert loop_load_runs(serial) == [1]
    assert loop_load_runs(batched) == [8]


@pytest.mark.parametrize("src", sorted(set(REDUCTIONS.values())))
def test_reductions_batch_their_loads(tmp_path, src):
    """Every load loop of these reduction kernels keeps >= 4 loads in flight per trip (a plain
    accumulate loop compiles to load / s_waitcnt vmcnt(0) / add per element: one memory latency each)."""
    from argus_amd.build import CSRC, FLAGS, HIPCC

    out = tmp_path / (src + ".s")
    cmd = [HIPCC, *[f for f in FLAGS if f != "-fPIC"], "--cuda-device-only", "-S", str(CSRC / src), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    fns = _function_bodies(out.read_text())
    for frag, s in REDUCTIONS.items():
        if s != src:
            continue
        hits = [name for name in fns if frag in name]
        assert hits, f"{frag} not found in {src}"
        for name in hits:
            runs = loop_load_runs(fns[name])
            assert runs, f"{name}: no load loop found (the check would be vacuous)"
            # the glds kernel's main loop (LDS DMA) is not a global_load loop; its bnfin merges are
            assert max(runs) >= 4 and all(n >= 4 for n in runs if n), f"{name}: loads in flight per loop trip {runs}"
