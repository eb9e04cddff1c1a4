"""Build libargus_hip.so in-tree: hipcc --offload-arch=gfx950, one object per source, parallel.

    python -m argus_amd.build [--verbose]

The shared library lands next to this file (argus_amd/libargus_hip.so) so it travels with the repo
snapshot to the GPU box (git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
OUT = HERE / "libargus_hip.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
SOURCES = ["capi.cpp", "ktimer.cpp", "conv.hip", "conv_glds.hip", "conv_halo.hip", "conv_dgw.hip", "conv_p1x1.hip", "conv_wgdma.hip", "reduce.hip", "stem.hip", "bn.hip", "head.hip", "loss.hip", "optim.hip", "augment.hip"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", "-Wno-unused-but-set-variable"]


def _compile(src: str, verbose: bool) -> Path:
    obj = CSRC / ".build" / (src + ".o")
    obj.parent.mkdir(exist_ok=True)
    srcp = CSRC / src
    deps = [srcp, *CSRC.glob("*.h"), HERE.parent / "include" / "argus_hip.h"]
    if obj.exists() and obj.stat().st_mtime > max(d.stat().st_mtime for d in deps):
        return obj
    cmd = [HIPCC, *FLAGS, "-c", str(srcp), "-o", str(obj)]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-x", "hip", *FLAGS, "-c", str(srcp), "-o", str(obj)]
    if verbose:
        cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    if verbose and r.stderr:
        print(r.stderr, file=sys.stderr)
    return obj


def build(verbose: bool = False) -> Path:
    with cf.ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), SOURCES))
    if OUT.exists() and OUT.stat().st_mtime > max(o.stat().st_mtime for o in objs):
        return OUT
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", str(OUT), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    return OUT


if __name__ == "__main__":
    print(build(verbose="--verbose" in sys.argv))
