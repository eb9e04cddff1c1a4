"""CPU: libargus_hip.so loads, reports its ABI, exports exactly what include/argus_hip.h declares,
and rejects bad arguments through the error channel (no compute call needs a GPU here)."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared():
    txt = (ROOT / "include" / "argus_hip.h").read_text()
    return sorted(set(re.findall(r"^(?:int|size_t|const char\*)\s+(argus_[a-z0-9_]+)\(", txt, re.M)))


def test_header_declares_and_library_exports_the_same_symbols():
    from argus_amd._lib import LIB_PATH, SIGNATURES

    assert declared() == sorted(SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB_PATH)], capture_output=True, text=True).stdout
    exported = sorted(set(re.findall(r" T (argus_[a-z0-9_]+)$", out, re.M)))
    assert exported == declared()


def test_library_loads_and_version():
    from argus_amd._lib import ABI_VERSION, lib

    L = lib()
    assert L.dll.argus_abi_version() == ABI_VERSION


def test_bad_arguments_are_reported():
    from argus_amd._lib import ArgusHipError, ConvDesc, lib

    L = lib()
    d = ConvDesc(2, 8, 8, 48, 64, 3, 3, 1, 1, 8, 8, 0)  # 48 channels: unsupported
    rc = L.dll.argus_conv_fwd(C.byref(d), 1, C.c_void_p(16), C.c_void_p(16), C.c_void_p(16), None, None, None, None)
    assert rc != 0 and b"multiples of 64" in L.dll.argus_last_error()
    bad = ConvDesc(2, 8, 8, 64, 64, 3, 3, 1, 1, 7, 8, 0)  # wrong ho
    with pytest.raises(ArgusHipError, match="ho/wo"):
        L.conv_fwd(C.byref(bad), 1, 16, 16, 16, None, None, None, None)
    fl = C.c_int64(0)
    good = ConvDesc(2, 8, 8, 64, 128, 3, 3, 2, 1, 4, 4, 0)
    tag = L.dll.argus_conv_launch_info(C.byref(good), 1, 0, C.byref(fl))
    assert fl.value == 2 * 2 * 4 * 4 * 128 * 9 * 64 and tag // 10000000 == 1
    assert L.dll.argus_conv_wgrad_workspace_bytes(C.byref(good), 1) > 0
    # kernel-selection policy: immutable defaults, per-call overrides on the descriptor only
    assert L.dll.argus_conv_policy_default(99) == -1 and L.dll.argus_conv_policy_default(20) == -1
    assert L.dll.argus_conv_policy_default(35) == 16384 and L.dll.argus_conv_policy_default(7) == 1024
    assert 0 <= L.dll.argus_conv_policy_default(37) <= 15
    assert L.dll.argus_conv_policy_default(45) in (0, 1, 2, 3) and L.dll.argus_conv_policy_default(52) == -1
    assert L.dll.argus_conv_policy_default(48) == 4 and L.dll.argus_conv_policy_default(47) == 131072
    # key 49: a 1x1 dgrad stages its apply prologue only up to that many 128-column tiles (host-only query)
    assert L.dll.argus_conv_policy_default(49) == 4 and L.dll.argus_conv_policy_default(50) == 0
    c1 = ConvDesc(2, 8, 8, 2048, 512, 1, 1, 1, 0, 8, 8, 0)
    assert [L.dll.argus_conv_dgrad_stages_prologue(C.byref(c1.with_tuning({49: v})), 1) for v in (0, 16, 8)] == [1, 1, 0]
    forced = good.with_tuning({1: 128, 4: 64})  # dgrad row / column tiles
    assert L.dll.argus_conv_launch_info(C.byref(forced), 1, 1, None) % 1000000 == 128 * 1000 + 64
    assert L.dll.argus_conv_launch_info(C.byref(good), 1, 1, None) % 1000000 == 64 * 1000 + 64
    # the MX-fp8 stored-operand convs (argus_conv_x8_ok, host-only): 3x3 stride-1 halo shapes whose
    # reduction channels are multiples of 128, under the fp8 pass bits (key 37: 8 forward, 2 dgrad)
    x8 = ConvDesc(8, 16, 16, 256, 256, 3, 3, 1, 1, 16, 16, 0)
    assert [L.dll.argus_conv_x8_ok(C.byref(x8.with_tuning({13: 1})), ps) for ps in (0, 1)] == [1, 1]
    assert [L.dll.argus_conv_x8_ok(C.byref(x8.with_tuning({13: 1, 37: 2})), ps) for ps in (0, 1)] == [0, 1]
    assert [L.dll.argus_conv_x8_ok(C.byref(x8.with_tuning({13: 1, 37: 8})), ps) for ps in (0, 1)] == [1, 0]
    s2 = ConvDesc(8, 16, 16, 256, 256, 3, 3, 2, 1, 8, 8, 0).with_tuning({13: 1})
    c64 = ConvDesc(8, 16, 16, 64, 64, 3, 3, 1, 1, 16, 16, 0).with_tuning({13: 1})
    assert [L.dll.argus_conv_x8_ok(C.byref(d_), ps) for d_ in (s2, c64) for ps in (0, 1)] == [0, 0, 0, 0]
    # the statistics-only forward's partial layout (host-only): the persistent kernel's ragged rows (one per
    # row split, negative tile) for bf16 1x1 stride-1 convs under key 44, the igemm layout otherwise
    so = ConvDesc(64, 64, 64, 64, 256, 1, 1, 1, 0, 64, 64, 0)
    rows, tile = L.dll.argus_conv_fwd_stats_only_rows(C.byref(so), 1), L.dll.argus_conv_fwd_stats_only_tile(C.byref(so), 1)
    assert tile < 0 and 0 < rows <= 1024 and rows * -tile >= 64 * 64 * 64
    so0 = so.with_tuning({44: 0})
    assert (L.dll.argus_conv_fwd_stats_only_rows(C.byref(so0), 1), L.dll.argus_conv_fwd_stats_only_tile(C.byref(so0), 1)) == \
        (L.dll.argus_conv_fwd_stat_rows(C.byref(so0), 1), L.dll.argus_conv_fwd_stat_tile(C.byref(so0), 1))
    assert L.dll.argus_conv_fwd_stats_only_tile(C.byref(good), 1) == L.dll.argus_conv_fwd_stat_tile(C.byref(good), 1)
    # stat_part sizing (ABI 17): the ragged layouts need the int32 counts after the float2 partials, so
    # rows*k*2 floats alone is too small for the persistent statistics-only forward and the ragged stem
    nb = L.dll.argus_conv_fwd_stat_part_bytes
    assert nb(C.byref(so), 1, 1) == rows * 256 * 8 + rows * 4
    r0 = L.dll.argus_conv_fwd_stat_rows(C.byref(so), 1)
    assert L.dll.argus_conv_fwd_stat_tile(C.byref(so), 1) > 0 and nb(C.byref(so), 1, 0) == r0 * 256 * 8
    stem = ConvDesc(8, 376, 672, 3, 64, 7, 7, 2, 3, 188, 336, 1)  # 188 x 336 output: ragged 8 x 32 tiles
    sr, st = L.dll.argus_conv_fwd_stat_rows(C.byref(stem), 1), L.dll.argus_conv_fwd_stat_tile(C.byref(stem), 1)
    assert st < 0 and nb(C.byref(stem), 1, 0) == sr * 64 * 8 + sr * 4 > sr * 64 * 8
    assert nb(C.byref(bad), 1, 0) == 0
    unknown = good.with_tuning({30: 1})  # removed key (the 64-channel halo variant is a constant)
    with pytest.raises(ArgusHipError, match="unknown tuning key 30"):
        L.conv_fwd(C.byref(unknown), 1, 16, 16, 16, None, None, None, None)


def test_product_path_has_no_cpu_fallback():
    import torch

    from argus_amd.losses import geometric_loss_fn
    from argus_amd.models import NCameraCNN

    m = NCameraCNN()
    with pytest.raises(RuntimeError, match="HIP"):
        m(torch.rand(1, 6, 32, 32))
    with pytest.raises(AssertionError):
        m(torch.rand(6, 32, 32))
    with pytest.raises(RuntimeError, match="HIP"):
        geometric_loss_fn(torch.zeros(2, 6), torch.zeros(2, 7))
