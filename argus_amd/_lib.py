"""ctypes binding of libargus_hip.so (include/argus_hip.h).

The product path has exactly one compute backend: these HIP kernels. If the library is missing or
fails to load, every op raises — there is no CPU or PyTorch fallback.

torch is imported before the library is opened: torch's bundled ``libamdhip64.so`` carries the same
SONAME (``libamdhip64.so.7``) as ROCm's, so the dynamic linker binds libargus_hip.so to the HIP
runtime torch already loaded — one runtime per process, and torch's streams/pointers are valid here.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL, see module docstring)

LIB_PATH = Path(os.environ.get("ARGUS_HIP_LIB", Path(__file__).resolve().parent / "libargus_hip.so"))

F32, BF16, FP8 = 0, 1, 2
ABI_VERSION = 19


class Tuning(C.Structure):
    """argus_tuning: one {key, value} override of the kernel-selection policy."""

    _fields_ = [("key", C.c_int32), ("value", C.c_int32)]


class ConvDesc(C.Structure):
    """argus_conv_desc. ``ConvDesc(n, h, w, c, k, r, s, stride, pad, ho, wo, stem)`` uses the library's
    kernel-selection defaults; ``with_tuning`` attaches per-call overrides."""

    _fields_ = [(n, C.c_int32) for n in ("n", "h", "w", "c", "k", "r", "s", "stride", "pad", "ho", "wo", "stem")] + [
        ("n_tuning", C.c_int32), ("tuning", C.POINTER(Tuning))]

    def with_tuning(self, tuning: dict | None) -> "ConvDesc":
        """A copy of this descriptor carrying ``tuning`` ({key: value}, argus_conv_policy_default keys) as
        its per-call overrides (None / {} = the defaults). The override array lives on the copy."""
        d = ConvDesc(*(getattr(self, f) for f, _ in self._fields_[:12]))
        items = sorted((tuning or {}).items())
        if items:
            arr = (Tuning * len(items))(*[Tuning(int(k), int(v)) for k, v in items])
            d._tuning_keep = arr
            d.n_tuning = len(items)
            d.tuning = C.cast(arr, C.POINTER(Tuning))
        return d


class BnBwdEpilogue(C.Structure):
    """argus_bn_bwd_epilogue (include/argus_hip.h)."""

    _fields_ = [("y", C.c_void_p), ("mean", C.c_void_p), ("invstd", C.c_void_p), ("mask_mode", C.c_int32),
                ("reserved", C.c_int32), ("scale", C.c_void_p), ("shift", C.c_void_p), ("mask_bits", C.c_void_p),
                ("y2", C.c_void_p), ("mean2", C.c_void_p), ("invstd2", C.c_void_p), ("part", C.c_void_p),
                ("part2", C.c_void_p), ("workspace", C.c_void_p), ("gamma", C.c_void_p), ("dgamma", C.c_void_p),
                ("dbeta", C.c_void_p), ("ca", C.c_void_p), ("cb", C.c_void_p), ("cc", C.c_void_p),
                ("gamma2", C.c_void_p), ("dgamma2", C.c_void_p), ("dbeta2", C.c_void_p), ("ca2", C.c_void_p),
                ("cb2", C.c_void_p), ("cc2", C.c_void_p), ("y_x", C.c_void_p), ("y_w", C.c_void_p),
                ("y_k", C.c_int32), ("reserved2", C.c_int32)]


class BnFwdFin(C.Structure):
    """argus_bn_fwd_fin (include/argus_hip.h): the train-mode BN finalize of argus_conv_fwd_fin."""

    _fields_ = [("workspace", C.c_void_p), ("gamma", C.c_void_p), ("beta", C.c_void_p), ("eps", C.c_float),
                ("momentum", C.c_float), ("running_mean", C.c_void_p), ("running_var", C.c_void_p),
                ("num_batches_tracked", C.c_void_p), ("mean", C.c_void_p), ("invstd", C.c_void_p),
                ("scale", C.c_void_p), ("shift", C.c_void_p)]


class BnBwdPrologue(C.Structure):
    """argus_bn_bwd_prologue (include/argus_hip.h)."""

    _fields_ = [("y", C.c_void_p), ("ca", C.c_void_p), ("cb", C.c_void_p), ("cc", C.c_void_p),
                ("dy_out", C.c_void_p)]


_P = C.c_void_p
_I = C.c_int
_I64 = C.c_int64
_F = C.c_float
_SZ = C.c_size_t
_DESC = C.POINTER(ConvDesc)

# name -> (restype, argtypes); must mirror include/argus_hip.h exactly (tests check the export list)
SIGNATURES = {
    "argus_abi_version": (_I, []),
    "argus_last_error": (C.c_char_p, []),
    "argus_images_to_nhwc4": (_I, [_I, _I64, _I, _I, _P, _P, _P]),
    "argus_images_u8_to_nhwc4": (_I, [_I, _I64, _I, _I, _P, _P, _P]),
    "argus_conv_weight_prep": (_I, [_DESC, _I, _P, _P, _P, _P, _P]),
    "argus_conv_weight_prep_table_bytes": (_SZ, [_I]),
    "argus_conv_weight_prep_table": (_I, [_I, _DESC, C.POINTER(_P), C.POINTER(C.c_int64), C.POINTER(_P),
                                          C.POINTER(_P), _P, _SZ, C.POINTER(_I)]),
    "argus_conv_weight_prep_batch": (_I, [_I, _I, _P, _I, _P]),
    "argus_conv_fwd": (_I, [_DESC, _I, _P, _P, _P, _P, _P, _P, _P]),
    "argus_conv_fwd_bn_out": (_I, [_DESC, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "argus_conv_x8_ok": (_I, [_DESC, _I]),
    "argus_conv_fwd_stats_only_rows": (_I, [_DESC, _I]),
    "argus_conv_fwd_stats_only_tile": (_I, [_DESC, _I]),
    "argus_conv_fwd_stat_part_bytes": (_SZ, [_DESC, _I, _I]),
    "argus_conv_fwd_fin": (_I, [_DESC, _I, _P, _P, _P, _P, _P, _P, C.POINTER(BnFwdFin), _P]),
    "argus_conv_fwd_apply_out": (_I, [_DESC, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "argus_conv_fwd_x8": (_I, [_DESC, _P, _P, _P, _P, _P]),
    "argus_conv_dgrad_bn_x8": (_I, [_DESC, _P, _P, _P, C.POINTER(BnBwdEpilogue), _P]),
    "argus_conv_fwd_stat_rows": (_I, [_DESC, _I]),
    "argus_conv_fwd_stat_tile": (_I, [_DESC, _I]),
    "argus_conv_policy_default": (_I, [_I]),
    "argus_conv_launch_info": (_I, [_DESC, _I, _I, C.POINTER(C.c_int64)]),
    "argus_conv_dgrad": (_I, [_DESC, _I, _P, _P, _P, _P, _P, _P]),
    "argus_conv_dgrad_bn_rows": (_I, [_DESC, _I]),
    "argus_conv_dgrad_stages_prologue": (_I, [_DESC, _I]),
    "argus_conv_dgrad_bn": (_I, [_DESC, _I, _P, _P, _P, _P, C.POINTER(BnBwdEpilogue), C.POINTER(BnBwdPrologue), _P]),
    "argus_conv_wgrad_workspace_bytes": (_SZ, [_DESC, _I]),
    "argus_conv_wgrad": (_I, [_DESC, _I, _P, _P, _P, _P, _P, _P, _SZ, _P]),
    "argus_conv_wgrad_apply": (_I, [_DESC, _I, _P, _P, C.POINTER(BnBwdPrologue), _P, _P, _SZ, _P]),
    "argus_conv_dgrad_wgrad_ok": (_I, [_DESC, _I]),
    "argus_conv_dgrad_wgrad_workspace_bytes": (_SZ, [_DESC, _I]),
    "argus_conv_dgrad_wgrad_bn_rows": (_I, [_DESC, _I]),
    "argus_conv_dgrad_wgrad_bn": (_I, [_DESC, _I, _P, _P, _P, _P, _P, C.POINTER(BnBwdEpilogue),
                                       C.POINTER(BnBwdPrologue), _P, _P, _SZ, _P]),
    "argus_event_create": (_I, [C.POINTER(C.c_void_p)]),
    "argus_event_record": (_I, [_P, _P]),
    "argus_stream_wait_event": (_I, [_P, _P]),
    "argus_event_destroy": (_I, [_P]),
    "argus_ktimer_enable": (_I, [C.c_char_p]),
    "argus_ktimer_enable_on": (_I, [C.c_char_p, _P]),
    "argus_ktimer_disable": (_I, []),
    "argus_ktimer_count": (_I, []),
    "argus_ktimer_get": (_I, [_I, C.c_char_p, _I, C.POINTER(C.c_int64), C.POINTER(C.c_double),
                              C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "argus_bn_workspace_bytes": (_SZ, [_I]),
    "argus_bn_finalize": (_I, [_I, _I, _I, _P, _I64, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "argus_bn_eval_coeffs": (_I, [_I, _P, _P, _P, _P, _F, _P, _P, _P]),
    "argus_bn_apply": (_I, [_I, _I64, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P]),
    "argus_bn_apply_x8": (_I, [_I64, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P]),
    "argus_bn_bwd_rows": (_I, [_I64, _I]),
    "argus_bn_bwd_reduce": (_I, [_I, _I64, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "argus_bn_bwd_finalize": (_I, [_I, _I, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "argus_bn_bwd_apply": (_I, [_I, _I64, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "argus_bn_bwd_apply_x8": (_I, [_I64, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "argus_maxpool_fwd": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "argus_maxpool_bwd": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "argus_maxpool_bwd_bn_rows": (_I, [_I, _I, _I, _I, _I]),
    "argus_maxpool_bwd_bn": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "argus_maxpool_bwd_bn_fin": (_I, [_I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                      _P, _P, _P]),
    "argus_avgpool_fwd": (_I, [_I, _I, _I, _I, _P, _P, _P]),
    "argus_avgpool_bwd": (_I, [_I, _I, _I, _I, _P, _P, _P]),
    "argus_gemm_f32_workspace_bytes": (_SZ, [_I, _I, _I]),
    "argus_augment_params_bytes": (_SZ, []),
    "argus_augment_scratch_bytes": (_SZ, [_I64, _I, _I]),
    "argus_augment_photometric": (_I, [_I64, _I, _I, _P, _P, _P, _P, _P]),
    "argus_gemm_f32": (_I, [_I, _I, _I, _P, _I, _I, _P, _I, _I, _P, _I, _P, _I, _P, _P, _SZ, _P]),
    "argus_colsum_f32": (_I, [_I, _I, _P, _I, _P, _P]),
    "argus_gelu_f32": (_I, [_I64, _P, _P, _P]),
    "argus_gelu_bwd_f32": (_I, [_I64, _P, _P, _P, _P]),
    "argus_se3_loss": (_I, [_I, _P, _P, _P, _P, _F, _P]),
    "argus_se3_exp": (_I, [_I, _P, _P, _I, _P]),
    "argus_sumsq_workspace_bytes": (_SZ, [_I64]),
    "argus_global_norm": (_I, [_I64, _P, _P, _P, _P]),
    "argus_adam_step": (_I, [_I64, _P, _P, _P, _P, _P, _F, _F, _F, _F, _F, _F, _F, _F, _F, _P]),
}


class ArgusHipError(RuntimeError):
    pass


class _Lib:
    def __init__(self) -> None:
        if not LIB_PATH.exists():
            raise ArgusHipError(
                f"{LIB_PATH} not found: build it with `python -m argus_amd.build` "
                "(the argus_amd GPU path has no fallback)"
            )
        self.dll = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(self.dll, name)
            fn.restype = res
            fn.argtypes = args
        v = self.dll.argus_abi_version()
        if v != ABI_VERSION:
            raise ArgusHipError(f"libargus_hip ABI {v} != expected {ABI_VERSION}")

    def __getattr__(self, name: str):
        fn = getattr(self.dll, "argus_" + name)
        if fn.restype is _I and not name.endswith(("rows", "tile", "version", "info", "default", "count")):
            def call(*args, _fn=fn, _name=name):
                rc = _fn(*args)
                if rc != 0:
                    msg = self.dll.argus_last_error().decode(errors="replace")
                    raise ArgusHipError(f"argus_{_name} failed ({rc}): {msg}")
                return rc
            setattr(self, name, call)
            return call
        setattr(self, name, fn)
        return fn


_LIB: _Lib | None = None


def lib() -> _Lib:
    global _LIB
    if _LIB is None:
        _LIB = _Lib()
    return _LIB


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


class DeviceEvent:
    """argus_event_t: orders two streams of this device with a device-scope release / acquire
    (hipEventDisableSystemFence), without the system-scope cache writeback a torch.cuda.Event record
    carries. ``record(stream)`` and ``wait(stream)`` take torch streams (None: the current stream)."""

    __slots__ = ("h",)

    def __init__(self) -> None:
        h = C.c_void_p()
        lib().event_create(C.byref(h))
        self.h = h.value

    def record(self, s=None) -> "DeviceEvent":
        lib().event_record(self.h, (s or torch.cuda.current_stream()).cuda_stream)
        return self

    def wait(self, s=None) -> None:
        lib().stream_wait_event((s or torch.cuda.current_stream()).cuda_stream, self.h)

    def __del__(self) -> None:
        if self.h and _LIB is not None:
            _LIB.dll.argus_event_destroy(self.h)
            self.h = None
