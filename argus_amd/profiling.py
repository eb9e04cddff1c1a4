"""Live per-launch kernel timing through the library's native timer (include/argus_hip.h
argus_ktimer_*): timed launches carry hipExtLaunchKernelGGL start/stop events in their dispatch
packet, so durations are the kernels' own execution on the launch stream, as rocprofv3 reports."""
from __future__ import annotations

import ctypes as C

from argus_amd._lib import lib


class KernelTimer:
    """``with KernelTimer(prefix) as t: ...; t.summary()`` -> per-instantiation timing of conv and BN kernels."""

    def __init__(self, prefix: str | None = None, stream: int | None = None):
        """``stream``: only launches on that HIP stream handle (e.g. the main stream's
        ``torch.cuda.current_stream().cuda_stream``); None = every stream."""
        self.prefix = prefix
        self.stream = stream

    def start(self) -> None:
        f = self.prefix.encode() if self.prefix else None
        if self.stream is None:
            lib().ktimer_enable(f)
        else:
            lib().ktimer_enable_on(f, self.stream)

    def stop(self) -> None:
        lib().ktimer_disable()

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *a):
        self.stop()

    def summary(self) -> dict:
        """name -> {launches, total_ms, avg_us, flops_per_launch, bytes_per_launch, tflops} (synchronizes)."""
        L = lib()
        n = L.ktimer_count()
        if n < 0:
            raise RuntimeError(L.dll.argus_last_error().decode())
        out = {}
        name = C.create_string_buffer(256)
        cnt, ms, work, nbytes = C.c_int64(), C.c_double(), C.c_double(), C.c_double()
        for i in range(n):
            L.ktimer_get(i, name, 256, C.byref(cnt), C.byref(ms), C.byref(work), C.byref(nbytes))
            k = cnt.value
            out[name.value.decode()] = {
                "launches": k, "total_ms": ms.value, "avg_us": 1e3 * ms.value / k,
                "flops_per_launch": work.value / k, "bytes_per_launch": nbytes.value / k,
                "tflops": work.value / (ms.value * 1e-3) / 1e12 if ms.value > 0 else 0.0}
        return out
