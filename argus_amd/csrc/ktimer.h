// Live per-launch kernel timing for bench.py's roofline: while enabled, every launch of a conv or
// BN / elementwise kernel
// whose instantiation name starts with the filter goes through hipExtLaunchKernelGGL with a
// start/stop event pair carried by the dispatch packet itself, so the measured span is the
// kernel's own execution on its stream (what rocprofv3 --kernel-trace reports), not the gap
// between host-enqueued markers. Names are the demangled template instantiations, e.g.
// "argus::igemm_kernel<__bf16, 128, 128, false, true>" (c++filt of rocprof's kernel name).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <string>

namespace argus {

bool ktimer_wants(const char* name, hipStream_t st);
// Returns the (start, stop) events for one timed launch of `name` doing `work` flops and moving
// `bytes` algorithmic HBM bytes.
void ktimer_slot(const char* name, double work, double bytes, hipEvent_t* start, hipEvent_t* stop);
// Algorithmic flops / bytes of the launch about to be issued (set by the C-ABI entry points).
extern thread_local double g_launch_work, g_launch_bytes;

template <typename K, typename... Args>
inline void timed_launch(const char* name, K kernel, dim3 grid, dim3 block, hipStream_t st, Args... args) {
  if (ktimer_wants(name, st)) {
    hipEvent_t a, b;
    ktimer_slot(name, g_launch_work, g_launch_bytes, &a, &b);
    hipExtLaunchKernelGGL(kernel, grid, block, 0, st, a, b, 0, args...);
  } else {
    hipLaunchKernelGGL(kernel, grid, block, 0, st, args...);
  }
}

template <typename T>
inline const char* type_name() { return sizeof(T) == 2 ? "__bf16" : "float"; }
inline const char* bool_name(bool b) { return b ? "true" : "false"; }

}  // namespace argus
