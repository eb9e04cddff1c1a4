// extern "C" surface of libargus_hip.so (include/argus_hip.h) + error reporting.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>

#include "internal.h"

namespace argus {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return ARGUS_ERR_HIP;
  }
  return ARGUS_OK;
}

}  // namespace argus

using namespace argus;

extern "C" {

int argus_abi_version(void) { return 19; }

const char* argus_last_error(void) { return g_last_error.c_str(); }

// cross-stream events: device-scope release / acquire only (hipEventDisableSystemFence)
int argus_event_create(argus_event_t* event) {
  if (!event) { set_error("event_create: null out pointer"); return ARGUS_ERR_ARG; }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
    set_error("event_create: hipEventCreateWithFlags failed");
    return ARGUS_ERR_HIP;
  }
  *event = e;
  return ARGUS_OK;
}

int argus_event_record(argus_event_t event, argus_stream_t stream) {
  if (!event) { set_error("event_record: null event"); return ARGUS_ERR_ARG; }
  if (hipEventRecord((hipEvent_t)event, (hipStream_t)stream) != hipSuccess) {
    set_error("event_record: hipEventRecord failed");
    return ARGUS_ERR_HIP;
  }
  return ARGUS_OK;
}

int argus_stream_wait_event(argus_stream_t stream, argus_event_t event) {
  if (!event) { set_error("stream_wait_event: null event"); return ARGUS_ERR_ARG; }
  if (hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0) != hipSuccess) {
    set_error("stream_wait_event: hipStreamWaitEvent failed");
    return ARGUS_ERR_HIP;
  }
  return ARGUS_OK;
}

int argus_event_destroy(argus_event_t event) {
  if (event && hipEventDestroy((hipEvent_t)event) != hipSuccess) {
    set_error("event_destroy: hipEventDestroy failed");
    return ARGUS_ERR_HIP;
  }
  return ARGUS_OK;
}

int argus_images_to_nhwc4(int dtype, int64_t nimg, int h, int w, const float* x, void* out, argus_stream_t stream) {
  if (nimg <= 0 || h <= 0 || w <= 0 || !x || !out) { set_error("images_to_nhwc4: bad arguments"); return ARGUS_ERR_ARG; }
  return images_to_nhwc4(dtype, nimg, h, w, x, out, (hipStream_t)stream);
}

int argus_images_u8_to_nhwc4(int dtype, int64_t nimg, int h, int w, const uint8_t* x, void* out,
                             argus_stream_t stream) {
  if (nimg <= 0 || h <= 0 || w <= 0 || !x || !out) { set_error("images_u8_to_nhwc4: bad arguments"); return ARGUS_ERR_ARG; }
  return images_u8_to_nhwc4(dtype, nimg, h, w, x, out, (hipStream_t)stream);
}

int argus_conv_weight_prep(const argus_conv_desc* d, int dtype, const float* w, const int64_t* strides, void* wf,
                           void* wd, argus_stream_t stream) {
  if (!d || !w) { set_error("conv_weight_prep: null argument"); return ARGUS_ERR_ARG; }
  return conv_weight_prep(*d, dtype, w, strides, wf, wd, (hipStream_t)stream);
}

size_t argus_conv_weight_prep_table_bytes(int count) { return conv_weight_prep_table_bytes(count); }

int argus_conv_weight_prep_table(int count, const argus_conv_desc* descs, const float* const* w_master,
                                 const int64_t* strides, void* const* w_fwd, void* const* w_dgrad, void* host_table,
                                 size_t table_bytes, int* nblocks) {
  return conv_weight_prep_table(count, descs, w_master, strides, w_fwd, w_dgrad, host_table, table_bytes, nblocks);
}

int argus_conv_weight_prep_batch(int dtype, int count, const void* device_table, int nblocks, argus_stream_t stream) {
  return conv_weight_prep_batch(dtype, count, device_table, nblocks, (hipStream_t)stream);
}

int argus_conv_fwd(const argus_conv_desc* d, int dtype, const void* x, const void* w, void* y, const float* sc,
                   const float* sh, float* stats, argus_stream_t stream) {
  if (!d || !x || !w || (!y && !stats) || (sc == nullptr) != (sh == nullptr)) {
    set_error("conv_fwd: bad arguments");
    return ARGUS_ERR_ARG;
  }
  return conv_fwd(*d, dtype, x, w, y, sc, sh, stats, (hipStream_t)stream);
}

int argus_conv_fwd_fin(const argus_conv_desc* d, int dtype, const void* x, const void* w, void* y, const float* sc,
                       const float* sh, float* stats, const argus_bn_fwd_fin* fin, argus_stream_t stream) {
  if (!d || !x || !w || !stats || !fin || !fin->workspace || !fin->gamma || !fin->beta ||
      (sc == nullptr) != (sh == nullptr)) {
    set_error("conv_fwd_fin: bad arguments");
    return ARGUS_ERR_ARG;
  }
  if (int e = conv_fwd(*d, dtype, x, w, y, sc, sh, stats, (hipStream_t)stream, nullptr, fin)) return e;
  if (g_ffin_folded) return ARGUS_OK;
  // not folded (the producer's tiles do not align with the merge groups): the separate finalize
  const bool so = y == nullptr && sc == nullptr;
  const int rows = so ? conv_fwd_stats_only_rows(*d, dtype) : conv_fwd_stat_rows(*d, dtype);
  const int tile = so ? conv_fwd_stats_only_tile(*d, dtype) : conv_fwd_stat_tile(*d, dtype == ARGUS_FP8 ? ARGUS_BF16 : dtype);
  return argus_bn_finalize(d->k, rows, tile, stats, (int64_t)d->n * d->ho * d->wo, fin->gamma, fin->beta, fin->eps,
                           fin->momentum, fin->running_mean, fin->running_var, fin->num_batches_tracked, fin->mean,
                           fin->invstd, fin->scale, fin->shift, fin->workspace, stream);
}

int argus_conv_fwd_apply_out(const argus_conv_desc* d, int dtype, const void* x, const void* w, void* y,
                             const float* sc, const float* sh, float* stats, void* x_out, argus_stream_t stream) {
  if (!d || !x || !w || (!y && !stats) || !sc || !sh || !x_out) {
    set_error("conv_fwd_apply_out: bad arguments");
    return ARGUS_ERR_ARG;
  }
  return conv_fwd(*d, dtype, x, w, y, sc, sh, stats, (hipStream_t)stream, x_out);
}

int argus_conv_fwd_bn_out(const argus_conv_desc* d, int dtype, const void* x, const void* w_fwd, const float* scale,
                          const float* shift, const void* res, const float* res_scale, const float* res_shift, void* out,
                          uint8_t* mask_bits, void* y, argus_stream_t stream) {
  if (!d) {
    set_error("conv_fwd_bn_out: bad arguments");
    return ARGUS_ERR_ARG;
  }
  return conv_fwd_bn_out(*d, dtype, x, w_fwd, scale, shift, res, res_scale, res_shift, out, mask_bits, y,
                         (hipStream_t)stream);
}
int argus_conv_fwd_stat_rows(const argus_conv_desc* d, int dtype) { return d ? conv_fwd_stat_rows(*d, dtype) : 0; }
int argus_conv_fwd_stats_only_rows(const argus_conv_desc* d, int dtype) {
  return d ? conv_fwd_stats_only_rows(*d, dtype) : 0;
}
int argus_conv_fwd_stats_only_tile(const argus_conv_desc* d, int dtype) {
  return d ? conv_fwd_stats_only_tile(*d, dtype) : 0;
}
size_t argus_conv_fwd_stat_part_bytes(const argus_conv_desc* d, int dtype, int stats_only) {
  if (!d || conv_check_desc(*d)) return 0;
  const int rows = stats_only ? conv_fwd_stats_only_rows(*d, dtype) : conv_fwd_stat_rows(*d, dtype);
  const int tile = stats_only ? conv_fwd_stats_only_tile(*d, dtype) : conv_fwd_stat_tile(*d, dtype);
  if (rows <= 0) return 0;
  // float2 {sum, M2} [rows][k], then int32 pixel counts [rows] when the tiling is ragged (tile < 0)
  return (size_t)rows * d->k * 2 * sizeof(float) + (tile < 0 ? (size_t)rows * sizeof(int32_t) : 0);
}

int argus_conv_policy_default(int key) { return policy_default(key); }

int argus_conv_launch_info(const argus_conv_desc* d, int dtype, int pass, int64_t* flops) {
  return d ? conv_launch_info(*d, dtype, pass, flops) : -1;
}

int argus_conv_fwd_stat_tile(const argus_conv_desc* d, int dtype) { return d ? conv_fwd_stat_tile(*d, dtype) : 0; }

int argus_conv_dgrad(const argus_conv_desc* d, int dtype, const void* dy, const void* wt, void* dx, const void* addend,
                     const uint8_t* addend_mask,
                     argus_stream_t stream) {
  if (!d || !dy || !wt || !dx) { set_error("conv_dgrad: bad arguments"); return ARGUS_ERR_ARG; }
  return conv_dgrad(*d, dtype, dy, wt, dx, addend, addend_mask, (hipStream_t)stream);
}

int argus_conv_dgrad_bn_rows(const argus_conv_desc* d, int dtype) { return d ? conv_dgrad_bn_rows(*d, dtype) : -1; }
int argus_conv_dgrad_stages_prologue(const argus_conv_desc* d, int dtype) {
  return d ? conv_dgrad_stages_prologue(*d, dtype) : 0;
}

int argus_conv_dgrad_bn(const argus_conv_desc* d, int dtype, const void* dy, const void* wt, void* dm,
                        const void* addend, const argus_bn_bwd_epilogue* bn, const argus_bn_bwd_prologue* pro,
                        argus_stream_t stream) {
  if (!d || !dy || !wt || !dm) { set_error("conv_dgrad_bn: bad arguments"); return ARGUS_ERR_ARG; }
  return conv_dgrad_bn(*d, dtype, dy, wt, dm, addend, bn, pro, (hipStream_t)stream);
}

int argus_conv_x8_ok(const argus_conv_desc* d, int pass) { return d ? conv_x8_ok(*d, pass) : 0; }

int argus_conv_fwd_x8(const argus_conv_desc* d, const void* x8, const void* w, void* y, float* stats,
                      argus_stream_t stream) {
  if (!d) { set_error("conv_fwd_x8: bad arguments"); return ARGUS_ERR_ARG; }
  return conv_fwd_x8(*d, x8, w, y, stats, (hipStream_t)stream);
}

int argus_conv_dgrad_bn_x8(const argus_conv_desc* d, const void* dy8, const void* wt, void* dm,
                           const argus_bn_bwd_epilogue* bn, argus_stream_t stream) {
  if (!d || !dy8 || !wt || !dm) { set_error("conv_dgrad_bn_x8: bad arguments"); return ARGUS_ERR_ARG; }
  return conv_dgrad_bn_x8(*d, dy8, wt, dm, bn, (hipStream_t)stream);
}

int argus_conv_wgrad_apply(const argus_conv_desc* d, int dtype, const void* x, const void* dm,
                           const argus_bn_bwd_prologue* ap, float* dw, void* ws, size_t ws_bytes, argus_stream_t stream) {
  if (!d || !x || !dm || !ap || !dw || !ws) { set_error("conv_wgrad_apply: bad arguments"); return ARGUS_ERR_ARG; }
  return conv_wgrad_apply(*d, dtype, x, dm, *ap, dw, ws, ws_bytes, (hipStream_t)stream);
}

int argus_conv_dgrad_wgrad_ok(const argus_conv_desc* d, int dtype) {
  return d && !conv_check_desc(*d) && conv_dgw_ok(*d, dtype) ? 1 : 0;
}

size_t argus_conv_dgrad_wgrad_workspace_bytes(const argus_conv_desc* d, int dtype) {
  return d && !conv_check_desc(*d) ? conv_dgw_ws_bytes(*d, dtype) : 0;
}

int argus_conv_dgrad_wgrad_bn_rows(const argus_conv_desc* d, int dtype) {
  return d && !conv_check_desc(*d) ? conv_dgw_rows(*d, dtype) : -1;
}

int argus_conv_dgrad_wgrad_bn(const argus_conv_desc* d, int dtype, const void* dm, const void* w_dgrad,
                              const void* x, void* dx, const void* addend, const argus_bn_bwd_epilogue* bn,
                              const argus_bn_bwd_prologue* pro, float* dw, void* workspace,
                              size_t workspace_bytes, argus_stream_t stream) {
  if (!d) { set_error("conv_dgrad_wgrad_bn: bad arguments"); return ARGUS_ERR_ARG; }
  return conv_dgw(*d, dtype, dm, w_dgrad, x, dx, addend, bn, pro, dw, workspace, workspace_bytes,
                  (hipStream_t)stream);
}

size_t argus_conv_wgrad_workspace_bytes(const argus_conv_desc* d, int dtype) { return d ? conv_wgrad_ws(*d, dtype) : 0; }

int argus_conv_wgrad(const argus_conv_desc* d, int dtype, const void* x, const float* sc, const float* sh,
                     const void* dy, float* dw, void* ws, size_t ws_bytes, argus_stream_t stream) {
  if (!d || !x || !dy || !dw || !ws || (sc == nullptr) != (sh == nullptr)) {
    set_error("conv_wgrad: bad arguments");
    return ARGUS_ERR_ARG;
  }
  return conv_wgrad(*d, dtype, x, sc, sh, dy, dw, ws, ws_bytes, (hipStream_t)stream);
}

}  // extern "C"
