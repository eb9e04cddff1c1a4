// Internal (C++) launcher declarations shared by the .hip translation units and capi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <string>

#include "../../include/argus_hip.h"

namespace argus {

void set_error(const std::string& msg);
int check_launch(const char* what);

int conv_fwd_bn_out(const argus_conv_desc& d, int dtype, const void* x, const void* w, const float* sc,
                    const float* sh, const void* res, const float* rsc, const float* rsh, void* out, uint8_t* bits,
                    void* y, hipStream_t st);
int conv_fwd(const argus_conv_desc& d, int dtype, const void* x, const void* w, void* y,
             const float* sc, const float* sh, float* stats, hipStream_t st, void* pro_out = nullptr,
             const argus_bn_fwd_fin* fin = nullptr);
// set by a forward launch that folded its statistics finalize (argus_conv_fwd_fin; conv.hip)
extern thread_local int g_ffin_folded;
int conv_fwd_stat_rows(const argus_conv_desc& d, int dtype);
int conv_fwd_x8(const argus_conv_desc& d, const void* x8, const void* w, void* y, float* stats, hipStream_t st);
int conv_dgrad_bn_x8(const argus_conv_desc& d, const void* dy8, const void* wt, void* dm, const argus_bn_bwd_epilogue* bn,
                     hipStream_t st);
int conv_x8_ok(const argus_conv_desc& d, int pass);
// BN workspace layout (bn.hip): [0, kBnCounterBytes) ticket counters, then double2 group results
constexpr size_t kBnCounterBytes = 16384;
// the folded weight-gradient reduction's counters at the end of a wgrad workspace (policy key 50)
constexpr size_t kWgFoldCtrBytes = 16384;
int conv_fwd_stat_tile(const argus_conv_desc& d, int dtype);
// the partial-row layout of a statistics-only forward (argus_conv_fwd with y == NULL)
int conv_fwd_stats_only_rows(const argus_conv_desc& d, int dtype);
int conv_fwd_stats_only_tile(const argus_conv_desc& d, int dtype);

// Kernel-selection policy (argus_conv_policy_default): the immutable library table overlaid with one
// call's overrides (argus_conv_desc.tuning). Host-only; built per call, never stored.
enum TuneKey : int {
  kForceBm = 0,         // 0..2: row tile of pass fwd / dgrad / wgrad (0 = heuristic)
  kForceBn = 3,         // 3..5: column tile
  kWgradTarget = 6,     // weight-gradient split target (workgroups)
  kSmallKMax = 7,       // largest K on the single-buffer OCC 3/4 igemm
  kGldsMinK = 8,        // smallest K on the glds forward / dgrad (0 = off)
  kGldsMinGrid = 9,     // fewest workgroups for the glds kernel
  kHaloEnable = 10,     // 3x3 stride-1 forward / dgrad on the LDS-halo kernel
  kWgHaloEnable = 11,   // 3x3 stride-1 weight gradient on the LDS-halo kernel
  kWgHaloTarget = 12,   // ... its split target
  kHaloMinGrid = 13,    // fewest workgroups for the forward / dgrad halo kernel
  kWgHaloMaxTiles = 14, // most 64 x 64 channel tiles for the halo weight gradient
  kStemLdsFwd = 19,     // bf16 stem forward on the LDS-patch kernel
  kWgradTarget3x3 = 27, // split target of the register-staged 3x3 weight gradient (Cout > 64)
  kStemLdsWgrad = 34,   // bf16 stem weight gradient on the LDS-patch kernel
  kFwdBm128Rows = 35,   // fewest forward GEMM rows for 128-row tiles
  kGldsMinRows = 36,    // fewest GEMM rows (largest phase) for the glds kernel
  kFp8Passes = 37,      // ARGUS_FP8: which passes take MX-fp8 operands (1 fwd | 2 3x3 dgrad | 4 1x1 dgrad | 8 3x3 s1 fwd)
  kDgradApStaged = 38,  // 1x1 dgrad with an apply prologue: register-staged (1) or apply kernel + glds (0)
  kGldsDgrad = 39,      // data gradients may run on the glds kernel (forwards: key 8 alone)
  kHaloDgrad = 40,      // 3x3 data gradients may run on the LDS-halo kernel (forwards: key 10 alone)
  kGldsDgradStages = 41,  // LDS ring depth of the glds data gradients (3, or 2: 96 KB)
  kBwdSmallKOcc = 42,     // workgroups per CU the small-K BN-epilogue / apply-prologue dgrads are built for (4 or 3)
  kP1x1Dgrad = 43,        // the persistent 1x1 dgrad (apply prologue + mask-bits BN epilogue) for conv1 (1 on)
  kP1x1FwdStats = 44,     // statistics-only 1x1 forwards on the persistent kernel (conv_p1x1.hip; 1 on)
  kWgradDma = 45,         // 1x1 bf16 weight gradients on the LDS-DMA ring kernel (conv_wgdma.hip)
  kWgradSmallP = 46,      // 1x1 weight gradients over at most this many pixels: half the split target
  kWgradDmaGather = 47,   // ... and the stride-2 (1x1 / 3x3) plain ones, x rows gathered (1 on, >1 pixel cap)
  kWgradDmaStages = 48,   // LDS ring stages of the 128 x 256 apply DMA weight gradient (2..5)
  kDgradApMaxCols = 49,   // 1x1 dgrads stage the apply prologue up to this many 128-column tiles (0: any)
  kWgradFold = 50,        // DMA weight gradients reduce their split partials in-launch (1 on)
  kHaloDeepRing = 51,     // 3x3 halo fwd / dgrad (128 columns, <= 384 halo positions): four weight stages (1 on)
  kNumTuneKeys = 52
};
struct Policy {
  int v[kNumTuneKeys];
  int operator[](int key) const { return v[key]; }
};
int policy_default(int key);  // -1: not a key
// The policy of one call: the defaults + d.tuning (the keys were validated by the conv entry point).
Policy policy_of(const argus_conv_desc& d);
// ARGUS_OK, or ARGUS_ERR_ARG (+ set_error) when d.tuning holds an unknown key or n_tuning < 0.
int check_tuning(const argus_conv_desc& d);
int conv_launch_info(const argus_conv_desc& d, int dtype, int pass, int64_t* flops);
size_t conv_weight_prep_table_bytes(int count);
int conv_weight_prep_table(int count, const argus_conv_desc* descs, const float* const* w, const int64_t* strides,
                           void* const* wf, void* const* wd, void* host_table, size_t bytes, int* nblocks);
int conv_weight_prep_batch(int dtype, int count, const void* device_table, int nblocks, hipStream_t st);
int conv_dgrad(const argus_conv_desc& d, int dtype, const void* dy, const void* wt, void* dx,
               const void* addend, const uint8_t* addend_mask, hipStream_t st);
int conv_dgrad_bn_rows(const argus_conv_desc& d, int dtype);
int conv_check_desc(const argus_conv_desc& d);  // conv.hip's descriptor validation (ARGUS_OK or an error)
// fused 1x1 data + weight gradient (conv_dgw.hip)
bool conv_dgw_ok(const argus_conv_desc& d, int dtype);
size_t conv_dgw_ws_bytes(const argus_conv_desc& d, int dtype);
int conv_dgw_rows(const argus_conv_desc& d, int dtype);
int conv_dgw(const argus_conv_desc& d, int dtype, const void* dm, const void* wd, const void* x, void* dx,
             const void* addend, const argus_bn_bwd_epilogue* bn, const argus_bn_bwd_prologue* pro, float* dw,
             void* ws, size_t ws_bytes, hipStream_t st);
int conv_dgrad_stages_prologue(const argus_conv_desc& d, int dtype);
int conv_dgrad_bn(const argus_conv_desc& d, int dtype, const void* dy, const void* wt, void* dm,
                  const void* addend, const argus_bn_bwd_epilogue* bn, const argus_bn_bwd_prologue* pro,
                  hipStream_t st);
size_t conv_wgrad_ws(const argus_conv_desc& d, int dtype);
int conv_wgrad_apply(const argus_conv_desc& d, int dtype, const void* x, const void* dm,
                     const argus_bn_bwd_prologue& ap, float* dw, void* ws, size_t ws_bytes, hipStream_t st);
int conv_wgrad(const argus_conv_desc& d, int dtype, const void* x, const float* sc,
               const float* sh, const void* dy, float* dw, void* ws, size_t ws_bytes,
               hipStream_t st);
int conv_weight_prep(const argus_conv_desc& d, int dtype, const float* w, const int64_t* strides,
                     void* wf, void* wd, hipStream_t st);
int images_to_nhwc4(int dtype, int64_t nimg, int h, int w, const float* x, void* out,
                    hipStream_t st);
int images_u8_to_nhwc4(int dtype, int64_t nimg, int h, int w, const uint8_t* x, void* out,
                       hipStream_t st);

}  // namespace argus
