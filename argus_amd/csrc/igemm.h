// Implicit-GEMM convolution parameters shared by the register-staged kernel (conv.hip) and the
// global->LDS (glds) kernel (conv_glds.hip).
#pragma once
#include "common.h"
#include "../../include/argus_hip.h"

namespace argus {

struct IgPhase {
  int M;          // GEMM rows of this phase = images * Hq * Wq
  int Hq, Wq;     // output grid of this phase
  int oh0, ow0;   // output pixel = (qh*osh + oh0, qw*osw + ow0)
  int K;          // ntaps * Cin (0: this phase has no taps -> output = addend or zeros)
  int dh[9], dw[9], boff[9];  // per tap: input offset (input = q*is + d) and B-row element offset
};

struct IgParams {
  const void* a;
  const void* b;
  void* c;
  const float* pro_scale;
  const float* pro_shift;
  float2* stats;
  const void* addend;          // C += addend (same layout as C; may alias C), masked by addend_mask
  const uint8_t* addend_mask;  // one byte per 16-byte chunk, bit j <-> element j (bn_apply mask)
  int N, Cin, lda, H, W, ish, isw, Ho, Wo, osh, osw, ldc, ldb;
  int stem, nphase;
  int stat_tile;  // rows per BN-statistics partial (forward with stats)
  IgPhase ph[4];
};

struct WgParams {
  const void* x;
  const void* dy;
  const float* pro_scale;
  const float* pro_shift;
  float* part;  // [splits][M][N]
  int M, N, Cin, lda, H, W, Ho, Wo, stride, pad, S;
  int P;
  int pps;  // pixels per split (multiple of the k-step)
  int stem;
};

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static ARGUS_DEV void run(f32x4& acc, u32x4 a, u32x4 b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  // lane group g supplies k = 4g + j at sub-step j (same mapping for A and B)
  static ARGUS_DEV void run(f32x4& acc, u32x4 a, u32x4 b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
};

ARGUS_DEV int swz8(int row) { return (row >> 1) & 7; }

ARGUS_DEV u32x4 sel(bool ok, u32x4 v) {
  const u32x4 z = {0u, 0u, 0u, 0u};
  return ok ? v : z;
}


// forward / dgrad launchers of the glds kernel (conv_glds.hip); return false when the shape is not
// served by it (then conv.hip's kernel runs)
bool igemm_glds_launch(const IgParams& p, int maxM, int maxK, hipStream_t st);
// 3x3 stride-1 forward / dgrad with an LDS-resident halo tile (conv_halo.hip); false = not served
bool conv3x3_halo_launch(const IgParams& p, hipStream_t st);
// 3x3 stride-1 weight gradient with an LDS-resident halo tile (conv_halo.hip): plan / launch of the
// split partials (fp32 [splits][K][9C]); false = not served
// bf16 weight gradient on global->LDS staged operands (conv_glds.hip): plan / launch; false = not served
bool wgrad_glds_plan(const argus_conv_desc& d, int dtype, bool pro, int* splits, int* pps);
bool wgrad_glds_launch(const argus_conv_desc& d, const WgParams& base, int splits, int pps, hipStream_t st);
bool wgrad3x3_halo_plan(const argus_conv_desc& d, int dtype, int* splits, int* tiles_per_split);
bool wgrad3x3_halo_launch(const argus_conv_desc& d, int dtype, const void* x, const float* sc, const float* sh,
                          const void* dy, void* ws, size_t ws_bytes, int* splits, hipStream_t st);

}  // namespace argus
