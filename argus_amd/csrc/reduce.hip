// Split-K sum of the weight-gradient partials (fp32 [splits][M][N] -> dW), shared by the
// register-staged, halo and stem weight-gradient kernels (conv.hip, conv_halo.hip, stem.hip). Its own
// translation unit so tests/test_isa.py can check its ISA (batched loads) in seconds.
#include "common.h"
#include "internal.h"
#include "igemm.h"

namespace argus {

// dw[e] = sum_s part[s][e] (fixed order: deterministic). Block = CW float4-columns x SL split lanes;
// lane l sums splits l, l+SL, ... then the SL lanes combine through LDS in lane order. For the stem
// the padded (r8, s8, c4) columns are scattered to OHWI 7x7x3.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int M, int N,
                                                           int stem, int CW, float* __restrict__ dw) {
  const int SL = 256 / CW;
  const int col = threadIdx.x % CW, sl = threadIdx.x / CW;
  const size_t e4 = (size_t)blockIdx.x * CW + col;
  const size_t total4 = (size_t)M * N / 4;
  const size_t stride = (size_t)M * N;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (e4 < total4)
    for (int kb = sl; kb < splits; kb += SL * kLoadBatch) {
      f32x4 v[kLoadBatch];  // in flight together (common.h kLoadBatch); clamped, masked below
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u)
        v[u] = *reinterpret_cast<const f32x4*>(part + (size_t)min(kb + u * SL, splits - 1) * stride + e4 * 4);
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) s += kb + u * SL < splits ? v[u] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  __shared__ f32x4 red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (sl != 0 || e4 >= total4) return;
  for (int l = 1; l < SL; ++l) s += red[l * CW + col];
  if (!stem) {
    *reinterpret_cast<f32x4*>(dw + e4 * 4) = s;
  } else {
    const size_t e = e4 * 4;
    const int m = (int)(e / N), c = (int)(e - (size_t)m * N);
    const int r = c >> 5, sp = (c & 31) >> 2;  // 4 consecutive cols = channels 0..3 of one (r, s)
    if (r < 7 && sp < 7) {
      float* o = dw + (size_t)m * 147 + (r * 7 + sp) * 3;
      o[0] = s.x; o[1] = s.y; o[2] = s.z;
    }
  }
}

// float4 columns per block: aim for >= 512 blocks, more split lanes when few columns
static int reduce_cw(int M, int N) {
  const size_t total4 = (size_t)M * N / 4;
  int cw = 64;
  while (cw > 4 && (total4 + cw - 1) / cw < 512) cw >>= 1;
  return cw;
}

// split lanes per float4 column (the summation order a folded reduction must repeat: conv_wgdma.hip)
int wgrad_reduce_lanes(int M, int N) { return 256 / reduce_cw(M, N); }

int wgrad_reduce_launch(const float* part, int splits, int M, int N, int stem, float* dw, hipStream_t st) {
  const size_t total4 = (size_t)M * N / 4;
  const int cw = reduce_cw(M, N);
  const int blocks = (int)((total4 + cw - 1) / cw);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, part, splits, M, N, stem, cw, dw);
  return check_launch("wgrad_reduce_kernel");
}

}  // namespace argus
