// Optimizer step over the flat fp32 parameter / gradient buffers: torch.nn.utils.clip_grad_norm_
// (max_norm 1.0, argus/train.py:318) + torch.optim.Adam (lr 1e-4, betas (0.9, 0.999), eps 1e-8,
// argus/train.py:232,319). One deterministic two-level norm reduction, then one fused
// clip-scale + Adam pass (reads g, p, m, v; writes p, m, v: 28 B per parameter — HBM-bound).
#include "common.h"
#include "internal.h"

namespace argus {

constexpr int kNormBlocks = 1024;

__global__ __launch_bounds__(256) void sumsq_kernel(int64_t n, const float* __restrict__ x, double* __restrict__ part) {
  double s = 0.0;
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + i * 4);
    s += (double)(v.x * v.x + v.y * v.y) + (double)(v.z * v.z + v.w * v.w);
  }
  for (int64_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    s += (double)x[i] * x[i];
  s = wave_sum(s);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void norm_finalize_kernel(int nparts, const double* __restrict__ part,
                                                            float* __restrict__ out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  s = wave_sum(s);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (float)sqrt(red[0] + red[1] + red[2] + red[3]);
}

__global__ __launch_bounds__(256) void adam_kernel(int64_t n, float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   const float* __restrict__ norm, float gscale, float max_norm, float lr,
                                                   float b1, float b2, float eps, float wd, float bc1, float bc2) {
  // g' = gscale * g (e.g. 1/world after a SUM all-reduce), then clip_grad_norm_ on g'
  float coef = gscale;
  if (norm) coef = gscale * fminf(1.f, max_norm / (norm[0] * gscale + 1e-6f));
  const float step = lr / bc1;
  const float bc2s = sqrtf(bc2);
  const int64_t n4 = n / 4;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f32x4 gp = *reinterpret_cast<const f32x4*>(g + i * 4);
    f32x4 pp = *reinterpret_cast<const f32x4*>(p + i * 4);
    f32x4 mm = *reinterpret_cast<const f32x4*>(m + i * 4);
    f32x4 vv = *reinterpret_cast<const f32x4*>(v + i * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = gp[j] * coef;
      if (wd != 0.f) gj += wd * pp[j];
      mm[j] = mm[j] + (1.f - b1) * (gj - mm[j]);  // torch: m.lerp_(g, 1-beta1)
      vv[j] = vv[j] * b2 + (1.f - b2) * gj * gj;
      const float denom = sqrtf(vv[j]) / bc2s + eps;
      pp[j] = pp[j] - step * (mm[j] / denom);
    }
    *reinterpret_cast<f32x4*>(p + i * 4) = pp;
    *reinterpret_cast<f32x4*>(m + i * 4) = mm;
    *reinterpret_cast<f32x4*>(v + i * 4) = vv;
  }
  for (int64_t i = n4 * 4 + blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float gj = g[i] * coef;
    if (wd != 0.f) gj += wd * p[i];
    m[i] = m[i] + (1.f - b1) * (gj - m[i]);
    v[i] = v[i] * b2 + (1.f - b2) * gj * gj;
    p[i] = p[i] - step * (m[i] / (sqrtf(v[i]) / bc2s + eps));
  }
}

}  // namespace argus

using namespace argus;

extern "C" {

size_t argus_sumsq_workspace_bytes(int64_t) { return kNormBlocks * sizeof(double); }

int argus_global_norm(int64_t count, const float* x, float* out, void* ws, argus_stream_t stream) {
  if (count <= 0 || !x || !out || !ws) { set_error("global_norm: bad arguments"); return ARGUS_ERR_ARG; }
  if (((uintptr_t)x) & 15) { set_error("global_norm: x must be 16-byte aligned"); return ARGUS_ERR_ARG; }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_kernel, dim3(kNormBlocks), dim3(256), 0, st, count, x, (double*)ws);
  if (int e = check_launch("sumsq_kernel")) return e;
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(256), 0, st, kNormBlocks, (const double*)ws, out);
  return check_launch("norm_finalize_kernel");
}

int argus_adam_step(int64_t count, float* p, const float* g, float* m, float* v, const float* norm, float gscale,
                    float max_norm, float lr, float b1, float b2, float eps, float wd, float bc1, float bc2,
                    argus_stream_t stream) {
  if (count <= 0 || !p || !g || !m || !v) { set_error("adam_step: bad arguments"); return ARGUS_ERR_ARG; }
  if ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) {
    set_error("adam_step: buffers must be 16-byte aligned");
    return ARGUS_ERR_ARG;
  }
  const int blocks = (int)std::min<int64_t>((count / 4 + 255) / 256 + 1, 4096);
  hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, count, p, g, m, v, norm, gscale,
                     max_norm, lr, b1, b2, eps, wd, bc1, bc2);
  return check_launch("adam_kernel");
}

}  // extern "C"
