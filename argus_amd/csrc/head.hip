// FC / MLP head (nn.Linear + exact-erf GELU): resnet.fc 2048->1024 (argus/models.py:56) and the
// output MLP 2048->128->128->6 (models.py:58-64, GELU at :88). fp32 throughout: these GEMMs are
// < 0.03 GFLOP/sample and latency-bound, so a simple LDS-tiled kernel on the exact
// f32 MFMA (v_mfma_f32_16x16x4_f32) keeps the head at fp32 accuracy in every precision mode.
#include "common.h"
#include "internal.h"

namespace argus {

ARGUS_DEV float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
ARGUS_DEV float gelu_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// 64x64 output tile, 256 threads (4 waves, 2x2, each 32x32 = 2x2 MFMA blocks), K-tile 32. The next
// K-tile's global loads are issued into registers before the current one's MFMAs (one exposed global
// latency per K-tile: these GEMMs have few tiles and are latency-bound, so the split heuristic below
// keeps every slice at <= 4 K-tiles).
ARGUS_DEV void epilogue_store(float v, int m, int n, float* __restrict__ C, int ldc, const float* __restrict__ bias,
                               int epi, float* __restrict__ aux) {
  float* dst = C + (size_t)m * ldc + n;
  switch (epi) {
    case 0: *dst = v; break;
    case 1: *dst = v + bias[n]; break;
    case 2: v += bias[n]; aux[(size_t)m * ldc + n] = v; *dst = gelu_f(v); break;
    case 3: *dst = v * gelu_grad(aux[(size_t)m * ldc + n]); break;
    default: *dst += v; break;
  }
}

constexpr int kGemmKT = 32;

// element e (0..7) of this thread's share of a 64 x 32 operand tile: (row 0..63, k 0..31); `t` = the
// operand is stored [k][row] (k-major: consecutive threads walk rows) instead of [row][k]
ARGUS_DEV void gemm_tile_pos(int tid, int e, int t, int& row, int& kk) {
  const int idx = tid + 256 * e;
  if (t) { kk = idx >> 6; row = idx & 63; } else { row = idx >> 5; kk = idx & 31; }
}

// split-K slice z covers k in [z*kc, min(K, (z+1)*kc)); with splits > 1 the raw partial tile goes to
// ws[z][M][N] and gemm_reduce_kernel applies the epilogue after a fixed-order sum.
__global__ __launch_bounds__(256) void gemm_f32_kernel(int M, int N, int K, const float* __restrict__ A, int lda,
                                                       int ta, const float* __restrict__ B, int ldb, int tb,
                                                       float* __restrict__ C, int ldc, const float* __restrict__ bias,
                                                       int epi, float* __restrict__ aux, int kc,
                                                       float* __restrict__ ws) {
  __shared__ float As[kGemmKT][65];  // [k][m]
  __shared__ float Bs[kGemmKT][65];  // [k][n]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kbeg = blockIdx.z * kc, kend = min(K, kbeg + kc);
  float ra[8], rb[8];
  auto load = [&](int k0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int mm, kk;
      gemm_tile_pos(tid, e, ta, mm, kk);
      const int gm = m0 + mm, gk = k0 + kk;
      ra[e] = (gm < M && gk < kend) ? (ta ? A[(size_t)gk * lda + gm] : A[(size_t)gm * lda + gk]) : 0.f;
      int nn, kb;
      gemm_tile_pos(tid, e, tb ? 0 : 1, nn, kb);
      const int gn = n0 + nn, gk2 = k0 + kb;
      rb[e] = (gn < N && gk2 < kend) ? (tb ? B[(size_t)gn * ldb + gk2] : B[(size_t)gk2 * ldb + gn]) : 0.f;
    }
  };
  if (kbeg < kend) load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += kGemmKT) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      int mm, kk, nn, kb;
      gemm_tile_pos(tid, e, ta, mm, kk);
      gemm_tile_pos(tid, e, tb ? 0 : 1, nn, kb);
      As[kk][mm] = ra[e];
      Bs[kb][nn] = rb[e];
    }
    __syncthreads();
    if (k0 + kGemmKT < kend) load(k0 + kGemmKT);  // in flight during this tile's MFMAs
#pragma unroll
    for (int s = 0; s < kGemmKT / 4; ++s) {
      const int kk = 4 * s + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float a = As[kk][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float b = Bs[kk][wn * 32 + j * 16 + (lane & 15)];
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i][j], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (m >= M || n >= N) continue;
        if (ws) ws[((size_t)blockIdx.z * M + m) * N + n] = acc[i][j][r];
        else epilogue_store(acc[i][j][r], m, n, C, ldc, bias, epi, aux);
      }
    }
}

__global__ __launch_bounds__(256) void gemm_reduce_kernel(int M, int N, int splits, const float* __restrict__ ws,
                                                          float* __restrict__ C, int ldc, const float* __restrict__ bias,
                                                          int epi, float* __restrict__ aux) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)M * N) return;
  float v = 0.f;
  for (int zb = 0; zb < splits; zb += kLoadBatch) {
    float t[kLoadBatch];  // in flight together (common.h kLoadBatch); clamped, masked below
#pragma unroll
    for (int u = 0; u < kLoadBatch; ++u) t[u] = ws[(size_t)min(zb + u, splits - 1) * M * N + e];
#pragma unroll
    for (int u = 0; u < kLoadBatch; ++u) v += zb + u < splits ? t[u] : 0.f;
  }
  const int m = (int)(e / N), n = (int)(e - (int64_t)m * N);
  epilogue_store(v, m, n, C, ldc, bias, epi, aux);
}

__global__ void colsum_kernel(int M, int N, const float* __restrict__ x, int ld, float* __restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int mb = 0; mb < M; mb += kLoadBatch) {
    float t[kLoadBatch];
#pragma unroll
    for (int u = 0; u < kLoadBatch; ++u) t[u] = x[(size_t)min(mb + u, M - 1) * ld + n];
#pragma unroll
    for (int u = 0; u < kLoadBatch; ++u) s += mb + u < M ? t[u] : 0.f;
  }
  out[n] = s;
}

__global__ void gelu_kernel(int64_t n, const float* __restrict__ x, float* __restrict__ y) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) y[i] = gelu_f(x[i]);
}
__global__ void gelu_bwd_kernel(int64_t n, const float* __restrict__ x, const float* __restrict__ dy,
                                float* __restrict__ dx) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    dx[i] = dy[i] * gelu_grad(x[i]);
}

}  // namespace argus

using namespace argus;

extern "C" {

// split-K slices: up to 512 workgroups, each slice >= 128 of K (<= 4 K-tiles once K allows)
static int gemm_splits(int m, int n, int k) {
  const int tiles = ((m + 63) / 64) * ((n + 63) / 64);
  int splits = 1;
  while (tiles * splits < 512 && k / (splits * 2) >= 128) splits *= 2;
  return splits;
}

size_t argus_gemm_f32_workspace_bytes(int m, int n, int k) {
  const int splits = gemm_splits(m, n, k);
  return splits > 1 ? (size_t)splits * m * n * sizeof(float) : 0;
}

int argus_gemm_f32(int m, int n, int k, const float* a, int lda, int ta, const float* b, int ldb, int tb, float* c,
                   int ldc, const float* bias, int epi, float* aux, void* ws, size_t ws_bytes, argus_stream_t stream) {
  if (m <= 0 || n <= 0 || k <= 0 || !a || !b || !c || epi < 0 || epi > 4 || ((epi == 1 || epi == 2) && !bias) ||
      ((epi == 2 || epi == 3) && !aux)) {
    set_error("gemm_f32: bad arguments");
    return ARGUS_ERR_ARG;
  }
  int splits = gemm_splits(m, n, k);
  if (splits > 1 && (!ws || ws_bytes < (size_t)splits * m * n * sizeof(float))) splits = 1;  // no workspace
  const int kc = ((k + splits - 1) / splits + kGemmKT - 1) / kGemmKT * kGemmKT;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((n + 63) / 64, (m + 63) / 64, splits);
  hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(256), 0, st, m, n, k, a, lda, ta, b, ldb, tb, c, ldc, bias, epi, aux,
                     kc, splits > 1 ? (float*)ws : (float*)nullptr);
  if (int e = check_launch("gemm_f32_kernel")) return e;
  if (splits > 1) {
    hipLaunchKernelGGL(gemm_reduce_kernel, dim3((unsigned)(((int64_t)m * n + 255) / 256)), dim3(256), 0, st, m, n,
                       splits, (const float*)ws, c, ldc, bias, epi, aux);
    return check_launch("gemm_reduce_kernel");
  }
  return ARGUS_OK;
}

int argus_colsum_f32(int m, int n, const float* x, int ld, float* out, argus_stream_t stream) {
  hipLaunchKernelGGL(colsum_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, m, n, x, ld, out);
  return check_launch("colsum_kernel");
}

int argus_gelu_f32(int64_t count, const float* x, float* y, argus_stream_t stream) {
  const int blocks = (int)std::min<int64_t>((count + 255) / 256, 4096);
  hipLaunchKernelGGL(gelu_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, count, x, y);
  return check_launch("gelu_kernel");
}

int argus_gelu_bwd_f32(int64_t count, const float* x, const float* dy, float* dx, argus_stream_t stream) {
  const int blocks = (int)std::min<int64_t>((count + 255) / 256, 4096);
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, count, x, dy, dx);
  return check_launch("gelu_bwd_kernel");
}

}  // extern "C"
