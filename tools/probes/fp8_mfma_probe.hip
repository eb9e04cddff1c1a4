// Probe (dev tool): operand layout and E8M0 scale semantics of v_mfma_scale_f32_16x16x128_f8f6f4
// (fp8 e4m3) and v_cvt_pk_fp8_f32 on gfx950, against a host GEMM. Tries layout hypotheses:
//   H1: lane (row = l%16, g = l/16) byte j <-> k = 32g + j
//   H2: byte j <-> k = 16g + j (j < 16), 64 + 16g + j - 16 (j >= 16)
//   H3: dword i (bytes 4i..4i+3) <-> k = 16i + 4g + (j%4)
//   H4: 8-byte chunk c <-> k = 32c + 8g + (j%8)
//   hipcc --offload-arch=gfx950 -O2 tools/probes/fp8_mfma_probe.hip -o tools/probes/fp8probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ int kmap(int h, int g, int j) {
  switch (h) {
    case 1: return 32 * g + j;
    case 2: return j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16);
    case 3: return 16 * (j / 4) + 4 * g + (j % 4);
    default: return 32 * (j / 8) + 8 * g + (j % 8);
  }
}

__global__ void mm(int h, const float* A, const float* Bt, const unsigned char* sa, const unsigned char* sb, float* D) {
  const int l = threadIdx.x, row = l % 16, g = l / 16;
  unsigned wa[8], wb[8];
  for (int i = 0; i < 8; ++i) {
    float a4[4], b4[4];
    for (int t = 0; t < 4; ++t) {
      a4[t] = A[row * 128 + kmap(h, g, 4 * i + t)];
      b4[t] = Bt[row * 128 + kmap(h, g, 4 * i + t)];
    }
    wa[i] = __builtin_amdgcn_cvt_pk_fp8_f32(a4[2], a4[3], __builtin_amdgcn_cvt_pk_fp8_f32(a4[0], a4[1], 0u, false), true);
    wb[i] = __builtin_amdgcn_cvt_pk_fp8_f32(b4[2], b4[3], __builtin_amdgcn_cvt_pk_fp8_f32(b4[0], b4[1], 0u, false), true);
  }
  v8i a = {(int)wa[0], (int)wa[1], (int)wa[2], (int)wa[3], (int)wa[4], (int)wa[5], (int)wa[6], (int)wa[7]};
  v8i b = {(int)wb[0], (int)wb[1], (int)wb[2], (int)wb[3], (int)wb[4], (int)wb[5], (int)wb[6], (int)wb[7]};
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, (int)sa[l], 0, (int)sb[l]);
  for (int r = 0; r < 4; ++r) D[(4 * (l / 16) + r) * 16 + l % 16] = acc[r];
}

int main() {
  static float A[16 * 128], Bt[16 * 128], D[256], R[256];
  unsigned char sa[64], sb[64];
  srand(1);
  for (int i = 0; i < 16 * 128; ++i) {
    A[i] = (float)((rand() % 17) - 8) / 4.f;
    Bt[i] = (float)((rand() % 9) - 4) / 2.f;
  }
  float *dA, *dB, *dD; unsigned char *dsa, *dsb;
  (void)hipMalloc(&dA, sizeof A); (void)hipMalloc(&dB, sizeof Bt); (void)hipMalloc(&dD, sizeof D);
  (void)hipMalloc(&dsa, 64); (void)hipMalloc(&dsb, 64);
  (void)hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice); (void)hipMemcpy(dB, Bt, sizeof Bt, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 3; ++mode) {  // 0: unit scales; 1: per-lane A scales; 2: per-lane B scales
    for (int l = 0; l < 64; ++l) {
      sa[l] = (unsigned char)(mode == 1 ? 127 + (l % 3) + (l / 16) : 127);
      sb[l] = (unsigned char)(mode == 2 ? 127 + (l % 2) + 2 * (l / 16 == 2) : 127);
    }
    (void)hipMemcpy(dsa, sa, 64, hipMemcpyHostToDevice); (void)hipMemcpy(dsb, sb, 64, hipMemcpyHostToDevice);
    for (int h = 1; h <= 4; ++h) {
      // reference with scale of (row, lane group holding that k under hypothesis h)
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          double s = 0;
          for (int g = 0; g < 4; ++g)
            for (int jj = 0; jj < 32; ++jj) {
              const int k = kmap(h, g, jj);
              s += (double)A[i * 128 + k] * std::ldexp(1.0, sa[g * 16 + i] - 127) * (double)Bt[j * 128 + k] *
                   std::ldexp(1.0, sb[g * 16 + j] - 127);
            }
          R[i * 16 + j] = (float)s;
        }
      hipLaunchKernelGGL(mm, dim3(1), dim3(64), 0, 0, h, dA, dB, dsa, dsb, dD);
      (void)hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
      double maxerr = 0, maxref = 0;
      for (int i = 0; i < 256; ++i) { maxerr = fmax(maxerr, fabs(D[i] - R[i])); maxref = fmax(maxref, fabs(R[i])); }
      printf("scales %d  H%d: max |D - ref| = %g (max |ref| = %g)\n", mode, h, maxerr, maxref);
    }
  }
  return 0;
}
