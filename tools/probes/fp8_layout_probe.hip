// Probe (dev tool): the k-block (E8M0 scale block) of every A operand byte of
// v_mfma_scale_f32_16x16x128_f8f6f4. A scale of lane M = 2^(M/16) (block b = M/16 of row M%16);
// A = a single 1.0 at (lane L, byte j), B = ones: D[L%16][*] = 2^block(L, j).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void mm(int L, int j, float* D) {
  const int l = threadIdx.x;
  unsigned w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (l == L) w[j / 4] = 0x38u << (8 * (j % 4));
  v8i a = {(int)w[0], (int)w[1], (int)w[2], (int)w[3], (int)w[4], (int)w[5], (int)w[6], (int)w[7]};
  const unsigned one4 = 0x38383838u;
  v8i b = {(int)one4, (int)one4, (int)one4, (int)one4, (int)one4, (int)one4, (int)one4, (int)one4};
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, 127 + l / 16, 0, 127);
  for (int r = 0; r < 4; ++r) D[(4 * (l / 16) + r) * 16 + l % 16] = acc[r];
}

int main() {
  float* dD;
  float D[256];
  (void)hipMalloc(&dD, sizeof D);
  for (int L = 0; L < 64; L += 16) {  // rows behave alike: one lane per lane group
    printf("lane %2d:", L);
    for (int j = 0; j < 32; ++j) {
      hipLaunchKernelGGL(mm, dim3(1), dim3(64), 0, 0, L, j, dD);
      (void)hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
      printf(" %d", (int)std::lround(std::log2(D[(L % 16) * 16])));
    }
    printf("\n");
  }
  return 0;
}
