// Probe (dev tool): which (row, k range) each lane's E8M0 scale byte of
// v_mfma_scale_f32_16x16x128_f8f6f4 applies to. A = B = all ones (fp8), every scale 1.0 (127)
// except lane L's A (or B) scale = 2.0 (128): D[i][j] - 128 shows the affected rows / columns and
// how many k (= the increase). hipcc --offload-arch=gfx950 -O2 ... -o tools/probes/fp8scale
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void mm(int which, int L, float* D) {
  const int l = threadIdx.x;
  const unsigned one4 = 0x38383838u;  // four e4m3 1.0
  v8i a = {(int)one4, (int)one4, (int)one4, (int)one4, (int)one4, (int)one4, (int)one4, (int)one4};
  const int sa = (which == 0 && l == L) ? 128 : 127, sb = (which == 1 && l == L) ? 128 : 127;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, a, acc, 0, 0, 0, sa, 0, sb);
  for (int r = 0; r < 4; ++r) D[(4 * (l / 16) + r) * 16 + l % 16] = acc[r];
}

int main() {
  float* dD;
  float D[256];
  (void)hipMalloc(&dD, sizeof D);
  for (int which = 0; which < 2; ++which)
    for (int L = 0; L < 64; ++L) {
      hipLaunchKernelGGL(mm, dim3(1), dim3(64), 0, 0, which, L, dD);
      (void)hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
      int nrow = 0, ncol = 0, r0 = -1, c0 = -1;
      float inc = 0;
      bool rows[16] = {}, cols[16] = {};
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j)
          if (D[i * 16 + j] != 128.f) { rows[i] = cols[j] = true; inc = D[i * 16 + j] - 128.f; }
      for (int i = 0; i < 16; ++i) { nrow += rows[i]; ncol += cols[i]; if (rows[i] && r0 < 0) r0 = i; if (cols[i] && c0 < 0) c0 = i; }
      printf("%s lane %2d: rows %d (first %d) cols %d (first %d) +%g\n", which ? "B" : "A", L, nrow, r0, ncol, c0, inc);
    }
  return 0;
}
