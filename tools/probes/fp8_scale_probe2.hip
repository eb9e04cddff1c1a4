// Probe (dev tool): does lane L's E8M0 scale apply to lane L's own operand bytes? A = B = ones,
// lane L's A (or B) bytes = 2.0 and lane L's scale = 0.5 (126): D stays 128 iff it does. For a
// mismatch, also searches the lane M whose scale = 0.5 cancels lane L's doubled bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void mm(int which, int L, int M, float* D) {
  const int l = threadIdx.x;
  const unsigned one4 = 0x38383838u, two4 = 0x40404040u;  // e4m3 1.0, 2.0
  const unsigned wa = (which == 0 && l == L) ? two4 : one4, wb = (which == 1 && l == L) ? two4 : one4;
  v8i a = {(int)wa, (int)wa, (int)wa, (int)wa, (int)wa, (int)wa, (int)wa, (int)wa};
  v8i b = {(int)wb, (int)wb, (int)wb, (int)wb, (int)wb, (int)wb, (int)wb, (int)wb};
  const int sa = (which == 0 && l == M) ? 126 : 127, sb = (which == 1 && l == M) ? 126 : 127;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, sa, 0, sb);
  for (int r = 0; r < 4; ++r) D[(4 * (l / 16) + r) * 16 + l % 16] = acc[r];
}

int main() {
  float* dD;
  float D[256];
  (void)hipMalloc(&dD, sizeof D);
  for (int which = 0; which < 2; ++which) {
    int own = 0;
    for (int L = 0; L < 64; ++L) {
      int found = -1;
      for (int M = 0; M < 64 && found < 0; ++M) {
        const int MM = (L + M) % 64;  // try the lane itself first
        hipLaunchKernelGGL(mm, dim3(1), dim3(64), 0, 0, which, L, MM, dD);
        (void)hipMemcpy(D, dD, sizeof D, hipMemcpyDeviceToHost);
        bool ok = true;
        for (int i = 0; i < 256; ++i) ok = ok && D[i] == 128.f;
        if (ok) found = MM;
      }
      own += found == L;
      if (found != L) printf("%s data lane %2d cancelled by scale lane %d\n", which ? "B" : "A", L, found);
    }
    printf("%s: %d of 64 lanes' scales apply to their own bytes\n", which ? "B" : "A", own);
  }
  return 0;
}
