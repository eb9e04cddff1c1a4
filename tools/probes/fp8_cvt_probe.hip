// Probe (dev tool): semantics of v_cvt_scalef32_pk_fp8_bf16 (is the scale a multiplier or a
// divisor?) and of u16x2 elementwise max (v_pk_max_u16).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__global__ void k(unsigned* o, const unsigned* in, const float* sc) {
  const int l = threadIdx.x;
  bf16x2 v = __builtin_bit_cast(bf16x2, in[l]);
  s16x2 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16((s16x2){0, 0}, v, sc[l], false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, v, sc[l], true);
  o[l] = __builtin_bit_cast(unsigned, r);
  u16x2 a = __builtin_bit_cast(u16x2, in[l]), b = __builtin_bit_cast(u16x2, in[(l + 1) % 4]);
  o[4 + l] = __builtin_bit_cast(unsigned, __builtin_elementwise_max(a, b));
}
int main() {
  // bf16 1.0 = 0x3f80, 3.0 = 0x4040
  unsigned in[4] = {0x40403f80u, 0x40403f80u, 0x40403f80u, 0xc0403f80u};
  float sc[4] = {1.f, 2.f, 0.5f, 0.25f};
  unsigned *dIn, *dO; float* dS; unsigned o[8];
  (void)hipMalloc(&dIn, 16); (void)hipMalloc(&dO, 32); (void)hipMalloc(&dS, 16);
  (void)hipMemcpy(dIn, in, 16, hipMemcpyHostToDevice); (void)hipMemcpy(dS, sc, 16, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(4), 0, 0, dO, dIn, dS);
  (void)hipMemcpy(o, dO, 32, hipMemcpyDeviceToHost);
  for (int i = 0; i < 4; ++i) printf("scale %g: in (1.0, 3.0%s) -> fp8 bytes %08x (1.0=0x38 2.0=0x40 0.5=0x30 3.0=0x44 6.0=0x4c 1.5=0x3c)\n", sc[i], i == 3 ? " neg" : "", o[i]);
  for (int i = 0; i < 4; ++i) printf("pk_max_u16 %08x %08x -> %08x\n", in[i], in[(i + 1) % 4], o[4 + i]);
  return 0;
}
