// Shared device helpers for the argus MI355X (gfx950 / CDNA4) kernels.
//
// Storage types: activations/weights are either fp32 (`float`, the parity path) or bf16
// (`__bf16`, the throughput path). Every reduction, BN statistic, loss and optimizer value is fp32
// (doubles where a reduction crosses many workgroups).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ARGUS_DEV __device__ __forceinline__
#define ARGUS_HOST_DEV __host__ __device__

typedef __bf16 bf16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

namespace argus {

// Loads issued together by the small cross-workgroup reductions (finalize merges, split-K sums): in a
// plain `for (...) s += p[i]` loop the compiler waits for each load (s_waitcnt vmcnt(0)) before
// issuing the next, so a 16-row merge paid 16 memory latencies in series (tools/isa_loopmix.py-style
// ISA check: tests/test_isa.py::test_reductions_batch_their_loads). These loops load a batch of
// kLoadBatch into registers (addresses clamped to a valid element), then accumulate in the same fixed
// order as before with selects (x + 0 = x), not branches: a branch per element lets the compiler sink
// each load into its branch and the waits come back.
#ifndef ARGUS_LOAD_BATCH
#define ARGUS_LOAD_BATCH 8  // (a build with 1 restores one load per trip: the A/B baseline)
#endif
constexpr int kLoadBatch = ARGUS_LOAD_BATCH;

constexpr int kWave = 64;

static inline __host__ __device__ int cdiv(int a, int b) { return (a + b - 1) / b; }

// Division of a non-negative int (< 2^31) by a runtime-constant divisor without the ~40-instruction
// integer division: q = umulhi(n, m) >> s with m = ceil(2^(31+l) / d), l = ceil(log2 d) (the
// round-up method of Granlund & Montgomery, exact for 31-bit numerators); d = 1 passes through.
struct FastDiv {
  int d;
  unsigned m;
  int s;
};
static inline FastDiv make_fastdiv(int d) {
  FastDiv f{d, 0u, 0};
  if (d > 1) {
    int l = 0;
    while ((1LL << l) < d) ++l;
    f.m = (unsigned)(((1ULL << (31 + l)) + (unsigned long long)d - 1) / (unsigned long long)d);
    f.s = l - 1;
  }
  return f;
}
ARGUS_DEV int fdiv(int n, const FastDiv& f) {
  return f.d == 1 ? n : (int)(__umulhi((unsigned)n, f.m) >> f.s);
}

ARGUS_DEV float to_f32(float x) { return x; }
ARGUS_DEV float to_f32(bf16 x) { return (float)x; }
template <typename T> ARGUS_DEV T from_f32(float x);
template <> ARGUS_DEV float from_f32<float>(float x) { return x; }
template <> ARGUS_DEV bf16 from_f32<bf16>(float x) { return (bf16)x; }

// A 16-byte "chunk": 8 bf16 or 4 fp32 elements. All activation and weight traffic moves in chunks.
template <typename T> struct Chunk;
template <> struct Chunk<float> { static constexpr int E = 4; };
template <> struct Chunk<bf16> { static constexpr int E = 8; };

ARGUS_DEV u32x4 ld16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }
ARGUS_DEV void st16(void* p, u32x4 v) { *reinterpret_cast<u32x4*>(p) = v; }
// Non-temporal 16-byte store: conv output tiles (written once, read by a later pass) stream past the
// caches instead of evicting operands. Measured on the write-heavy 1x1 convs (K=64 -> 256 channels):
// 2.4 -> 3.1 TB/s (tools/convbench.py).
ARGUS_DEV void st16_nt(void* p, u32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p)); }

// unpack / pack a chunk to fp32 lanes
ARGUS_DEV void unpack(u32x4 v, float (&f)[4]) {
  f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y);
  f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
}
ARGUS_DEV void unpack(u32x4 v, float (&f)[8]) {
  unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
ARGUS_DEV u32x4 pack(const float (&f)[4]) {
  u32x4 v; v.x = __float_as_uint(f[0]); v.y = __float_as_uint(f[1]);
  v.z = __float_as_uint(f[2]); v.w = __float_as_uint(f[3]); return v;
}
ARGUS_DEV unsigned pack2_bf16(float a, float b) {
  bf16 x = (bf16)a, y = (bf16)b;
  unsigned short ux = __builtin_bit_cast(unsigned short, x), uy = __builtin_bit_cast(unsigned short, y);
  return (unsigned)ux | ((unsigned)uy << 16);
}
ARGUS_DEV u32x4 pack(const float (&f)[8]) {
  u32x4 v; v.x = pack2_bf16(f[0], f[1]); v.y = pack2_bf16(f[2], f[3]);
  v.z = pack2_bf16(f[4], f[5]); v.w = pack2_bf16(f[6], f[7]); return v;
}

typedef int v8i __attribute__((ext_vector_type(8)));
ARGUS_DEV v8i cat8(u32x4 lo, u32x4 hi) {
  return v8i{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

// OCP MX-fp8 quantization of 16 bf16 (two chunks, this thread's half of a 32-element block): the
// block amax (bf16 bit patterns: |x| ordered as unsigned, v_pk_max_u16) is shared with the partner
// lane (lane ^ 1 holds the other half); its E8M0 exponent e is the smallest with amax * 2^-e < 448
// (the e4m3 maximum, so nothing saturates): amax = 2^(E-127) (1 + f/128) gives e = E - 135, + 1 when
// f >= 96. v_cvt_scalef32_pk_fp8_bf16 divides by 2^e and rounds to e4m3 (probed:
// tools/probes/fp8_cvt_probe.hip). Returns e through `e`.
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef short s16x2v __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2v __attribute__((ext_vector_type(2)));
ARGUS_DEV u32x4 mx_fp8_quant(u32x4 lo, u32x4 hi, int& e) {
  const unsigned w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  u16x2v m = __builtin_bit_cast(u16x2v, w[0] & 0x7fff7fffu);
#pragma unroll
  for (int j = 1; j < 8; ++j) m = __builtin_elementwise_max(m, __builtin_bit_cast(u16x2v, w[j] & 0x7fff7fffu));
  unsigned mb = m.x > m.y ? m.x : m.y;
  const unsigned mo = (unsigned)__shfl_xor((int)mb, 1, 64);
  mb = mb > mo ? mb : mo;
  const int E = (int)(mb >> 7), f = (int)(mb & 127u);
  int ex = E == 0 ? 0 : E - 135 + (f >= 96 ? 1 : 0);
  ex = ex < -126 ? -126 : (ex > 127 ? 127 : ex);
  e = ex;
  const float sc = __int_as_float((127 + ex) << 23);
  unsigned o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    s16x2v r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16((s16x2v){0, 0}, __builtin_bit_cast(bf16x2v, w[2 * q]), sc,
                                                          false);
    r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, __builtin_bit_cast(bf16x2v, w[2 * q + 1]), sc, true);
    o[q] = __builtin_bit_cast(unsigned, r);
  }
  return u32x4{o[0], o[1], o[2], o[3]};
}

// The same quantization for 8 bf16 (one chunk; a 32-element block spans the 4 lanes l & ~3 .. l | 3,
// which must all be active): the block amax over the 4 lanes, then 8 e4m3 bytes. Used by the
// elementwise passes that store an MX-fp8 copy of their output (argus_bn_apply_x8 / _bwd_apply_x8):
// the bytes and the exponent equal what mx_fp8_quant gives for the same 32 values.
ARGUS_DEV uint2 mx_fp8_quant8(u32x4 v, int& e) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
  u16x2v m = __builtin_bit_cast(u16x2v, w[0] & 0x7fff7fffu);
#pragma unroll
  for (int j = 1; j < 4; ++j) m = __builtin_elementwise_max(m, __builtin_bit_cast(u16x2v, w[j] & 0x7fff7fffu));
  unsigned mb = m.x > m.y ? m.x : m.y;
  unsigned mo = (unsigned)__shfl_xor((int)mb, 1, 64);
  mb = mb > mo ? mb : mo;
  mo = (unsigned)__shfl_xor((int)mb, 2, 64);
  mb = mb > mo ? mb : mo;
  const int E = (int)(mb >> 7), f = (int)(mb & 127u);
  int ex = E == 0 ? 0 : E - 135 + (f >= 96 ? 1 : 0);
  ex = ex < -126 ? -126 : (ex > 127 ? 127 : ex);
  e = ex;
  const float sc = __int_as_float((127 + ex) << 23);
  unsigned o[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    s16x2v r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16((s16x2v){0, 0}, __builtin_bit_cast(bf16x2v, w[2 * q]), sc,
                                                          false);
    r = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(r, __builtin_bit_cast(bf16x2v, w[2 * q + 1]), sc, true);
    o[q] = __builtin_bit_cast(unsigned, r);
  }
  return uint2{o[0], o[1]};
}

// ReLU mask of a stored chunk: bit j set <=> element j > 0 (one byte per 16-byte chunk).
template <typename T>
ARGUS_DEV uint8_t chunk_positive_bits(u32x4 v) {
  float f[Chunk<T>::E];
  unpack(v, f);
  unsigned b = 0;
#pragma unroll
  for (int j = 0; j < Chunk<T>::E; ++j) b |= (f[j] > 0.f ? 1u : 0u) << j;
  return (uint8_t)b;
}

// wave-level sum (64 lanes)
ARGUS_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
ARGUS_DEV double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware remap of a 1-D block id (MI355X: 8 XCDs, blocks dealt round-robin).
// Consecutive remapped ids land on the same XCD so neighbouring tiles share that XCD's L2.
ARGUS_DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

// Flattened split-K grid (1-D, nwg * splits workgroups): work item w = split * nwg + tile, remapped so
// that consecutive w share an XCD. All output tiles of one pixel split then run on one XCD and share
// its L2 copy of that split's dy / x rows (the split's operands are re-read by every tile).
// With group == false the split index is the slow dimension of the dispatch order instead (a split's
// tiles spread over the XCDs) — measured faster for the 3x3 filters, whose 18+ tiles per split
// contend for the same dy lines when they share one L2.
ARGUS_DEV void split_tile(int nwg, int splits, bool group, int& tile, int& split) {
  if (group) {
    const int w = xcd_remap(blockIdx.x, nwg * splits);
    split = w / nwg;
    tile = w - split * nwg;
  } else {
    split = blockIdx.x / nwg;
    tile = xcd_remap(blockIdx.x - split * nwg, nwg);
  }
}

}  // namespace argus
