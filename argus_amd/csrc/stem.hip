// ResNet-50 stem convolution (torchvision conv1: 7x7, stride 2, pad 3, 3 -> 64 channels, bias=False;
// argus/models.py:43) forward, bf16, with the input patch of each output tile staged in LDS once.
//
// Why: the implicit GEMM (conv.hip, STEM variant) gathers its im2col operand from global memory per
// k-step: every input pixel is fetched by ~12 output pixels (49 taps at stride 2), and its K of 256
// = (8 rows x 8 cols x 4 channels) carries a zero filter row. Here a workgroup owns an 8 x 32 output
// tile (256 pixels x 64 channels): it loads the (2*8+5) x (2*32+6) input patch (NHWC4, 8 bytes a
// pixel) and the 64 x 224 filter once, then runs K = 7 filter rows x 32 (8 columns x 4 channels, the
// 8th column's weights are zero) straight from LDS: the A fragment of lane (pixel j, group g) for
// filter row r is the two adjacent input pixels (2j + 2g, 2j + 2g + 1) of patch row 2i + r, one
// 16-byte read.
//
// Epilogue as igemm_kernel's forward: BN statistics {sum, M2} per 128 output pixels (the tile's two
// halves: rows 0-3 and 4-7), the C tile staged through LDS and written as 16-byte non-temporal stores.
// Served: bf16, any output size whose 8 x 32 tiling is >= 75 % useful. Ragged edge tiles (the 376 x 672
// frame's 188 x 336 output: 4 spare rows, 16 spare columns) compute their spare pixels but neither
// store them nor count them: such a half-tile's partial is {sum, M2} over its n valid pixels (M2 about
// their own mean, as a full tile's), and every half-tile also writes its pixel count n to the int32
// row-count array that follows the partials (stat tile -128: argus_bn_finalize merges each row with
// its own n in fp64; ADVICE r4: re-centring M2 to 128 pixels in fp32 lost the within-tile variance
// when |mean| >> std).
//
// The weight gradient (stem_wgrad_kernel) uses the same tile: dW[oc][(r, s, c)] = sum over pixels of
// dy[px][oc] * patch(2i + r, 2j + s)[c]. Both MFMA operands need 8 consecutive PIXELS per lane, which
// ds_read_b64_tr_b16 provides from pixel-major LDS rows: for dy (rows of 64 channels) and for the
// patch, where the 16 k-columns (s0..s0+3) x 4 channels of filter row r at output pixel (i, j) are
// the 32 contiguous bytes at patch(2i + r, 2j + s0). So the im2col operand is never materialised:
// a workgroup stages dy (staged through the BN-backward apply when fused) and the patch once per
// 256-pixel tile, loops over its run of tiles with the next tile's loads in flight, and writes one
// fp32 64 x 256 partial per split for wgrad_reduce_kernel.
#include "common.h"
#include "bnfin.h"
#include "internal.h"
#include "ktimer.h"

namespace argus {

namespace {
constexpr int kTH = 8, kTW = 32;           // output tile
constexpr int kPR = 2 * kTH + 5;           // patch rows (21)
constexpr int kPC = 2 * kTW + 6;           // patch columns (70): column pc = input column 2*ow0 - 3 + pc
constexpr int kWS = 7 * 32 + 8;            // LDS weight row stride, elements (224 + 8: 464 B, conflict-free)
constexpr int kPatchB = kPR * kPC * 8;     // 11760
constexpr int kWB = 64 * kWS * 2;          // 29696
constexpr int kLD = 64 + 8;                // C staging row stride, elements
constexpr int kLdsB = (kPatchB + kWB) > 256 * kLD * 2 ? (kPatchB + kWB) : 256 * kLD * 2;
}  // namespace

struct StemParams {
  const bf16* x;   // (n, H, W, 4) bf16, channel 3 zero
  const bf16* w;   // w_fwd of the stem: [64][8][8][4] (r, s, c), padding zero
  bf16* y;         // (n, Ho, Wo, 64)
  float2* stats;   // {sum, M2} per 128 output pixels x 64 channels, or null
  int* counts;     // ragged tilings: pixels per partial row (after the partials), else null
  int n, H, W, Ho, Wo;
  BnFwdFin ffin;   // the statistics finalize folded in (argus_conv_fwd_fin; ffin.mode != 0)
};

ARGUS_HOST_DEV inline int stem_tpr(int wo) { return (wo + kTW - 1) / kTW; }
ARGUS_HOST_DEV inline int stem_tpi(int ho, int wo) { return ((ho + kTH - 1) / kTH) * stem_tpr(wo); }

__global__ __launch_bounds__(256, 3) void stem_fwd_kernel(const StemParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsB];
  uint2* patch = reinterpret_cast<uint2*>(lds);
  bf16* wl = reinterpret_cast<bf16*>(lds + kPatchB);

  const int tpr = stem_tpr(p.Wo), tpi = stem_tpi(p.Ho, p.Wo);  // tiles per tile-row, per image
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int img = tile / tpi, rem = tile - img * tpi;
  const int oh0 = (rem / tpr) * kTH, ow0 = (rem % tpr) * kTW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // ---- stage the input patch (zero outside the image) and the 64 x 224 filter ----
  const uint2* X = reinterpret_cast<const uint2*>(p.x) + (size_t)img * p.H * p.W;
  const int ih0 = 2 * oh0 - 3, iw0 = 2 * ow0 - 3;
  uint2 pv[(kPR * kPC + 255) / 256];
#pragma unroll
  for (int i = 0; i < (kPR * kPC + 255) / 256; ++i) {
    const int q = tid + 256 * i;
    const int pr = q / kPC, pc = q - pr * kPC;
    const int ih = ih0 + pr, iw = iw0 + pc;
    const bool ok = q < kPR * kPC && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
    const uint2 v = X[ok ? ih * p.W + iw : 0];
    pv[i] = ok ? v : make_uint2(0u, 0u);
  }
  u32x4 wv[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) {  // 64 rows x 28 chunks of 16 B (filter rows 0..6)
    const int q = tid + 256 * i;
    const int n = q / 28, ch = q - n * 28;
    wv[i] = ld16(p.w + n * 256 + ch * 8);
  }
#pragma unroll
  for (int i = 0; i < (kPR * kPC + 255) / 256; ++i) {
    const int q = tid + 256 * i;
    if (q < kPR * kPC) patch[q] = pv[i];
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int q = tid + 256 * i;
    const int n = q / 28, ch = q - n * 28;
    *reinterpret_cast<u32x4*>(wl + n * kWS + ch * 8) = wv[i];
  }
  __syncthreads();

  // ---- MFMA: wave w owns tile rows 2w, 2w+1 (64 pixels) x 64 channels ----
  const int g = lane >> 4, i16 = lane & 15;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint8_t* pb = lds;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    u32x4 fa[4], fb[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int tr = 2 * wave + (mi >> 1), j = (mi & 1) * 16 + i16;
      fa[mi] = *reinterpret_cast<const u32x4*>(pb + ((2 * tr + r) * kPC + 2 * j + 2 * g) * 8);
    }
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      fb[ni] = *reinterpret_cast<const u32x4*>(wl + (ni * 16 + i16) * kWS + r * 32 + g * 8);
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[mi]),
                                                              __builtin_bit_cast(bf16x8, fb[ni]), acc[mi][ni], 0, 0, 0);
  }
  __syncthreads();  // LDS is reused below

  // ---- BN statistics: {sum, M2} per 64-pixel wave, merged per 128-pixel half (waves 2h, 2h+1) ----
  const size_t tile_lin = (size_t)img * tpi + rem;
  // valid output rows / columns of this tile (ragged edge tiles: fewer than 8 / 32)
  const int vr = min(kTH, p.Ho - oh0), vc = min(kTW, p.Wo - ow0);
  const bool full = vr == kTH && vc == kTW;
  if (p.stats) {
    float2* red = reinterpret_cast<float2*>(lds);  // [4 waves][64]
    // this wave's tile rows 2w, 2w+1: valid pixels, and which of its accumulator rows are valid
    const int nw = (min(max(vr - 2 * wave, 0), 2)) * vc;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      float s = 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = full || (2 * wave + (mi >> 1) < vr && (mi & 1) * 16 + g * 4 + r < vc);
          s += ok ? acc[mi][ni][r] : 0.f;
        }
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const float mean_w = full ? s * (1.f / 64.f) : (nw > 0 ? s / (float)nw : 0.f);
      float q = 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = full || (2 * wave + (mi >> 1) < vr && (mi & 1) * 16 + g * 4 + r < vc);
          const float d = acc[mi][ni][r] - mean_w;
          q = ok ? fmaf(d, d, q) : q;
        }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < 16) red[wave * 64 + ni * 16 + lane] = make_float2(s, q);
    }
    __syncthreads();
    if (tid < 128) {
      const int h = tid >> 6, col = tid & 63;
      const float2 a0 = red[(2 * h) * 64 + col], a1 = red[(2 * h + 1) * 64 + col];
      float2 o;
      if (full) {
        const float d = (a0.x - a1.x) * (1.f / 64.f);
        o = make_float2(a0.x + a1.x, a0.y + a1.y + d * d * 32.f);
      } else {  // Chan's merge over the valid counts; the count goes to the row-count array
        const int na = min(max(vr - 4 * h, 0), 2) * vc, nb = min(max(vr - 4 * h - 2, 0), 2) * vc;
        const int n = na + nb;
        float m2 = a0.y + a1.y;
        if (na > 0 && nb > 0) {
          const float d = a0.x / (float)na - a1.x / (float)nb;
          m2 += d * d * ((float)na * (float)nb / (float)n);
        }
        o = n > 0 ? make_float2(a0.x + a1.x, m2) : make_float2(0.f, 0.f);
      }
      store_part(p.stats + (tile_lin * 2 + h) * 64 + col, o);
      if (p.counts && col == 0) {
        const int n = full ? 128 : (min(max(vr - 4 * h, 0), 4) * vc);
        store_count(p.counts + tile_lin * 2 + h, n);  // write-through (the folded finalize)
      }
    }
    __syncthreads();
    if (p.ffin.mode) {  // the statistics finalize folded in (bnfin.h): two partial rows a tile
      __shared__ int fin_flag;
      bn_fwd_fin_arrive<256, 64>(p.ffin, tile_lin, 0, reinterpret_cast<double2*>(lds), &fin_flag);
      __syncthreads();
    }
  }

  // ---- epilogue: C tile through LDS, 16-byte coalesced non-temporal stores ----
  bf16* Cs = reinterpret_cast<bf16*>(lds);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wave * 64 + mi * 16 + g * 4 + r) * kLD + ni * 16 + i16] = (bf16)acc[mi][ni][r];
  __syncthreads();
  const int c = tid & 7;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int m = (tid >> 3) + 32 * i;  // C row: tile row m / 32, column m % 32
    if ((m >> 5) >= vr || (m & 31) >= vc) continue;  // a ragged tile's spare pixel
    const int oh = oh0 + (m >> 5), ow = ow0 + (m & 31);
    const u32x4 v = *reinterpret_cast<const u32x4*>(Cs + m * kLD + c * 8);
    st16_nt(p.y + (((size_t)img * p.Ho + oh) * p.Wo + ow) * 64 + c * 8, v);
  }
}

// ------------------------------------------------------------------------------------------------
// weight gradient
// ------------------------------------------------------------------------------------------------
namespace {
constexpr int kDyB = 256 * 128;  // dy tile: 256 pixel rows x 64 channels bf16
constexpr int kWgLdsB = kDyB + kPatchB;
constexpr int kPatchPT = (kPR * kPC + 255) / 256;  // patch pixels per thread (6)
// dy row slot swizzle (4 slots of 32 B per 128-B row): the 8 rows one ds_read_b64_tr_b16 half-wave
// touches (q = 0..3 of two 8-row groups) land on 8 distinct (row parity, slot) bank spans
ARGUS_DEV int dswz(int row) { return ((row >> 1) & 1) | (((row >> 3) & 1) << 1); }
}  // namespace

struct StemWgParams {
  const bf16* x;    // (n, H, W, 4)
  const bf16* dm;   // dy, or dm of the fused BN-backward apply: (n, Ho, Wo, 64)
  const bf16* y;    // apply: y (same layout), else null
  const float *ca, *cb, *cc;  // apply: dy = ca*dm + cb*y + cc per channel
  float* part;      // [splits][64][256] fp32 (columns (r, s, c) = r*32 + s*4 + c; s = 7 and r = 7 unused)
  int n, H, W, Ho, Wo, tiles, tps;
};

template <bool AP>
__global__ __launch_bounds__(256, 2) void stem_wgrad_kernel(const StemWgParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWgLdsB];
  uint8_t* dyl = lds;
  uint2* patch = reinterpret_cast<uint2*>(lds + kDyB);

  const int split = blockIdx.x;
  const int t0 = split * p.tps, t1 = min(p.tiles, t0 + p.tps);
  const int tpr = stem_tpr(p.Wo), tpi = stem_tpi(p.Ho, p.Wo);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c8 = tid & 7;  // this thread's 8-channel chunk of every dy row it stages

  float ca[8], cb[8], cc[8];
  if constexpr (AP) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { ca[j] = p.ca[c8 * 8 + j]; cb[j] = p.cb[c8 * 8 + j]; cc[j] = p.cc[c8 * 8 + j]; }
  }

  struct Stage {
    u32x4 d[8], y[AP ? 8 : 1];
    uint2 x[kPatchPT];
    unsigned ok;  // bit i: staged dy row i is a pixel of the image (ragged edge tiles: spare ones are 0)
  } S;
  auto load = [&](int tile) {
    const int img = tile / tpi, rem = tile - img * tpi;
    const int oh0 = (rem / tpr) * kTH, ow0 = (rem % tpr) * kTW;
    S.ok = 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = (tid >> 3) + 32 * i;  // tile pixel: row i of the tile, column tid >> 3
      const bool ok = oh0 + (row >> 5) < p.Ho && ow0 + (row & 31) < p.Wo;
      const size_t off = ok ? (((size_t)img * p.Ho + oh0 + (row >> 5)) * p.Wo + ow0 + (row & 31)) * 64 + c8 * 8 : 0;
      S.d[i] = ld16(p.dm + off);
      if constexpr (AP) S.y[i] = ld16(p.y + off);
      S.ok |= ok ? 1u << i : 0u;
    }
    const uint2* X = reinterpret_cast<const uint2*>(p.x) + (size_t)img * p.H * p.W;
    const int ih0 = 2 * oh0 - 3, iw0 = 2 * ow0 - 3;
#pragma unroll
    for (int i = 0; i < kPatchPT; ++i) {
      const int q = tid + 256 * i;
      const int pr = q / kPC, pc = q - pr * kPC;
      const int ih = ih0 + pr, iw = iw0 + pc;
      const bool ok = q < kPR * kPC && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      const uint2 v = X[ok ? ih * p.W + iw : 0];
      S.x[i] = ok ? v : make_uint2(0u, 0u);
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = (tid >> 3) + 32 * i;
      u32x4 v = S.d[i];
      if constexpr (AP) {  // argus_bn_bwd_apply's formula, fp32, rounded to bf16 (as wgrad_kernel's AP)
        float d[8], yv[8];
        unpack(v, d);
        unpack(S.y[i], yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = fmaf(ca[j], d[j], fmaf(cb[j], yv[j], cc[j]));
        v = pack(d);
      }
      if (!((S.ok >> i) & 1u)) v = u32x4{0u, 0u, 0u, 0u};  // a spare pixel's dy is zero (after the apply)
      *reinterpret_cast<u32x4*>(dyl + row * 128 + (((c8 >> 1) ^ dswz(row)) << 5) + (c8 & 1) * 16) = v;
    }
#pragma unroll
    for (int i = 0; i < kPatchPT; ++i) {
      const int q = tid + 256 * i;
      if (q < kPR * kPC) patch[q] = S.x[i];
    }
  };

  // wave w: output channels 32*(w & 1) .. +31 (two 16-blocks) x k-column blocks 7*(w >> 1) .. +6
  // (block nb: filter row nb >> 1, columns s0 = 4*(nb & 1) .. s0+3, 4 channels each)
  const int wm = wave & 1, wn = wave >> 1;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pq = i16 & 3;
  f32x4 acc[2][7];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto tr_read = [](const uint8_t* a0, const uint8_t* a1) {
    const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(uint32_t)(uintptr_t)a0);
    const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(uint32_t)(uintptr_t)a1);
    const uint2 u0 = __builtin_bit_cast(uint2, t0), u1 = __builtin_bit_cast(uint2, t1);
    return __builtin_bit_cast(bf16x8, u32x4{u0.x, u0.y, u1.x, u1.y});
  };

  if (t0 < t1) load(t0);
  for (int t = t0; t < t1; ++t) {
    store();
    __syncthreads();
    if (t + 1 < t1) load(t + 1);  // in flight while this tile's MFMAs run
#pragma unroll 1
    for (int ks = 0; ks < kTH; ++ks) {  // k-step = one tile row (32 pixels)
      // lane (g, i16) reads pixels j = 8g + 4h + q, h = 0, 1: its operand's 8 k-values (pixels 8g .. 8g+7)
      bf16x8 fa[2], fb[7];
#pragma unroll
      for (int m2 = 0; m2 < 2; ++m2) {
        const int mi = 2 * wm + m2;
        const int r0 = 32 * ks + 8 * g + q, r1 = r0 + 4;
        fa[m2] = tr_read(dyl + r0 * 128 + ((mi ^ dswz(r0)) << 5) + pq * 8,
                         dyl + r1 * 128 + ((mi ^ dswz(r1)) << 5) + pq * 8);
      }
      const uint8_t* pb = lds + kDyB;
#pragma unroll
      for (int t7 = 0; t7 < 7; ++t7) {
        const int nb = 7 * wn + t7, r = nb >> 1, s0 = (nb & 1) * 4;
        const int j0 = 8 * g + q;
        const uint8_t* a0 = pb + ((2 * ks + r) * kPC + 2 * j0 + s0 + pq) * 8;
        fb[t7] = tr_read(a0, a0 + 8 * 8);  // pixel j0 + 4: 8 patch columns further
      }
#pragma unroll
      for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
        for (int t7 = 0; t7 < 7; ++t7)
          acc[m2][t7] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[m2], fb[t7], acc[m2][t7], 0, 0, 0);
    }
    __syncthreads();
  }

  // C[oc = 16*mi + 4g + e][col = 16*nb + i16]
  float* out = p.part + (size_t)split * 64 * 256;
#pragma unroll
  for (int m2 = 0; m2 < 2; ++m2)
#pragma unroll
    for (int t7 = 0; t7 < 7; ++t7)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        out[(16 * (2 * wm + m2) + 4 * g + e) * 256 + 16 * (7 * wn + t7) + i16] = acc[m2][t7][e];
}

// bf16, 64 output channels, and an 8 x 32 tiling of the output that is >= 75 % pixels of the image
static bool stem_shape_ok(const argus_conv_desc& d, int dtype) {
  if (dtype != ARGUS_BF16 || !d.stem || d.k != 64) return false;
  const long tiled = (long)stem_tpi(d.ho, d.wo) * kTH * kTW;
  return 4L * d.ho * d.wo >= 3L * tiled;
}

int stem_stat_rows(const argus_conv_desc& d) { return 2 * d.n * stem_tpi(d.ho, d.wo); }
bool stem_ragged(const argus_conv_desc& d) { return d.ho % kTH != 0 || d.wo % kTW != 0; }

// splits: ~2 workgroups per CU (the LDS of two 43.5 KB tiles), each a run of whole tiles
bool stem_wgrad_plan(const argus_conv_desc& d, int dtype, int* splits, int* tps) {
  if (!stem_shape_ok(d, dtype)) return false;
  const int tiles = d.n * stem_tpi(d.ho, d.wo);
  int t = (tiles + 511) / 512;
  *tps = t;
  *splits = (tiles + t - 1) / t;
  return true;
}

bool stem_wgrad_launch(const argus_conv_desc& d, int dtype, const void* x, const void* dm,
                       const argus_bn_bwd_prologue* ap, void* ws, size_t ws_bytes, int* splits, hipStream_t st) {
  int s, tps;
  if (!stem_wgrad_plan(d, dtype, &s, &tps)) return false;
  if (ws_bytes < (size_t)s * 64 * 256 * sizeof(float)) return false;
  StemWgParams p;
  p.x = reinterpret_cast<const bf16*>(x);
  p.dm = reinterpret_cast<const bf16*>(dm);
  p.y = ap ? reinterpret_cast<const bf16*>(ap->y) : nullptr;
  p.ca = ap ? ap->ca : nullptr; p.cb = ap ? ap->cb : nullptr; p.cc = ap ? ap->cc : nullptr;
  p.part = reinterpret_cast<float*>(ws);
  p.n = d.n; p.H = d.h; p.W = d.w; p.Ho = d.ho; p.Wo = d.wo;
  p.tiles = d.n * stem_tpi(d.ho, d.wo); p.tps = tps;
  if (ap) timed_launch("argus::stem_wgrad_kernel<true>", stem_wgrad_kernel<true>, dim3(s), dim3(256), st, p);
  else timed_launch("argus::stem_wgrad_kernel<false>", stem_wgrad_kernel<false>, dim3(s), dim3(256), st, p);
  *splits = s;
  return true;
}

bool stem_fwd_ok(const argus_conv_desc& d, int dtype) { return stem_shape_ok(d, dtype); }

// The partial-row layout this kernel writes is argus_conv_fwd_stat_rows / _stat_tile: stem_stat_rows
// rows of 128 pixels (-128 when ragged: int32 pixel counts per row follow the float2[rows][64] partials)
bool stem_fwd_launch(const argus_conv_desc& d, int dtype, const void* x, const void* w, void* y, float* stats,
                     hipStream_t st, const BnFwdFin* ffin) {
  if (!stem_fwd_ok(d, dtype)) return false;
  StemParams p;
  p.ffin = BnFwdFin{};
  if (ffin && stats) {  // the folded finalize: two partial rows a tile (argus_conv_fwd_fin)
    p.ffin = *ffin;
    const int T = d.n * stem_tpi(d.ho, d.wo);
    if (bn_fwd_fin_plan(p.ffin, T, 2, stem_stat_rows(d))) {
      p.ffin.tile_rows = stem_ragged(d) ? -128 : 128;
      p.ffin.part = reinterpret_cast<const float2*>(stats);
      g_ffin_folded = 1;
    } else {
      p.ffin.mode = 0;
    }
  }
  p.x = reinterpret_cast<const bf16*>(x);
  p.w = reinterpret_cast<const bf16*>(w);
  p.y = reinterpret_cast<bf16*>(y);
  p.stats = reinterpret_cast<float2*>(stats);
  p.counts = stats && stem_ragged(d) ? reinterpret_cast<int*>(p.stats + (size_t)stem_stat_rows(d) * 64) : nullptr;
  p.n = d.n; p.H = d.h; p.W = d.w; p.Ho = d.ho; p.Wo = d.wo;
  const int grid = d.n * stem_tpi(d.ho, d.wo);
  timed_launch("argus::stem_fwd_kernel", stem_fwd_kernel, dim3(grid), dim3(256), st, p);
  return true;
}

}  // namespace argus
