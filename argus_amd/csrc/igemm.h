// Implicit-GEMM convolution parameters shared by the register-staged kernel (conv.hip) and the
// global->LDS (glds) kernel (conv_glds.hip).
#pragma once
#include "common.h"
#include "bnfin.h"
#include "internal.h"
#include "../../include/argus_hip.h"

namespace argus {

struct IgPhase {
  int M;          // GEMM rows of this phase = images * Hq * Wq
  int Hq, Wq;     // output grid of this phase
  int oh0, ow0;   // output pixel = (qh*osh + oh0, qw*osw + ow0)
  int K;          // ntaps * Cin (0: this phase has no taps -> output = addend or zeros)
  int dh[9], dw[9], boff[9];  // per tap: input offset (input = q*is + d) and B-row element offset
};

// BatchNorm-backward epilogue of a dgrad whose output feeds BN backward (argus_bn_bwd_epilogue):
// store dm = output * relu-mask and emit per-(row tile, channel) {sum dm, sum dm*(y-mean)*invstd}.
struct BnBwdEpi {
  const void* y;
  const float* mean;
  const float* invstd;
  const float* sc;        // mode 2: mask = y*sc+sh > 0
  const float* sh;
  const uint8_t* bits;    // mode 3: argus_bn_apply mask bits of y's block output
  const void* y2;         // optional second branch (mode 3): the downsample BN
  const float* mean2;
  const float* invstd2;
  float2* part;           // [nphase * prow][N]
  float2* part2;
  int mode;               // 0 = off, 2, 3
  int prow;               // partial rows per dgrad phase
  const void* yx;         // kYrecBit: y = conv1x1(yx, yw) recomputed in the epilogue (yk input channels)
  const void* yw;
  int yk;
};

// BN-backward apply folded into the A-operand staging of a dgrad (argus_bn_bwd_prologue): the A
// operand `a` holds dm; the kernel consumes dy = ca*dm + cb*y + cc (per channel of A) and the
// workgroups of column tile 0 also store that dy (center tap, phase 0: each element once) to `out`
// for the weight gradient.
struct BnApplyPro {
  const void* y;
  const float* ca;
  const float* cb;
  const float* cc;
  void* out;
};

// Forward epilogue of the bottleneck tail (argus_conv_fwd_bn_out): out = relu(y*sc + sh + res*rsc + rsh)
// (rsc null: + res) with its ReLU mask bits, from the conv's own output tile (y need not be stored)
struct BnOutEpi {
  const float* sc;
  const float* sh;
  const void* res;
  const float* rsc;
  const float* rsh;
  void* out;
  uint8_t* bits;
};

struct IgParams {
  const void* a;
  const void* b;
  void* c;
  const float* pro_scale;
  const float* pro_shift;
  void* pro_out;  // forward with a prologue: the staged relu(x*scale+shift) stored here (1x1 stride 1)
  float2* stats;
  const void* addend;          // C += addend (same layout as C; may alias C), masked by addend_mask
  const uint8_t* addend_mask;  // one byte per 16-byte chunk, bit j <-> element j (bn_apply mask)
  int N, Cin, lda, H, W, ish, isw, Ho, Wo, osh, osw, ldc, ldb;
  int stem, nphase;
  int stat_tile;  // rows per BN-statistics partial (forward with stats)
  IgPhase ph[4];
  BnBwdEpi bb;    // dgrad only
  BnFin fin;      // BN finalize folded into this launch (fin.mode != 0)
  BnFwdFin ffin;  // forward: the statistics finalize folded into this launch (ffin.mode != 0, argus_conv_fwd_fin)
  BnApplyPro ap;  // dgrad only: the A operand is dm (ap.y != nullptr)
  BnOutEpi oe;    // forward only (kOutBit): the block output from the C tile
  int f8;         // ARGUS_FP8: MX-fp8 operands where the shape allows (host dispatch only)
  int fwd;        // host: forward params (1) or data gradient (0) - the fp8 pass policy (key 37)
  int ksz;        // host: filter size of the conv (1 or 3; the fp8 pass policy)
  int epi_pre;    // halo dgrad: prefetch the BN-backward epilogue operands under the last chunk
  int x8;         // A and B stored as MX-fp8 (e4m3 rows + E8M0 scales): the F8 halo kernel (conv_halo.hip)
  const Policy* pol;  // host only (kernel selection of this call; never read on the device)
};

// compile-time epilogue/prologue variant of the dgrad kernels: low 3 bits = BN-backward epilogue
// (BwdMode), bit 4 = BN-backward apply prologue (BnApplyPro)
constexpr int kApplyBit = 16;
// bit 5: MX-fp8 operands (OCP e4m3 + one E8M0 scale per 32 K-elements of a row, quantized while
// staging from the bf16 tensors; v_mfma_scale_f32_16x16x128_f8f6f4)
constexpr int kFp8Bit = 32;
// bit 6: forward epilogue BnOutEpi (the bottleneck's bn3 + residual + ReLU applied to the C tile)
constexpr int kOutBit = 64;
// bit 7: the BN-backward epilogue's y recomputed from its producing 1x1 conv (BnBwdEpi::yx / yw)
constexpr int kYrecBit = 128;

struct WgParams {
  const void* x;
  const void* dy;
  const float* pro_scale;
  const float* pro_shift;
  float* part;  // [splits][M][N]
  int M, N, Cin, lda, H, W, Ho, Wo, stride, pad, S;
  int P;
  int pps;  // pixels per split (multiple of the k-step)
  int stem;
  // BN-backward apply prologue (AP kernels): dy holds dm; the A operand is ca*dm + cb*ap_y + cc
  const void* ap_y;
  const float *ap_ca, *ap_cb, *ap_cc;
  FastDiv fd_hw, fd_w;  // Ho*Wo and Wo (pixel -> (image, row, column) without integer division)
  int group;            // split_tile: a split's tiles on one XCD (1x1 filters; 3x3 with tuning key 31)
  // folded split reduction of the LDS-DMA kernel (policy key 50; cnt == nullptr: off): arrival / done
  // counters [2 * tiles + 1] (zero before the launch, zero again after it), dW [M][N], the lane count of
  // wgrad_reduce_kernel's order for this M x N and the reducing workgroups per tile
  struct {
    unsigned* cnt;
    float* dw;
    int sl, rpt;
  } fold;
};

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static ARGUS_DEV void run(f32x4& acc, u32x4 a, u32x4 b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  // lane group g supplies k = 4g + j at sub-step j (same mapping for A and B)
  static ARGUS_DEV void run(f32x4& acc, u32x4 a, u32x4 b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
};

ARGUS_DEV int swz8(int row) { return (row >> 1) & 7; }

// Per-thread state of the BN-backward epilogue: a thread owns one 16-byte channel chunk (fixed
// across the rows it stores), keeps that chunk's coefficients and its column sums in registers.
// BW (compile time, so the plain forward / dgrad kernels keep their register budget): 2 = mask from
// y*scale+shift > 0; 3 = mask bits; 4 = mask bits + the second (downsample) BN branch.
template <int BW> struct BwdMode {
  static constexpr bool ON = BW != 0, RECOMPUTE = BW == 2, DUAL = BW == 4;
};

template <typename T, int BW>
struct BwdEpiAcc {
  static constexpr int E = Chunk<T>::E;
  static constexpr int EM = BwdMode<BW>::RECOMPUTE ? E : 1;  // mask coefficients
  static constexpr int ED = BwdMode<BW>::DUAL ? E : 1;       // second branch
  float s[E], t[E], mu[E], is[E], S[EM], H[EM], t2[ED], mu2[ED], is2[ED];

  ARGUS_DEV static void ld(float* dst, const float* src) {
#pragma unroll
    for (int j = 0; j < E; j += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(src + j);
      dst[j] = v.x; dst[j + 1] = v.y; dst[j + 2] = v.z; dst[j + 3] = v.w;
    }
  }

  ARGUS_DEV void init(const BnBwdEpi& b, int ch) {
    ld(mu, b.mean + ch);
    ld(is, b.invstd + ch);
    if constexpr (BwdMode<BW>::RECOMPUTE) { ld(S, b.sc + ch); ld(H, b.sh + ch); }
    if constexpr (BwdMode<BW>::DUAL) {
      ld(mu2, b.mean2 + ch);
      ld(is2, b.invstd2 + ch);
#pragma unroll
      for (int j = 0; j < E; ++j) t2[j] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < E; ++j) { s[j] = 0.f; t[j] = 0.f; }
  }

  // v = the output chunk as it would be stored (rounded to T); yv / y2v / mb = the BN input chunk(s)
  // and mask byte at the same element offset (loaded by epi_load): returns the masked chunk dm and
  // accumulates the column sums.
  ARGUS_DEV u32x4 step(u32x4 v, u32x4 yraw, u32x4 y2raw, unsigned mb) {
    float d[E], yv[E];
    unpack(v, d);
    unpack(yraw, yv);
    if constexpr (BwdMode<BW>::RECOMPUTE) {
#pragma unroll
      for (int j = 0; j < E; ++j) d[j] = fmaf(yv[j], S[j], H[j]) > 0.f ? d[j] : 0.f;
    } else {
#pragma unroll
      for (int j = 0; j < E; ++j) d[j] = (mb >> j) & 1u ? d[j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < E; ++j) {
      s[j] += d[j];
      t[j] = fmaf(d[j], (yv[j] - mu[j]) * is[j], t[j]);
    }
    if constexpr (BwdMode<BW>::DUAL) {
      float y2v[E];
      unpack(y2raw, y2v);
#pragma unroll
      for (int j = 0; j < E; ++j) t2[j] = fmaf(d[j], (y2v[j] - mu2[j]) * is2[j], t2[j]);
    }
    return pack(d);
  }

  // Fixed-order reduction over the RG row groups of the workgroup (thread = (row group rg, chunk c))
  // through LDS red[E][RG][CPR] (float2; CPR = COLS / E chunks), written as partial row `row` of
  // columns col0..col0+COLS. Element j of every thread's chunk goes to its own [RG][CPR] plane, so the
  // 16 lanes of a ds_write_b64 group (consecutive chunks, one row group) fill 128 contiguous bytes and
  // the summing lanes (consecutive chunks of one element plane) read contiguous slots: no bank
  // conflicts (a [RG][COLS] layout put a wave's lanes 64 bytes apart: 8-way on the writes).
  template <int COLS, int NT>
  ARGUS_DEV void reduce(const BnBwdEpi& b, float2* red, int rg, int RG, int c, size_t row, int N, int col0) {
    constexpr int CPR = COLS / E;
#pragma unroll
    for (int br = 0; br < (BwdMode<BW>::DUAL ? 2 : 1); ++br) {
#pragma unroll
      for (int j = 0; j < E; ++j) {
        float tv = t[j];
        if constexpr (BwdMode<BW>::DUAL) tv = br == 0 ? t[j] : t2[j];
        red[(j * RG + rg) * CPR + c] = make_float2(s[j], tv);
      }
      __syncthreads();
      float2* out = (br == 0 ? b.part : b.part2) + row * N + col0;
      for (int idx = threadIdx.x; idx < COLS; idx += NT) {
        const int cc = idx % CPR, j = idx / CPR;  // column cc * E + j
        const float2* plane = red + j * RG * CPR + cc;
        float2 a = plane[0];
        for (int g = 1; g < RG; ++g) { a.x += plane[g * CPR].x; a.y += plane[g * CPR].y; }
        store_part(out + cc * E + j, a);  // write-through: the folded finalize (bnfin.h) reads it cross-CU
      }
      __syncthreads();
    }
  }
};

// Global operands of one epilogue output chunk (addend, BN-backward inputs). The conv epilogues load
// them for a batch of rows before storing any (epi_load, then epi_apply): the addend may alias the
// output, so loads could not otherwise be hoisted above earlier rows' stores, and one dependent HBM
// round trip per row left the epilogue latency-bound.
struct EpiIn {
  u32x4 add, y, y2;
  unsigned amask, bits;
};

template <typename T, int BW, bool LOADY = true>
ARGUS_DEV void epi_load(const IgParams& p, size_t off, EpiIn& in) {
  constexpr int E = Chunk<T>::E;
  if (p.addend) {
    in.add = ld16(reinterpret_cast<const T*>(p.addend) + off);
    in.amask = p.addend_mask ? p.addend_mask[off / E] : 0xffu;
  }
  if constexpr (BW != 0) {
    if constexpr (LOADY) in.y = ld16(reinterpret_cast<const T*>(p.bb.y) + off);
    if constexpr (!BwdMode<BW>::RECOMPUTE) in.bits = p.bb.bits[off / E];
    if constexpr (BwdMode<BW>::DUAL) in.y2 = ld16(reinterpret_cast<const T*>(p.bb.y2) + off);
  }
}

template <typename T, int BW>
ARGUS_DEV u32x4 epi_apply(const IgParams& p, u32x4 v, const EpiIn& in, BwdEpiAcc<T, BW>& bwd) {
  constexpr int E = Chunk<T>::E;
  if (p.addend) {
    float f[E], o[E];
    unpack(v, f);
    unpack(in.add, o);
#pragma unroll
    for (int j = 0; j < E; ++j) f[j] += (in.amask >> j) & 1u ? o[j] : 0.f;
    v = pack(f);
  }
  if constexpr (BW != 0) v = bwd.step(v, in.y, in.y2, in.bits);
  return v;
}

// host: group plan of a folded BN-backward finalize (one partial row per (phase, row tile))
inline void plan_fin(IgParams& p, int) {
  if (!p.fin.mode) return;
  bn_fin_plan(p.fin, p.nphase * p.bb.prow, 1);
  p.fin.rows = p.fin.T;
}

// host: plan the folded forward statistics finalize (p.ffin) of a producer with BM-row tiles, each
// BM / p.stat_tile partial rows; mode 0 (argus_conv_fwd_fin then launches argus_bn_finalize) where the
// fold's groups cannot repeat argus_bn_finalize's (bnfin.h bn_fwd_fin_plan)
inline void plan_ffin(IgParams& p, int BM) {
  if (!p.ffin.mode) return;
  const int M = p.ph[0].M;
  if (!p.stats || p.nphase != 1 || p.stat_tile <= 0 || BM % p.stat_tile ||
      !bn_fwd_fin_plan(p.ffin, (M + BM - 1) / BM, BM / p.stat_tile, (M + p.stat_tile - 1) / p.stat_tile)) {
    p.ffin.mode = 0;
    return;
  }
  p.ffin.tile_rows = p.stat_tile;
  p.ffin.part = p.stats;
  g_ffin_folded = 1;
}

// host: the epilogue variant of a BnBwdEpi (0 when off)
inline int bwd_variant(const BnBwdEpi& b) { return b.mode == 0 ? 0 : (b.mode == 2 ? 2 : (b.y2 ? 4 : 3)); }

// Partial rows of tiles that do not exist in a smaller dgrad phase (grid sized for the largest):
// workgroup e past the phase's tiles zeroes row (mtiles + e / ntiles), columns of tile e % ntiles.
template <int COLS, int NT>
ARGUS_DEV void bwd_epi_zero_rows(const BnBwdEpi& b, int e, int mtiles, int ntiles, int N) {
  const int mt = mtiles + e / ntiles, nt = e - (e / ntiles) * ntiles;
  if (mt >= b.prow) return;
  const size_t row = (size_t)blockIdx.z * b.prow + mt;
  for (int idx = threadIdx.x; idx < COLS; idx += NT) {
    store_part(b.part + row * N + nt * COLS + idx, make_float2(0.f, 0.f));  // write-through (bnfin.h)
    if (b.y2) store_part(b.part2 + row * N + nt * COLS + idx, make_float2(0.f, 0.f));
  }
}

ARGUS_DEV u32x4 sel(bool ok, u32x4 v) {
  const u32x4 z = {0u, 0u, 0u, 0u};
  return ok ? v : z;
}


// dW = fixed-order sum of the fp32 split partials [splits][M][N] (reduce.hip); the stem's padded
// (r8, s8, c4) columns are scattered to OHWI 7x7x3
int wgrad_reduce_launch(const float* part, int splits, int M, int N, int stem, float* dw, hipStream_t st);

// forward / dgrad launchers of the glds kernel (conv_glds.hip); return false when the shape is not
// served by it (then conv.hip's kernel runs). _ok: the same choice without launching.
bool igemm_glds_ok(const IgParams& p, int maxM, int maxK);
bool igemm_glds_launch(const IgParams& p, int maxM, int maxK, hipStream_t st);
// persistent 1x1 stride-1 dgrad with an apply prologue and a mask-bits BN-backward epilogue (the
// bottleneck conv1 data gradients, conv_p1x1.hip): shape check, BN partial rows, launch
bool p1x1_ok(const argus_conv_desc& d, int dtype);
bool p1x1_fwd_stats_ok(const argus_conv_desc& d, int dtype, int enabled);
int p1x1_fwd_stats_rows(const argus_conv_desc& d);
int p1x1_fwd_stats_tile(const argus_conv_desc& d);
int p1x1_fwd_stats_launch(const argus_conv_desc& d, const void* x, const void* w, float* stats, hipStream_t st,
                          const BnFwdFin* ffin = nullptr);
// conv_wgdma.hip: 1x1 stride-1 bf16 weight gradients (optionally with the BN-backward apply) by LDS-DMA
bool wgrad_dma_ok(const argus_conv_desc& d, int dtype, int bm, int bn, int enabled, bool ap, int gather_key);
// its column-tile width (128 / 256) for the plain (ap false) or the apply form; 0 = not served
int wgrad_dma_width(const argus_conv_desc& d, int dtype, int bm, int bn, int key, bool ap, int gather_key);
void wgrad_dma_launch(const argus_conv_desc& d, const WgParams& p, int key, int gather_key, int splits, int ns,
                      hipStream_t st);
// output tiles of the LDS-DMA weight gradient of d (its folded reduction's counters: 2 per tile + 1)
int wgrad_dma_fold_tiles(const argus_conv_desc& d, int key, int gather_key, bool ap);
// the lane count of wgrad_reduce_kernel's summation order for an M x N dW (reduce.hip)
int wgrad_reduce_lanes(int M, int N);
int p1x1_rows(const argus_conv_desc& d);
int p1x1_launch(const argus_conv_desc& d, const void* dm, const void* wd, void* out, const void* addend,
                const argus_bn_bwd_epilogue* bn, const argus_bn_bwd_prologue* pro, hipStream_t st);
// 3x3 stride-1 forward / dgrad with an LDS-resident halo tile (conv_halo.hip); false = not served.
// _ok returns the column tile it would launch (128 / 64) or 0.
int conv3x3_halo_ok(const IgParams& p);
// workgroup row tiles of the halo fwd/dgrad for these params (BN-backward partial rows of its dgrad)
int conv3x3_halo_tiles(const IgParams& p);
bool conv3x3_halo_launch(const IgParams& p, hipStream_t st);
int conv3x3_halo_x8_ok(const IgParams& p);
// 3x3 stride-1 weight gradient with an LDS-resident halo tile (conv_halo.hip): plan / launch of the
// split partials (fp32 [splits][K][9C]); false = not served
bool wgrad3x3_halo_plan(const argus_conv_desc& d, int dtype, int* splits, int* tiles_per_split);
// stem forward on an LDS input patch (stem.hip): false = shape / dtype not served
bool stem_fwd_ok(const argus_conv_desc& d, int dtype);
// its BN-statistics partial rows, and whether its tiling is ragged (stat tile -128: argus_bn_finalize)
int stem_stat_rows(const argus_conv_desc& d);
bool stem_ragged(const argus_conv_desc& d);
bool stem_fwd_launch(const argus_conv_desc& d, int dtype, const void* x, const void* w, void* y, float* stats,
                     hipStream_t st, const BnFwdFin* ffin = nullptr);
// stem weight gradient on the LDS patch + dy tile (stem.hip): split plan and launch of the fp32
// partials [splits][64][256]; ap = the fused BN-backward apply (dy = ca*dm + cb*y + cc) or null
bool stem_wgrad_plan(const argus_conv_desc& d, int dtype, int* splits, int* tiles_per_split);
bool stem_wgrad_launch(const argus_conv_desc& d, int dtype, const void* x, const void* dm,
                       const argus_bn_bwd_prologue* ap, void* ws, size_t ws_bytes, int* splits, hipStream_t st);
bool wgrad3x3_halo_launch(const argus_conv_desc& d, int dtype, const void* x, const float* sc, const float* sh,
                          const void* dy, void* ws, size_t ws_bytes, int* splits, hipStream_t st);

}  // namespace argus
