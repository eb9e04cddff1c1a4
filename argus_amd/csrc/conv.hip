// Convolution kernels for the ResNet-50 backbone (torchvision Conv2d, bias=False; the 53 convs of
// argus/models.py:43 — SURVEY.md Appendix B), NHWC activations, OHWI weights, MFMA on gfx950.
//
//  igemm_kernel  : implicit GEMM  C[m][n] = sum_k A[m][k] * B[n][k]
//                  forward:  m = output pixel, n = output channel, k = (tap, input channel);
//                            A = im2col(x) gathered on the fly (optionally BN+ReLU applied while
//                            staging), B = w[k][r][s][c]; epilogue stores y and per-tile BN stats.
//                  dgrad:    the same kernel on dy with the transposed weights w_t[c][r][s][k],
//                            one grid.z slice per output phase (ph, pw) of a strided conv so every
//                            tile sees a dense, uniform tap set (no zero-insertion).
//  wgrad_kernel  : dW[k][(r,s,c)] = sum_pixels dy[p][k] * im2col(x)[p][(r,s,c)], split over pixel
//                  ranges; both operands are pixel-major in LDS and are read transposed with
//                  ds_read_b64_tr_b16 (bf16) — fp32 partial slabs, then a deterministic reduce.
//
// Tiles: 256 threads = 4 waves (2 x 2), wave tile (BM/2) x (BN/2) of 16x16 MFMA blocks.
// bf16: v_mfma_f32_16x16x32_bf16, K-step 64; fp32 (parity path): v_mfma_f32_16x16x4_f32, K-step 32.
// LDS rows are 8 x 16-byte chunks, XOR-swizzled (chunk ^ ((row>>1)&7)) so the ds_read_b128
// fragment reads are bank-conflict free. Register-staged double buffering: the global loads of
// k-step t+1 are issued before the MFMAs of step t and written to the other LDS buffer after.
#include "common.h"
#include "internal.h"
#include "ktimer.h"
#include "igemm.h"

namespace argus {

// ------------------------------------------------------------------------------------------------
// implicit GEMM (forward / dgrad)
// ------------------------------------------------------------------------------------------------
template <typename T>
ARGUS_DEV u32x4 bn_relu_chunk(u32x4 v, const float* __restrict__ sc, const float* __restrict__ sh, int ch) {
  constexpr int E = Chunk<T>::E;
  float f[E];
  unpack(v, f);
#pragma unroll
  for (int j = 0; j < E; ++j) f[j] = fmaxf(fmaf(f[j], sc[ch + j], sh[ch + j]), 0.f);
  return pack(f);
}

// Input channels whose BN+ReLU prologue coefficients the implicit GEMM keeps in LDS (staged once per
// workgroup: per-k-step global coefficient loads would wait behind the k-step's operand loads)
constexpr int kProLds = 512;

// Per-thread BN+ReLU coefficients for one 16-byte chunk of channels.
template <typename T> struct ProCoef {
  float s[Chunk<T>::E], h[Chunk<T>::E];
  ARGUS_DEV void load(const float* __restrict__ sc, const float* __restrict__ sh, int ch) {
#pragma unroll
    for (int j = 0; j < Chunk<T>::E; j += 4) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(sc + ch + j);
      const f32x4 b = *reinterpret_cast<const f32x4*>(sh + ch + j);
      s[j] = a.x; s[j + 1] = a.y; s[j + 2] = a.z; s[j + 3] = a.w;
      h[j] = b.x; h[j + 1] = b.y; h[j + 2] = b.z; h[j + 3] = b.w;
    }
  }
  // from the LDS copy [scale 0..kProLds) [shift 0..kProLds) staged at kernel start
  ARGUS_DEV void load_lds(const float* lds_sc, int ch) {
#pragma unroll
    for (int j = 0; j < Chunk<T>::E; j += 4) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(lds_sc + ch + j);
      const f32x4 b = *reinterpret_cast<const f32x4*>(lds_sc + kProLds + ch + j);
      s[j] = a.x; s[j + 1] = a.y; s[j + 2] = a.z; s[j + 3] = a.w;
      h[j] = b.x; h[j + 1] = b.y; h[j + 2] = b.z; h[j + 3] = b.w;
    }
  }
  ARGUS_DEV u32x4 apply(u32x4 v) const {
    constexpr int E = Chunk<T>::E;
    float f[E];
    unpack(v, f);
#pragma unroll
    for (int j = 0; j < E; ++j) f[j] = fmaxf(fmaf(f[j], s[j], h[j]), 0.f);
    return pack(f);
  }
};

// C tile of the implicit GEMM, staged through LDS for 16-byte coalesced global stores.
// Returns the LDS element stride of a staged row.
template <typename T, int BN> constexpr int epi_ld() { return BN + 16 / (int)sizeof(T); }

// OCC = workgroups per CU the kernel is built for: 2 -> double-buffered LDS + 2-deep register
// prefetch ring (deep-K GEMMs); 3 or 4 -> one LDS buffer, no ring, <= 168 / 128 VGPRs (K <= 2
// k-steps: the 1x1 convs whose time is load/epilogue latency, hidden by more resident workgroups).
template <typename T, int BM, int BN, bool STEM, bool PRO, int OCC, int BWX>
__global__ __launch_bounds__(256, OCC) void igemm_kernel(const IgParams p) {
  constexpr int BW = BWX & 7;                   // BN-backward epilogue variant
  constexpr bool AP = (BWX & kApplyBit) != 0;   // BN-backward apply prologue
  constexpr bool F8 = (BWX & kFp8Bit) != 0;     // MX-fp8 operands (bf16 activations, fp8 weights)
  constexpr bool OUT = (BWX & kOutBit) != 0;    // forward: bn3 + residual + ReLU epilogue (BnOutEpi)
  static_assert(!OUT || (BW == 0 && !AP && !F8 && !STEM && !PRO), "block-output epilogue: plain forward");
  constexpr bool YREC = (BWX & kYrecBit) != 0;  // BN-backward epilogue: y recomputed (BnBwdEpi::yx)
  static_assert(!YREC || ((BW == 3 || BW == 4) && !F8 && !STEM && !PRO && sizeof(T) == 2), "y recompute: bf16 dgrad");
  static_assert(!F8 || (sizeof(T) == 2 && !STEM && !PRO), "fp8: bf16 tensors, no BN+ReLU prologue");
  constexpr int E = Chunk<T>::E;
  constexpr int EF = F8 ? 2 * E : E;  // elements one thread stages per row per k-step
  constexpr int BKE = 8 * EF;  // K elements per k-step (8 chunks of 16 B per LDS row)
  constexpr int MI = BM / 32, NI = BN / 32;
  constexpr int AR = BM / 32, BR = BN / 32;
  // fp8: one LDS buffer, no register ring (the bf16 pair per chunk doubles the staging registers;
  // an LDS double buffer with one staged copy measured slower: fwd+dgrad 7.37 vs 6.62 ms)
  constexpr int NBUF = (OCC >= 3 || F8) ? 1 : 2;
  __shared__ uint8_t lds_sc[1][F8 ? BM + BN : 1][4];  // fp8: E8M0 scale of (row, 32-element block)
  constexpr int HALF_C = (BM / 2) * (BN + 16 / (int)sizeof(T)) * (int)sizeof(T);  // epilogue pass of BM/2 rows
  constexpr int RED_B = (256 / (BN * (int)sizeof(T) / 16)) * BN * 8;            // BN-backward column sums
  // y recompute: the full C tile and the recomputed y tile side by side (BM x (BN + 8) bf16 each)
  constexpr int YREC_B = YREC ? 2 * BM * (BN + 8) * 2 : 0;
  constexpr int LDS0 = NBUF * (BM + BN) * 128 > HALF_C ? NBUF * (BM + BN) * 128 : HALF_C;
  constexpr int LDS1 = LDS0 > RED_B ? LDS0 : RED_B;
  constexpr int LDS_BYTES = LDS1 > YREC_B ? LDS1 : YREC_B;
  __shared__ __attribute__((aligned(16))) u32x4 lds[LDS_BYTES / 16];
  __shared__ __attribute__((aligned(16))) float pro_lds[(PRO && !STEM) ? 2 * kProLds : 4];

  const IgPhase& ph = p.ph[blockIdx.z];
  const int mtiles = (ph.M + BM - 1) / BM;
  const int ntiles = p.N / BN;
  const int nwg = mtiles * ntiles;
  __shared__ int fin_flag;
  if ((int)blockIdx.x >= nwg) {
    if constexpr (BW != 0) {
      const int e = blockIdx.x - nwg;
      bwd_epi_zero_rows<BN, 256>(p.bb, e, mtiles, ntiles, p.N);
      if (p.fin.mode && mtiles + e / ntiles < p.bb.prow)
        bn_fin_arrive<256, BN>(p.fin, blockIdx.z * p.bb.prow + mtiles + e / ntiles, e % ntiles,
                               reinterpret_cast<double2*>(lds), &fin_flag);
    }
    return;
  }
  if (ph.K == 0 && p.addend == p.c && !p.addend_mask && BW == 0) return;  // in-place += 0
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int cidx = tid & 7;
  const bool pro_in_lds = (PRO && !STEM) && p.Cin <= kProLds;
  if constexpr (PRO && !STEM) {
    if (pro_in_lds) {
      for (int c = tid; c < p.Cin; c += 256) {
        pro_lds[c] = p.pro_scale[c];
        pro_lds[kProLds + c] = p.pro_shift[c];
      }
      __syncthreads();
    }
  }
  const T* __restrict__ A = reinterpret_cast<const T*>(p.a);
  const T* __restrict__ B = reinterpret_cast<const T*>(p.b);

  // per-thread A rows (output pixels) and B rows (output channels); element offsets fit int32
  // (checked on the host)
  int a_off[AR], a_ih[AR], a_iw[AR];
  bool a_ok[AR];
  const int HWq = ph.Hq * ph.Wq;
  // 1x1 / stride-1 GEMM (one tap at offset 0, input grid = GEMM row grid): input pixel = GEMM row, so
  // no (image, row, column) split is needed (its integer divisions made the small-K 1x1 convs
  // VALU-bound: SQ_INSTS_VALU 9-20x SQ_INSTS_MFMA)
  const bool a_ident = !STEM && ph.K == p.Cin && ph.dh[0] == 0 && ph.dw[0] == 0 && p.ish == 1 && p.isw == 1 &&
                       ph.Hq == p.H && ph.Wq == p.W;
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = mt * BM + (tid >> 3) + 32 * i;
    a_ok[i] = m < ph.M;
    const int mm = a_ok[i] ? m : 0;
    if (a_ident) {
      a_ih[i] = 0;
      a_iw[i] = 0;
      a_off[i] = mm * p.lda;
    } else {
      const int nimg = mm / HWq, rem = mm - nimg * HWq;
      const int qh = rem / ph.Wq, qw = rem - qh * ph.Wq;
      a_ih[i] = qh * p.ish;
      a_iw[i] = qw * p.isw;
      a_off[i] = ((nimg * p.H + a_ih[i]) * p.W + a_iw[i]) * p.lda;
    }
  }
  const T* b_row[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i)
    b_row[i] = B + (size_t)(nt * BN + (tid >> 3) + 32 * i) * p.ldb + cidx * EF;
  // fp8: B is the pre-quantized weight copy (argus_conv_weight_prep, ARGUS_FP8): e4m3 rows of ldb bytes,
  // then the E8M0 scales [N][ldb / 32]
  const uint8_t* b8_row[F8 ? BR : 1];
  const uint8_t* b8_sc[F8 ? BR : 1];
  if constexpr (F8) {
    const uint8_t* B8 = reinterpret_cast<const uint8_t*>(p.b);
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const size_t row = (size_t)(nt * BN + (tid >> 3) + 32 * i);
      b8_row[i] = B8 + row * p.ldb + cidx * 16;
      b8_sc[i] = B8 + (size_t)p.N * p.ldb + row * (p.ldb / 32) + (cidx >> 1);
    }
  }

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one k-step of staged operands (two named copies form the 2-deep prefetch ring)
  struct Stage {
    u32x4 a[AR], b[BR];
    u32x4 a2[F8 ? AR : 1];  // fp8: the second bf16 chunk of the thread's 16 A elements
    uint8_t sb[F8 ? BR : 1];  // fp8: the E8M0 scale of the thread's B block (even cidx)
    u32x4 y[AP ? AR : 1];  // apply prologue: the BN input rows beside the dm rows
    u32x4 y2[(AP && F8) ? AR : 1];
    bool ok[AR];
    int ch, tap0;  // tap0: this k-step is the center tap of phase 0 (the dy store)
  };

  auto load = [&](int kt, Stage& S) {
    const int k0 = kt * BKE;
    if constexpr (STEM) {
      // K = (r, s(8), c(4)); a chunk is 2 pixels x 4 channels (bf16) or 1 pixel x 4 channels (fp32)
      const int k = k0 + cidx * E;
      const int r = k >> 5, s0 = (k & 31) >> 2;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int ih = a_ih[i] + r - 3;
        const bool rok = a_ok[i] && (unsigned)ih < (unsigned)p.H;
        const int rowoff = a_off[i] + ((r - 3) * p.W + s0 - 3) * 4;
        if constexpr (E == 8) {
          const int iw0 = a_iw[i] + s0 - 3, iw1 = iw0 + 1;
          const bool ok0 = rok && (unsigned)iw0 < (unsigned)p.W, ok1 = rok && (unsigned)iw1 < (unsigned)p.W;
          const uint2 v0 = *reinterpret_cast<const uint2*>(A + (ok0 ? rowoff : 0));
          const uint2 v1 = *reinterpret_cast<const uint2*>(A + (ok1 ? rowoff + 4 : 0));
          S.a[i] = u32x4{ok0 ? v0.x : 0u, ok0 ? v0.y : 0u, ok1 ? v1.x : 0u, ok1 ? v1.y : 0u};
        } else {
          const int iw = a_iw[i] + s0 - 3;
          const bool ok = rok && (unsigned)iw < (unsigned)p.W;
          S.a[i] = sel(ok, ld16(A + (ok ? rowoff : 0)));
        }
      }
#pragma unroll
      for (int i = 0; i < BR; ++i) S.b[i] = ld16(b_row[i] + k0);
    } else {
      const int t = k0 / p.Cin;
      const int ci0 = k0 - t * p.Cin;
      const int dh = ph.dh[t], dw = ph.dw[t], boff = ph.boff[t];
      const int ch = ci0 + cidx * EF;
      const int tap = (dh * p.W + dw) * p.lda + ch;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int ih = a_ih[i] + dh, iw = a_iw[i] + dw;
        const bool ok = a_ok[i] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        S.a[i] = ld16(A + (ok ? a_off[i] + tap : ch));
        if constexpr (F8) S.a2[i] = ld16(A + (ok ? a_off[i] + tap + E : ch));
        if constexpr (AP) S.y[i] = ld16(reinterpret_cast<const T*>(p.ap.y) + (ok ? a_off[i] + tap : ch));
        if constexpr (AP && F8) S.y2[i] = ld16(reinterpret_cast<const T*>(p.ap.y) + (ok ? a_off[i] + tap + E : ch));
        S.ok[i] = ok;  // rows outside the image are zeroed in store(): load() only issues loads
      }
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        if constexpr (F8) {
          S.b[i] = ld16(b8_row[i] + boff + ci0);
          if ((cidx & 1) == 0) S.sb[i] = b8_sc[i][(boff + ci0) / 32];
        } else {
          S.b[i] = ld16(b_row[i] + boff + ci0);
        }
      }
      S.ch = ch;
      if constexpr (AP || PRO) S.tap0 = dh == 0 && dw == 0 && blockIdx.z == 0 && nt == 0;
    }
  };

  auto store = [&](int buf, Stage& S) {
    u32x4* L = lds + buf * (BM + BN) * 8;
    if constexpr (!PRO && !AP && !STEM) {
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        S.a[i] = sel(S.ok[i], S.a[i]);
        if constexpr (F8) S.a2[i] = sel(S.ok[i], S.a2[i]);
      }
    }
    if constexpr (PRO && !STEM) {
      ProCoef<T> pc;
      if (pro_in_lds) pc.load_lds(pro_lds, S.ch);
      else pc.load(p.pro_scale, p.pro_shift, S.ch);
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        S.a[i] = sel(S.ok[i], pc.apply(S.a[i]));
        // the applied input stored once (column tile 0; 1x1 stride-1 convs only: argus_conv_fwd_apply_out)
        if (p.pro_out && S.tap0 && S.ok[i]) st16(reinterpret_cast<T*>(p.pro_out) + a_off[i] + S.ch, S.a[i]);
      }
    }
    if constexpr (AP) {  // dy = ca*dm + cb*y + cc; zero outside the image (dgrad's zero padding of dy)
#pragma unroll
      for (int h = 0; h < (F8 ? 2 : 1); ++h) {  // fp8: the thread's two chunks
        float ca[E], cb[E], cc[E];
        BwdEpiAcc<T, 3>::ld(ca, p.ap.ca + S.ch + h * E);
        BwdEpiAcc<T, 3>::ld(cb, p.ap.cb + S.ch + h * E);
        BwdEpiAcc<T, 3>::ld(cc, p.ap.cc + S.ch + h * E);
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          u32x4& av = h == 0 ? S.a[i] : S.a2[F8 ? i : 0];
          float d[E], yv[E];
          unpack(av, d);
          unpack(h == 0 ? S.y[i] : S.y2[(AP && F8) ? i : 0], yv);
#pragma unroll
          for (int j = 0; j < E; ++j) d[j] = fmaf(ca[j], d[j], fmaf(cb[j], yv[j], cc[j]));
          av = sel(S.ok[i], pack(d));
          if (p.ap.out && S.tap0 && S.ok[i]) st16(reinterpret_cast<T*>(p.ap.out) + a_off[i] + S.ch + h * E, av);
        }
      }
    }
    if constexpr (F8) {  // A: 16 bf16 -> 16 e4m3 with the 32-element block scale shared with lane ^ 1
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int row = (tid >> 3) + 32 * i;
        int e;
        L[row * 8 + (cidx ^ swz8(row))] = mx_fp8_quant(S.a[i], S.a2[i], e);
        if ((cidx & 1) == 0) lds_sc[buf][row][cidx >> 1] = (uint8_t)(127 + e);
      }
#pragma unroll
      for (int i = 0; i < BR; ++i) {  // B: pre-quantized
        const int row = (tid >> 3) + 32 * i;
        L[BM * 8 + row * 8 + (cidx ^ swz8(row))] = S.b[i];
        if ((cidx & 1) == 0) lds_sc[buf][BM + row][cidx >> 1] = S.sb[i];
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int row = (tid >> 3) + 32 * i;
      L[row * 8 + (cidx ^ swz8(row))] = S.a[i];
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int row = (tid >> 3) + 32 * i;
      L[BM * 8 + row * 8 + (cidx ^ swz8(row))] = S.b[i];
    }
  };

  const int g = lane >> 4, i16 = lane & 15;
  auto compute = [&](int buf) {
    const u32x4* L = lds + buf * (BM + BN) * 8;
    if constexpr (F8) {
      // v_mfma_scale_f32_16x16x128_f8f6f4 operand layout (probed, tools/probes/): lane (row i16,
      // group g) holds K bytes [16g, 16g+16) and [64+16g, 64+16g+16) = LDS chunks g and g+4; the
      // scale operand of lane (i16, g) is the E8M0 scale of (row i16, 32-element block g)
      v8i fb[NI];
      int sb[NI];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int row = wn * (BN / 2) + ni * 16 + i16;
        fb[ni] = cat8(L[BM * 8 + row * 8 + (g ^ swz8(row))], L[BM * 8 + row * 8 + ((g + 4) ^ swz8(row))]);
        sb[ni] = lds_sc[buf][BM + row][g];
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int row = wm * (BM / 2) + mi * 16 + i16;
        const v8i fa = cat8(L[row * 8 + (g ^ swz8(row))], L[row * 8 + ((g + 4) ^ swz8(row))]);
        const int sa = lds_sc[buf][row][g];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa, fb[ni], acc[mi][ni], 0, 0, 0, sa, 0,
                                                                          sb[ni]);
      }
      return;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      u32x4 fa[MI], fb[NI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int row = wm * (BM / 2) + mi * 16 + i16;
        fa[mi] = L[row * 8 + ((4 * s2 + g) ^ swz8(row))];
      }
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int row = wn * (BN / 2) + ni * 16 + i16;
        fb[ni] = L[BM * 8 + row * 8 + ((4 * s2 + g) ^ swz8(row))];
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) Mma<T>::run(acc[mi][ni], fa[mi], fb[ni]);
    }
  };

  // Main loop: LDS double buffer + 2-deep register prefetch ring (S0/S1). At the MFMAs of step kt,
  // the global loads of steps kt+1 and kt+2 are in flight.
  const int nk = ph.K / BKE;
  // one LDS buffer: the next k-step's loads are issued into the same staging registers once this step's
  // are in LDS, and land under its MFMAs - except for the apply-prologue variants built for 4 workgroups
  // per CU, where the live staging registers (dm and y rows) across the MFMAs would spill
  constexpr bool PREF = !(AP && OCC >= 4);
  if constexpr (NBUF == 1 && PREF) {
    Stage S0;
    if (nk > 0) load(0, S0);
    for (int kt = 0; kt < nk; ++kt) {
      store(0, S0);
      __syncthreads();
      if (kt + 1 < nk) load(kt + 1, S0);
      compute(0);
      __syncthreads();
    }
  } else if constexpr (NBUF == 1) {
    for (int kt = 0; kt < nk; ++kt) {
      Stage S0;
      load(kt, S0);
      store(0, S0);
      __syncthreads();
      compute(0);
      __syncthreads();
    }
  } else if (nk > 0) {
    Stage S0, S1;
    load(0, S0);
    store(0, S0);
    if (nk > 1) load(1, S1);
    if (nk > 2) load(2, S0);
    __syncthreads();
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      compute(0);
      store(1, S1);
      if (kt + 3 < nk) load(kt + 3, S1);
      __syncthreads();
      compute(1);
      if (kt + 2 < nk) {
        store(0, S0);
        if (kt + 4 < nk) load(kt + 4, S0);
      }
      __syncthreads();
    }
    if (kt < nk) {
      compute(0);
      __syncthreads();
    }
  }

  // ---- BN statistics of this tile: {sum, M2} per column (fp32 accumulators) ----
  if (p.stats) {
    float2* red = reinterpret_cast<float2*>(lds);  // [2][BN]
    int nvalid_w = ph.M - (mt * BM + wm * (BM / 2));
    nvalid_w = nvalid_w < 0 ? 0 : (nvalid_w > BM / 2 ? BM / 2 : nvalid_w);
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      float s = 0.f;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool ok = mi * 16 + g * 4 + r < nvalid_w;
          s += ok ? acc[mi][ni][r] : 0.f;
        }
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const float mean_w = nvalid_w > 0 ? s / (float)nvalid_w : 0.f;
      float q = 0.f;
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = acc[mi][ni][r] - mean_w;
          q = mi * 16 + g * 4 + r < nvalid_w ? fmaf(d, d, q) : q;
        }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < 16) red[wm * BN + wn * (BN / 2) + ni * 16 + lane] = make_float2(s, q);
    }
    __syncthreads();
    if (tid < BN) {
      int na = ph.M - mt * BM;
      na = na < 0 ? 0 : (na > BM / 2 ? BM / 2 : na);
      int nb = ph.M - (mt * BM + BM / 2);
      nb = nb < 0 ? 0 : (nb > BM / 2 ? BM / 2 : nb);
      const float2 a0 = red[tid], a1 = red[BN + tid];
      float m2 = a0.y + a1.y;
      if (na > 0 && nb > 0) {
        const float d = a0.x / (float)na - a1.x / (float)nb;
        m2 += d * d * ((float)na * (float)nb / (float)(na + nb));
      }
      store_part(p.stats + (size_t)mt * p.N + nt * BN + tid, make_float2(a0.x + a1.x, m2));
    }
    __syncthreads();
    if (p.ffin.mode) {  // the statistics finalize folded in (bnfin.h): one partial row per row tile
      bn_fwd_fin_arrive<256, BN>(p.ffin, mt, nt, reinterpret_cast<double2*>(lds), &fin_flag);
      __syncthreads();
    }
  }
  if constexpr (BW == 0 && !OUT) {
    if (!p.c) return;  // statistics-only forward (argus_conv_fwd with y == NULL)
  }

  // ---- epilogue: stage the C tile in LDS, then 16-byte coalesced (+accumulating) stores ----
  constexpr int LD = epi_ld<T, BN>();
  constexpr int EPASS = (BM * LD * (int)sizeof(T) > LDS_BYTES) ? 2 : 1;
  constexpr int ROWS = BM / EPASS;
  static_assert(ROWS * LD * (int)sizeof(T) <= LDS_BYTES, "epilogue C tile exceeds the LDS array");
  static_assert(!YREC || (EPASS == 1 && 2 * BM * LD * (int)sizeof(T) <= LDS_BYTES), "y recompute: C + y tiles");
  constexpr int CPR = BN * (int)sizeof(T) / 16;  // 16-byte chunks per row
  constexpr int RPP = 256 / CPR;                  // rows per store pass
  T* Cs = reinterpret_cast<T*>(lds);
  T* Ys = Cs + BM * LD;  // YREC: the recomputed y tile
  T* __restrict__ Cg = reinterpret_cast<T*>(p.c);
  // output pixel = GEMM row (forward, stride-1 dgrad): no division per stored row
  const bool c_ident = p.osh == 1 && p.osw == 1 && ph.oh0 == 0 && ph.ow0 == 0 && ph.Hq == p.Ho && ph.Wq == p.Wo;
  if constexpr (YREC) {
    // y = conv1x1(yx, yw) of this tile's rows and columns, accumulated exactly as the forward GEMM does
    // (k-steps of 64 in order, two 32-k MFMAs each, operands as the forward's LDS fragments), so the
    // bf16-rounded result equals the y the forward would have stored, bit for bit. Runs while no other
    // epilogue state is live (acc is still held; one B fragment at a time keeps the register budget).
    const T* __restrict__ X2 = reinterpret_cast<const T*>(p.bb.yx);
    const T* __restrict__ W2 = reinterpret_cast<const T*>(p.bb.yw);
    const int K2 = p.bb.yk;
    int xo[MI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int m = mt * BM + wm * (BM / 2) + mi * 16 + i16;
      const int mm = m < ph.M ? m : 0;
      int px = mm;
      if (!c_ident) {
        const int nimg = mm / HWq, rem = mm - nimg * HWq;
        const int qh = rem / ph.Wq, qw = rem - qh * ph.Wq;
        px = (nimg * p.Ho + qh * p.osh + ph.oh0) * p.Wo + qw * p.osw + ph.ow0;
      }
      xo[mi] = px * K2;
    }
    const T* wrow = W2 + (size_t)(nt * BN + wn * (BN / 2) + i16) * K2;
    f32x4 acc2[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < K2; k0 += 64) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int kk = k0 + (4 * s2 + g) * 8;
        u32x4 fa[MI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) fa[mi] = ld16(X2 + xo[mi] + kk);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const u32x4 fb = ld16(wrow + (size_t)ni * 16 * K2 + kk);
#pragma unroll
          for (int mi = 0; mi < MI; ++mi) Mma<T>::run(acc2[mi][ni], fa[mi], fb);
        }
      }
    }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Ys[(wm * (BM / 2) + mi * 16 + g * 4 + r) * LD + wn * (BN / 2) + ni * 16 + i16] = from_f32<T>(acc2[mi][ni][r]);
  }
  BwdEpiAcc<T, BW> bwd;
  if constexpr (BW != 0) bwd.init(p.bb, nt * BN + (tid % CPR) * E);
  // block-output epilogue: this thread's chunk coefficients (its chunk column is fixed)
  float oa[OUT ? E : 1], ob[OUT ? E : 1], ra[OUT ? E : 1], rb[OUT ? E : 1];
  if constexpr (OUT) {
    const int ch = nt * BN + (tid % CPR) * E;
    BwdEpiAcc<T, 3>::ld(oa, p.oe.sc + ch);
    BwdEpiAcc<T, 3>::ld(ob, p.oe.sh + ch);
    if (p.oe.rsc) {
      BwdEpiAcc<T, 3>::ld(ra, p.oe.rsc + ch);
      BwdEpiAcc<T, 3>::ld(rb, p.oe.rsh + ch);
    } else {
#pragma unroll
      for (int j = 0; j < E; ++j) { ra[j] = 1.f; rb[j] = 0.f; }
    }
  }
#pragma unroll
  for (int q = 0; q < EPASS; ++q) {
    if (EPASS == 1 || wm == q) {
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = (EPASS == 1 ? wm * (BM / 2) : 0) + mi * 16 + g * 4 + r;
            const int col = wn * (BN / 2) + ni * 16 + i16;
            Cs[row * LD + col] = from_f32<T>(acc[mi][ni][r]);
          }
    }
    __syncthreads();
    const int c = tid % CPR;
    constexpr int NIT = ROWS / RPP, U = NIT < 4 ? NIT : 4;
    static_assert(NIT * RPP == ROWS && NIT % U == 0, "epilogue row partition");
#pragma unroll
    for (int i0 = 0; i0 < NIT; i0 += U) {
      size_t off[U];
      bool ok[U];
      EpiIn in[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = tid / CPR + RPP * (i0 + u);
        const int m = mt * BM + q * ROWS + rr;
        ok[u] = m < ph.M;
        const int mm = ok[u] ? m : 0;
        if (c_ident) {
          off[u] = (size_t)mm * p.ldc + nt * BN + c * E;
        } else {
          const int nimg = mm / HWq, rem = mm - nimg * HWq;
          const int qh = rem / ph.Wq, qw = rem - qh * ph.Wq;
          const int oh = qh * p.osh + ph.oh0, ow = qw * p.osw + ph.ow0;
          off[u] = (((size_t)nimg * p.Ho + oh) * p.Wo + ow) * p.ldc + nt * BN + c * E;
        }
        if constexpr (OUT) {
          if (ok[u]) in[u].add = ld16(reinterpret_cast<const T*>(p.oe.res) + off[u]);
        } else if constexpr (YREC) {
          if (ok[u]) {
            epi_load<T, BW, false>(p, off[u], in[u]);
            in[u].y = *reinterpret_cast<const u32x4*>(Ys + rr * LD + c * E);
          }
        } else if (ok[u]) {
          epi_load<T, BW>(p, off[u], in[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        const int rr = tid / CPR + RPP * (i0 + u);
        const u32x4 v = *reinterpret_cast<const u32x4*>(Cs + rr * LD + c * E);
        if constexpr (OUT) {  // argus_bn_apply's arithmetic on the stored (rounded) y, bit for bit
          if (Cg) st16_nt(Cg + off[u], v);
          float f[E], r[E];
          unpack(v, f);
          unpack(in[u].add, r);
#pragma unroll
          for (int j = 0; j < E; ++j) f[j] = fmaxf(fmaf(f[j], oa[j], ob[j]) + fmaf(r[j], ra[j], rb[j]), 0.f);
          const u32x4 o = pack(f);
          st16(reinterpret_cast<T*>(p.oe.out) + off[u], o);
          p.oe.bits[off[u] / E] = chunk_positive_bits<T>(o);
        } else {
          st16_nt(Cg + off[u], epi_apply<T, BW>(p, v, in[u], bwd));
        }
      }
    }
    if (EPASS > 1) __syncthreads();
  }
  if constexpr (BW != 0) {
    __syncthreads();  // the C staging area becomes the reduction buffer
    bwd.template reduce<BN, 256>(p.bb, reinterpret_cast<float2*>(lds), tid / CPR, RPP, tid % CPR,
                                 (size_t)blockIdx.z * p.bb.prow + mt, p.N, nt * BN);
  }
  if constexpr (BW != 0) {
    if (p.fin.mode) {
      __syncthreads();
      bn_fin_arrive<256, BN>(p.fin, blockIdx.z * p.bb.prow + mt, nt, reinterpret_cast<double2*>(lds), &fin_flag);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// weight gradient (split over pixel ranges)
// ------------------------------------------------------------------------------------------------
// bf16 LDS image: rows of 256 B = 8 slots of 32 B; slot XOR swz32(row) makes the 8 rows a
// ds_read_b64_tr_b16 half-wave touches land on 8 distinct slots.
ARGUS_DEV int swz32(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }

// Two workgroups per CU; the 128x128 tile keeps a single staged k-step in registers (the 2-deep ring
// would not fit two waves per SIMD without spilling; with it at one or two waves per SIMD, or as two
// 256-thread sub-pipelines per workgroup, it measured slower: DESIGN.md §5).
// Register budget of the weight gradient: launch bounds for 3 workgroups per CU. Its LDS (64 KB) still
// admits 2 per CU, but the 128x128 apply-staging variant drops from 204 to 142 VGPRs (no spill), so
// the main stream's 1x1 data gradients (128 VGPRs, 25 KB LDS) can share a CU with two of them instead
// of waiting for them to retire: paired bench runs on one box 9068 / 9078 vs 9012 / 9014 img/s (B=64),
// 376x672 and B=256 level (profiles/r04_pairs_lb1_occ3.txt, r04_pairs_occ3.txt).
#ifndef ARGUS_WGRAD_OCC
#define ARGUS_WGRAD_OCC 3
#endif
template <typename T, int BM, int BN, bool STEM, bool PRO, bool FAST, bool AP = false>
__global__ __launch_bounds__(256, ARGUS_WGRAD_OCC) void wgrad_kernel(const WgParams p) {
  constexpr int E = Chunk<T>::E;
  constexpr bool BF = (E == 8);
  constexpr int BKP = BF ? 64 : 32;               // pixels per k-step
  constexpr int CA = BM * (int)sizeof(T) / 16;    // chunks per A row
  constexpr int CB = BN * (int)sizeof(T) / 16;
  constexpr int RSA = BF ? 16 : CA;               // LDS row stride (chunks)
  constexpr int RSB = BF ? 16 : CB;
  constexpr int RPA = 256 / CA, RPB = 256 / CB;   // rows per staging pass
  constexpr int PA = BKP / RPA, PB = BKP / RPB;   // passes
  constexpr int MI = BM / 32, NI = BN / 32;
  __shared__ __attribute__((aligned(16))) u32x4 lds[2][BKP * (RSA + RSB)];

  const int mtiles = p.M / BM, ntiles = p.N / BN;
  const int nwg = mtiles * ntiles;
  int bid, split;
  split_tile(nwg, (p.P + p.pps - 1) / p.pps, p.group != 0, bid, split);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int pbeg = split * p.pps;
  const int pend = min(p.P, pbeg + p.pps);
  const int nkh = pend > pbeg ? (pend - pbeg + BKP - 1) / BKP : 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const T* __restrict__ X = reinterpret_cast<const T*>(p.x);
  const T* __restrict__ DY = reinterpret_cast<const T*>(p.dy);

  // A staging: dy[p][mt*BM + ca*E .. +E)
  const int ca = tid % CA, ra0 = tid / CA;
  const T* a_col = DY + mt * BM + ca * E;
  // B staging: column chunk fixed per thread -> tap / channel fixed
  const int cb = tid % CB, rb0 = tid / CB;
  const int kcol = nt * BN + cb * E;
  int tap_r, tap_s, ci;
  if constexpr (STEM) {
    tap_r = kcol >> 5; tap_s = (kcol & 31) >> 2; ci = 0;
  } else {
    const int t = kcol / p.Cin;
    ci = kcol - t * p.Cin;
    tap_r = t / p.S; tap_s = t - tap_r * p.S;
  }
  const int HWo = p.Ho * p.Wo;
  const int ldrow = p.W * p.lda;  // elements per input row
  // FAST: per-thread (row, col) offsets of its B rows inside a k-step
  int dr[PB], dc[PB];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int r = rb0 + RPB * i;
    if (p.Wo >= BKP) { dr[i] = 0; dc[i] = r; } else { dr[i] = r / p.Wo; dc[i] = r - dr[i] * p.Wo; }
  }

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  ProCoef<T> pc;
  if constexpr (PRO) pc.load(p.pro_scale, p.pro_shift, ci);
  // apply prologue: this thread's A chunk is a fixed channel chunk -> coefficients in registers
  float apa[AP ? E : 1], apb[AP ? E : 1], apc[AP ? E : 1];
  if constexpr (AP) {
    BwdEpiAcc<T, 3>::ld(apa, p.ap_ca + mt * BM + ca * E);
    BwdEpiAcc<T, 3>::ld(apb, p.ap_cb + mt * BM + ca * E);
    BwdEpiAcc<T, 3>::ld(apc, p.ap_cc + mt * BM + ca * E);
  }
  const T* ap_col = AP ? reinterpret_cast<const T*>(p.ap_y) + mt * BM + ca * E : nullptr;

  // load() only issues the global loads of a k-step; everything that consumes the loaded registers (the
  // apply, the BN prologue, zeroing rows past the split's range) runs in store(), after the previous
  // k-step's MFMAs: a transform in load() made the wave wait for its loads there (s_waitcnt vmcnt(0)
  // ahead of every MFMA of the k-step), so no load latency overlapped the MFMAs
  struct Stage {
    u32x4 a[PA], b[PB];
    u32x4 y[AP ? PA : 1];  // the apply's y rows beside the dm rows
    bool oka[PA], okb[PB];
  };

  auto load = [&](int p0, Stage& S) {
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int pix = p0 + ra0 + RPA * i;
      const bool ok = pix < pend;
      S.a[i] = ld16(a_col + (size_t)(ok ? pix : pbeg) * p.M);  // pbeg < P: a safe clamp
      if constexpr (AP) S.y[i] = ld16(ap_col + (size_t)(ok ? pix : pbeg) * p.M);
      S.oka[i] = ok;
    }
    int n0 = 0, oh0 = 0, ow0 = 0;
    if constexpr (FAST) {  // uniform: the k-step lies inside one image
      n0 = fdiv(p0, p.fd_hw);
      const int rem0 = p0 - n0 * HWo;
      oh0 = fdiv(rem0, p.fd_w);
      ow0 = rem0 - oh0 * p.Wo;
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int pix = p0 + rb0 + RPB * i;
      const bool pok = pix < pend;
      int nimg, oh, ow;
      if constexpr (FAST) {
        nimg = n0; oh = oh0 + dr[i]; ow = ow0 + dc[i];
      } else {
        const int pp = pok ? pix : pbeg;
        nimg = fdiv(pp, p.fd_hw);
        const int rem = pp - nimg * HWo;
        oh = fdiv(rem, p.fd_w);
        ow = rem - oh * p.Wo;
      }
      const int ih = oh * p.stride - p.pad + tap_r;
      const int iw0 = ow * p.stride - p.pad + tap_s;
      const bool hok = pok && (unsigned)ih < (unsigned)p.H;
      const int rowoff = (nimg * p.H + ih) * ldrow;
      if constexpr (STEM) {
        if constexpr (BF) {
          const int iw1 = iw0 + 1;
          const bool ok0 = hok && (unsigned)iw0 < (unsigned)p.W, ok1 = hok && (unsigned)iw1 < (unsigned)p.W;
          const uint2 v0 = *reinterpret_cast<const uint2*>(X + (ok0 ? rowoff + iw0 * 4 : 0));
          const uint2 v1 = *reinterpret_cast<const uint2*>(X + (ok1 ? rowoff + iw1 * 4 : 0));
          S.b[i] = u32x4{ok0 ? v0.x : 0u, ok0 ? v0.y : 0u, ok1 ? v1.x : 0u, ok1 ? v1.y : 0u};
          S.okb[i] = true;
        } else {
          const bool ok = hok && (unsigned)iw0 < (unsigned)p.W;
          S.b[i] = ld16(X + (ok ? rowoff + iw0 * 4 : 0));
          S.okb[i] = ok;
        }
      } else {
        const bool ok = hok && (unsigned)iw0 < (unsigned)p.W;
        S.b[i] = ld16(X + (ok ? rowoff + iw0 * p.lda + ci : 0));
        S.okb[i] = ok;
      }
    }
  };
  auto store = [&](int buf, const Stage& S) {
#pragma unroll
    for (int i = 0; i < PA; ++i) {
      const int row = ra0 + RPA * i;
      int c = ca;
      if constexpr (BF) c = (((ca >> 1) ^ swz32(row)) << 1) | (ca & 1);
      u32x4 v = S.a[i];
      if constexpr (AP) {  // dy = ca*dm + cb*y + cc (argus_bn_bwd_apply's formula, fp32, rounded to T)
        float d[E], yv[E];
        unpack(v, d);
        unpack(S.y[i], yv);
#pragma unroll
        for (int j = 0; j < E; ++j) d[j] = fmaf(apa[j], d[j], fmaf(apb[j], yv[j], apc[j]));
        v = pack(d);
      }
      lds[buf][row * RSA + c] = sel(S.oka[i], v);
    }
#pragma unroll
    for (int i = 0; i < PB; ++i) {
      const int row = rb0 + RPB * i;
      int c = cb;
      if constexpr (BF) c = (((cb >> 1) ^ swz32(row)) << 1) | (cb & 1);
      u32x4 v = S.b[i];
      if constexpr (PRO && !STEM) v = pc.apply(v);
      lds[buf][BKP * RSA + row * RSB + c] = sel(S.okb[i], v);
    }
  };

  const int g = lane >> 4, i16 = lane & 15;
  auto compute = [&](int buf) {
    if constexpr (BF) {
      const char* base = reinterpret_cast<const char*>(&lds[buf][0]);
      const int q = i16 >> 2, pq = i16 & 3;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x4 fa[MI], fb[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) {
          const int slot = (wm * (BM / 2) + mi * 16) >> 4;
          unsigned w[4];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int row = 32 * s2 + 8 * g + 4 * h + q;
            const char* addr = base + row * 256 + ((slot ^ swz32(row)) << 5) + pq * 8;
            const s16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(uint32_t)(uintptr_t)addr);
            const uint2 u = __builtin_bit_cast(uint2, t);
            w[2 * h] = u.x; w[2 * h + 1] = u.y;
          }
          fa[mi] = u32x4{w[0], w[1], w[2], w[3]};
        }
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const int slot = (wn * (BN / 2) + ni * 16) >> 4;
          unsigned w[4];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int row = 32 * s2 + 8 * g + 4 * h + q;
            const char* addr = base + BKP * RSA * 16 + row * 256 + ((slot ^ swz32(row)) << 5) + pq * 8;
            const s16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(uint32_t)(uintptr_t)addr);
            const uint2 u = __builtin_bit_cast(uint2, t);
            w[2 * h] = u.x; w[2 * h + 1] = u.y;
          }
          fb[ni] = u32x4{w[0], w[1], w[2], w[3]};
        }
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) Mma<bf16>::run(acc[mi][ni], fa[mi], fb[ni]);
      }
    } else {
      const float* fa = reinterpret_cast<const float*>(&lds[buf][0]);
      const float* fb = reinterpret_cast<const float*>(&lds[buf][BKP * RSA]);
#pragma unroll
      for (int sub = 0; sub < BKP / 4; ++sub) {
        const int row = 4 * sub + g;
        float av[MI], bv[NI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) av[mi] = fa[row * RSA * 4 + wm * (BM / 2) + mi * 16 + i16];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) bv[ni] = fb[row * RSB * 4 + wn * (BN / 2) + ni * 16 + i16];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mi], bv[ni], acc[mi][ni], 0, 0, 0);
      }
    }
  };

  // LDS double buffer + 2-deep register prefetch ring (as igemm_kernel); the 128x128 tile keeps a
  // single staged k-step (the ring would not fit two waves per SIMD without spilling)
  constexpr bool RING = !(BM == 128 && BN == 128);
  const int nk = nkh;
  if (!RING && nk > 0) {
    Stage S0;
    load(pbeg, S0);
    store(0, S0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load(pbeg + (kt + 1) * BKP, S0);
      compute(cur);
      if (kt + 1 < nk) store(cur ^ 1, S0);
      __syncthreads();
    }
  } else if (nk > 0) {
    Stage S0, S1;
    load(pbeg, S0);
    store(0, S0);
    if (nk > 1) load(pbeg + BKP, S1);
    if (nk > 2) load(pbeg + 2 * BKP, S0);
    __syncthreads();
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      compute(0);
      store(1, S1);
      if (kt + 3 < nk) load(pbeg + (kt + 3) * BKP, S1);
      __syncthreads();
      compute(1);
      if (kt + 2 < nk) {
        store(0, S0);
        if (kt + 4 < nk) load(pbeg + (kt + 4) * BKP, S0);
      }
      __syncthreads();
    }
    if (kt < nk) compute(0);
  }

  float* out = p.part + (size_t)split * p.M * p.N;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int n = nt * BN + wn * (BN / 2) + ni * 16 + i16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * BM + wm * (BM / 2) + mi * 16 + g * 4 + r;
        out[(size_t)m * p.N + n] = acc[mi][ni][r];  // cached: the split reduce reads it next
      }
    }
}

// ------------------------------------------------------------------------------------------------
// layout kernels
// ------------------------------------------------------------------------------------------------
// Input pixel -> fp32: fp32 images pass through; uint8 images are divided by 255 exactly as the
// reference's `.to(torch.float32) / 255.0` (argus/data.py:214-215), so both paths give equal bits.
ARGUS_DEV float pixel_f32(float v) { return v; }
ARGUS_DEV float pixel_f32(uint8_t v) { return (float)v / 255.0f; }

template <typename T, typename In>
__global__ __launch_bounds__(256) void images_to_nhwc4_kernel(const In* __restrict__ x, T* __restrict__ out,
                                                              int64_t nimg, int hw) {
  const int64_t total = nimg * hw;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t img = i / hw, pix = i - img * hw;
    const In* src = x + img * 3 * hw + pix;
    if constexpr (sizeof(T) == 2) {  // the pixel's 4 bf16 as one 8-byte store
      const T v[4] = {from_f32<T>(pixel_f32(src[0])), from_f32<T>(pixel_f32(src[hw])),
                      from_f32<T>(pixel_f32(src[2 * hw])), from_f32<T>(0.f)};
      *reinterpret_cast<uint2*>(out + i * 4) = __builtin_bit_cast(uint2, v);
    } else {
      T* dst = out + i * 4;
      dst[0] = from_f32<T>(pixel_f32(src[0]));
      dst[1] = from_f32<T>(pixel_f32(src[hw]));
      dst[2] = from_f32<T>(pixel_f32(src[2 * hw]));
      dst[3] = from_f32<T>(0.f);
    }
  }
}

// fp32 master weight (any strides: element (k, c, r, s) at k*sk + c*sc + r*sr + s*ss) -> forward
// copy w_fwd[k][r][s][c] (dtype; stem padded [k][8][8][4]) and dgrad copy w_dgrad[c][r][s][k].
struct WStrides { long long sk, sc, sr, ss; };

template <typename T>
__global__ __launch_bounds__(256) void weight_prep_kernel(const float* __restrict__ w, WStrides st,
                                                          T* __restrict__ wf, T* __restrict__ wd, int K, int R,
                                                          int S, int C, int stem) {
  if (stem) {
    const int total = K * 256;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
      const int k = i >> 8, col = i & 255;
      const int r = col >> 5, s = (col & 31) >> 2, c = col & 3;
      float v = 0.f;
      if (r < 7 && s < 7 && c < 3) v = w[k * st.sk + c * st.sc + r * st.sr + s * st.ss];
      wf[i] = from_f32<T>(v);
    }
    return;
  }
  const int RSC = R * S * C;
  const int total = K * RSC;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int k = i / RSC, rem = i - k * RSC;
    const int rs = rem / C, c = rem - rs * C;
    const int r = rs / S, s = rs - r * S;
    const float v = w[k * st.sk + c * st.sc + r * st.sr + s * st.ss];
    if (wf) wf[i] = from_f32<T>(v);
    if (wd) wd[((size_t)c * R * S + rs) * K + k] = from_f32<T>(v);
  }
}

// Batched weight_prep: one launch converts every conv of the network. Non-stem convs go in 64(k) x
// 64(c) tiles of one tap: the tile is read once (rows of c), written to w_fwd[k][tap][c] as rows and
// transposed through LDS into w_dgrad[c][tap][k] as rows, so both writes are coalesced. The stem
// (C = 3, no w_dgrad) is an element-wise pad + convert, kWpChunk elements per workgroup.
struct WpEntry {
  const float* w;
  long long sk, sc, sr, ss;
  void* wf;
  void* wd;
  int K, R, S, C, stem, blk0;  // blk0: first workgroup of this entry
  int f8f, f8d;                 // ARGUS_FP8: the MX-fp8 layout for w_fwd / w_dgrad (wp_f8_layouts)
};
constexpr int kWpChunk = 4096;

ARGUS_HOST_DEV inline int wp_blocks(int K, int R, int S, int C, int stem) {
  return stem ? (K * 256 + kWpChunk - 1) / kWpChunk : (K / 64) * (C / 64) * R * S;
}

// MX-fp8 weight layout (argus_conv_weight_prep with ARGUS_FP8, for the passes whose reduction channels
// are multiples of 128: forward when C % 128 == 0, dgrad when K % 128 == 0): in the buffer of the bf16
// copy, bytes [0, rows * cols) hold the e4m3 values row-major, followed by one E8M0 scale byte per 32
// consecutive elements of a row ([rows][cols / 32]). The values are the bf16-rounded weights quantized
// exactly as the conv kernel would quantize them while staging (mx_fp8_quant): pre-quantizing only
// moves that work out of every forward / dgrad launch.
// policy key 37 bit of a pass: 1 forward, 2 data gradient of a 3x3 conv, 4 data gradient of a 1x1 conv
// (with or without the apply prologue: one weight copy serves both)
// Bit 8: the forward of 3x3 stride-1 convs only (the convs argus_conv_fwd_x8 serves from an MX-fp8
// stored input; the other forwards stay bf16)
static int fp8_pass_bits(int fwd, int ksz) { return fwd ? 1 : (ksz == 1 ? 4 : 2); }
static bool fp8_pass(int passes, int fwd, int ksz, int stride) {
  return (passes & fp8_pass_bits(fwd, ksz)) || (fwd && ksz == 3 && stride == 1 && (passes & 8));
}

// the passes of conv d that take fp8 operands under its policy: their weight copies get the fp8 layout
static void wp_f8_layouts(const argus_conv_desc& d, int& f8f, int& f8d) {
  const int passes = policy_of(d)[kFp8Passes];
  f8f = !d.stem && d.c % 128 == 0 && fp8_pass(passes, 1, d.r, d.stride);
  f8d = !d.stem && d.k % 128 == 0 && fp8_pass(passes, 0, d.r, d.stride);
}

// 16 fp32 weights of one row -> bf16 (as the bf16 copy) -> 16 e4m3 + the 32-element block's scale
// (shared with lane ^ 1, which holds the other half of the block); returns the scale byte.
ARGUS_DEV unsigned wp_quant16(const float (&f)[16], uint8_t* dst) {
  float lo[8], hi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { lo[j] = f[j]; hi[j] = f[8 + j]; }
  int e;
  st16(dst, mx_fp8_quant(pack(lo), pack(hi), e));
  return (unsigned)(127 + e);
}

// One 64 (k) x 64 (c) tile of one tap (or a stem chunk) of entry e: workgroup `local` of the entry.
// F8: fp8 layout for the passes wp_f8_fwd / wp_f8_dgrad select, bf16 otherwise (T = bf16).
template <typename T, bool F8>
ARGUS_DEV void weight_prep_tile(const WpEntry& e, int local) {
  T* __restrict__ wf = reinterpret_cast<T*>(e.wf);
  T* __restrict__ wd = reinterpret_cast<T*>(e.wd);
  if (e.stem) {
    const int total = e.K * 256;
    for (int i = local * kWpChunk + threadIdx.x; i < (local + 1) * kWpChunk && i < total; i += 256) {
      const int k = i >> 8, col = i & 255;
      const int r = col >> 5, s = (col & 31) >> 2, c = col & 3;
      float v = 0.f;
      if (r < 7 && s < 7 && c < 3) v = e.w[k * e.sk + c * e.sc + r * e.sr + s * e.ss];
      wf[i] = from_f32<T>(v);
    }
    return;
  }
  const int RS = e.R * e.S, ct = e.C / 64;
  const int rs = local % RS, rem = local / RS;
  const int c0 = (rem % ct) * 64, k0 = (rem / ct) * 64;
  const int r = rs / e.S, s = rs - r * e.S;
  __shared__ T tile[64][65];
  const int row = threadIdx.x >> 2, cq = (threadIdx.x & 3) * 16;  // 4 threads x 16 elements per row
  const bool f8f = F8 && e.f8f, f8d = F8 && e.f8d;
  {
    const float* src = e.w + (long long)(k0 + row) * e.sk + r * e.sr + s * e.ss + (long long)(c0 + cq) * e.sc;
    float f[16];
    if (e.sc == 1 && ((uintptr_t)src & 15) == 0) {  // channel-contiguous master (OHWI storage): 16-byte loads
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(src + j);
        f[j] = v.x; f[j + 1] = v.y; f[j + 2] = v.z; f[j + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) f[j] = src[j * e.sc];
    }
    constexpr int E = Chunk<T>::E;
#pragma unroll
    for (int j = 0; j < 16; ++j) tile[row][cq + j] = from_f32<T>(f[j]);
    if (f8f) {  // e4m3 row [k][RS*C] + scales [k][RS*C/32]
      const long long cols = (long long)RS * e.C, at = (long long)(k0 + row) * cols + rs * e.C + c0 + cq;
      uint8_t* base = reinterpret_cast<uint8_t*>(e.wf);
      const unsigned sb = wp_quant16(f, base + at);
      if ((threadIdx.x & 1) == 0) base[(long long)e.K * cols + at / 32] = (uint8_t)sb;
    } else {
      T* dst = wf + ((size_t)(k0 + row) * RS + rs) * e.C + c0 + cq;
#pragma unroll
      for (int j = 0; j < 16; j += E) {
        float g[E];
#pragma unroll
        for (int u = 0; u < E; ++u) g[u] = f[j + u];
        st16(dst + j, pack(g));
      }
    }
  }
  if (!wd) return;
  __syncthreads();
  constexpr int E = Chunk<T>::E;
  float g16[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) g16[j] = to_f32(tile[cq + j][row]);  // row = c, 16 consecutive k
  if (f8d) {  // e4m3 row [c][RS*K] + scales [c][RS*K/32]
    const long long cols = (long long)RS * e.K, at = (long long)(c0 + row) * cols + rs * e.K + k0 + cq;
    uint8_t* base = reinterpret_cast<uint8_t*>(e.wd);
    const unsigned sb = wp_quant16(g16, base + at);
    if ((threadIdx.x & 1) == 0) base[(long long)e.C * cols + at / 32] = (uint8_t)sb;
    return;
  }
  T* dst = wd + ((size_t)(c0 + row) * RS + rs) * e.K + k0 + cq;
#pragma unroll
  for (int j = 0; j < 16; j += E) {
    float g[E];
#pragma unroll
    for (int u = 0; u < E; ++u) g[u] = g16[j + u];
    st16(dst + j, pack(g));
  }
}

template <typename T, bool F8>
__global__ __launch_bounds__(256) void weight_prep_batch_kernel(const WpEntry* __restrict__ tab, int count) {
  int lo = 0, hi = count - 1;
  const int b = blockIdx.x;
  while (lo < hi) {  // last entry with blk0 <= b
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].blk0 <= b) lo = mid; else hi = mid - 1;
  }
  const WpEntry e = tab[lo];
  weight_prep_tile<T, F8>(e, b - e.blk0);
}

// one conv (argus_conv_weight_prep with ARGUS_FP8): the entry by value
__global__ __launch_bounds__(256) void weight_prep_one_f8_kernel(const WpEntry e) {
  weight_prep_tile<bf16, true>(e, blockIdx.x);
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------

static int check_desc(const argus_conv_desc& d);
int conv_check_desc(const argus_conv_desc& d) { return check_desc(d); }

static int check_desc(const argus_conv_desc& d) {
  if (int e = check_tuning(d)) return e;
  if (d.n <= 0 || d.h <= 0 || d.w <= 0 || d.k <= 0 || d.r <= 0 || d.s <= 0 || d.stride <= 0) {
    set_error("conv: non-positive dimension in descriptor");
    return ARGUS_ERR_ARG;
  }
  if (d.ho != (d.h + 2 * d.pad - d.r) / d.stride + 1 || d.wo != (d.w + 2 * d.pad - d.s) / d.stride + 1) {
    set_error("conv: ho/wo inconsistent with h/w/r/s/stride/pad");
    return ARGUS_ERR_SHAPE;
  }
  if (d.stem) {
    if (d.c != 3 || d.r != 7 || d.s != 7 || d.stride != 2 || d.pad != 3 || d.k % 64) {
      set_error("conv: stem must be 3->k (k%64==0) 7x7/2 p3");
      return ARGUS_ERR_SHAPE;
    }
  } else if (d.c % 64 || d.k % 64 || d.r > 3 || d.s > 3 || d.stride > 2) {
    set_error("conv: channels must be multiples of 64, filters <= 3x3, stride <= 2");
    return ARGUS_ERR_SHAPE;
  }
  if ((int64_t)d.n * d.h * d.w * (d.stem ? 4 : d.c) >= (1LL << 31) || (int64_t)d.n * d.ho * d.wo * d.k >= (1LL << 31)) {
    set_error("conv: tensor too large for 32-bit element offsets (split the batch)");
    return ARGUS_ERR_SHAPE;
  }
  return ARGUS_OK;
}

template <typename T, int BM, int BN, bool STEM, bool PRO, int OCC, int BW>
static const char* ig_name() {
  static const std::string s = std::string("argus::igemm_kernel<") + type_name<T>() + ", " + std::to_string(BM) +
                               ", " + std::to_string(BN) + ", " + bool_name(STEM) + ", " + bool_name(PRO) + ", " +
                               std::to_string(OCC) + ", " + std::to_string(BW) + ">";
  return s.c_str();
}

template <typename T, int BM, int BN, bool STEM, bool PRO, int OCC, int BW = 0>
static void launch_ig(const IgParams& p0, int maxM, hipStream_t st) {
  IgParams p = p0;
  plan_fin(p, BM);
  plan_ffin(p, BM);
  const int ntiles = p.N / BN;
  dim3 grid(cdiv(maxM, BM) * ntiles, 1, p.nphase);
  timed_launch(ig_name<T, BM, BN, STEM, PRO, OCC, BW>(), igemm_kernel<T, BM, BN, STEM, PRO, OCC, BW>, grid,
               dim3(256), st, p);
}

template <typename T, bool PRO, int OCC, int BW = 0>
static void dispatch_ig(const IgParams& p, int maxM, int bm, int bn, hipStream_t st) {
  const bool bn128 = bn == 128;
  if (bm == 128) {
    // the single-buffer 128x128 tile needs > 128 VGPRs: 3 workgroups per CU instead of 4
    if (bn128) launch_ig<T, 128, 128, false, PRO, (OCC == 4 ? 3 : OCC), BW>(p, maxM, st);
    else launch_ig<T, 128, 64, false, PRO, OCC, BW>(p, maxM, st);
  } else {
    if (bn128) launch_ig<T, 64, 128, false, PRO, OCC, BW>(p, maxM, st);
    else launch_ig<T, 64, 64, false, PRO, OCC, BW>(p, maxM, st);
  }
}

// BN-backward epilogue (+ apply prologue) variants (dgrad only: no stem, no BN+ReLU prologue)
template <typename T, int OCC, int APB>
static void dispatch_ig_bwd1(const IgParams& p, int maxM, int bm, int bn, hipStream_t st) {
  if constexpr (sizeof(T) == 2 && !(APB & kFp8Bit)) {
    if (p.bb.yx) {  // y recomputed in the epilogue (block-output BN: mask bits, + the downsample branch)
      if (bwd_variant(p.bb) == 4) dispatch_ig<T, false, OCC, 4 | APB | kYrecBit>(p, maxM, bm, bn, st);
      else dispatch_ig<T, false, OCC, 3 | APB | kYrecBit>(p, maxM, bm, bn, st);
      return;
    }
  }
  switch (bwd_variant(p.bb)) {
    case 2: dispatch_ig<T, false, OCC, 2 | APB>(p, maxM, bm, bn, st); break;
    case 3: dispatch_ig<T, false, OCC, 3 | APB>(p, maxM, bm, bn, st); break;
    case 4: dispatch_ig<T, false, OCC, 4 | APB>(p, maxM, bm, bn, st); break;
    default: dispatch_ig<T, false, OCC, APB>(p, maxM, bm, bn, st);
  }
}

template <typename T, int OCC>
static void dispatch_ig_bwd(const IgParams& p, int maxM, int bm, int bn, hipStream_t st) {
  if (p.ap.y) dispatch_ig_bwd1<T, OCC, kApplyBit>(p, maxM, bm, bn, st);
  else dispatch_ig_bwd1<T, OCC, 0>(p, maxM, bm, bn, st);
}

// ------------------------------------------------------------------------------------------------
// kernel-selection policy (argus_conv_policy_default): an immutable table + per-call overrides
// ------------------------------------------------------------------------------------------------
// Defaults, each the measured best:
//  7: K <= 1024 on the single-buffer OCC=3/4 kernel (convbench B=64: 128 -> 1024 took fwd+dgrad from
//     6.13 to 5.87 ms/step: more resident workgroups hide the global-load latency better than the OCC=2
//     register ring);
//  6 / 27: weight-gradient split targets 512 (1x1) / 512 (register-staged 3x3, Cout > 64: isolated
//     sweeps favoured 1024, in the full step 512 wins +0.7 % - fewer fp32 split partials contending with
//     the main stream for HBM); 3x3 with Cout = 64: 2048;
//  19 / 34: the bf16 stem forward / weight gradient on the LDS-patch kernels (stem.hip);
//  35: 128-row forward tiles from 16 K GEMM rows; 36: the glds kernel from 4 256-row tiles;
//  37: ARGUS_FP8 runs the MX-fp8 MFMA on the 3x3 data gradients only (2). Full B=512 steps per
//      setting (profiles/r04_b512_fp8_policy.txt): 2 -> 10203 img/s, 0 (no fp8) 10170, 4 (1x1 dgrads,
//      apply prologue staged then quantized) 9583, 6 9668, 7 (every pass) 9486; bf16 10190. Per layer
//      (tools/convbench.py, profiles/r04_convbench_b512_*.txt) the register-staged fp8 kernel loses to
//      the bf16 kernels on every forward but one (OCC 2 against OCC 3-4 or LDS-DMA staging, plus the
//      per-row quantization of the activation operand) and the 1x1 data gradients with the apply
//      prologue (four staged chunks per row: OCC 2) take 1.4 ms where the bf16 kernel takes 1.0 ms.
static constexpr int kUnset = -1;
static const Policy kDefaultPolicy = [] {
  Policy p;
  for (int& v : p.v) v = kUnset;
  for (int k = 0; k < 6; ++k) p.v[k] = 0;
  p.v[kWgradTarget] = 512;
  p.v[kSmallKMax] = 1024;
  p.v[kGldsMinK] = 1024;
  p.v[kGldsMinGrid] = 256;
  p.v[kHaloEnable] = 1;
  p.v[kWgHaloEnable] = 1;
  // 12: split target of the 3x3 halo weight gradient: 128 (round 6; 256 before): engine A/B, best of 3
  //     interleaved rounds, B=64 13.24 vs 13.48-13.54 ms, B=256 45.49 vs 45.63-45.66 ms, 376x672 88.27 vs
  //     88.06-88.39 ms; 64 slower, 192 between (profiles/r06h_*, r06i_*). Half the workgroups hold the CUs
  //     beside the main stream's chain for longer, and write half the fp32 split partials
  p.v[kWgHaloTarget] = 128;
  p.v[kHaloMinGrid] = 256;
  // 14: the halo weight gradient for 3x3 convs of up to 64 (64 x 64) channel tiles, i.e. every layer
  //     (round 4; 4 = layers 1-2 only before): engine A/B 13.86-14.05 vs 14.07-14.20 ms (B=64),
  //     48.0 vs 48.5-48.9 ms (B=256), 93.6 vs 95.5-96.0 ms (376x672 B=128): profiles/r04_ab_key14.txt
  p.v[kWgHaloMaxTiles] = 64;
  p.v[kStemLdsFwd] = 1;
  p.v[kWgradTarget3x3] = 512;
  p.v[kStemLdsWgrad] = 1;
  p.v[kFwdBm128Rows] = 16 * 1024;
  p.v[kGldsMinRows] = 4 * 256;
  // 37: the 3x3 data gradients (2) and the 3x3 stride-1 forwards (8) on MX-fp8 operands; where the
  //     engine stores their inputs as MX-fp8 copies (argus_conv_fwd_x8 / _dgrad_bn_x8) they run on the
  //     halo kernel's F8 variant (B=512: forward 3x3 3.49 -> 2.32 ms/step, the step 90.8 -> 90.1 ms
  //     median of 3, profiles/r05l_*)
  p.v[kFp8Passes] = 10;
  // 38: a 1x1 dgrad with an apply prologue (dy = ca*dm + cb*y + cc) on the glds kernel after the
  //     apply kernel materialises dy (0), rather than staging the apply in the register-staged kernel
  //     (1): 1 saves the dy round trip but the register-staged kernel is slower at K >= 1024;
  //     engine A/B 14.73-14.96 vs 14.76-14.88 ms (B=64), 51.5 vs 51.6 (B=256), 99.6 vs 100.2-100.6
  //     (376x672 B=128): profiles/r04_ab_key38.txt
  p.v[kDgradApStaged] = 0;
  // 39 / 40: data gradients may use the glds / LDS-halo kernels (0 = register-staged igemm): 39 = 0
  //     14.02-14.05 vs 14.03-14.20 ms at B=64 but 96.6-96.9 vs 95.5-96.0 ms at 376x672; 40 = 0 within
  //     the instance spread at both (profiles/r04_ab_coresidency.txt)
  p.v[kGldsDgrad] = 1;
  p.v[kHaloDgrad] = 1;
  p.v[kGldsDgradStages] = 3;
  // 42: the small-K dgrads with a BN-backward epilogue or an apply prologue built for 4 workgroups per CU
  //     (128 VGPRs: the 64 x 128 apply + mask-bits variants spill 6 registers) or 3 (168 VGPRs)
  p.v[kBwdSmallKOcc] = 4;
  // 44: statistics-only 1x1 forwards (the bottleneck conv3 before argus_conv_fwd_bn_out) on the
  //     persistent kernel of conv_p1x1.hip (1) or the register-staged igemm (0): layer 1 44.5-47.7 ->
  //     32.2 us, layers 2-4 31-33 -> 26-29 us per launch (B=64, profiles/r05q_timeline/); the step
  //     within drift (13.921 vs 13.924 ms under the profiler, r05p_ab_key44.txt)
  p.v[kP1x1FwdStats] = 1;
  // 43: the bottleneck conv1 data gradients (1x1, apply prologue, mask-bits BN epilogue with the folded
  //     finalize) on the persistent kernel of conv_p1x1.hip (1) or the register-staged igemm (0)
  p.v[kP1x1Dgrad] = 1;
  // 45: 1x1 bf16 weight gradients on the LDS-DMA ring kernel of conv_wgdma.hip with 128 x 128 tiles (1),
  //     128 x 256 tiles where Cin % 256 == 0 for the apply variant (2) or both (3), or the
  //     register-staged wgrad_kernel (0): engine A/B 2 vs 0: B=256 46.05-46.21 vs 46.54-46.57 ms,
  //     376x672 89.6-89.9 vs 90.6-91.2 ms, B=64 within drift (profiles/r05ai_ab_key45_*.txt). Round 6: 3
  //     (key 49 = 4 sends layer 3-4 conv1 weight gradients to the plain form): B=64 13.34-13.36 vs
  //     13.39-13.40 ms best of 4, B=256 and 376x672 level (profiles/r06e_*, r06f_*)
  p.v[kWgradDma] = 3;
  // 46: 1x1 weight gradients over at most this many pixels take half the split target (256): engine
  //     A/B at B=64 (layers 2-4) 13.69-13.74 vs 13.79-13.85 ms, B=256 (layers 3-4) 46.95-47.01 vs
  //     47.02-47.07, 376x672 (layer 4) within drift; 262144 no better; a global target of 256 gains
  //     at B=64 but costs 376x672 0.7 % (profiles/r05ap_*, r05ar_*)
  p.v[kWgradSmallP] = 65536;
  // 47: the stride-2 plain weight gradients (1x1 downsample, 3x3 conv2) on the gathering DMA kernel
  //     (0 off, 1 every size, > 1 up to that many output pixels): engine A/B with every size on, B=64
  //     13.42-13.46 vs 13.51-13.57 ms, 376x672 within drift (profiles/r05as_*), but B=256 46.56-46.86 vs
  //     46.43-46.60 ms (r05at_*: its 524,288-pixel layer-2 launches lose); served up to 131,072 pixels:
  //     B=64 every layer, B=256 layers 3-4, 376x672 B=128 layer 4
  p.v[kWgradDmaGather] = 131072;
  // 48: LDS ring stages of the 128 x 256 apply weight gradient (32 KB each; 4 = 128 KB, one workgroup
  //     per CU; 5 = all 160 KB, one more stage in flight; 2 / 3 leave room for main-stream workgroups)
  p.v[kWgradDmaStages] = 4;
  // 49: 1x1 BN-backward-apply prologues are staged by the dgrad only up to this many 128-column tiles
  //     (0: always): beyond it the redundant per-tile apply (VALU) costs more than materialising dy.
  //     4 (the conv1 dgrads of layers 3-4 materialise dy1): engine A/B, best of 3-4 interleaved rounds,
  //     B=64 13.65 vs 13.68-13.72 ms, B=256 46.21 vs 47.03-47.13 ms, 376x672 B=128 90.23 vs 90.71-91.56 ms;
  //     8 level, 2 slower (14.6 ms at B=64): profiles/r06a_ab_keys.txt, r06b_ab_*_key49*.txt
  p.v[kDgradApMaxCols] = 4;
  // 50: the LDS-DMA weight gradients sum their split partials inside the launch (reducing workgroups
  //     after the compute grid, conv_wgdma.hip) instead of a wgrad_reduce launch; the caller's workspace
  //     must end in kWgFoldCtrBytes of zeros (argus_conv_wgrad_workspace_bytes includes them). Engine
  //     A/B at B=64: 14.50 vs 13.78-13.85 ms (profiles/r06a_ab_keys.txt): the reducing workgroups wait
  //     for their tile's last split while holding a CU's LDS, and the write-through partials leave L2:
  //     off (dW bit-identical either way)
  p.v[kWgradFold] = 0;
  // 51: the 3x3 halo forward / data gradient (128-column tiles) with a four-stage weight ring on
  //     384-position halo images where the tile's halo fits (the 32- and 16-wide layers at 256 x 256):
  //     alone (tools/dgradbench.py --convs conv2, B=64) layer 2 51.5 / 68.5 vs 51.6 / 68.9 us (plain /
  //     BN epilogue + fold), layer 3 43.4 vs 43.9 us; engine A/B level at B=64 and B=256
  //     (profiles/r06d_*): off. The halo loop is not waiting on weight stages in flight
  p.v[kHaloDeepRing] = 0;
  return p;
}();

int policy_default(int key) {
  return key >= 0 && key < kNumTuneKeys ? kDefaultPolicy.v[key] : -1;
}

int check_tuning(const argus_conv_desc& d) {
  if (d.n_tuning < 0 || (d.n_tuning > 0 && !d.tuning)) {
    set_error("conv: bad tuning array");
    return ARGUS_ERR_ARG;
  }
  for (int i = 0; i < d.n_tuning; ++i) {
    const int k = d.tuning[i].key;
    if (policy_default(k) == kUnset) {
      set_error("conv: unknown tuning key " + std::to_string(k));
      return ARGUS_ERR_ARG;
    }
  }
  return ARGUS_OK;
}

Policy policy_of(const argus_conv_desc& d) {
  Policy p = kDefaultPolicy;
  for (int i = 0; i < d.n_tuning; ++i) p.v[d.tuning[i].key] = d.tuning[i].value;
  return p;
}

// MX-fp8 operands (ARGUS_FP8) need whole 128-element k-steps inside one filter tap and no BN+ReLU
// prologue (the BN-backward apply prologue is staged before the quantization); other convs of an fp8
// network run the bf16 kernels. The weights are then the pre-quantized copy (argus_conv_weight_prep
// with ARGUS_FP8: wp_f8_fwd / wp_f8_dgrad pick the same convs).
static bool f8_ok(const IgParams& p) {
  if (!p.f8 || p.stem || p.pro_scale || p.Cin % 128) return false;
  if (!fp8_pass((*p.pol)[kFp8Passes], p.fwd, p.ksz, p.fwd ? p.ish : 0)) return false;
  for (int i = 0; i < p.nphase; ++i)
    if (p.ph[i].K % 128) return false;
  return true;
}

template <typename T>
static int run_ig(const IgParams& p, hipStream_t st, int bm, int bn) {
  int maxM = 0, maxK = 0;
  for (int i = 0; i < p.nphase; ++i) {
    maxM = p.ph[i].M > maxM ? p.ph[i].M : maxM;
    maxK = p.ph[i].K > maxK ? p.ph[i].K : maxK;
  }
  const bool smallk = maxK <= (*p.pol)[kSmallKMax];
  if constexpr (sizeof(T) == 2) {
    if (p.x8) {  // MX-fp8 stored operands: the F8 halo kernel only (argus_conv_fwd_x8 checked the shape)
      if (conv3x3_halo_launch(p, st)) return check_launch("conv3x3_halo_kernel");
      set_error("conv x8: not a halo-eligible conv");
      return ARGUS_ERR_SHAPE;
    }
    if (f8_ok(p) && !p.bb.yx) {  // single-buffered (the staged bf16 pair per chunk doubles the staging registers)
      if (p.ap.y) dispatch_ig_bwd1<T, 2, kFp8Bit | kApplyBit>(p, maxM, bm, bn, st);
      else dispatch_ig_bwd1<T, 2, kFp8Bit>(p, maxM, bm, bn, st);
      return check_launch("igemm_kernel");
    }
    // the statistics-only forward and the block-output epilogue exist on the register-staged kernel only
    if ((p.c || !p.fwd) && !p.oe.out && !p.bb.yx && !p.pro_out) {
      if (conv3x3_halo_launch(p, st)) return check_launch("conv3x3_halo_kernel");
      if (igemm_glds_launch(p, maxM, maxK, st)) return check_launch("igemm_glds_kernel");
    }
  }
  if (p.oe.out) {
    if (p.stem || p.pro_scale || p.bb.mode || p.ap.y) { set_error("conv_fwd_bn_out: plain forward only"); return ARGUS_ERR_ARG; }
    if (smallk) dispatch_ig<T, false, 4, kOutBit>(p, maxM, bm, bn, st);
    else dispatch_ig<T, false, 2, kOutBit>(p, maxM, bm, bn, st);
    return check_launch("igemm_kernel");
  }
  if (p.stem) {
    if (p.N != 64 || bm != 128) { set_error("igemm: stem expects 64 output channels"); return ARGUS_ERR_SHAPE; }
    launch_ig<T, 128, 64, true, false, 4>(p, maxM, st);  // single buffer (convbench B=64: 214 -> 179 us)
  } else if (p.pro_scale) {
    if (smallk) dispatch_ig<T, true, 4>(p, maxM, bm, bn, st);
    else dispatch_ig<T, true, 2>(p, maxM, bm, bn, st);
  } else if (p.bb.mode || p.ap.y) {
    if (smallk && (*p.pol)[kBwdSmallKOcc] == 3) dispatch_ig_bwd<T, 3>(p, maxM, bm, bn, st);
    else if (smallk) dispatch_ig_bwd<T, 4>(p, maxM, bm, bn, st);
    else dispatch_ig_bwd<T, 2>(p, maxM, bm, bn, st);
  } else {
    if (smallk) dispatch_ig<T, false, 4>(p, maxM, bm, bn, st);
    else dispatch_ig<T, false, 2>(p, maxM, bm, bn, st);
  }
  return check_launch("igemm_kernel");
}

// column tile of pass {0 fwd, 1 dgrad, 2 wgrad} (policy keys 3..5 force 64 | 128)
static int pick_bn(const Policy& pol, int pass, int n) {
  const int f = pol[kForceBn + pass];
  if (f == 64 || (f == 128 && n % 128 == 0)) return f;
  return n % 128 == 0 ? 128 : 64;
}

// row-tile size of the forward GEMM (drives the BN-statistics partial count)
static int fwd_bm(const argus_conv_desc& d, const Policy& pol) {
  if (d.stem) return 128;
  if (pol[kForceBm]) return pol[kForceBm];
  const long M = (long)d.n * d.ho * d.wo;
  return M >= pol[kFwdBm128Rows] ? 128 : 64;
}

// the stem forward runs on the LDS-patch kernel (stem.hip)
static bool stem_lds_fwd(const argus_conv_desc& d, int dtype, const Policy& pol) {
  return d.stem && pol[kStemLdsFwd] && stem_fwd_ok(d, dtype == ARGUS_FP8 ? ARGUS_BF16 : dtype);
}

int conv_fwd_stats_only_rows(const argus_conv_desc& d, int dtype) {
  if (check_desc(d)) return 0;
  if (p1x1_fwd_stats_ok(d, dtype, policy_of(d)[kP1x1FwdStats])) return p1x1_fwd_stats_rows(d);
  return conv_fwd_stat_rows(d, dtype);
}

int conv_fwd_stats_only_tile(const argus_conv_desc& d, int dtype) {
  if (check_desc(d)) return 0;
  if (p1x1_fwd_stats_ok(d, dtype, policy_of(d)[kP1x1FwdStats])) return -p1x1_fwd_stats_tile(d);
  return conv_fwd_stat_tile(d, dtype);
}

int conv_fwd_stat_rows(const argus_conv_desc& d, int dtype) {
  if (check_desc(d)) return 0;
  const Policy pol = policy_of(d);
  if (stem_lds_fwd(d, dtype, pol)) return stem_stat_rows(d);
  return cdiv(d.n * d.ho * d.wo, fwd_bm(d, pol));
}

// rows of the forward statistics partials; negative when every partial row is to be merged as a full
// one (the ragged LDS-patch stem: argus_bn_finalize)
int conv_fwd_stat_tile(const argus_conv_desc& d, int dtype) {
  if (check_desc(d)) return 0;
  const Policy pol = policy_of(d);
  if (stem_lds_fwd(d, dtype, pol)) return stem_ragged(d) ? -128 : 128;
  return fwd_bm(d, pol);
}

// dgrad row tile: 64 (swept: 64-row tiles beat 128 on every non-glds/non-halo dgrad at B=64, the
// extra workgroups outweigh the re-read weight tile; dgrad has no statistics partials to multiply)
static int dgrad_bm(const Policy& pol) {
  if (pol[kForceBm + 1]) return pol[kForceBm + 1];
  return 64;
}

// implicit-GEMM parameters of a forward conv (operand pointers left null)
static void fwd_params(const argus_conv_desc& d, const Policy& pol, IgParams& p) {
  p = IgParams{};
  p.pol = &pol;
  p.fwd = 1;
  p.ksz = d.r;
  p.N = d.k; p.H = d.h; p.W = d.w; p.ish = d.stride; p.isw = d.stride;
  p.Ho = d.ho; p.Wo = d.wo; p.osh = 1; p.osw = 1; p.ldc = d.k;
  p.addend = nullptr; p.addend_mask = nullptr; p.stem = d.stem; p.nphase = 1;
  IgPhase& ph = p.ph[0];
  ph.M = d.n * d.ho * d.wo; ph.Hq = d.ho; ph.Wq = d.wo; ph.oh0 = 0; ph.ow0 = 0;
  if (d.stem) {
    p.Cin = 256; p.lda = 4; p.ldb = 256; ph.K = 256;
    ph.dh[0] = 0; ph.dw[0] = 0; ph.boff[0] = 0;
  } else {
    p.Cin = d.c; p.lda = d.c; p.ldb = d.r * d.s * d.c; ph.K = d.r * d.s * d.c;
    for (int r = 0; r < d.r; ++r)
      for (int s = 0; s < d.s; ++s) {
        const int t = r * d.s + s;
        ph.dh[t] = r - d.pad; ph.dw[t] = s - d.pad; ph.boff[t] = t * d.c;
      }
  }
}

thread_local int g_ffin_folded = 0;

int conv_fwd(const argus_conv_desc& d, int dtype, const void* x, const void* w, void* y,
             const float* sc, const float* sh, float* stats, hipStream_t st, void* pro_out,
             const argus_bn_fwd_fin* fin) {
  if (int e = check_desc(d)) return e;
  if (pro_out && (!sc || d.stem || d.r != 1 || d.s != 1 || d.stride != 1 || d.pad != 0 || pro_out == x ||
                  dtype == ARGUS_FP8)) {
    set_error("conv_fwd_apply_out: a BN+ReLU prologue on a 1x1 stride-1 bf16/fp32 conv, x_out != x");
    return ARGUS_ERR_ARG;
  }
  const bool f8 = dtype == ARGUS_FP8;  // bf16 tensors, MX-fp8 GEMM operands where the shape allows
  if (f8) dtype = ARGUS_BF16;
  g_launch_work = 2.0 * d.n * d.ho * d.wo * d.k * d.r * d.s * d.c;  // algorithmic flops / bytes (ktimer)
  g_launch_bytes = (double)(dtype == ARGUS_BF16 ? 2 : 4) *
                       ((double)d.n * d.h * d.w * (d.stem ? 4 : d.c) + (double)d.k * d.r * d.s * d.c +
                        (double)d.n * d.ho * d.wo * d.k) +
                   (stats ? 8.0 * conv_fwd_stat_rows(d, dtype) * d.k : 0.0);
  if (d.stem && sc) { set_error("conv_fwd: stem has no prologue"); return ARGUS_ERR_ARG; }
  if (!y && (!stats || d.stem || f8 || dtype != ARGUS_BF16)) {
    set_error("conv_fwd: y may be NULL only for a bf16 non-stem forward with statistics");
    return ARGUS_ERR_ARG;
  }
  if (!y) g_launch_bytes -= 2.0 * d.n * d.ho * d.wo * d.k;  // nothing stored
  if (pro_out) g_launch_bytes += (dtype == ARGUS_BF16 ? 2.0 : 4.0) * d.n * d.h * d.w * d.c;  // x' stored
  const Policy pol = policy_of(d);
  if (f8 && sc) {
    int f8f, f8d;
    wp_f8_layouts(d, f8f, f8d);
    if (f8f) { set_error("conv_fwd: an fp8 forward takes no BN+ReLU prologue"); return ARGUS_ERR_ARG; }
  }
  // argus_conv_fwd_fin: the statistics finalize, folded into the launch where its planner allows
  g_ffin_folded = 0;
  BnFwdFin ff{};
  if (fin && stats) {
    ff.mode = 1;
    ff.C = d.k;
    ff.count = (long long)d.n * d.ho * d.wo;
    ff.cnt = reinterpret_cast<unsigned*>(fin->workspace);
    ff.red = reinterpret_cast<double2*>(reinterpret_cast<char*>(fin->workspace) + kBnCounterBytes);
    ff.gamma = fin->gamma; ff.beta = fin->beta; ff.eps = fin->eps; ff.momentum = fin->momentum;
    ff.running_mean = fin->running_mean; ff.running_var = fin->running_var;
    ff.nbt = reinterpret_cast<long long*>(fin->num_batches_tracked);
    ff.mean_o = fin->mean; ff.invstd_o = fin->invstd; ff.scale_o = fin->scale; ff.shift_o = fin->shift;
  }
  const BnFwdFin* ffp = ff.mode ? &ff : nullptr;
  if (stem_lds_fwd(d, dtype, pol) && stem_fwd_launch(d, dtype, x, w, y, stats, st, ffp))  // stem.hip (bf16)
    return check_launch("stem_fwd_kernel");
  if (!y && !sc && p1x1_fwd_stats_ok(d, dtype, pol[kP1x1FwdStats]))  // statistics only: conv_p1x1.hip
    return p1x1_fwd_stats_launch(d, x, w, stats, st, ffp);
  IgParams p;
  fwd_params(d, pol, p);
  p.ffin = ff;
  p.a = x; p.b = w; p.c = y; p.pro_scale = sc; p.pro_shift = sh; p.pro_out = pro_out;
  p.stats = reinterpret_cast<float2*>(stats);
  const int bm = fwd_bm(d, pol), bn = d.stem ? 64 : pick_bn(pol, 0, d.k);
  p.stat_tile = bm;
  p.f8 = f8;
  return dtype == ARGUS_BF16 ? run_ig<bf16>(p, st, bm, bn) : run_ig<float>(p, st, bm, bn);
}

int conv_fwd_bn_out(const argus_conv_desc& d, int dtype, const void* x, const void* w, const float* sc,
                    const float* sh, const void* res, const float* rsc, const float* rsh, void* out, uint8_t* bits,
                    void* y, hipStream_t st) {
  if (int e = check_desc(d)) return e;
  if (dtype != ARGUS_BF16 || d.stem || d.r != 1 || d.s != 1 || d.stride != 1 || d.pad != 0 || d.k % 64) {
    set_error("conv_fwd_bn_out: bf16 1x1 stride-1 convs only");
    return ARGUS_ERR_ARG;
  }
  if (!x || !w || !sc || !sh || !res || !out || !bits || (rsc == nullptr) != (rsh == nullptr)) {
    set_error("conv_fwd_bn_out: null operand");
    return ARGUS_ERR_ARG;
  }
  const double px = (double)d.n * d.ho * d.wo;
  g_launch_work = 2.0 * px * d.k * d.c;
  g_launch_bytes = 2.0 * (px * d.c + (double)d.k * d.c + px * d.k * (y ? 3 : 2)) + px * d.k / 8;
  const Policy pol = policy_of(d);
  IgParams p;
  fwd_params(d, pol, p);
  p.a = x; p.b = w; p.c = y;
  p.oe.sc = sc; p.oe.sh = sh; p.oe.res = res; p.oe.rsc = rsc; p.oe.rsh = rsh; p.oe.out = out; p.oe.bits = bits;
  const int bm = fwd_bm(d, pol), bn = pick_bn(pol, 0, d.k);
  p.stat_tile = bm;
  return run_ig<bf16>(p, st, bm, bn);
}

static void dgrad_params(const argus_conv_desc& d, const Policy& pol, const void* dy, const void* wt, void* dx,
                         const void* addend, const uint8_t* addend_mask, IgParams& p) {
  p = IgParams{};
  p.pol = &pol;
  p.ksz = d.r;
  p.a = dy; p.b = wt; p.c = dx;
  p.N = d.c; p.Cin = d.k; p.lda = d.k; p.H = d.ho; p.W = d.wo; p.ish = 1; p.isw = 1;
  p.Ho = d.h; p.Wo = d.w; p.osh = d.stride; p.osw = d.stride; p.ldc = d.c; p.ldb = d.r * d.s * d.k;
  p.addend = addend; p.addend_mask = addend_mask; p.stem = 0;
  const int s = d.stride;
  int np = 0;
  for (int phh = 0; phh < s; ++phh)
    for (int pww = 0; pww < s; ++pww) {
      IgPhase& ph = p.ph[np++];
      ph.Hq = cdiv(d.h - phh, s); ph.Wq = cdiv(d.w - pww, s);
      ph.oh0 = phh; ph.ow0 = pww; ph.M = d.n * ph.Hq * ph.Wq;
      int t = 0;
      for (int r = 0; r < d.r; ++r) {
        const int a = phh + d.pad - r;
        if (((a % s) + s) % s) continue;
        for (int c = 0; c < d.s; ++c) {
          const int b = pww + d.pad - c;
          if (((b % s) + s) % s) continue;
          ph.dh[t] = a / s; ph.dw[t] = b / s;  // exact division (a, b divisible by s)
          ph.boff[t] = (r * d.s + c) * d.k;
          ++t;
        }
      }
      ph.K = t * d.k;
    }
  p.nphase = np;
}

// BN-backward partial rows per phase of the kernel run_ig will choose for these dgrad params
static int dgrad_prow(const IgParams& p, int dtype) {
  int maxM = 0, maxK = 0;
  for (int i = 0; i < p.nphase; ++i) {
    maxM = p.ph[i].M > maxM ? p.ph[i].M : maxM;
    maxK = p.ph[i].K > maxK ? p.ph[i].K : maxK;
  }
  if (p.x8) return conv3x3_halo_tiles(p);
  if (dtype == ARGUS_BF16 && !f8_ok(p) && !p.bb.yx) {
    if (conv3x3_halo_ok(p)) return conv3x3_halo_tiles(p);
    if (igemm_glds_ok(p, maxM, maxK)) return cdiv(maxM, 256);
  }
  return cdiv(maxM, dgrad_bm(*p.pol));
}

static void dgrad_work(const argus_conv_desc& d, int dtype, bool addend, bool mask, bool bn, bool dual) {
  const double E = dtype == ARGUS_BF16 ? 2.0 : 4.0;
  const double px_in = (double)d.n * d.h * d.w * d.c;
  g_launch_work = 2.0 * d.n * d.ho * d.wo * d.k * d.r * d.s * d.c;  // algorithmic flops / bytes (ktimer)
  g_launch_bytes = E * ((double)d.n * d.ho * d.wo * d.k + (double)d.k * d.r * d.s * d.c +
                        (addend ? 2.0 : 1.0) * px_in) +
                   (mask ? px_in / (dtype == ARGUS_BF16 ? 8 : 4) : 0.0) +
                   (bn ? E * px_in * (dual ? 2.0 : 1.0) : 0.0);  // BN input(s) y read by the epilogue
}

int conv_dgrad(const argus_conv_desc& d, int dtype, const void* dy, const void* wt, void* dx,
               const void* addend, const uint8_t* addend_mask, hipStream_t st) {
  if (int e = check_desc(d)) return e;
  const bool f8 = dtype == ARGUS_FP8;
  if (f8) dtype = ARGUS_BF16;
  dgrad_work(d, dtype, addend != nullptr, addend_mask != nullptr, false, false);
  if (d.stem) { set_error("conv_dgrad: the stem input has no gradient"); return ARGUS_ERR_ARG; }
  const Policy pol = policy_of(d);
  IgParams p;
  dgrad_params(d, pol, dy, wt, dx, addend, addend_mask, p);
  p.f8 = f8;
  const int bm = dgrad_bm(pol), bn = pick_bn(pol, 1, d.c);
  return dtype == ARGUS_BF16 ? run_ig<bf16>(p, st, bm, bn) : run_ig<float>(p, st, bm, bn);
}

int conv_dgrad_bn_rows(const argus_conv_desc& d, int dtype) {
  if (check_desc(d) || d.stem) return -1;
  const Policy pol = policy_of(d);
  IgParams p;
  dgrad_params(d, pol, nullptr, nullptr, nullptr, nullptr, nullptr, p);
  p.f8 = dtype == ARGUS_FP8;
  return p.nphase * dgrad_prow(p, p.f8 ? ARGUS_BF16 : dtype);
}

// Whether argus_conv_dgrad_bn stages the apply prologue inside the (register-staged) dgrad kernel:
// the halo / glds kernels (LDS DMA, no staging transform) get dy materialised by the apply kernel
// first, and a 3x3 dgrad would stage each dy element once per tap (9x the apply work, measured slower
// than the separate pass), so only 1x1 dgrads on the register-staged kernel stage it.
static bool dgrad_stages_prologue(const argus_conv_desc& d, int dtype, IgParams& p) {
  if (d.r != 1 || d.s != 1) return false;
  if (f8_ok(p)) return true;  // the fp8 register-staged kernel stages the apply, then quantizes
  int maxM = 0, maxK = 0;
  for (int i = 0; i < p.nphase; ++i) {
    maxM = p.ph[i].M > maxM ? p.ph[i].M : maxM;
    maxK = p.ph[i].K > maxK ? p.ph[i].K : maxK;
  }
  if ((*p.pol)[kDgradApStaged]) return true;  // the glds kernel is not used: no dy to materialise
  if (dtype == ARGUS_BF16 && (conv3x3_halo_ok(p) || igemm_glds_ok(p, maxM, maxK))) return false;
  // key 49: every 128-column tile of the dgrad (d.c / 128 of them) redoes the apply of the same A rows
  // (the register-staged igemm and the persistent conv1 kernel alike); past that many tiles the apply
  // kernel materialises dy once instead (0: no limit)
  const int maxcols = (*p.pol)[kDgradApMaxCols];
  return !(dtype == ARGUS_BF16 && maxcols > 0 && d.c / 128 > maxcols);
}

int conv_dgrad_stages_prologue(const argus_conv_desc& d, int dtype) {
  if (check_desc(d) || d.stem) return 0;
  const Policy pol = policy_of(d);
  IgParams p;
  dgrad_params(d, pol, nullptr, nullptr, nullptr, nullptr, nullptr, p);
  p.f8 = dtype == ARGUS_FP8;
  return dgrad_stages_prologue(d, p.f8 ? ARGUS_BF16 : dtype, p) ? 1 : 0;
}

static int dgrad_bn_impl(const argus_conv_desc& d, int dtype, const void* dy, const void* wt, void* dm,
                         const void* addend, const argus_bn_bwd_epilogue* bn, const argus_bn_bwd_prologue* pro,
                         bool x8, hipStream_t st) {
  if (int e = check_desc(d)) return e;
  const bool f8 = dtype == ARGUS_FP8;
  if (f8) dtype = ARGUS_BF16;
  if (d.stem) { set_error("conv_dgrad_bn: the stem input has no gradient"); return ARGUS_ERR_ARG; }
  static const argus_bn_bwd_epilogue no_epilogue = {};
  const bool epi = bn != nullptr;
  if (!epi) bn = &no_epilogue;
  const bool yrec = epi && bn->y_x;
  if (yrec && (dtype != ARGUS_BF16 || bn->y || !bn->y_w || bn->mask_mode != 3 || bn->y_k <= 0 || bn->y_k % 64)) {
    set_error("conv_dgrad_bn: y recompute needs bf16, mask mode 3, y == NULL, y_w and y_k % 64 == 0");
    return ARGUS_ERR_ARG;
  }
  if ((epi && ((!bn->y && !yrec) || !bn->mean || !bn->invstd || !bn->part || (bn->mask_mode != 2 && bn->mask_mode != 3))) ||
      (bn->mask_mode == 2 && (!bn->scale || !bn->shift || bn->y2)) || (bn->mask_mode == 3 && !bn->mask_bits) ||
      (bn->y2 && (!bn->mean2 || !bn->invstd2 || !bn->part2)) || (bn->y && bn->y == dm)) {
    set_error("conv_dgrad_bn: bad BN-backward epilogue arguments");
    return ARGUS_ERR_ARG;
  }
  if (pro && (!pro->y || !pro->ca || !pro->cb || !pro->cc || (pro->dy_out && (pro->dy_out == dy || pro->dy_out == dm)))) {
    set_error("conv_dgrad_bn: bad apply-prologue arguments");
    return ARGUS_ERR_ARG;
  }
  const Policy pol = policy_of(d);
  if (x8 && (pro || yrec || addend || (epi && bn->mask_mode != 2))) {
    set_error("conv_dgrad_bn_x8: no apply prologue, addend or y recompute; BN epilogue mask mode 2 only");
    return ARGUS_ERR_ARG;
  }
  // the persistent conv1 data gradient (conv_p1x1.hip): the same dm bits, fewer partial rows
  if (!x8 && pol[kP1x1Dgrad] && epi && !yrec && bn->mask_mode == 3 && pro && !pro->dy_out && p1x1_ok(d, dtype) &&
      !(f8 && (pol[kFp8Passes] & 4)) && bn->workspace && bn->gamma && bn->ca && bn->cb && bn->cc &&
      (!bn->y2 || (bn->gamma2 && bn->ca2 && bn->cb2 && bn->cc2))) {
    dgrad_work(d, dtype, addend != nullptr, true, true, bn->y2 != nullptr);
    g_launch_bytes += 2.0 * d.n * d.ho * d.wo * d.k;  // the apply's y
    return p1x1_launch(d, dy, wt, dm, addend, bn, pro, st);
  }
  IgParams p;
  dgrad_params(d, pol, dy, wt, dm, addend, nullptr, p);
  p.f8 = f8 && !yrec;
  if (x8) {
    int f8f, f8d;
    wp_f8_layouts(d, f8f, f8d);
    p.x8 = 1;
    p.bb.mode = epi ? 2 : 0;  // (the shape check below sees the epilogue variant)
    if (!f8d || !conv3x3_halo_x8_ok(p)) {
      set_error("conv_dgrad_bn_x8: not served (3x3 stride-1 halo shapes, K % 128, MX-fp8 dgrad weights: "
                "policy key 37 bit 2)");
      return ARGUS_ERR_ARG;
    }
    p.bb.mode = 0;
  }
  if (yrec) { p.bb.yx = bn->y_x; p.bb.yw = bn->y_w; p.bb.yk = bn->y_k; }
  if (pro) {
    // the register-staged kernel stages dy = ca*dm + cb*y + cc itself; the halo / glds kernels (LDS
    // DMA, no staging transform) get it materialised by the apply kernel first
    if (!dgrad_stages_prologue(d, dtype, p)) {
      if (!pro->dy_out) {
        set_error("conv_dgrad_bn: this dgrad cannot stage the apply prologue; dy_out is required");
        return ARGUS_ERR_ARG;
      }
      if (int e = argus_bn_bwd_apply(dtype, (int64_t)d.n * d.ho * d.wo, d.k, dy, 0, nullptr, pro->y, nullptr,
                                     nullptr, pro->ca, pro->cb, pro->cc, pro->dy_out, nullptr, nullptr, nullptr,
                                     nullptr, nullptr, nullptr, st))
        return e;
      p.a = pro->dy_out;
    } else {
      p.ap.y = pro->y; p.ap.ca = pro->ca; p.ap.cb = pro->cb; p.ap.cc = pro->cc; p.ap.out = pro->dy_out;
    }
  }
  dgrad_work(d, dtype, addend != nullptr, bn->mask_mode == 3, epi, bn->y2 != nullptr);
  if (x8)  // dy and the weights as e4m3 + E8M0 scales
    g_launch_bytes -= (double)d.n * d.ho * d.wo * d.k * (2.0 - 33.0 / 32) + (double)d.k * 9 * d.c * (2.0 - 33.0 / 32);
  if (yrec) {  // y not read: its producing conv's input instead (+ the recompute flops)
    g_launch_bytes -= 2.0 * (double)d.n * d.h * d.w * (d.c - bn->y_k);
    g_launch_work += 2.0 * d.n * d.h * d.w * d.c * bn->y_k;
  }
  if (p.ap.y)  // y in (+ dy out)
    g_launch_bytes += (dtype == ARGUS_BF16 ? 2.0 : 4.0) * (p.ap.out ? 2.0 : 1.0) * d.n * d.ho * d.wo * d.k;
  BnBwdEpi& b = p.bb;
  b.y = bn->y; b.mean = bn->mean; b.invstd = bn->invstd; b.sc = bn->scale; b.sh = bn->shift;
  b.bits = bn->mask_bits; b.y2 = bn->y2; b.mean2 = bn->mean2; b.invstd2 = bn->invstd2;
  b.part = reinterpret_cast<float2*>(bn->part); b.part2 = reinterpret_cast<float2*>(bn->part2);
  b.mode = bn->mask_mode;
  b.prow = dgrad_prow(p, dtype);
  if (bn->workspace) {  // the BN-backward finalize folded into this launch
    if (!bn->gamma || !bn->ca || !bn->cb || !bn->cc || (bn->y2 && (!bn->gamma2 || !bn->ca2 || !bn->cb2 || !bn->cc2)) ||
        d.c / 64 * 65 * 4 > (int)kBnCounterBytes) {
      set_error("conv_dgrad_bn: bad finalize arguments");
      return ARGUS_ERR_ARG;
    }
    BnFin& f = p.fin;
    f.mode = 2; f.C = d.c; f.count = (long long)d.n * d.h * d.w;
    f.cnt = reinterpret_cast<unsigned*>(bn->workspace);
    f.red = reinterpret_cast<double2*>(reinterpret_cast<char*>(bn->workspace) + kBnCounterBytes);
    f.part = reinterpret_cast<const float2*>(bn->part); f.part2 = reinterpret_cast<const float2*>(bn->part2);
    f.gamma = bn->gamma; f.bmean = bn->mean; f.binvstd = bn->invstd;
    f.dgamma = bn->dgamma; f.dbeta = bn->dbeta; f.ca = bn->ca; f.cb = bn->cb; f.cc = bn->cc;
    f.gamma2 = bn->gamma2; f.bmean2 = bn->mean2; f.binvstd2 = bn->invstd2;
    f.dgamma2 = bn->dgamma2; f.dbeta2 = bn->dbeta2; f.ca2 = bn->ca2; f.cb2 = bn->cb2; f.cc2 = bn->cc2;
  }
  const int bm = dgrad_bm(pol), bn_ = pick_bn(pol, 1, d.c);
  return dtype == ARGUS_BF16 ? run_ig<bf16>(p, st, bm, bn_) : run_ig<float>(p, st, bm, bn_);
}

int conv_dgrad_bn(const argus_conv_desc& d, int dtype, const void* dy, const void* wt, void* dm,
                  const void* addend, const argus_bn_bwd_epilogue* bn, const argus_bn_bwd_prologue* pro,
                  hipStream_t st) {
  return dgrad_bn_impl(d, dtype, dy, wt, dm, addend, bn, pro, false, st);
}

int conv_dgrad_bn_x8(const argus_conv_desc& d, const void* dy8, const void* wt, void* dm, const argus_bn_bwd_epilogue* bn,
                     hipStream_t st) {
  return dgrad_bn_impl(d, ARGUS_FP8, dy8, wt, dm, nullptr, bn, nullptr, true, st);
}

// MX-fp8 stored-operand forward (argus_conv_fwd_x8): the input as e4m3 [P][C] + E8M0 [P][C/32] (the
// x8 copy argus_bn_apply_x8 writes beside the bf16 activation), the forward weights in the fp8 layout
// (policy key 37 bit 8 or 1), bf16 y and the BN statistics partials as argus_conv_fwd
int conv_fwd_x8(const argus_conv_desc& d, const void* x8, const void* w, void* y, float* stats, hipStream_t st) {
  if (int e = check_desc(d)) return e;
  if (!x8 || !w || !y) { set_error("conv_fwd_x8: bad arguments"); return ARGUS_ERR_ARG; }
  const Policy pol = policy_of(d);
  int f8f, f8d;
  wp_f8_layouts(d, f8f, f8d);
  IgParams p;
  fwd_params(d, pol, p);
  p.a = x8; p.b = w; p.c = y;
  p.stats = reinterpret_cast<float2*>(stats);
  p.stat_tile = fwd_bm(d, pol);
  p.f8 = 1;
  p.x8 = 1;
  if (d.stem || !f8f || !conv3x3_halo_x8_ok(p)) {
    set_error("conv_fwd_x8: not served (3x3 stride-1 halo shapes, C % 128, MX-fp8 forward weights: policy key 37 "
              "bit 8)");
    return ARGUS_ERR_ARG;
  }
  const double px = (double)d.n * d.ho * d.wo;
  g_launch_work = 2.0 * px * d.k * 9 * d.c;
  g_launch_bytes = 33.0 / 32 * ((double)d.n * d.h * d.w * d.c + (double)d.k * 9 * d.c) + 2.0 * px * d.k +
                   (stats ? 8.0 * conv_fwd_stat_rows(d, ARGUS_FP8) * d.k : 0.0);
  return run_ig<bf16>(p, st, p.stat_tile, 128);
}

// 1 when argus_conv_fwd_x8 (pass 0) / argus_conv_dgrad_bn_x8 (pass 1) serves conv d under its policy
int conv_x8_ok(const argus_conv_desc& d, int pass) {
  if (check_desc(d) || d.stem) return 0;
  const Policy pol = policy_of(d);
  int f8f, f8d;
  wp_f8_layouts(d, f8f, f8d);
  IgParams p;
  if (pass == 0) {
    fwd_params(d, pol, p);
    if (!f8f) return 0;
  } else {
    dgrad_params(d, pol, nullptr, nullptr, nullptr, nullptr, nullptr, p);
    if (!f8d) return 0;
  }
  p.x8 = 1;
  return conv3x3_halo_x8_ok(p) ? 1 : 0;
}

struct WgPlan {
  int bm, bn, mt, nt, splits, pps, kstep;
  int N;
};

// ap: the BN-backward-apply form (argus_conv_wgrad_apply), which may pick another DMA tile width
static WgPlan wgrad_plan(const argus_conv_desc& d, int dtype, bool ap = false) {
  const Policy pol = policy_of(d);
  WgPlan pl;
  pl.N = d.stem ? 256 : d.r * d.s * d.c;
  pl.bm = (pol[kForceBm + 2] == 64 || d.k % 128) ? 64 : 128;
  pl.bn = pick_bn(pol, 2, pl.N);
  if (d.stem) { pl.bm = 64; pl.bn = 128; }
  pl.mt = d.k / pl.bm;
  pl.nt = pl.N / pl.bn;
  pl.kstep = dtype == ARGUS_BF16 ? 64 : 32;
  const long P = (long)d.n * d.ho * d.wo;
  // the plain 128 x 256 DMA kernel runs two workgroups per CU: the target counts its wider tiles (the
  // apply form's runs one per CU, so the 128 x 128 count, i.e. half the grid, is its target)
  const bool wide2 = !ap && wgrad_dma_width(d, dtype, pl.bm, pl.bn, pol[kWgradDma], false, pol[kWgradDmaGather]) == 256;
  const long tiles = (long)pl.mt * (wide2 ? pl.nt / 2 : pl.nt);
  // measured (tools/tilesweep.py, MI355X): 1x1 convs peak near 512 workgroups, 3x3 near 1024
  // (2048 when Cout = 64: one row tile, 9 column tiles)
  long target = pol[kWgradTarget];
  if (target == 512 && d.r == 3) target = d.k <= 64 ? 2048 : pol[kWgradTarget3x3];
  // key 46: 1x1 weight gradients over few pixels take half the split target: the side stream then
  // holds fewer CUs beside the main stream's chain, and writes half the split partials
  if (target == 512 && d.r == 1 && P <= pol[kWgradSmallP]) target = 256;
  // the grid (tiles x splits) stays within the target: a grid just past it (e.g. 36 tiles x 15 splits
  // = 540 for 512 two-per-CU slots) runs a second, nearly empty round of workgroups
  long splits = target / tiles;
  const long max_splits = (P + pl.kstep * 4 - 1) / (pl.kstep * 4);  // >= 4 k-steps per split
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  long pps = (P + splits - 1) / splits;
  pps = (pps + pl.kstep - 1) / pl.kstep * pl.kstep;
  splits = (P + pps - 1) / pps;
  pl.splits = (int)splits;
  pl.pps = (int)pps;
  return pl;
}

size_t conv_wgrad_ws(const argus_conv_desc& d, int dtype) {
  if (check_desc(d)) return 0;
  const WgPlan pl = wgrad_plan(d, dtype), pla = wgrad_plan(d, dtype, true);
  size_t b = (size_t)(pl.splits > pla.splits ? pl.splits : pla.splits) * d.k * pl.N * sizeof(float);
  int hs, htps;
  if (stem_wgrad_plan(d, dtype, &hs, &htps)) {
    const size_t sb = (size_t)hs * 64 * 256 * sizeof(float);
    b = sb > b ? sb : b;
  }
  if (wgrad3x3_halo_plan(d, dtype, &hs, &htps)) {
    const size_t hb = (size_t)hs * d.k * 9 * d.c * sizeof(float);
    b = hb > b ? hb : b;
  }
  // + the folded reduction's counters (key 50): the last kWgFoldCtrBytes, past every kernel's partials
  return b + kWgFoldCtrBytes;
}

template <typename T, int BM, int BN, bool STEM, bool PRO, bool FAST, bool AP>
static const char* wg_name() {
  static const std::string s = std::string("argus::wgrad_kernel<") + type_name<T>() + ", " + std::to_string(BM) +
                               ", " + std::to_string(BN) + ", " + bool_name(STEM) + ", " + bool_name(PRO) + ", " +
                               bool_name(FAST) + ", " + bool_name(AP) + ">";
  return s.c_str();
}

template <typename T, int BM, int BN, bool STEM, bool PRO, bool FAST, bool AP = false>
static void launch_wg(const WgParams& p, const WgPlan& pl, hipStream_t st) {
  timed_launch(wg_name<T, BM, BN, STEM, PRO, FAST, AP>(), wgrad_kernel<T, BM, BN, STEM, PRO, FAST, AP>,
               dim3(pl.mt * pl.nt * pl.splits), dim3(256), st, p);
}

template <typename T, bool PRO, bool FAST, bool AP = false>
static void dispatch_wg_tiles(const WgParams& p, const WgPlan& pl, hipStream_t st) {
  if (pl.bm == 128 && pl.bn == 128) launch_wg<T, 128, 128, false, PRO, FAST, AP>(p, pl, st);
  else if (pl.bm == 128) launch_wg<T, 128, 64, false, PRO, FAST, AP>(p, pl, st);
  else if (pl.bn == 128) launch_wg<T, 64, 128, false, PRO, FAST, AP>(p, pl, st);
  else launch_wg<T, 64, 64, false, PRO, FAST, AP>(p, pl, st);
}

template <typename T>
static void dispatch_wg(const WgParams& p, const WgPlan& pl, hipStream_t st) {
  // FAST pixel indexing: every k-step lies in one image and rows tile the k-step evenly
  const int bkp = pl.kstep;
  const bool fast = (p.Ho * p.Wo) % bkp == 0 && (p.Wo % bkp == 0 || bkp % p.Wo == 0);
  if (p.stem) {  // stem: M = 64 channels, N = 256; with the BN-backward apply of dy staged (AP) or not
    if (p.ap_y) {
      if (fast) launch_wg<T, 64, 128, true, false, true, true>(p, pl, st);
      else launch_wg<T, 64, 128, true, false, false, true>(p, pl, st);
    } else {
      if (fast) launch_wg<T, 64, 128, true, false, true>(p, pl, st);
      else launch_wg<T, 64, 128, true, false, false>(p, pl, st);
    }
  } else if (p.ap_y) {  // the BN-backward apply of dy staged from dm (argus_conv_wgrad_apply)
    if (fast) dispatch_wg_tiles<T, false, true, true>(p, pl, st);
    else dispatch_wg_tiles<T, false, false, true>(p, pl, st);
  } else if (p.pro_scale) {
    if (fast) dispatch_wg_tiles<T, true, true>(p, pl, st);
    else dispatch_wg_tiles<T, true, false>(p, pl, st);
  } else {
    if (fast) dispatch_wg_tiles<T, false, true>(p, pl, st);
    else dispatch_wg_tiles<T, false, false>(p, pl, st);
  }
}

// ap != nullptr: argus_conv_wgrad_apply (dy staged as ca*dm + cb*y + cc from dm = `dy`)
static int conv_wgrad_impl(const argus_conv_desc& d, int dtype, const void* x, const float* sc, const float* sh,
                           const void* dy, const argus_bn_bwd_prologue* ap, float* dw, void* ws, size_t ws_bytes,
                           hipStream_t st) {
  if (int e = check_desc(d)) return e;
  const Policy pol = policy_of(d);
  g_launch_work = 2.0 * d.n * d.ho * d.wo * d.k * d.r * d.s * d.c;  // algorithmic flops / bytes (ktimer)
  const WgPlan pl = wgrad_plan(d, dtype, ap != nullptr);
  // algorithmic bytes: x + dy read once, the fp32 dW written once (the split partials and their
  // reduction are this implementation's overhead, visible in the PMC traffic, not algorithmic work)
  g_launch_bytes = (double)(dtype == ARGUS_BF16 ? 2 : 4) *
                       ((double)d.n * d.h * d.w * (d.stem ? 4 : d.c) + (double)d.n * d.ho * d.wo * d.k) +
                   4.0 * d.k * d.r * d.s * d.c;
  if (ws_bytes < (size_t)pl.splits * d.k * pl.N * sizeof(float)) {
    set_error("conv_wgrad: workspace too small");
    return ARGUS_ERR_ARG;
  }
  WgParams p = {};
  p.x = x; p.dy = dy; p.pro_scale = sc; p.pro_shift = sh; p.part = reinterpret_cast<float*>(ws);
  if (ap) {
    p.ap_y = ap->y; p.ap_ca = ap->ca; p.ap_cb = ap->cb; p.ap_cc = ap->cc;
    g_launch_bytes += (dtype == ARGUS_BF16 ? 2.0 : 4.0) * (double)d.n * d.ho * d.wo * d.k;  // y of the apply
  }
  p.M = d.k; p.N = pl.N; p.Cin = d.stem ? 4 : d.c; p.lda = d.stem ? 4 : d.c;
  p.H = d.h; p.W = d.w; p.Ho = d.ho; p.Wo = d.wo; p.stride = d.stride; p.pad = d.pad; p.S = d.s;
  p.P = d.n * d.ho * d.wo; p.pps = pl.pps; p.stem = d.stem;
  // a split's tiles on one XCD for the 1x1 convs and the stem (its two 128-column tiles then share the
  // XCD's L2 copy of the split's dy: read once from HBM, not twice); 3x3: spread (measured faster)
  p.group = (d.s == 1 && pl.N == d.c) || d.stem ? 1 : 0;
  p.fd_hw = make_fastdiv(d.ho * d.wo); p.fd_w = make_fastdiv(d.wo);
  if (d.stem && sc) { set_error("conv_wgrad: stem has no prologue"); return ARGUS_ERR_ARG; }
  int splits = pl.splits;
  if (d.stem && pol[kStemLdsWgrad] && stem_wgrad_launch(d, dtype, x, dy, ap, ws, ws_bytes, &splits, st)) {
    if (int e = check_launch("stem_wgrad_kernel")) return e;
  } else if (!sc && wgrad_dma_ok(d, dtype, pl.bm, pl.bn, pol[kWgradDma], ap != nullptr, pol[kWgradDmaGather])) {
    // key 50: the split sum folded into the launch (its last kWgFoldCtrBytes of ws hold the counters,
    // zero before the first launch; every launch leaves them zero)
    const int ft = wgrad_dma_fold_tiles(d, pol[kWgradDma], pol[kWgradDmaGather], ap != nullptr);
    const size_t need = (size_t)pl.splits * d.k * pl.N * sizeof(float);
    const bool fold = pol[kWgradFold] && ft > 0 && (2 * ft + 1) * 4 <= (int)kWgFoldCtrBytes &&
                      ws_bytes >= need + kWgFoldCtrBytes;
    if (fold) {
      p.fold.cnt = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(ws) + ((ws_bytes - kWgFoldCtrBytes) & ~(size_t)255));
      p.fold.dw = dw;
      p.fold.sl = wgrad_reduce_lanes(d.k, pl.N);
    }
    wgrad_dma_launch(d, p, pol[kWgradDma], pol[kWgradDmaGather], pl.splits, pol[kWgradDmaStages], st);  // LDS-DMA ring
    if (int e = check_launch("wgrad_dma_kernel")) return e;
    if (fold) return ARGUS_OK;
  } else if (ap) {  // the register-staged kernel stages the apply; no halo / glds variant does
    if (dtype == ARGUS_BF16) dispatch_wg<bf16>(p, pl, st);
    else dispatch_wg<float>(p, pl, st);
    if (int e = check_launch("wgrad_kernel")) return e;
  } else if (wgrad3x3_halo_launch(d, dtype, x, sc, sh, dy, ws, ws_bytes, &splits, st)) {
    if (int e = check_launch("wgrad3x3_halo_kernel")) return e;
  } else {
    if (dtype == ARGUS_BF16) dispatch_wg<bf16>(p, pl, st);
    else dispatch_wg<float>(p, pl, st);
    if (int e = check_launch("wgrad_kernel")) return e;
  }
  return wgrad_reduce_launch(reinterpret_cast<const float*>(ws), splits, d.k, pl.N, d.stem, dw, st);
}

int conv_wgrad(const argus_conv_desc& d, int dtype, const void* x, const float* sc, const float* sh,
               const void* dy, float* dw, void* ws, size_t ws_bytes, hipStream_t st) {
  return conv_wgrad_impl(d, dtype, x, sc, sh, dy, nullptr, dw, ws, ws_bytes, st);
}

int conv_wgrad_apply(const argus_conv_desc& d, int dtype, const void* x, const void* dm,
                     const argus_bn_bwd_prologue& ap, float* dw, void* ws, size_t ws_bytes, hipStream_t st) {
  if (!ap.y || !ap.ca || !ap.cb || !ap.cc) { set_error("conv_wgrad_apply: bad apply arguments"); return ARGUS_ERR_ARG; }
  return conv_wgrad_impl(d, dtype, x, nullptr, nullptr, dm, &ap, dw, ws, ws_bytes, st);
}

int conv_launch_info(const argus_conv_desc& d, int dtype, int pass, int64_t* flops) {
  if (check_desc(d)) return -1;
  const Policy pol = policy_of(d);
  if (flops) *flops = 2LL * d.n * d.ho * d.wo * d.k * d.r * d.s * d.c;
  const int dtag = (dtype == ARGUS_BF16 || dtype == ARGUS_FP8) ? 1 : 0;
  if (pass == 0) return 10000000 + dtag * 1000000 + fwd_bm(d, pol) * 1000 + (d.stem ? 64 : pick_bn(pol, 0, d.k));
  if (pass == 1) return 10000000 + dtag * 1000000 + dgrad_bm(pol) * 1000 + pick_bn(pol, 1, d.c);
  const WgPlan pl = wgrad_plan(d, dtype);
  return 20000000 + dtag * 1000000 + pl.bm * 1000 + pl.bn;
}

int conv_weight_prep(const argus_conv_desc& d, int dtype, const float* w, const int64_t* strides, void* wf,
                     void* wd, hipStream_t st) {
  if (int e = check_desc(d)) return e;
  WStrides ws;
  if (strides) {
    ws = {strides[0], strides[1], strides[2], strides[3]};
  } else {  // OHWI contiguous
    ws = {(long long)d.r * d.s * d.c, 1, (long long)d.s * d.c, d.c};
  }
  if (d.stem && !wf) { set_error("weight_prep: stem needs w_fwd"); return ARGUS_ERR_ARG; }
  if (dtype == ARGUS_FP8) {  // the MX-fp8 layout where a pass takes fp8 operands (weight_prep_tile)
    if (!wf) { set_error("weight_prep: fp8 needs w_fwd"); return ARGUS_ERR_ARG; }
    WpEntry e{w, ws.sk, ws.sc, ws.sr, ws.ss, wf, d.stem ? nullptr : wd, d.k, d.r, d.s, d.c, d.stem, 0, 0, 0};
    wp_f8_layouts(d, e.f8f, e.f8d);
    hipLaunchKernelGGL(weight_prep_one_f8_kernel, dim3(wp_blocks(d.k, d.r, d.s, d.c, d.stem)), dim3(256), 0, st, e);
    return check_launch("weight_prep_one_f8_kernel");
  }
  const int total = d.stem ? d.k * 256 : d.k * d.r * d.s * d.c;
  const int blocks = std::min(cdiv(total, 256), 4096);
  if (dtype == ARGUS_BF16)
    hipLaunchKernelGGL(weight_prep_kernel<bf16>, dim3(blocks), dim3(256), 0, st, w, ws, (bf16*)wf,
                       (bf16*)(d.stem ? nullptr : wd), d.k, d.r, d.s, d.c, d.stem);
  else
    hipLaunchKernelGGL(weight_prep_kernel<float>, dim3(blocks), dim3(256), 0, st, w, ws, (float*)wf,
                       (float*)(d.stem ? nullptr : wd), d.k, d.r, d.s, d.c, d.stem);
  return check_launch("weight_prep_kernel");
}

size_t conv_weight_prep_table_bytes(int count) { return count > 0 ? (size_t)count * sizeof(WpEntry) : 0; }

int conv_weight_prep_table(int count, const argus_conv_desc* descs, const float* const* w, const int64_t* strides,
                           void* const* wf, void* const* wd, void* host_table, size_t bytes, int* nblocks) {
  if (count <= 0 || !descs || !w || !wf || !host_table || bytes < conv_weight_prep_table_bytes(count)) {
    set_error("conv_weight_prep_table: bad arguments");
    return ARGUS_ERR_ARG;
  }
  WpEntry* tab = reinterpret_cast<WpEntry*>(host_table);
  int blk = 0;
  for (int i = 0; i < count; ++i) {
    const argus_conv_desc& d = descs[i];
    if (int e = check_desc(d)) return e;
    if (!w[i] || !wf[i]) { set_error("conv_weight_prep_table: null pointer"); return ARGUS_ERR_ARG; }
    WpEntry& t = tab[i];
    t.w = w[i];
    if (strides) { t.sk = strides[4 * i]; t.sc = strides[4 * i + 1]; t.sr = strides[4 * i + 2]; t.ss = strides[4 * i + 3]; }
    else { t.sk = (long long)d.r * d.s * d.c; t.sc = 1; t.sr = (long long)d.s * d.c; t.ss = d.c; }
    t.wf = wf[i];
    t.wd = (d.stem || !wd) ? nullptr : wd[i];
    t.K = d.k; t.R = d.r; t.S = d.s; t.C = d.c; t.stem = d.stem; t.blk0 = blk;
    wp_f8_layouts(d, t.f8f, t.f8d);  // used by the ARGUS_FP8 batch only
    if (!d.stem && (d.k % 64 || d.c % 64)) { set_error("conv_weight_prep_table: channels must be multiples of 64"); return ARGUS_ERR_SHAPE; }
    blk += wp_blocks(d.k, d.r, d.s, d.c, d.stem);
  }
  if (nblocks) *nblocks = blk;
  return ARGUS_OK;
}

int conv_weight_prep_batch(int dtype, int count, const void* device_table, int nblocks, hipStream_t st) {
  if (count <= 0 || nblocks <= 0 || !device_table) { set_error("conv_weight_prep_batch: bad arguments"); return ARGUS_ERR_ARG; }
  g_launch_work = 0.0;
  const WpEntry* tab = reinterpret_cast<const WpEntry*>(device_table);
  if (dtype == ARGUS_FP8)
    hipLaunchKernelGGL((weight_prep_batch_kernel<bf16, true>), dim3(nblocks), dim3(256), 0, st, tab, count);
  else if (dtype == ARGUS_BF16)
    hipLaunchKernelGGL((weight_prep_batch_kernel<bf16, false>), dim3(nblocks), dim3(256), 0, st, tab, count);
  else
    hipLaunchKernelGGL((weight_prep_batch_kernel<float, false>), dim3(nblocks), dim3(256), 0, st, tab, count);
  return check_launch("weight_prep_batch_kernel");
}

template <typename In>
static int launch_images(int dtype, int64_t nimg, int h, int w, const In* x, void* out, hipStream_t st) {
  const int64_t total = nimg * h * w;
  const int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  if (dtype == ARGUS_BF16)
    hipLaunchKernelGGL((images_to_nhwc4_kernel<bf16, In>), dim3(blocks), dim3(256), 0, st, x, (bf16*)out, nimg, h * w);
  else
    hipLaunchKernelGGL((images_to_nhwc4_kernel<float, In>), dim3(blocks), dim3(256), 0, st, x, (float*)out, nimg,
                       h * w);
  return check_launch("images_to_nhwc4_kernel");
}

int images_to_nhwc4(int dtype, int64_t nimg, int h, int w, const float* x, void* out, hipStream_t st) {
  return launch_images(dtype, nimg, h, w, x, out, st);
}

int images_u8_to_nhwc4(int dtype, int64_t nimg, int h, int w, const uint8_t* x, void* out, hipStream_t st) {
  return launch_images(dtype, nimg, h, w, x, out, st);
}

}  // namespace argus
