// 3x3 stride-1 pad-1 convolution (forward and dgrad, bf16) with the input tile held in LDS once per
// 64-channel chunk, halo included, and the nine taps read as shifted windows of it.
//
// Why: the implicit GEMM (conv.hip / conv_glds.hip) re-fetches its A tile from L2 once per tap, 9x
// per channel chunk; measured on MI355X (SQ counters, tools/convbench.py) both of those kernels sit
// at ~38 % MFMA utilisation on the 3x3 layers with waves parked on loads, and a 256x128x64 step needs
// ~96 GB/s per CU of L2->LDS traffic against the ~70 GB/s per CU an L2-resident gather sustains
// (MI355X_MICROARCH.md, "Indexed rows: gather into LDS"). With the halo tile, per chunk a workgroup
// loads (rows+2) x (W+2) input pixels once plus 9 weight tiles: L2 intensity ~190 FLOP/B instead of
// ~87.
//
// Geometry: a workgroup owns 256 consecutive output pixels (NHW order) x BN output channels; the 256
// pixels are whole rows of one image (W in {16, 32, 64, ...}) or whole images (H*W in {64, 128}).
// Waves: 4 x (BN/64), each a 64x64 tile of 4x4 v_mfma_f32_16x16x32_bf16. Per chunk cc (64 input
// channels) and tap t, A[m][k] = halo[pos(m) + off(t)][k], B = w[n][tap t][cc*64 + k].
// LDS: two halo images (double-buffered over chunks, 448 positions x 128 B; slot j of position q holds
// channel chunk j ^ swz8(q)) + a 3-stage ring of weight tiles, all filled by global_load_lds_dwordx4
// (lane-linear 1 KB pieces, swizzle on the source address, zero page for halo positions outside the
// image). The input is the materialised BN + ReLU output of the producer (bf16 schedule: engine.py).
#include "common.h"
#include "igemm.h"
#include "internal.h"
#include "ktimer.h"

namespace argus {

namespace {

__device__ __attribute__((aligned(64))) u32x4 halo_zero_page[4];  // zero-initialised (static storage)

template <int N> ARGUS_DEV void waitvm() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
ARGUS_DEV void gl16(const void* src, uint32_t lds_byte_addr) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(uintptr_t)lds_byte_addr, 16, 0,
                                   0);
}
ARGUS_DEV void sbar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

}  // namespace

constexpr int kHaloPos = 448;  // halo positions per image buffer (max (rows+2)*(W+2) over the shapes served)
constexpr int kHaloPos1 = 416;  // single-buffer variant: 2 x (416 x 128 B + 3 x 8 KB weight stages) fit one CU
// F8 variant: 400 positions per halo image (the fp8 shapes: 340 / 324 / 400 at W = 32 / 16x16 / 8x8),
// so two images, their scales and three weight stages fit one CU
constexpr int kHaloPosF8 = 400;
// DEEP variant (policy key 51): 384-position halo images (the 256 x 256 frame's 32- and 16-wide layers
// need 340 / 324) free LDS for a fourth weight stage: 2 x 48 KB + 4 x 16 KB = 160 KB, so three weight
// taps are in flight under each tap's MFMAs instead of two (the loop waits on L2 -> LDS weight latency:
// a 16 KB stage per ~0.4 us tap at one workgroup per CU)
constexpr int kHaloPosDeep = 384;

// HB = halo image buffers: 2 (double-buffered over 64-channel chunks) or 1 (Cin = 64: a single chunk,
// nothing to prefetch; the 64-column tile then fits two workgroups per CU in LDS)
// F8 (round 5): the A operand (the conv input / the data gradient's dy) and the weights are stored in the
// OCP MX-fp8 x8 layout (e4m3 bytes [pixel][C] followed by one E8M0 scale per 32 channels [pixel][C/32],
// written by argus_bn_apply_x8 / argus_bn_bwd_apply_x8 and argus_conv_weight_prep): a 128-channel chunk
// is 128 bytes per halo position (the bf16 chunk's LDS footprint), its E8M0 scales 4 bytes per position
// in their own LDS image, and each tap runs v_mfma_scale_f32_16x16x128_f8f6f4 (K = 128) per 16 x 16 tile:
// twice the bf16 MFMA rate and half its LDS fragment reads per channel. The images hold 400 positions
// (not 448: the fp8 shapes need no more), which leaves room for the scale images and three weight
// stages; a wave whose last halo DMA would cover positions past 400 sends it to a 1 KB dummy slot (every
// wave issues the same DMAs, so the counted waits hold).
template <int N> ARGUS_DEV void waitvm_le(int n) {  // vmcnt(n) for a runtime n <= N (the next lower count)
  if constexpr (N == 0) {
    waitvm<0>();
  } else {
    if (n >= N) waitvm<N>();
    else waitvm_le<N - 1>(n);
  }
}

template <int BN, int BW, int HB, bool F8 = false, bool DEEP = false>
__global__ __launch_bounds__(4 * (BN / 64) * 64, HB == 1 ? 2 : 1) void conv3x3_halo_kernel(const IgParams p) {
  static_assert(!DEEP || (!F8 && HB == 2 && BN == 128), "deep weight ring: the bf16 128-column double-halo form");
  constexpr int WN = BN / 64, NW = 4 * WN, NT = NW * 64;
  constexpr int HPOS = F8 ? kHaloPosF8 : (HB == 1 ? kHaloPos1 : (DEEP ? kHaloPosDeep : kHaloPos));  // per image buffer
  constexpr int HALO = HPOS * 128;              // bytes per halo image
  constexpr int BST = BN * 128;                 // bytes per weight stage
  constexpr int NBS = DEEP ? 4 : 3;             // weight ring stages
  constexpr int CH = F8 ? 128 : 64;             // channels per chunk (128 bytes per halo position either way)
  constexpr int ES = F8 ? 1 : 2;                // bytes per element
  constexpr int HSI = F8 ? (HPOS + 64 * NW - 1) / (64 * NW) : 0;  // halo scale DMAs per wave per chunk
  // F8: E8M0 scales of one halo image (4 per position; padded to whole DMAs, so every wave issues the
  // same number and the counted waits hold) and of one weight stage (4 per row)
  constexpr int HSB = F8 ? HSI * NW * 256 : 0;
  constexpr int BSB = F8 ? BN * 4 : 0;
  constexpr int HS_OFF = HB * HALO + NBS * BST, BS_OFF = HS_OFF + HB * HSB;
  constexpr int DUMMY = BS_OFF + NBS * BSB;  // F8: 1 KB sink of the halo DMAs past HPOS
  constexpr int LD = BN + 8;
  constexpr int EPI = 256 * LD * 2;
  constexpr int MAIN = HB * HALO + NBS * BST + HB * HSB + NBS * BSB + (F8 ? 1024 : 0);
  constexpr int LDS0 = MAIN > EPI ? MAIN : EPI;
  constexpr int RED_B = (NT / (BN / 8)) * BN * 8;  // BN-backward column sums
  constexpr int LDS_BYTES = LDS0 > RED_B ? LDS0 : RED_B;
  constexpr int HG = (HPOS + 8 * NW - 1) / (8 * NW);  // halo glds per wave per chunk
  constexpr int BG = BN * 8 / NT;               // weight glds per wave per tap
  static_assert((F8 || HG * 8 * NW == HPOS) && HPOS % 8 == 0 && BG * NT == BN * 8, "halo / tile partition");
  constexpr int HGC = HG + HSI, BGC = BG + (F8 ? 1 : 0);  // DMAs per wave: one chunk's halo, one tap's weights
  static_assert(!F8 || (BN / NW == 16 && LDS_BYTES <= 163840 && BW != 3 && BW != 4), "fp8 halo: 16 weight rows per wave");
  static_assert(LDS_BYTES <= 163840, "halo LDS");
  __shared__ __attribute__((aligned(1024))) u32x4 lds[LDS_BYTES / 16];

  const IgPhase& ph = p.ph[0];
  const int mtiles = ph.M / 256;
  const int ntiles = p.N / BN;
  const int nwg = mtiles * ntiles;
  if ((int)blockIdx.x >= nwg) return;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - wm * WN;
  const char* __restrict__ X = reinterpret_cast<const char*>(p.a);
  const char* __restrict__ Wt = reinterpret_cast<const char*>(p.b);
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;

  // tile geometry: NI images x R rows x W columns of output = input (stride 1): 256 consecutive pixels
  const int H = p.H, W = p.W, HWi = H * W;
  int NI, R, r0, img0;
  if (HWi >= 256) { NI = 1; R = 256 / W; img0 = (mt * 256) / HWi; r0 = (mt * 256 - img0 * HWi) / W; }
  else { NI = 256 / HWi; R = H; img0 = mt * NI; r0 = 0; }
  const int HWD = W + 2, HR = R + 2, IMGP = HR * HWD;
  const int npos = NI * IMGP;
  const int RTW = R * W;
  auto slot_px = [&](int m) -> long { return (long)mt * 256 + m; };  // output pixel of tile slot m

  // halo glds sources: position q = 8*(i*NW + wave) + lane/8, channel chunk (lane&7)^swz8(q)
  int h_off[HG];
  bool h_ok[HG];
#pragma unroll
  for (int i = 0; i < HG; ++i) {
    const int q = 8 * (i * NW + wave) + (lane >> 3);
    const int ii = q / IMGP, rem = q - ii * IMGP;
    const int hr = rem / HWD, hc = rem - hr * HWD;
    const int ih = r0 + hr - 1, iw = hc - 1;
    h_ok[i] = q < npos && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
    h_off[i] = h_ok[i] ? (((img0 + ii) * H + ih) * W + iw) * p.lda * ES + ((lane & 7) ^ swz8(q)) * 16 : 0;
  }
  const char* b_src[BG];
#pragma unroll
  for (int i = 0; i < BG; ++i) {
    const int row = 8 * (i * NW + wave) + (lane >> 3);
    b_src[i] = Wt + (size_t)(nt * BN + row) * p.ldb * ES + ((lane & 7) ^ swz8(row)) * 16;
  }
  const void* zero = (const void*)halo_zero_page;
  const int nch = p.Cin / CH;
  const int nk = 9 * nch;
  // F8: the scale DMAs (4 bytes a lane): halo position qs = 64*(j*NW + wave) + lane; weight row
  // 16*wave + lane (lanes < 16)
  const uint8_t* XS = reinterpret_cast<const uint8_t*>(p.a) + (size_t)ph.M * p.Cin;
  const uint8_t* WS = reinterpret_cast<const uint8_t*>(p.b) + (size_t)p.N * p.ldb;
  int hs_off[F8 ? HSI : 1];
  bool hs_ok[F8 ? HSI : 1];
  if constexpr (F8) {
#pragma unroll
    for (int j = 0; j < HSI; ++j) {
      const int q = 64 * (j * NW + wave) + lane;
      const int ii = q / IMGP, rem = q - ii * IMGP;
      const int hr = rem / HWD, hc = rem - hr * HWD;
      const int ih = r0 + hr - 1, iw = hc - 1;
      hs_ok[j] = q < npos && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      hs_off[j] = hs_ok[j] ? (((img0 + ii) * H + ih) * W + iw) * (p.Cin / 32) : 0;
    }
  }
  const uint8_t* ws_row = WS + (size_t)(nt * BN + 16 * wave + (lane & 15)) * (p.ldb / 32);

  auto issue_halo = [&](int cc) {
    const uint32_t base = lds0 + (HB == 2 ? (cc & 1) * HALO : 0) + wave * 1024;
    const int ci0 = cc * CH * ES;
#pragma unroll
    for (int i = 0; i < HG; ++i)
      gl16(h_ok[i] ? (const void*)(X + h_off[i] + ci0) : zero,
           (!F8 || 8 * (i * NW + wave) < HPOS) ? base + i * NW * 1024 : lds0 + DUMMY);
    if constexpr (F8) {
      const uint32_t sb = lds0 + HS_OFF + (HB == 2 ? (cc & 1) * HSB : 0);
#pragma unroll
      for (int j = 0; j < HSI; ++j)
        __builtin_amdgcn_global_load_lds(hs_ok[j] ? (const void*)(XS + hs_off[j] + cc * 4) : zero,
                                         (__attribute__((address_space(3))) void*)(uintptr_t)(sb + (j * NW + wave) * 256),
                                         4, 0, 0);
    }
  };
  auto issue_b = [&](int kt) {
    const int cc = kt / 9, t = kt - cc * 9;
    const int off = (ph.boff[t] + cc * CH) * ES;
    const uint32_t base = lds0 + HB * HALO + (kt % NBS) * BST + wave * 1024;
#pragma unroll
    for (int i = 0; i < BG; ++i) gl16(b_src[i] + off, base + i * NW * 1024);
    if constexpr (F8) {  // this wave's 16 weight rows: 4 scale bytes each (lanes >= 16 masked)
      if (lane < 16)
        __builtin_amdgcn_global_load_lds((const void*)(ws_row + off / 32),
                                         (__attribute__((address_space(3))) void*)(uintptr_t)(
                                             lds0 + BS_OFF + (kt % NBS) * BSB + wave * 64),
                                         4, 0, 0);
    }
  };

  // per-thread fragment rows: halo position of output pixel m at tap (0,0)
  const int g = lane >> 4, i16 = lane & 15;
  int hb[4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int m = wm * 64 + mi * 16 + i16;
    const int ii = m / RTW, rem = m - ii * RTW;
    const int lr = rem / W, lc = rem - lr * W;
    hb[mi] = ii * IMGP + lr * HWD + lc;
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int kt) {
    const int cc = kt / 9, t = kt - cc * 9;
    const int toff = (ph.dh[t] + 1) * HWD + (ph.dw[t] + 1);
    const char* Hl = reinterpret_cast<const char*>(lds) + (HB == 2 ? (cc & 1) * HALO : 0);
    const char* Bl = reinterpret_cast<const char*>(lds) + HB * HALO + (kt % NBS) * BST;
    if constexpr (F8) {
      // lane (i16, g): K bytes [16g, 16g+16) and [64+16g, 64+16g+16) of the 128-channel chunk = 16-byte
      // chunks g and g + 4; the scale operand: the E8M0 scale of (row i16, 32-channel block g)
      const uint8_t* Hs = reinterpret_cast<const uint8_t*>(lds) + HS_OFF + (HB == 2 ? (cc & 1) * HSB : 0);
      const uint8_t* Bs = reinterpret_cast<const uint8_t*>(lds) + BS_OFF + (kt % NBS) * BSB;
      v8i fb[4];
      int sb[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int row = wn * 64 + ni * 16 + i16;
        fb[ni] = cat8(*reinterpret_cast<const u32x4*>(Bl + row * 128 + ((g ^ swz8(row)) << 4)),
                      *reinterpret_cast<const u32x4*>(Bl + row * 128 + (((g + 4) ^ swz8(row)) << 4)));
        sb[ni] = Bs[row * 4 + g];
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int q = hb[mi] + toff;
        const v8i fa = cat8(*reinterpret_cast<const u32x4*>(Hl + q * 128 + ((g ^ swz8(q)) << 4)),
                            *reinterpret_cast<const u32x4*>(Hl + q * 128 + (((g + 4) ^ swz8(q)) << 4)));
        const int sa = Hs[q * 4 + g];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa, fb[ni], acc[mi][ni], 0, 0, 0, sa, 0,
                                                                          sb[ni]);
      }
      return;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      u32x4 fa[4], fb[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int q = hb[mi] + toff;
        fa[mi] = *reinterpret_cast<const u32x4*>(Hl + q * 128 + (((4 * s2 + g) ^ swz8(q)) << 4));
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int row = wn * 64 + ni * 16 + i16;
        fb[ni] = *reinterpret_cast<const u32x4*>(Bl + row * 128 + (((4 * s2 + g) ^ swz8(row)) << 4));
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) Mma<bf16>::run(acc[mi][ni], fa[mi], fb[ni]);
    }
  };

  // ---- main loop over k-steps kt = chunk*9 + tap ----
  // issue order: H(0) B(0) .. B(NBS-2) | per step j: [H(chunk(j)+1) if tap(j)==0] [B(j+NBS-1)]
  // BN-backward epilogue operands (y, mask bits, y2) of this thread's output rows, loaded at the start
  // of the last channel chunk (step kpre) so they arrive under its nine taps instead of after the loop
  // (one workgroup per CU: nothing else would hide that latency). NLD = the loads that certainly
  // issue (an addend adds more: the wait below then only waits longer).
  constexpr int CPR_ = BN / 8, NITP = 256 / (NT / CPR_);
  // (BW 2 only, the 3x3 dgrads of the step: the mask-bit variants would spill the extra registers)
  constexpr bool PRE = BW == 2 && !F8;
  constexpr int NLD = PRE ? NITP : 0;
  EpiIn pre[PRE ? NITP : 1];
  const int kpre = p.epi_pre ? nk - 9 : -2;
  issue_halo(0);
  issue_b(0);
  if (nk > 1) issue_b(1);
  if (NBS > 3 && nk > 2) issue_b(2);
  for (int kt = 0; kt < nk; ++kt) {
    const int t = kt % 9, cc = kt / 9;
    // loads allowed to stay in flight: everything issued after B(kt)
    if constexpr (NBS == 3) {
      bool halo_after = false;
      if (kt >= 1) {
        const int j = kt - 1;
        halo_after = (j % 9 == 0) && (j / 9 + 1 < nch);
      }
      const bool b_after = kt + 1 < nk;
      const bool after_pre = PRE && kt == kpre + 1;  // the prefetch went out after B(kt)
      if (halo_after && b_after) waitvm<HGC + BGC>();
      else if (halo_after) waitvm<HGC>();
      else if (b_after) { if (after_pre) waitvm<BGC + NLD>(); else waitvm<BGC>(); }
      else waitvm<0>();
    } else {
      // after B(kt): B(kt+1) .. B(kt+NBS-2) and the halos steps kt-NBS+2 .. kt-1 issued (at most one: a
      // halo goes out at tap 0 of a chunk), and the epilogue prefetch of step kpre
      const int nb = min(NBS - 2, nk - 1 - kt);
      int nh = 0;
#pragma unroll
      for (int j = kt - (NBS - 2); j < kt; ++j) nh += (j >= 0 && j % 9 == 0 && j / 9 + 1 < nch) ? 1 : 0;
      const int npre = (PRE && kpre >= 0 && kt > kpre && kt <= kpre + NBS - 2) ? NLD : 0;
      waitvm_le<(NBS - 2) * BGC + HGC + NLD>(nb * BGC + nh * HGC + npre);
    }
    sbar();
    if constexpr (PRE) {
      if (kt == kpre) {
#pragma unroll
        for (int i = 0; i < NITP; ++i) {
          const int rr = tid / CPR_ + (NT / CPR_) * i;
          const long px = slot_px(rr);
          epi_load<bf16, BW>(p, (size_t)px * p.ldc + nt * BN + (tid % CPR_) * 8, pre[i]);
        }
      }
    }
    if (t == 0 && cc + 1 < nch) issue_halo(cc + 1);
    if (kt + NBS - 1 < nk) issue_b(kt + NBS - 1);
    compute(kt);
  }
  waitvm<0>();
  __syncthreads();

  // ---- BN statistics (forward): one partial per 64-row wave tile or 128-row pair ----
  if (p.stats) {
    float2* red = reinterpret_cast<float2*>(lds);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      float s = 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += acc[mi][ni][r];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const float mean_w = s * (1.f / 64.f);
      float q = 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = acc[mi][ni][r] - mean_w;
          q = fmaf(d, d, q);
        }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      const int col = wn * 64 + ni * 16 + lane;
      if (p.stat_tile == 64) {
        if (lane < 16) store_part(p.stats + (size_t)(mt * 4 + wm) * p.N + nt * BN + col, make_float2(s, q));
      } else if (lane < 16) {
        red[wm * BN + col] = make_float2(s, q);
      }
    }
    __syncthreads();
    if (p.stat_tile == 128) {
      for (int idx = tid; idx < 2 * BN; idx += NT) {
        const int h = idx / BN, col = idx - h * BN;
        const float2 a0 = red[(2 * h) * BN + col], a1 = red[(2 * h + 1) * BN + col];
        const float d = (a0.x - a1.x) * (1.f / 64.f);
        store_part(p.stats + (size_t)(mt * 2 + h) * p.N + nt * BN + col,
                   make_float2(a0.x + a1.x, a0.y + a1.y + d * d * 32.f));
      }
    }
    __syncthreads();
    if (p.ffin.mode) {  // the statistics finalize folded in (bnfin.h): 256 / stat_tile partial rows a tile
      bn_fwd_fin_arrive<NT, BN>(p.ffin, mt, nt, reinterpret_cast<double2*>(lds),
                                reinterpret_cast<int*>(reinterpret_cast<char*>(lds) + NT * 32));
      __syncthreads();
    }
  }

  // ---- epilogue: LDS-staged C tile, 16-byte coalesced (+addend) stores; output pixels are contiguous ----
  bf16* Cs = reinterpret_cast<bf16*>(lds);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * 64 + mi * 16 + g * 4 + r) * LD + wn * 64 + ni * 16 + i16] = (bf16)acc[mi][ni][r];
  __syncthreads();
  constexpr int CPR = BN / 8, RPP = NT / CPR;
  bf16* __restrict__ Cg = reinterpret_cast<bf16*>(p.c);
  const int c = tid % CPR;
  BwdEpiAcc<bf16, BW> bwd;
  if constexpr (BW != 0) bwd.init(p.bb, nt * BN + c * 8);
  constexpr int NIT = 256 / RPP, U = 4;
  static_assert(NIT * RPP == 256 && NIT % U == 0 && NIT == NITP, "epilogue row partition");
#pragma unroll
  for (int i0 = 0; i0 < NIT; i0 += U) {
    size_t off[U];
    EpiIn in[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = tid / CPR + RPP * (i0 + u);
      off[u] = (size_t)slot_px(rr) * p.ldc + nt * BN + c * 8;
      if (PRE && p.epi_pre) in[u] = pre[PRE ? i0 + u : 0];
      else epi_load<bf16, BW>(p, off[u], in[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = tid / CPR + RPP * (i0 + u);
      const u32x4 v = *reinterpret_cast<const u32x4*>(Cs + rr * LD + c * 8);
      st16_nt(Cg + off[u], epi_apply<bf16, BW>(p, v, in[u], bwd));
    }
  }
  if constexpr (BW != 0) {
    __syncthreads();
    bwd.template reduce<BN, NT>(p.bb, reinterpret_cast<float2*>(lds), tid / CPR, RPP, c, (size_t)mt, p.N, nt * BN);
  }
  if (p.fin.mode) {  // LDS is free now: scratch [2 NT] double2, then the ticket flag
    __syncthreads();
    bn_fin_arrive<NT, BN>(p.fin, mt, nt, reinterpret_cast<double2*>(lds),
                          reinterpret_cast<int*>(reinterpret_cast<char*>(lds) + NT * 32));
  }
}

// the demangled instantiation name (as rocprofv3 reports it: the kernel timer's labels join the PMC summaries)
template <int BN, int BW, int HB, bool F8, bool DEEP>
static const char* halo_name() {
  static const std::string s = std::string("argus::conv3x3_halo_kernel<") + std::to_string(BN) + ", " +
                               std::to_string(BW) + ", " + std::to_string(HB) + (F8 ? ", true" : ", false") +
                               (DEEP ? ", true>" : ", false>");
  return s.c_str();
}

// The BN-backward epilogue operands of the halo dgrad are prefetched under its last channel chunk on
// the single-buffer 64-column variant (layer 1: 172 -> 163 us); on the 128-column one it measured
// 83 -> 100 us (the step within noise), so that variant loads them after the loop.
template <int BN, int BW, int HB, bool F8 = false, bool DEEP = false>
static void launch_halo2(const IgParams& p0, hipStream_t st) {
  IgParams p = p0;
  p.epi_pre = HB == 1;
  plan_fin(p, 256);
  plan_ffin(p, 256);
  dim3 grid(conv3x3_halo_tiles(p) * (p.N / BN));
  timed_launch(halo_name<BN, BW, HB, F8, DEEP>(), conv3x3_halo_kernel<BN, BW, HB, F8, DEEP>, grid,
               dim3(4 * (BN / 64) * 64), st, p);
}

template <int BN, int BW>
static void launch_halo1(const IgParams& p, hipStream_t st) {
  if constexpr (BW == 0 || BW == 2) {
    if (p.x8) {  // conv3x3_halo_x8_ok: 128-channel chunks, two halo buffers
      launch_halo2<BN, BW, 2, true>(p, st);
      return;
    }
  }
  const int HWi = p.H * p.W;
  const int npos = HWi >= 256 ? (256 / p.W + 2) * (p.W + 2) : (256 / HWi) * (p.H + 2) * (p.W + 2);
  if constexpr (BN == 64) {
    if (p.Cin == 64 && npos <= kHaloPos1) {  // one channel chunk: one halo buffer, two workgroups per CU
      launch_halo2<BN, BW, 1>(p, st);
      return;
    }
  } else {
    if ((*p.pol)[kHaloDeepRing] && npos <= kHaloPosDeep) {  // key 51: the four-stage weight ring
      launch_halo2<BN, BW, 2, false, true>(p, st);
      return;
    }
  }
  launch_halo2<BN, BW, 2>(p, st);
}

template <int BN>
static void launch_halo(const IgParams& p, hipStream_t st) {
  switch (bwd_variant(p.bb)) {
    case 2: launch_halo1<BN, 2>(p, st); break;
    case 3: launch_halo1<BN, 3>(p, st); break;
    case 4: launch_halo1<BN, 4>(p, st); break;
    default: launch_halo1<BN, 0>(p, st);
  }
}

// Tile geometry of a halo-eligible conv: 256 consecutive output pixels = whole rows of one image or
// whole images (false = not servable). (TH x TW block tiles for frames whose width does not divide 256
// - the 376 x 672 frame's 168-, 84-, 42- and 21-wide layers - were built and measured: at B=128 they
// moved 11 of 21 dgrads off the 256 x 128 GEMM for no net gain, 2518.6 vs 2524.4 img/s; removed.)
static bool halo_geom(const IgParams& p, int& npos, int& tiles) {
  const IgPhase& ph = p.ph[0];
  const int HWi = p.H * p.W;
  if (ph.M % 256) return false;
  bool rows;
  if (HWi >= 256) {
    rows = 256 % p.W == 0 && HWi % 256 == 0;
    npos = (256 / p.W + 2) * (p.W + 2);
  } else {
    rows = 256 % HWi == 0;
    npos = (256 / HWi) * (p.H + 2) * (p.W + 2);
  }
  if (!rows || npos > kHaloPos) return false;
  tiles = ph.M / 256;
  return true;
}

// 3x3 / stride 1 / pad 1, same input and output grid, one phase; 256-pixel tiles (whole rows / whole
// images). Policy keys 10 (enable) and 13 (fewest workgroups; 1 also allows the 4-wave 64-column
// variant on any shape: tests).
int conv3x3_halo_ok(const IgParams& p) {
  const Policy& pol = *p.pol;
  if (!pol[kHaloEnable] || (!p.fwd && !pol[kHaloDgrad]) || p.stem || p.pro_scale || p.ap.y || p.nphase != 1 || p.ish != 1 || p.isw != 1 || p.osh != 1 ||
      p.osw != 1)
    return 0;
  const IgPhase& ph = p.ph[0];
  if (ph.K != 9 * p.Cin || p.Cin % 64 || p.lda % 8 || p.ldb % 8 || p.H != p.Ho || p.W != p.Wo) return 0;
  for (int t = 0; t < 9; ++t)
    if (ph.dh[t] < -1 || ph.dh[t] > 1 || ph.dw[t] < -1 || ph.dw[t] > 1) return 0;
  int npos, tiles;
  if (!halo_geom(p, npos, tiles)) return 0;
  if (p.stats && p.stat_tile != 64 && p.stat_tile != 128) return 0;
  // measured (tools/convbench.py, B=64): wins only with 8-wave workgroups (N % 128) filling every CU;
  // the 4-wave BN=64 tile and sub-CU-count grids lose to the register-staged kernel - except the
  // 64-channel layer-1 3x3 convs on the single-halo-buffer variant (two workgroups per CU; B=64 in the
  // full step: fwd 80 -> 71 us, dgrad + BN epilogue 147 -> 132 us per layer; 8245 -> 8302 img/s)
  const int min_grid = pol[kHaloMinGrid];
  if (p.N % 128 == 0 && tiles * (p.N / 128) >= min_grid) return 128;
  if (p.N == 64 && p.Cin == 64 && tiles >= min_grid) return 64;
  if (min_grid <= 1 && p.N % 64 == 0) return 64;  // forced (tests): the 4-wave variant
  return 0;
}

int conv3x3_halo_tiles(const IgParams& p) {
  int npos, tiles;
  return halo_geom(p, npos, tiles) ? tiles : 0;
}

// the MX-fp8 stored-operand variant (argus_conv_fwd_x8 / argus_conv_dgrad_bn_x8): the halo shapes with
// 128-channel chunks (Cin % 128), the plain forward or the BN-backward epilogue of mask mode 2, and
// tightly packed x8 rows (lda == Cin; the scales follow the M x Cin bytes)
int conv3x3_halo_x8_ok(const IgParams& p) {
  const int bn = conv3x3_halo_ok(p);
  int npos, tiles;
  if (!bn || !halo_geom(p, npos, tiles) || npos > kHaloPosF8 || p.Cin % 128 || p.lda != p.Cin || p.ldb % 128 ||
      p.addend || p.addend_mask)
    return 0;
  const int bw = bwd_variant(p.bb);
  return bw == 0 || bw == 2 ? bn : 0;
}

bool conv3x3_halo_launch(const IgParams& p, hipStream_t st) {
  const int bn = p.x8 ? conv3x3_halo_x8_ok(p) : conv3x3_halo_ok(p);
  if (!bn) return false;
  if (bn == 128) launch_halo<128>(p, st);
  else launch_halo<64>(p, st);
  return true;
}


// ================================================================================================
// 3x3 stride-1 weight gradient with the input halo tile in LDS (dW[k][tap][c] = sum_p dy[p][k] *
// x[p + off(tap)][c]). A workgroup (8 waves, 2 x 4) owns 64
// output channels x 9 taps x 64 input channels (a 64 x 576 tile; wave (wm, wn) holds rows 32wm..+31
// and the 9 column blocks of 16 at 9wn..9wn+8) and reduces over a range of 128-pixel-slot tiles: a
// TH x TW block of one image (TW divides W; 256 x 256 frames: 4 x 32 blocks of the 64-wide layer,
// whole rows of the 32- and 16-wide ones; 376 x 672 frames: 3 x 42 blocks of the 168- and 84-wide
// layers; slots past TH*TW or below the image carry zero dy; wg_halo_geom), or NI
// whole images when H*W < 128. Per tile it glds-loads dy [128 slots][64 k] and the x halo
// [(TH+2)*(TW+2) positions][64 c] once (7 uniform 1 KB pieces per wave, double-buffered
// over tiles with a counted vmcnt); both MFMA operands are k(=pixel)-major, read with
// ds_read_b64_tr_b16. Images are [row][128 B], 16-byte slot j of row r at slot j ^ wsw(r): the eight
// rows a 32-lane half touches in one transposed read (r0..r0+3, r0+8..r0+11) hit distinct banks.
// fp32 partials go to part[split][K][9C]; wgrad_reduce_kernel sums them in fixed order.
// ================================================================================================
struct WgHaloParams {
  const bf16* x;
  const bf16* dy;
  float* part;
  int n, H, W, C, K;
  int ptiles, tps;  // 128-slot tiles in total, tiles per split
  int TH, TW, NI;   // tile block (TH x TW pixels of one image), images per tile (NI > 1: TH = H, TW = W)
  int RT, CT;       // row / column blocks per image (NI == 1)
};

constexpr int kWgHaloPos = 256;  // halo positions per stage ((TH+2) x (TW+2) <= 256)
constexpr int kWgStages = 3;     // tiles in flight: LDS 3 x 48 KB (two tiles' loads overlap each tile's MFMAs)

ARGUS_DEV int wsw(int r) { return (r & 2) | ((r >> 1) & 4); }  // bit 1 -> bit 1, bit 3 -> bit 2

// Transposed LDS reads (ds_read_b64_tr_b16) issued as inline asm. The compiler treats a ds_read_tr16_b64 builtin
// as possibly aliasing the global_load_lds stages in flight and put an `s_waitcnt vmcnt(0)` in front
// of the first one of every k-step, which drained the next tiles' loads each time (the ring overlapped
// nothing). As asm the reads are invisible to that analysis: the ring's own counted vmcnt waits and
// barriers order them, and lgkm_tie() waits for their data before the MFMAs use it.
ARGUS_DEV uint2 ds_tr_asm(uint32_t addr) {
  uint2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr) : "memory");
  return r;
}
// every LDS read issued so far has landed. The tie takes the asm reads' own uint2 results (not the
// u32x4 fragments assembled from them): the compiler's waitcnt pass does not see inline-asm loads, so a
// copy made before the wait (e.g. to pair two results into the 4-register tuple an MFMA operand needs)
// would read registers whose data has not arrived. Tied here, no use or copy moves above the wait; the
// fragments are assembled from the tied values afterwards.
ARGUS_DEV void lgkm_tie(uint2 (&a)[2][2], uint2 (&b)[9][2]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(a[0][0]), "+v"(a[0][1]), "+v"(a[1][0]), "+v"(a[1][1]), "+v"(b[0][0]), "+v"(b[0][1]),
                 "+v"(b[1][0]), "+v"(b[1][1]), "+v"(b[2][0]), "+v"(b[2][1]), "+v"(b[3][0]), "+v"(b[3][1]),
                 "+v"(b[4][0]), "+v"(b[4][1]), "+v"(b[5][0]), "+v"(b[5][1]), "+v"(b[6][0]), "+v"(b[6][1]),
                 "+v"(b[7][0]), "+v"(b[7][1]), "+v"(b[8][0]), "+v"(b[8][1])
               :
               : "memory");
}

__global__ __launch_bounds__(512, 1) void wgrad3x3_halo_kernel(const WgHaloParams p) {
  constexpr int DYB = 128 * 128;                // dy image bytes
  constexpr int HXB = kWgHaloPos * 128;         // halo image bytes
  constexpr int STG = DYB + HXB;                // one stage
  constexpr int PIECES = STG / 1024;            // 1 KB glds pieces per stage (48)
  constexpr int GPW = PIECES / 8;               // per wave (6)
  static_assert(GPW * 8 == PIECES && DYB / 1024 == 16, "stage partition");
  __shared__ __attribute__((aligned(1024))) u32x4 lds[(kWgStages * STG + 512) / 16];

  const int ctiles = p.C / 64;
  int tile, split;
  split_tile((p.K / 64) * ctiles, (p.ptiles + p.tps - 1) / p.tps, false, tile, split);
  const int kt = tile / ctiles, ct = tile - kt * ctiles;
  const int t0 = split * p.tps, t1 = min(p.ptiles, t0 + p.tps);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;

  const int H = p.H, W = p.W, TH = p.TH, TW = p.TW, NI = p.NI, THW = TH * TW;
  const int HWD = TW + 2, IMGP = (TH + 2) * HWD, npos = NI * IMGP;

  // fragment geometry: slot 32*s2 + 8g + 4h + q of the tile -> halo row at tap (0,0); slots past the
  // tile's pixels read position 0 (loaded, finite) against their zero dy
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
  const int half8 = (pp & 1) * 8;
  auto halo_row = [&](int m) {
    const int ii = m / THW, rem = m - ii * THW;
    const int lr = rem / TW, lc = rem - lr * TW;
    return ii < NI ? ii * IMGP + lr * HWD + lc : 0;
  };
  // glds pieces of this wave: i = 0, 1 -> dy rows; i = 2.. -> halo positions. Their element offsets from
  // the tile's corner (image img0, row r0, column c0) and the coordinates the bounds checks need are the
  // same in every tile: computed once (per tile only a scalar base and two compares per piece remain).
  constexpr int HP = GPW - 2;
  int dy_off[2], dy_lr[2];
  int hx_off[HP], hx_rc[HP];  // hx_rc: halo row - 1 (high 16 bits, signed) | halo column - 1 (low, signed)
  bool hx_in[HP];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 8 * (wave + 8 * i) + (lane >> 3);
    const int ii = row / THW, rem = row - ii * THW, lr = rem / TW, lc = rem - lr * TW;
    dy_lr[i] = ii < NI ? lr : (1 << 30);  // slots past the tile's pixels: never in the image (zero dy)
    dy_off[i] = ((ii * H + lr) * W + lc) * p.K + kt * 64 + ((lane & 7) ^ wsw(row)) * 8;
  }
#pragma unroll
  for (int i = 0; i < HP; ++i) {
    const int qq = 8 * (wave + 8 * i) + (lane >> 3);
    const int ii = qq / IMGP, rem = qq - ii * IMGP;
    const int hr = rem / HWD, hc = rem - hr * HWD;
    hx_in[i] = qq < npos;
    hx_rc[i] = ((hr - 1) << 16) | ((hc - 1) & 0xffff);
    hx_off[i] = ((ii * H + hr - 1) * W + hc - 1) * p.C + ct * 64 + ((lane & 7) ^ wsw(qq)) * 8;
  }
  const void* zero = (const void*)halo_zero_page;

  auto issue = [&](int tile, int stage) {
    int img0, r0 = 0, c0 = 0;
    if (NI > 1) {
      img0 = tile * NI;
    } else {
      const int tpi = p.RT * p.CT;
      img0 = tile / tpi;
      const int rem = tile - img0 * tpi, rt = rem / p.CT;
      r0 = rt * TH;
      c0 = (rem - rt * p.CT) * TW;
    }
    const size_t corner = ((size_t)img0 * H + r0) * W + c0;
    const bf16* dyb = p.dy + corner * p.K;
    const bf16* xb = p.x + corner * p.C;
    const uint32_t base = lds0 + stage * STG;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool ok = r0 + dy_lr[i] < H;
      gl16(ok ? (const void*)(dyb + dy_off[i]) : zero, base + (wave + 8 * i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < HP; ++i) {
      const int ih = r0 + (hx_rc[i] >> 16), iw = c0 + (int)(short)(hx_rc[i] & 0xffff);
      const bool ok = hx_in[i] && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      gl16(ok ? (const void*)(xb + hx_off[i]) : zero, base + DYB + (wave + 8 * i) * 1024);
    }
  };

  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LDS byte offsets of this lane's transposed reads, relative to its stage's dy / halo image. They are
  // the same in every tile (fixed geometry), so they are computed once and kept packed as two 16-bit
  // halves per VGPR (images < 64 KB): per read one unpack + one add instead of the row / swizzle math
  // that made the k-step VALU-bound (SQ_INSTS_VALU 16x SQ_INSTS_MFMA).
  auto tr_off = [&](int r, int slot) { return r * 128 + ((slot ^ wsw(r)) << 4) + half8; };
  unsigned offa[4][2], offb[4][9];
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) {
    const int rlo = 32 * s2 + 8 * g + q;
    const int h0 = halo_row(rlo), h1 = halo_row(rlo + 4);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int slot = 2 * (2 * wm + mi) + (pp >> 1);
      offa[s2][mi] = (unsigned)tr_off(rlo, slot) | ((unsigned)tr_off(rlo + 4, slot) << 16);
    }
#pragma unroll
    for (int ni = 0; ni < 9; ++ni) {
      const int nb = 9 * wn + ni;  // 16-column block of the 576 columns: tap nb/4, channels 16*(nb%4)
      const int t = nb >> 2, cb = nb & 3;
      const int toff = (t / 3) * HWD + (t % 3);
      const int slot = 2 * cb + (pp >> 1);
      offb[s2][ni] = (unsigned)tr_off(h0 + toff, slot) | ((unsigned)tr_off(h1 + toff, slot) << 16);
    }
  }
  auto frag = [&](uint32_t img, unsigned packed, uint2 (&u)[2]) {
    u[0] = ds_tr_asm(img + (packed & 0xffffu));
    u[1] = ds_tr_asm(img + (packed >> 16));
  };
  auto join = [](const uint2 (&u)[2]) { return u32x4{u[0].x, u[0].y, u[1].x, u[1].y}; };

  // 3-stage ring: tile i lands in stage i % 3; tiles i+1 and i+2 stay in flight over tile i's MFMAs
  if (t0 < t1) issue(t0, 0);
  if (t0 + 1 < t1) issue(t0 + 1, 1);
  int stage = 0;
  for (int tile = t0; tile < t1; ++tile) {
    const int ahead = min(t1 - 1 - tile, kWgStages - 1);  // tiles issued after this one
    if (ahead == kWgStages - 1) {
      // stage (stage + 2) % 3 was last read in the previous iteration, before its closing barrier
      issue(tile + 2, stage == 0 ? 2 : stage - 1);
      waitvm<2 * GPW>();
    } else if (ahead == 1) {
      waitvm<GPW>();
    } else {
      waitvm<0>();
    }
    sbar();
    const uint32_t DYI = lds0 + stage * STG;
    const uint32_t HXI = DYI + DYB;
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      uint2 ra[2][2], rb[9][2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) frag(DYI, offa[s2][mi], ra[mi]);
#pragma unroll
      for (int ni = 0; ni < 9; ++ni) frag(HXI, offb[s2][ni], rb[ni]);
      lgkm_tie(ra, rb);
      u32x4 fa[2], fb[9];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) fa[mi] = join(ra[mi]);
#pragma unroll
      for (int ni = 0; ni < 9; ++ni) fb[ni] = join(rb[ni]);
#pragma unroll
      for (int ni = 0; ni < 9; ++ni)
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) Mma<bf16>::run(acc[mi][ni], fa[mi], fb[ni]);
    }
    sbar();  // every wave is done with this stage before it is refilled
    stage = stage == kWgStages - 1 ? 0 : stage + 1;
  }

  // ---- fp32 partial tile: part[split][k][tap*C + c] ----
  float* out = p.part + (size_t)split * p.K * (9 * p.C);
#pragma unroll
  for (int ni = 0; ni < 9; ++ni) {
    const int nb = 9 * wn + ni;
    const int t = nb >> 2, cb = nb & 3;
    const int col = t * p.C + ct * 64 + cb * 16 + i16;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        out[(size_t)(kt * 64 + wm * 32 + mi * 16 + g * 4 + r) * (9 * p.C) + col] = acc[mi][ni][r];
  }
}


// Tile geometry of the halo weight gradient. H*W < 128: NI = 128 / (H*W) whole images per tile
// (128 % HW == 0). Otherwise a TH x TW block of one image: over the divisors TW of W (<= 128) with
// TH = min(128 / TW, H) rows and a (TH+2) x (TW+2) halo within kWgHaloPos, the most useful pixels per
// 128 slots (ragged last row block included), ties to the wider block. 256 x 256 frames: the 64-wide
// layer 1 gets 4 x 32 blocks ((2+2) x (64+2) = 264 positions would exceed kWgHaloPos = 256), the 32-
// and 16-wide layers whole rows (4 x 32, 8 x 16), the 8 x 8 layer two whole images; 168- and 84-wide
// frames: 3 x 42.
struct WgHaloGeom {
  int TH, TW, NI, RT, CT;
  long ptiles;
};
static bool wg_halo_geom(const argus_conv_desc& d, WgHaloGeom& gm) {
  const int H = d.h, W = d.w, HW = H * W;
  if (HW < 128) {
    if (128 % HW || (d.n * 128 / HW) == 0 || d.n % (128 / HW)) return false;
    gm.NI = 128 / HW; gm.TH = H; gm.TW = W; gm.RT = gm.CT = 1;
    if (gm.NI * (H + 2) * (W + 2) > kWgHaloPos) return false;
    gm.ptiles = (long)d.n / gm.NI;
    return true;
  }
  double best = 0.0;
  for (int tw = W < 128 ? W : 128; tw >= 1; --tw) {
    if (W % tw) continue;
    int th = 128 / tw;
    if (th > H) th = H;
    if ((th + 2) * (tw + 2) > kWgHaloPos) continue;
    const int rt = (H + th - 1) / th;
    const double eff = (double)H * tw / ((double)rt * 128.0);  // image pixels per slot
    if (eff > best + 1e-9) {
      best = eff;
      gm.TH = th; gm.TW = tw; gm.RT = rt; gm.CT = W / tw;
    }
  }
  if (best < 0.75) return false;  // mostly padding: the register-staged kernel
  gm.NI = 1;
  gm.ptiles = (long)d.n * gm.RT * gm.CT;
  return true;
}

// Plan for a 3x3 / stride 1 / pad 1 bf16 weight gradient: false when not served. splits * K * 9C
// fp32 partials. Policy keys 11 (enable), 12 (split target: 512 -> 256 once it ran on the side stream
// beside the main-stream chain, bench B=64 +0.6-0.9 %) and 14 (most channel tiles).
bool wgrad3x3_halo_plan(const argus_conv_desc& d, int dtype, int* splits, int* tps) {
  const Policy pol = policy_of(d);
  if (!pol[kWgHaloEnable] || dtype != ARGUS_BF16 || d.stem || d.r != 3 || d.s != 3 || d.stride != 1 || d.pad != 1 ||
      d.c % 64 || d.k % 64 || d.ho != d.h || d.wo != d.w)
    return false;
  WgHaloGeom gm;
  if (!wg_halo_geom(d, gm)) return false;
  const long ptiles = gm.ptiles;
  const long tiles = (long)(d.k / 64) * (d.c / 64);
  // measured: a win for <= 4 (k, c) tiles (the 64- and 128-channel layers); beyond, its two tr16
  // operand streams make it LDS-read-bound and the register-staged wgrad_kernel is faster
  if (tiles > pol[kWgHaloMaxTiles]) return false;
  long s = (pol[kWgHaloTarget] + tiles - 1) / tiles;
  if (s < 1) s = 1;
  if (s > ptiles) s = ptiles;
  const long per = (ptiles + s - 1) / s;
  *tps = (int)per;
  *splits = (int)((ptiles + per - 1) / per);
  return true;
}

bool wgrad3x3_halo_launch(const argus_conv_desc& d, int dtype, const void* x, const float* sc, const float* sh,
                          const void* dy, void* ws, size_t ws_bytes, int* splits_out, hipStream_t st) {
  int splits, tps;
  if (sc || sh || !wgrad3x3_halo_plan(d, dtype, &splits, &tps)) return false;  // inputs are materialised
  if (ws_bytes < (size_t)splits * d.k * 9 * d.c * sizeof(float)) return false;
  WgHaloParams p;
  p.x = reinterpret_cast<const bf16*>(x);
  p.dy = reinterpret_cast<const bf16*>(dy);
  p.part = reinterpret_cast<float*>(ws);
  p.n = d.n; p.H = d.h; p.W = d.w; p.C = d.c; p.K = d.k;
  WgHaloGeom gm;
  wg_halo_geom(d, gm);
  p.ptiles = (int)gm.ptiles;
  p.TH = gm.TH; p.TW = gm.TW; p.NI = gm.NI; p.RT = gm.RT; p.CT = gm.CT;
  p.tps = tps;
  dim3 grid((d.k / 64) * (d.c / 64) * splits);
  timed_launch("argus::wgrad3x3_halo_kernel", wgrad3x3_halo_kernel, grid, dim3(512), st, p);
  *splits_out = splits;
  return true;
}

}  // namespace argus
