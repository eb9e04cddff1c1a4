// Implicit-GEMM convolution (forward / dgrad, bf16, no BN prologue) with global->LDS DMA staging.
//
// Why a second kernel: the register-staged igemm_kernel (conv.hip) moves every operand byte
// global -> VGPR -> LDS; on gfx950 a ds_write_b128 costs ~13 cycles of VGPR->LDS transfer per wave
// instruction (~79 B/clk/CU, MI355X_MICROARCH.md §LDS), which for its 128x128 tile exceeds the MFMA
// time per k-step. Here both operands go straight to LDS with global_load_lds_dwordx4 (no VGPR, no
// ds_write), through a 3-stage LDS ring with a counted vmcnt and raw s_barrier, so two k-steps of
// loads are in flight while the MFMAs of the current one run (cdna_hip_programming.md §5,
// "Pipelining across barriers").
//
// Geometry: each wave computes a 64x64 output tile (4x4 v_mfma_f32_16x16x32_bf16 blocks); the
// workgroup is (BM/64) x (BN/64) waves: 256x128 (8 waves) or 256x64 (4 waves). K-step = one tap x 64
// input channels. LDS images are [row][64 k] bf16 (128 B rows), 16-byte slot j of row r holding
// k-chunk j ^ swz8(r) (conflict-free ds_read_b128 fragment reads); glds writes lane-linear 1 KB
// pieces (8 rows), so the swizzle is applied on the per-lane global source address. Out-of-image
// taps and rows past M read a 16-byte zero page. BN statistics are emitted per 64-row wave tile or
// per 128-row half tile, in the same partial layout as igemm_kernel's 64- / 128-row tiles.
#include "common.h"
#include "igemm.h"
#include "internal.h"
#include "ktimer.h"

namespace argus {

__device__ __attribute__((aligned(64))) u32x4 g_zero_page[4];  // zero-initialised (static storage)

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left at their maxima (gfx9 encoding).
template <int N> ARGUS_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

ARGUS_DEV void glds16(const void* src, uint32_t lds_byte_addr) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(uintptr_t)lds_byte_addr, 16, 0,
                                   0);
}

ARGUS_DEV void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// NSTAGE 3: k-steps kt+1 and kt+2 in flight during compute(kt) (144 KB LDS for 256 x 128); 2: kt+1
// only, 96 KB, so a workgroup fits beside one side-stream weight-gradient workgroup (64 KB) on a CU
template <int BM, int BN, int BW, int NSTAGE = 3>
__global__ __launch_bounds__((BM / 64) * (BN / 64) * 64, 1) void igemm_glds_kernel(const IgParams p) {
  constexpr int WM = BM / 64, WN = BN / 64, NW = WM * WN, NT = NW * 64;
  constexpr int STAGE = (BM + BN) * 128;      // bytes per pipeline stage (A image, then B image)
  static_assert(NSTAGE == 2 || NSTAGE == 3, "glds ring depth");
  constexpr int LD = BN + 8;                   // epilogue C row stride (elements)
  constexpr int EPI = BM * LD * 2;
  constexpr int LDS0 = NSTAGE * STAGE > EPI ? NSTAGE * STAGE : EPI;
  constexpr int RED_B = (NT / (BN / 8)) * BN * 8;  // BN-backward column sums
  constexpr int LDS_BYTES = LDS0 > RED_B ? LDS0 : RED_B;
  constexpr int AI = BM * 8 / NT;              // A glds per thread per stage
  constexpr int BI = BN * 8 / NT;              // B glds per thread per stage
  constexpr int GPS = AI + BI;                 // glds per wave per stage (vmcnt unit)
  static_assert(AI * NT == BM * 8 && BI * NT == BN * 8, "tile / thread mismatch");
  __shared__ __attribute__((aligned(1024))) u32x4 lds[LDS_BYTES / 16];

  const IgPhase& ph = p.ph[blockIdx.z];
  const int mtiles = (ph.M + BM - 1) / BM;
  const int ntiles = p.N / BN;
  const int nwg = mtiles * ntiles;
  // the folded finalize's ticket flag: the last 16 bytes of the LDS array (bn_fin_arrive's scratch is its
  // first NT * 32 bytes), so the 2-stage ring stays at exactly 96 KB
  int& fin_flag = *reinterpret_cast<int*>(&lds[LDS_BYTES / 16 - 1]);
  if ((int)blockIdx.x >= nwg) {
    if constexpr (BW != 0) {
      const int e = blockIdx.x - nwg;
      bwd_epi_zero_rows<BN, NT>(p.bb, e, mtiles, ntiles, p.N);
      if (p.fin.mode && mtiles + e / ntiles < p.bb.prow)
        bn_fin_arrive<NT, BN>(p.fin, blockIdx.z * p.bb.prow + mtiles + e / ntiles, e % ntiles,
                              reinterpret_cast<double2*>(lds), &fin_flag);
    }
    return;
  }
  if (ph.K == 0 && p.addend == p.c && !p.addend_mask && BW == 0) return;  // in-place += 0
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave - wm * WN;
  const bf16* __restrict__ A = reinterpret_cast<const bf16*>(p.a);
  const bf16* __restrict__ B = reinterpret_cast<const bf16*>(p.b);
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;

  // this thread's A rows (output pixels) and the k-chunk each of its glds fetches
  const int HWq = ph.Hq * ph.Wq;
  int a_off[AI], a_ih[AI], a_iw[AI], a_ch[AI];
  bool a_ok[AI];
  // 1x1 / stride-1 GEMM: input pixel = GEMM row (no per-row integer divisions; igemm_kernel, conv.hip)
  const bool a_ident = ph.K == p.Cin && ph.dh[0] == 0 && ph.dw[0] == 0 && p.ish == 1 && p.isw == 1 &&
                       ph.Hq == p.H && ph.Wq == p.W;
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int row = 8 * (i * NW + wave) + (lane >> 3);
    const int m = mt * BM + row;
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
    a_ch[i] = ((lane & 7) ^ swz8(row)) * 8;
  }
  const bf16* b_src[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int row = 8 * (i * NW + wave) + (lane >> 3);
    b_src[i] = B + (size_t)(nt * BN + row) * p.ldb + ((lane & 7) ^ swz8(row)) * 8;
  }
  const void* zero = (const void*)g_zero_page;

  auto issue = [&](int kt, int stage) {
    const int k0 = kt * 64;
    const int t = k0 / p.Cin;
    const int ci0 = k0 - t * p.Cin;
    const int dh = ph.dh[t], dw = ph.dw[t], boff = ph.boff[t];
    const int tap = (dh * p.W + dw) * p.lda + ci0;
    const uint32_t base = lds0 + stage * STAGE + wave * 1024;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int ih = a_ih[i] + dh, iw = a_iw[i] + dw;
      const bool ok = a_ok[i] && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
      glds16(ok ? (const void*)(A + a_off[i] + tap + a_ch[i]) : zero, base + i * NW * 1024);
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) glds16(b_src[i] + boff + ci0, base + BM * 128 + i * NW * 1024);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, i16 = lane & 15;
  auto compute = [&](int stage) {
    const char* L = reinterpret_cast<const char*>(lds) + stage * STAGE;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      u32x4 fa[4], fb[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        const int row = wm * 64 + mi * 16 + i16;
        fa[mi] = *reinterpret_cast<const u32x4*>(L + row * 128 + (((4 * s2 + g) ^ swz8(row)) << 4));
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int row = wn * 64 + ni * 16 + i16;
        fb[ni] = *reinterpret_cast<const u32x4*>(L + BM * 128 + row * 128 + (((4 * s2 + g) ^ swz8(row)) << 4));
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) Mma<bf16>::run(acc[mi][ni], fa[mi], fb[ni]);
    }
  };

  // ---- main loop: NSTAGE-deep ring ----
  const int nk = ph.K / 64;
  if (nk > 0) issue(0, 0);
  if constexpr (NSTAGE == 3) {  // k-steps kt+1 and kt+2 in flight during compute(kt)
    if (nk > 1) issue(1, 1);
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) wait_vmcnt<GPS>(); else wait_vmcnt<0>();
      raw_barrier();  // stage kt landed for every wave; every wave finished reading stage kt-1
      if (kt + 2 < nk) issue(kt + 2, (kt + 2) % NSTAGE);
      compute(kt % NSTAGE);
    }
  } else {  // k-step kt+1 in flight during compute(kt)
    for (int kt = 0; kt < nk; ++kt) {
      wait_vmcnt<0>();
      raw_barrier();  // stage kt landed for every wave; every wave finished reading stage kt-1 (= kt+1's)
      if (kt + 1 < nk) issue(kt + 1, (kt + 1) & 1);
      compute(kt & 1);
    }
  }
  wait_vmcnt<0>();
  __syncthreads();  // LDS is reused below

  // ---- BN statistics per 64-row (one wave) or 128-row (two waves) tile: {sum, M2} per column ----
  if (p.stats) {
    float2* red = reinterpret_cast<float2*>(lds);  // [WM][BN]
    int nvalid_w = ph.M - (mt * BM + wm * 64);
    nvalid_w = nvalid_w < 0 ? 0 : (nvalid_w > 64 ? 64 : nvalid_w);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      float s = 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += mi * 16 + g * 4 + r < nvalid_w ? acc[mi][ni][r] : 0.f;
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const float mean_w = nvalid_w > 0 ? s / (float)nvalid_w : 0.f;
      float q = 0.f;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = acc[mi][ni][r] - mean_w;
          q = mi * 16 + g * 4 + r < nvalid_w ? fmaf(d, d, q) : q;
        }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (p.stat_tile == 64) {  // a wave's 64 rows are one partial row
        if (lane < 16 && nvalid_w > 0)
          store_part(p.stats + (size_t)(mt * WM + wm) * p.N + nt * BN + wn * 64 + ni * 16 + lane, make_float2(s, q));
      } else if (lane < 16) {
        red[wm * BN + wn * 64 + ni * 16 + lane] = make_float2(s, q);
      }
    }
    __syncthreads();
    constexpr int HALVES = BM / 128;
    if (p.stat_tile == 128)
    for (int idx = tid; idx < HALVES * BN; idx += NT) {
      const int h = idx / BN, col = idx - h * BN;
      const int r0 = mt * BM + h * 128;
      if (r0 >= ph.M) continue;
      int na = ph.M - r0;
      na = na > 64 ? 64 : na;
      int nb = ph.M - (r0 + 64);
      nb = nb < 0 ? 0 : (nb > 64 ? 64 : nb);
      const float2 a0 = red[(2 * h) * BN + col], a1 = red[(2 * h + 1) * BN + col];
      float m2 = a0.y + a1.y;
      if (na > 0 && nb > 0) {
        const float d = a0.x / (float)na - a1.x / (float)nb;
        m2 += d * d * ((float)na * (float)nb / (float)(na + nb));
      }
      store_part(p.stats + (size_t)(mt * HALVES + h) * p.N + nt * BN + col, make_float2(a0.x + a1.x, m2));
    }
    __syncthreads();
    if (p.ffin.mode) {  // the statistics finalize folded in (bnfin.h): BM / stat_tile partial rows a tile
      bn_fwd_fin_arrive<NT, BN>(p.ffin, mt, nt, reinterpret_cast<double2*>(lds), &fin_flag);
      __syncthreads();
    }
  }

  // ---- epilogue: stage the C tile in LDS, then 16-byte coalesced (+addend) stores ----
  bf16* Cs = reinterpret_cast<bf16*>(lds);
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + mi * 16 + g * 4 + r;
        const int col = wn * 64 + ni * 16 + i16;
        Cs[row * LD + col] = (bf16)acc[mi][ni][r];
      }
  __syncthreads();
  constexpr int CPR = BN / 8;   // 16-byte chunks per row
  constexpr int RPP = NT / CPR;  // rows per store pass
  bf16* __restrict__ Cg = reinterpret_cast<bf16*>(p.c);
  const int c = tid % CPR;
  BwdEpiAcc<bf16, BW> bwd;
  if constexpr (BW != 0) bwd.init(p.bb, nt * BN + c * 8);
  // output pixel = GEMM row (forward, stride-1 dgrad): no division per stored row
  const bool c_ident = p.osh == 1 && p.osw == 1 && ph.oh0 == 0 && ph.ow0 == 0 && ph.Hq == p.Ho && ph.Wq == p.Wo;
  constexpr int NIT = BM / RPP, U = 4;
  static_assert(NIT * RPP == BM && NIT % U == 0, "epilogue row partition");
  for (int i0 = 0; i0 < NIT; i0 += U) {
    size_t off[U];
    bool ok[U];
    EpiIn in[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int rr = tid / CPR + RPP * (i0 + u);
      const int m = mt * BM + rr;
      ok[u] = m < ph.M;
      const int mm = ok[u] ? m : 0;
      if (c_ident) {
        off[u] = (size_t)mm * p.ldc + nt * BN + c * 8;
      } else {
        const int nimg = mm / HWq, rem = mm - nimg * HWq;
        const int qh = rem / ph.Wq, qw = rem - qh * ph.Wq;
        const int oh = qh * p.osh + ph.oh0, ow = qw * p.osw + ph.ow0;
        off[u] = (((size_t)nimg * p.Ho + oh) * p.Wo + ow) * p.ldc + nt * BN + c * 8;
      }
      if (ok[u]) epi_load<bf16, BW>(p, off[u], in[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) continue;
      const int rr = tid / CPR + RPP * (i0 + u);
      const u32x4 v = *reinterpret_cast<const u32x4*>(Cs + rr * LD + c * 8);
      st16_nt(Cg + off[u], epi_apply<bf16, BW>(p, v, in[u], bwd));
    }
  }
  if constexpr (BW != 0) {
    __syncthreads();
    bwd.template reduce<BN, NT>(p.bb, reinterpret_cast<float2*>(lds), tid / CPR, RPP, c,
                                (size_t)blockIdx.z * p.bb.prow + mt, p.N, nt * BN);
  }
  if constexpr (BW != 0) {
    if (p.fin.mode) {
      __syncthreads();
      bn_fin_arrive<NT, BN>(p.fin, blockIdx.z * p.bb.prow + mt, nt, reinterpret_cast<double2*>(lds), &fin_flag);
    }
  }
}

template <int BM, int BN, int BW, int NS>
static const char* glds_name() {
  static const std::string s = std::string("argus::igemm_glds_kernel<") + std::to_string(BM) + ", " +
                               std::to_string(BN) + ", " + std::to_string(BW) + ", " + std::to_string(NS) + ">";
  return s.c_str();
}

template <int BM, int BN, int BW, int NS>
static void launch_glds1(const IgParams& p0, int maxM, hipStream_t st) {
  IgParams p = p0;
  plan_fin(p, BM);
  plan_ffin(p, BM);
  dim3 grid(cdiv(maxM, BM) * (p.N / BN), 1, p.nphase);
  timed_launch(glds_name<BM, BN, BW, NS>(), igemm_glds_kernel<BM, BN, BW, NS>, grid,
               dim3((BM / 64) * (BN / 64) * 64), st, p);
}

template <int BM, int BN, int NS>
static void launch_glds_ns(const IgParams& p, int maxM, hipStream_t st) {
  switch (bwd_variant(p.bb)) {
    case 2: launch_glds1<BM, BN, 2, NS>(p, maxM, st); break;
    case 3: launch_glds1<BM, BN, 3, NS>(p, maxM, st); break;
    case 4: launch_glds1<BM, BN, 4, NS>(p, maxM, st); break;
    default: launch_glds1<BM, BN, 0, NS>(p, maxM, st);
  }
}

// policy key 41: ring depth of the data gradients (the forwards keep 3: no side stream beside them)
template <int BM, int BN>
static void launch_glds(const IgParams& p, int maxM, hipStream_t st) {
  if (!p.fwd && (*p.pol)[kGldsDgradStages] == 2) launch_glds_ns<BM, BN, 2>(p, maxM, st);
  else launch_glds_ns<BM, BN, 3>(p, maxM, st);
}

// policy key 8: smallest K (taps*C) served by the glds kernel (0 = off); 512 -> 1024 after the
// non-temporal epilogue stores (convbench B=64: fwd+dgrad 5.32 -> 5.20 ms). Key 9: fewest workgroups.
bool igemm_glds_ok(const IgParams& p, int maxM, int maxK) {
  const int min_k = (*p.pol)[kGldsMinK];
  if (min_k <= 0 || p.stem || p.pro_scale || p.ap.y || (!p.fwd && !(*p.pol)[kGldsDgrad]) || maxK < min_k || p.Cin % 64 || p.lda % 8 ||
      p.ldb % 8 || maxM < (*p.pol)[kGldsMinRows])
    return false;
  if (p.stats && p.stat_tile != 128 && p.stat_tile != 64) return false;
  for (int i = 0; i < p.nphase; ++i)
    if (p.ph[i].K % 64) return false;
  // measured (tools/convbench.py): a win only with >= one 8-wave workgroup per CU; the 4-wave
  // 256x64 tile and sub-CU-count grids lose to the register-staged kernel
  return !(p.N % 128 || cdiv(maxM, 256) * (p.N / 128) < (*p.pol)[kGldsMinGrid]);
}

bool igemm_glds_launch(const IgParams& p, int maxM, int maxK, hipStream_t st) {
  if (!igemm_glds_ok(p, maxM, maxK)) return false;
  launch_glds<256, 128>(p, maxM, st);
  return true;
}

}  // namespace argus
