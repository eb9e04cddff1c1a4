// Persistent 1x1 data gradient of a bottleneck's conv1 into the previous block's output BatchNorm:
// the BN-backward apply staged on its input (dy1 = ca*dm1 + cb*y1 + cc) and the block-output BN's
// backward in its epilogue (dm3 = (dx + dh) * relu'(out), partial sums {sum dm3, sum dm3*xhat3}, plus
// the downsample BN's second branch), with the finalize folded in.
//
// Why: the register-staged implicit GEMM (conv.hip, igemm_kernel<bf16, 64, 128, ..., 4, 19 | 20>)
// runs these as 64 x 128 tiles with one K-step each (K = the block width, 64..256): at B=64 the
// layer-1 launch is 16,384 workgroups, each of which stages its own copy of the weight tile, waits
// for its operands with nothing in flight, writes one BN partial row and takes one finalize ticket
// (bench.py slack table, profiles/r05a_slack.txt: 2.5 TB/s in the step, 1.0 ms of slack per step over
// the HBM bound; 6 VGPRs spilled at its 4-workgroups-per-CU budget). Here a workgroup owns one
// 128-column block for the whole launch: the weight block [128][K] stays in LDS, the workgroup walks
// its share of the 64-row tiles with the next tile's dm1 / y1 rows and epilogue operands (dh, y3,
// mask bits, yd) loaded under the current tile's MFMAs and stores, keeps the BN partial sums of its
// fixed channel chunk in registers across tiles and writes one partial row (one finalize ticket) per
// workgroup.
//
// Arithmetic is igemm_kernel's: the same apply (fp32 FMA, rounded to bf16), the same MFMA sequence per
// output element (K in 64-element steps, two 32-k MFMAs each), the same bf16 C tile, addend and mask:
// dm3 is bit-identical; the partial sums differ only in their summation grouping.
//
// Reference: the backward of Bottleneck.conv1 (+ bn3 / downsample BN backward of the previous block)
// of torchvision resnet50 (argus/models.py:43) under loss.backward() (argus/train.py:316).
#include "common.h"
#include "igemm.h"
#include "internal.h"
#include "ktimer.h"

namespace argus {

namespace {
constexpr int kP1BM = 64, kP1BN = 128, kP1LDC = kP1BN + 8;

// 16-byte chunk `chunk` of LDS row `row` (KC chunks per row): XOR-swizzled so the 16 rows one MFMA
// fragment read touches land on 16 distinct bank slots (KC = 8: igemm_kernel's 128-byte-row swizzle)
template <int KC> ARGUS_DEV int p1_pos(int row, int chunk) {
  return row * KC + (chunk ^ (KC >= 16 ? (row & 15) : ((row >> 1) & 7)));
}
}  // namespace

struct P1Params {
  const bf16* dm;   // [P][K] the A operand before the apply (dm1)
  const bf16* ay;   // [P][K] the apply's y (y1)
  const float *ca, *cb, *cc;  // [K]
  const bf16* wd;   // [N][K] w_dgrad of the 1x1 conv
  const bf16* addend;  // [P][N] or null (dh: the block input's gradient from the residual path)
  bf16* out;        // [P][N] dm3
  BnBwdEpi bb;      // mask mode 3 (+ second branch); partial rows = G
  BnFin fin;
  int P, N, G, NB, tiles;
};

template <int K, int BW>
__global__ __launch_bounds__(256, K >= 256 ? 1 : 2) void p1x1_dgrad_kernel(const P1Params p) {
  constexpr bool DUAL = BW == 4;
  constexpr int KC = K / 8;           // 16-byte chunks per A / W row
  constexpr int ARP = 256 / KC;       // A rows per staging pass
  constexpr int APS = kP1BM / ARP;    // A passes (= K / 32)
  constexpr int W_B = kP1BN * K * 2, A_B = kP1BM * K * 2, C_B = kP1BM * kP1LDC * 2;
  constexpr int RED_B = 8 * 16 * 16 * 8;  // BwdEpiAcc::reduce scratch: [E][RG][CPR] float2
  static_assert(C_B >= RED_B && A_B + C_B >= 256 * 32, "scratch");
  __shared__ __attribute__((aligned(16))) u32x4 lds[(W_B + A_B + C_B) / 16];
  __shared__ int fin_flag;
  u32x4* Wl = lds;
  u32x4* Al = lds + W_B / 16;
  bf16* Cs = reinterpret_cast<bf16*>(lds + (W_B + A_B) / 16);

  const int total = p.G * p.NB;
  const int wid = xcd_remap(blockIdx.x, total);  // the NB column blocks of one row split share an XCD
  const int nb = wid % p.NB, g0 = wid / p.NB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, i16 = lane & 15;

  // the weight block: rows nb*128 .. +127 of w_dgrad (resident for the launch)
#pragma unroll
  for (int i = 0; i < kP1BN * KC / 256; ++i) {
    const int idx = tid + 256 * i, r = idx / KC, c = idx - r * KC;
    Wl[p1_pos<KC>(r, c)] = ld16(p.wd + (size_t)(nb * kP1BN + r) * K + c * 8);
  }
  // A staging: a fixed channel chunk per thread (its apply coefficients in registers)
  const int ac = tid % KC, ar0 = tid / KC;
  float ca[8], cb[8], cc[8];
  BwdEpiAcc<bf16, 3>::ld(ca, p.ca + ac * 8);
  BwdEpiAcc<bf16, 3>::ld(cb, p.cb + ac * 8);
  BwdEpiAcc<bf16, 3>::ld(cc, p.cc + ac * 8);
  // epilogue: a fixed 8-channel chunk per thread, rows rg + 16 i
  const int ec = tid % 16, rg = tid / 16;
  const int col = nb * kP1BN + ec * 8;
  BwdEpiAcc<bf16, BW> bwd;
  bwd.init(p.bb, col);

  struct APre { u32x4 dm[APS], y[APS]; };
  struct EPre { u32x4 add[4], y[4], y2[DUAL ? 4 : 1]; unsigned bits[4]; };
  auto load_a = [&](int t, APre& S) {
#pragma unroll
    for (int i = 0; i < APS; ++i) {
      const int m = min(t * kP1BM + ar0 + ARP * i, p.P - 1);  // clamped; rows >= P are zeroed at staging
      S.dm[i] = ld16(p.dm + (size_t)m * K + ac * 8);
      S.y[i] = ld16(p.ay + (size_t)m * K + ac * 8);
    }
  };
  auto load_e = [&](int t, EPre& S) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t off = (size_t)min(t * kP1BM + rg + 16 * i, p.P - 1) * p.N + col;
      if (p.addend) S.add[i] = ld16(p.addend + off);
      S.y[i] = ld16(reinterpret_cast<const bf16*>(p.bb.y) + off);
      if constexpr (DUAL) S.y2[i] = ld16(reinterpret_cast<const bf16*>(p.bb.y2) + off);
      S.bits[i] = p.bb.bits[off / 8];
    }
  };

  APre A;
  EPre Ep;
  int t = g0;
  if (t < p.tiles) {
    load_a(t, A);
    load_e(t, Ep);
  }
  __syncthreads();  // the weight block
  for (; t < p.tiles; t += p.G) {
    // ---- stage dy = ca*dm + cb*y + cc (fp32, rounded to bf16), rows >= P zero ----
#pragma unroll
    for (int i = 0; i < APS; ++i) {
      const int r = ar0 + ARP * i;
      float d[8], yv[8];
      unpack(A.dm[i], d);
      unpack(A.y[i], yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = fmaf(ca[j], d[j], fmaf(cb[j], yv[j], cc[j]));
      Al[p1_pos<KC>(r, ac)] = sel(t * kP1BM + r < p.P, pack(d));
    }
    const int tn = t + p.G;
    if (tn < p.tiles) load_a(tn, A);  // the next tile's rows in flight during the MFMAs and the epilogue
    __syncthreads();

    // ---- 64 x 128 tile: wave (wm, wn) owns rows 32 wm .. +31, columns 64 wn .. +63 ----
    f32x4 acc[2][4];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < K / 32; ++kk) {  // igemm_kernel's order: 64-k steps, chunks 4*s2 + g
      const int ch = 4 * kk + g;
      u32x4 fa[2], fb[4];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) fa[mi] = Al[p1_pos<KC>(32 * wm + 16 * mi + i16, ch)];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) fb[ni] = Wl[p1_pos<KC>(64 * wn + 16 * ni + i16, ch)];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) Mma<bf16>::run(acc[mi][ni], fa[mi], fb[ni]);
    }
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          Cs[(32 * wm + 16 * mi + 4 * g + r) * kP1LDC + 64 * wn + 16 * ni + i16] = (bf16)acc[mi][ni][r];
    __syncthreads();

    // ---- epilogue: (dx + dh) * mask -> dm3, partial sums in registers; 16-byte non-temporal stores ----
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = rg + 16 * i;
      const int m = t * kP1BM + r;
      if (m >= p.P) continue;
      u32x4 v = *reinterpret_cast<const u32x4*>(Cs + r * kP1LDC + ec * 8);
      if (p.addend) {
        float f[8], o[8];
        unpack(v, f);
        unpack(Ep.add[i], o);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += o[j];
        v = pack(f);
      }
      st16_nt(p.out + (size_t)m * p.N + col, bwd.step(v, Ep.y[i], DUAL ? Ep.y2[DUAL ? i : 0] : Ep.y[i], Ep.bits[i]));
    }
    if (tn < p.tiles) load_e(tn, Ep);
  }
  __syncthreads();  // the C tile area becomes the reduction scratch
  bwd.template reduce<kP1BN, 256>(p.bb, reinterpret_cast<float2*>(Cs), rg, 16, ec, (size_t)g0, p.N, nb * kP1BN);
  if (p.fin.mode) {
    __syncthreads();
    bn_fin_arrive<256, kP1BN>(p.fin, g0, nb, reinterpret_cast<double2*>(Al), &fin_flag);
  }
}

// host ------------------------------------------------------------------------------------------

static int p1_occ(int K) { return K >= 256 ? 1 : 2; }

bool p1x1_ok(const argus_conv_desc& d, int dtype) {
  return dtype == ARGUS_BF16 && !d.stem && d.r == 1 && d.s == 1 && d.stride == 1 && d.pad == 0 &&
         (d.k == 64 || d.k == 128 || d.k == 256) && d.c % kP1BN == 0 && d.h == d.ho && d.w == d.wo &&
         (long)d.n * d.h * d.w > 0;
}

// row splits (= BN partial rows) of the persistent launch
int p1x1_rows(const argus_conv_desc& d) {
  const int tiles = (int)(((long)d.n * d.h * d.w + kP1BM - 1) / kP1BM);
  const int nb = d.c / kP1BN;
  int G = p1_occ(d.k) * 256 / nb;
  if (G < 1) G = 1;
  return G < tiles ? G : tiles;
}

int p1x1_launch(const argus_conv_desc& d, const void* dm, const void* wd, void* out, const void* addend,
                const argus_bn_bwd_epilogue* bn, const argus_bn_bwd_prologue* pro, hipStream_t st) {
  P1Params p{};
  p.dm = reinterpret_cast<const bf16*>(dm);
  p.ay = reinterpret_cast<const bf16*>(pro->y);
  p.ca = pro->ca; p.cb = pro->cb; p.cc = pro->cc;
  p.wd = reinterpret_cast<const bf16*>(wd);
  p.addend = reinterpret_cast<const bf16*>(addend);
  p.out = reinterpret_cast<bf16*>(out);
  p.P = d.n * d.h * d.w;
  p.N = d.c;
  p.NB = d.c / kP1BN;
  p.tiles = (p.P + kP1BM - 1) / kP1BM;
  p.G = p1x1_rows(d);
  BnBwdEpi& b = p.bb;
  b.y = bn->y; b.mean = bn->mean; b.invstd = bn->invstd; b.bits = bn->mask_bits; b.y2 = bn->y2;
  b.mean2 = bn->mean2; b.invstd2 = bn->invstd2;
  b.part = reinterpret_cast<float2*>(bn->part); b.part2 = reinterpret_cast<float2*>(bn->part2);
  b.mode = 3; b.prow = p.G;
  if (bn->workspace) {
    BnFin& f = p.fin;
    f.mode = 2; f.C = d.c; f.count = (long long)p.P;
    f.cnt = reinterpret_cast<unsigned*>(bn->workspace);
    f.red = reinterpret_cast<double2*>(reinterpret_cast<char*>(bn->workspace) + kBnCounterBytes);
    f.part = reinterpret_cast<const float2*>(bn->part); f.part2 = reinterpret_cast<const float2*>(bn->part2);
    f.gamma = bn->gamma; f.bmean = bn->mean; f.binvstd = bn->invstd;
    f.dgamma = bn->dgamma; f.dbeta = bn->dbeta; f.ca = bn->ca; f.cb = bn->cb; f.cc = bn->cc;
    f.gamma2 = bn->gamma2; f.bmean2 = bn->mean2; f.binvstd2 = bn->invstd2;
    f.dgamma2 = bn->dgamma2; f.dbeta2 = bn->dbeta2; f.ca2 = bn->ca2; f.cb2 = bn->cb2; f.cc2 = bn->cc2;
    bn_fin_plan(f, p.G, 1);
    f.rows = f.T;
  }
  const dim3 grid(p.G * p.NB);
  const bool dual = bn->y2 != nullptr;
  static const char* names[3][2] = {{"argus::p1x1_dgrad_kernel<64, 3>", "argus::p1x1_dgrad_kernel<64, 4>"},
                                    {"argus::p1x1_dgrad_kernel<128, 3>", "argus::p1x1_dgrad_kernel<128, 4>"},
                                    {"argus::p1x1_dgrad_kernel<256, 3>", "argus::p1x1_dgrad_kernel<256, 4>"}};
  const int ki = d.k == 64 ? 0 : (d.k == 128 ? 1 : 2);
  const char* nm = names[ki][dual];
  if (d.k == 64) {
    if (dual) timed_launch(nm, p1x1_dgrad_kernel<64, 4>, grid, dim3(256), st, p);
    else timed_launch(nm, p1x1_dgrad_kernel<64, 3>, grid, dim3(256), st, p);
  } else if (d.k == 128) {
    if (dual) timed_launch(nm, p1x1_dgrad_kernel<128, 4>, grid, dim3(256), st, p);
    else timed_launch(nm, p1x1_dgrad_kernel<128, 3>, grid, dim3(256), st, p);
  } else {
    if (dual) timed_launch(nm, p1x1_dgrad_kernel<256, 4>, grid, dim3(256), st, p);
    else timed_launch(nm, p1x1_dgrad_kernel<256, 3>, grid, dim3(256), st, p);
  }
  return check_launch("p1x1_dgrad_kernel");
}

// ================================================================================================
// Persistent statistics-only 1x1 forward (the bottleneck conv3 before argus_conv_fwd_bn_out): per-channel
// {sum, M2} of y = x w^T over all pixels, y never stored.
//
// Why: on the register-staged igemm (128 x 128 tiles, one or two K-steps) this pass is latency-bound:
// at B=64 the layer-1 launch is 8,192 workgroups that each stage a weight tile, run one K-step and
// write a partial row, 45 us for a 67 MB read (profiles/r05n_*). Here a workgroup keeps a column block
// of the weights [BNC][K] in LDS for the launch, walks its share of the 64-row tiles with the next
// two tiles' rows in flight in registers, and accumulates per-lane moments of its column values about a
// per-lane shift (no per-tile reductions); the lanes and row halves are Chan-merged once at the end:
// one partial row and one pixel count per row split. Products are igemm_kernel's (the same bf16
// operands, the same MFMA K order); only the moment grouping differs.
// ================================================================================================
struct P1FParams {
  const bf16* x;   // [P][K]
  const bf16* w;   // [N][K] w_fwd of the 1x1 conv
  float2* part;    // [G][N] {sum, M2}
  int* counts;     // [G] pixels per partial row (after the partials)
  int P, N, G, NB, tiles;
  BnFwdFin ffin;   // the statistics finalize folded in (argus_conv_fwd_fin; ffin.mode != 0)
};

template <int K, int BNC>
__global__ __launch_bounds__(256) void p1x1_fwd_stats_kernel(const P1FParams p) {
  constexpr int KC = K / 8;           // 16-byte chunks per row
  constexpr int ARP = 256 / KC;       // A rows per staging pass
  constexpr int APS = kP1BM / ARP;    // A passes
  constexpr int NI = BNC / 32;        // 16-column blocks per wave (waves 2 x 2: 32 rows x BNC/2 columns)
  constexpr int DEPTH = K <= 256 ? 2 : 1;  // tiles of A rows in flight in registers
  constexpr int W_B = BNC * K * 2, A_B = kP1BM * K * 2;
  static_assert(A_B >= 2 * BNC * 16, "reduction scratch");
  __shared__ __attribute__((aligned(16))) u32x4 lds[(W_B + A_B) / 16];
  u32x4* Wl = lds;
  u32x4* Al = lds + W_B / 16;

  const int total = p.G * p.NB;
  const int wid = xcd_remap(blockIdx.x, total);
  const int nb = wid % p.NB, g0 = wid / p.NB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int g = lane >> 4, i16 = lane & 15;

#pragma unroll
  for (int i = 0; i < BNC * KC / 256; ++i) {
    const int idx = tid + 256 * i, r = idx / KC, c = idx - r * KC;
    Wl[p1_pos<KC>(r, c)] = ld16(p.w + (size_t)(nb * BNC + r) * K + c * 8);
  }
  const int ac = tid % KC, ar0 = tid / KC;
  auto load_a = [&](int t, u32x4 (&A)[APS]) {
#pragma unroll
    for (int i = 0; i < APS; ++i) {
      const int m = min(t * kP1BM + ar0 + ARP * i, p.P - 1);
      A[i] = ld16(p.x + (size_t)m * K + ac * 8);
    }
  };
  // per-lane moments of its column values (rows 4g + r of its 16-row groups), about a per-lane shift
  // (the lane's first value of the column: sums of differences, no cancellation at large means)
  float shf[NI], ls[NI], lq[NI];
  int ln = 0;
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) { shf[ni] = 0.f; ls[ni] = 0.f; lq[ni] = 0.f; }

  auto tile = [&](int t, u32x4 (&A)[APS], int tnext) {
#pragma unroll
    for (int i = 0; i < APS; ++i) {
      const int r = ar0 + ARP * i;
      Al[p1_pos<KC>(r, ac)] = A[i];
    }
    if (tnext < p.tiles) load_a(tnext, A);  // DEPTH tiles ahead, under this tile's MFMAs
    __syncthreads();  // the A tile (and, first time round, the weight block)
    f32x4 acc[2][NI];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < K / 32; ++kk) {  // igemm_kernel's order: 64-k steps, chunks 4*s2 + g
      const int ch = 4 * kk + g;
      u32x4 fa[2], fb[NI];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) fa[mi] = Al[p1_pos<KC>(32 * wm + 16 * mi + i16, ch)];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) fb[ni] = Wl[p1_pos<KC>((BNC / 2) * wn + 16 * ni + i16, ch)];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) Mma<bf16>::run(acc[mi][ni], fa[mi], fb[ni]);
    }
    __syncthreads();  // every wave is done with the A tile before the next one is staged
    const int row0 = t * kP1BM + 32 * wm + 4 * g;
    if (row0 + 19 < p.P) {  // all 8 of this lane's rows (row0 + 16 mi + r) valid
      if (ln == 0) {
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) shf[ni] = acc[0][ni][0];
      }
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = acc[mi][ni][r] - shf[ni];
            ls[ni] += d;
            lq[ni] = fmaf(d, d, lq[ni]);
          }
      ln += 8;
    } else {  // the ragged last tile
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (row0 + 16 * mi + r >= p.P) continue;
          if (ln == 0) {
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) shf[ni] = acc[mi][ni][r];
          }
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            const float d = acc[mi][ni][r] - shf[ni];
            ls[ni] += d;
            lq[ni] = fmaf(d, d, lq[ni]);
          }
          ++ln;
        }
    }
  };

  u32x4 A0[APS], A1[DEPTH == 2 ? APS : 1];
  int t = g0;
  if (t < p.tiles) load_a(t, A0);
  if constexpr (DEPTH == 2) {
    if (t + p.G < p.tiles) load_a(t + p.G, A1);
    for (; t < p.tiles; t += 2 * p.G) {
      tile(t, A0, t + 2 * p.G);
      if (t + p.G < p.tiles) tile(t + p.G, A1, t + 3 * p.G);
    }
  } else {
    for (; t < p.tiles; t += p.G) tile(t, A0, t + p.G);
  }

  // lane moments -> {n, mean, M2}, Chan-merged over the 4 lanes of a column (g) and the two row
  // halves (wm, through LDS): one {sum, M2} row and pixel count per row split
  float* red = reinterpret_cast<float*>(Al);  // [wm][BNC] {n, mean, m2}
#pragma unroll
  for (int ni = 0; ni < NI; ++ni) {
    float n = (float)ln;
    float mean = ln ? shf[ni] + ls[ni] / n : 0.f;
    float m2 = ln ? fmaxf(lq[ni] - ls[ni] * ls[ni] / n, 0.f) : 0.f;
#pragma unroll
    for (int x = 16; x <= 32; x *= 2) {
      const float no = __shfl_xor(n, x, 64), mo = __shfl_xor(mean, x, 64), qo = __shfl_xor(m2, x, 64);
      const float nn = n + no;
      if (nn > 0.f) {
        const float d = mo - mean;
        m2 = m2 + qo + d * d * (n * no / nn);
        mean = mean + d * (no / nn);
      }
      n = nn;
    }
    if (g == 0) {
      const int col = (BNC / 2) * wn + 16 * ni + i16;
      red[(wm * BNC + col) * 3 + 0] = n;
      red[(wm * BNC + col) * 3 + 1] = mean;
      red[(wm * BNC + col) * 3 + 2] = m2;
    }
  }
  __syncthreads();
  if (tid < BNC) {
    const float na = red[tid * 3], ma = red[tid * 3 + 1], qa = red[tid * 3 + 2];
    const float nb_ = red[(BNC + tid) * 3], mb = red[(BNC + tid) * 3 + 1], qb = red[(BNC + tid) * 3 + 2];
    const float n = na + nb_;
    float sum = 0.f, m2 = 0.f;
    if (n > 0.f) {
      const float d = mb - ma;
      sum = na * ma + nb_ * mb;
      m2 = qa + qb + d * d * (na * nb_ / n);
    }
    store_part(p.part + (size_t)g0 * p.N + nb * BNC + tid, make_float2(sum, m2));
    // the row count, write-through: with the finalize folded in, every column block's workgroup writes it
    // (the same value), since the last arriver of column block nb reads the counts of its own group's
    // row splits, which only that column block's workgroups are ordered before
    if (tid == 0 && (nb == 0 || p.ffin.mode)) store_count(p.counts + g0, (int)n);
  }
  if (p.ffin.mode) {  // the statistics finalize folded in (bnfin.h): one partial row per row split
    __shared__ int fin_flag;
    __syncthreads();
    bn_fwd_fin_arrive<256, BNC>(p.ffin, g0, nb, reinterpret_cast<double2*>(Al), &fin_flag);
  }
}

static bool p1f_shape(const argus_conv_desc& d, int dtype) {
  return dtype == ARGUS_BF16 && !d.stem && d.r == 1 && d.s == 1 && d.stride == 1 && d.pad == 0 &&
         (d.c == 64 || d.c == 128 || d.c == 256 || d.c == 512) && d.k % (d.c == 512 ? 64 : 128) == 0 &&
         d.h == d.ho && d.w == d.wo && (long)d.n * d.h * d.w > 0;
}

static int p1f_bnc(const argus_conv_desc& d) { return d.c == 512 ? 64 : 128; }

// workgroups per CU the LDS admits (W block + A tile), at most 4 (registers: 90-104 VGPRs at K <= 128)
static int p1f_occ(const argus_conv_desc& d) {
  const int bytes = p1f_bnc(d) * d.c * 2 + kP1BM * d.c * 2;
  const int o = 160 * 1024 / bytes;
  return o < 1 ? 1 : (o > 4 ? 4 : o);
}

bool p1x1_fwd_stats_ok(const argus_conv_desc& d, int dtype, int enabled) { return enabled && p1f_shape(d, dtype); }

int p1x1_fwd_stats_rows(const argus_conv_desc& d) {
  const int tiles = (int)(((long)d.n * d.h * d.w + kP1BM - 1) / kP1BM);
  const int nb = d.k / p1f_bnc(d);
  int G = p1f_occ(d) * 256 / nb;
  if (G < 1) G = 1;
  return G < tiles ? G : tiles;
}

// the most pixels one partial row holds (argus_conv_fwd_stat_tile reports it negated: ragged rows)
int p1x1_fwd_stats_tile(const argus_conv_desc& d) {
  const int tiles = (int)(((long)d.n * d.h * d.w + kP1BM - 1) / kP1BM);
  const int G = p1x1_fwd_stats_rows(d);
  return ((tiles + G - 1) / G) * kP1BM;
}

int p1x1_fwd_stats_launch(const argus_conv_desc& d, const void* x, const void* w, float* stats, hipStream_t st,
                          const BnFwdFin* ffin) {
  P1FParams p{};
  p.x = reinterpret_cast<const bf16*>(x);
  p.w = reinterpret_cast<const bf16*>(w);
  p.P = d.n * d.h * d.w;
  p.N = d.k;
  p.NB = d.k / p1f_bnc(d);
  p.tiles = (p.P + kP1BM - 1) / kP1BM;
  p.G = p1x1_fwd_stats_rows(d);
  p.part = reinterpret_cast<float2*>(stats);
  p.counts = reinterpret_cast<int*>(stats + (size_t)2 * p.G * p.N);
  if (ffin) {  // the folded finalize: one ragged partial row per row split (argus_conv_fwd_fin)
    p.ffin = *ffin;
    if (bn_fwd_fin_plan(p.ffin, p.G, 1, p.G)) {
      p.ffin.tile_rows = -p1x1_fwd_stats_tile(d);
      p.ffin.part = p.part;
      g_ffin_folded = 1;
    } else {
      p.ffin.mode = 0;
    }
  }
  const dim3 grid(p.G * p.NB);
  switch (d.c) {
    case 64: timed_launch("argus::p1x1_fwd_stats_kernel<64, 128>", p1x1_fwd_stats_kernel<64, 128>, grid, dim3(256), st, p); break;
    case 128: timed_launch("argus::p1x1_fwd_stats_kernel<128, 128>", p1x1_fwd_stats_kernel<128, 128>, grid, dim3(256), st, p); break;
    case 256: timed_launch("argus::p1x1_fwd_stats_kernel<256, 128>", p1x1_fwd_stats_kernel<256, 128>, grid, dim3(256), st, p); break;
    default: timed_launch("argus::p1x1_fwd_stats_kernel<512, 64>", p1x1_fwd_stats_kernel<512, 64>, grid, dim3(256), st, p);
  }
  return check_launch("p1x1_fwd_stats_kernel");
}

}  // namespace argus
