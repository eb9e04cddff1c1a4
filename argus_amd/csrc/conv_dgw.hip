// Fused data + weight gradient of a 1x1 stride-1 conv between two BatchNorms (ResNet-50 layer-1
// conv3: 64 -> 256 channels), one pass over the conv's output gradient.
//
// The unfused backward of this conv reads the bn3 input gradient dm3 and bn3's input y3 twice: once
// in the dgrad (which stages dy3 = ca*dm3 + cb*y3 + cc in its A-operand prologue) and once more in
// the side stream's weight gradient (which stages the same dy3). At layer 1 those are two 256-channel
// tensors (2 x 268 MB per block at B=64): the second read is the largest avoidable HBM traffic of the
// backward. Here every workgroup stages a 32-row tile of dy3 once into LDS and runs both GEMMs on it:
//   dgrad  dx[32 x 64]   = dy3[32 x 256] . W[256 x 64]     (B operand: W, LDS-resident for the kernel)
//   wgrad  dW[256 x 64] += dy3^T[256 x 32] . a2[32 x 64]   (transposed LDS reads of the same tile)
// The dgrad output goes through the BN-backward epilogue of bn2 (ReLU mask recomputed from
// y2*scale+shift > 0, partial sums {sum dm, sum dm*xhat}, optional folded finalize: bnfin.h); the
// weight gradient stays in registers across the workgroup's tiles (persistent grid, at most two
// workgroups per CU) and is written once per workgroup as an fp32 partial [G][256][64], summed in
// fixed order by wgrad_reduce_launch (deterministic).
//
// LDS (56 KB, two workgroups per CU): the 32-row dy3 tile as two images of 128 channels (256-byte
// rows, 32-byte slots XOR-swizzled per row as in wgrad_kernel, conv.hip: conflict-free
// ds_read_b64_tr_b16 for the transposed weight-gradient operand); the a2 tile in the same format; W as
// two 64-row images of 128 input-gradient channels. The dgrad's C tile and the BN / finalize scratch
// reuse the dy3 images after the MFMAs of a tile. Registers: the 256 x 64 weight-gradient tile (64
// fp32 per lane) plus the next tile's prefetched dm / y / a2 (36).
//
// Reference: the backward of Bottleneck.conv3 (torchvision resnet50, argus/models.py:43) under
// loss.backward() (argus/train.py:316): torch computes grad_input and grad_weight of that conv.
#include "common.h"
#include "igemm.h"
#include "internal.h"
#include "ktimer.h"

namespace argus {

namespace {

constexpr int kKo = 256;  // conv output channels = dy3 channels (GEMM K of the dgrad)
constexpr int kCi = 64;   // conv input channels = dx channels
constexpr int kBr = 32;   // rows (pixels) per tile
constexpr int kImg = kBr * 16;   // u32x4 per tile image of 256-byte rows
constexpr int kImgW = kCi * 16;  // u32x4 per W image (64 rows)

struct DgwParams {
  const bf16* dm;   // [P][256] bn3 input gradient (masked)
  const bf16* y;    // [P][256] bn3 input
  const float *ca, *cb, *cc;  // dy3 = ca*dm + cb*y + cc (bn3 backward coefficients)
  const bf16* wd;   // [64][256] dgrad weight (argus_conv_weight_prep w_dgrad)
  const bf16* x;    // [P][64] conv input (a2)
  bf16* out;        // [P][64] masked bn2 input gradient (BNE) or the plain dx (+ addend)
  const bf16* addend;  // !BNE: dx += addend (may alias out)
  float* part_w;    // [G][256][64] weight-gradient partials
  BnBwdEpi bb;      // bn2 (mode 2); partial rows = G
  BnFin fin;
  int P;
};

ARGUS_DEV int dgw_swz(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }

// u32x4 index of 16-byte chunk c (0..15) of row `row` in a 256-byte-row image
ARGUS_DEV int dgw_pos(int row, int c) { return row * 16 + ((((c >> 1) ^ dgw_swz(row)) << 1) | (c & 1)); }

// MFMA A/B fragment (lane (i16, g): row i16 of the block, k = 8g .. +7 of the 32-k step) from an image
// whose rows are the fragment rows: 16-byte chunk `chunk` of row `row`
ARGUS_DEV u32x4 dgw_frag(const u32x4* img, int row, int chunk) { return img[dgw_pos(row, chunk)]; }

// transposed fragment: lane (i16, g) gets channels slot*16 + i16 of image rows 8g .. 8g+7 (the image
// rows are the GEMM K dimension, 32 of them), as wgrad_kernel's reads (conv.hip)
ARGUS_DEV u32x4 dgw_frag_tr(const u32x4* img, int slot, int g, int i16) {
  const char* base = reinterpret_cast<const char*>(img);
  const int q = i16 >> 2, pq = i16 & 3;
  unsigned w[4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 8 * g + 4 * h + q;
    const char* addr = base + row * 256 + ((slot ^ dgw_swz(row)) << 5) + pq * 8;
    const s16x4 t = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (s16x4 __attribute__((address_space(3)))*)(uintptr_t)(uint32_t)(uintptr_t)addr);
    const uint2 u = __builtin_bit_cast(uint2, t);
    w[2 * h] = u.x;
    w[2 * h + 1] = u.y;
  }
  return u32x4{w[0], w[1], w[2], w[3]};
}

struct DgwStage {
  u32x4 dm[4], y[4];  // rows tid/32 + 8i, channel chunk tid%32
  u32x4 x;            // row tid/8, channel chunk tid%8
  u32x4 y2;           // BNE: the epilogue's BN input at the same (row, chunk) as x
};

}  // namespace

// BNE: the dx epilogue is bn2's backward (mask mode 2, partial sums, optional folded finalize); else a
// plain store of dx (+ addend: the first block's downsample, accumulated onto conv1's dgrad)
// YR: y (bn3's input, = this conv's own forward output conv(x, W)) is not read but recomputed from the
// staged a2 tile and W (the transposed dgrad images), with the forward GEMM's accumulation order, so the
// bf16 values equal what argus_conv_fwd would have stored (y need not exist: argus_conv_fwd_bn_out)
template <bool BNE, bool YR>
__global__ __launch_bounds__(256, 2) void dgw1x1_kernel(const DgwParams p) {
  // dy3 tile (2 images of 128 channels), a2 tile, W (2 images): 56 KB, two workgroups per CU; the
  // per-channel constants (apply coefficients of dy3, bn2's mean / invstd / scale / shift): 4 KB
  __shared__ __attribute__((aligned(16))) u32x4 lds[3 * kImg + 2 * kImgW];
  __shared__ __attribute__((aligned(16))) float cst[3 * kKo + 4 * kCi];
  u32x4* DY = lds;
  u32x4* XA = lds + 2 * kImg;
  u32x4* WD = lds + 3 * kImg;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int ntiles = (p.P + kBr - 1) / kBr;

  // W: 64 rows (dx channels) x 256 k (dy3 channels) -> two 128-k images
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = tid / 32 + 8 * i, c = tid % 32;
    WD[(c >> 4) * kImgW + dgw_pos(row, c & 15)] = ld16(p.wd + row * kKo + c * 8);
  }

  for (int i = tid; i < kKo; i += 256) {
    cst[i] = p.ca[i];
    cst[kKo + i] = p.cb[i];
    cst[2 * kKo + i] = p.cc[i];
  }
  if (BNE && tid < kCi) {
    float* b2 = cst + 3 * kKo;
    b2[tid] = p.bb.mean[tid];
    b2[kCi + tid] = p.bb.invstd[tid];
    b2[2 * kCi + tid] = p.bb.sc[tid];
    b2[3 * kCi + tid] = p.bb.sh[tid];
  }
  const int ca_c = tid % 32;  // this thread's dy3 channel chunk (apply)
  const int xc = tid % 8;     // its a2 / dx channel chunk (staging, epilogue)
  float esum[8], exs[8];  // bn2 partial sums of this thread's channel chunk: sum dm, sum dm*xhat
#pragma unroll
  for (int j = 0; j < 8; ++j) { esum[j] = 0.f; exs[j] = 0.f; }

  auto load = [&](int t, DgwStage& S) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = min(t * kBr + tid / 32 + 8 * i, p.P - 1);  // clamped; rows >= P are zeroed at staging
      S.dm[i] = ld16(p.dm + (size_t)m * kKo + ca_c * 8);
      if constexpr (!YR) S.y[i] = ld16(p.y + (size_t)m * kKo + ca_c * 8);
    }
    const size_t xo = (size_t)min(t * kBr + tid / 8, p.P - 1) * kCi + xc * 8;
    S.x = ld16(p.x + xo);
    if constexpr (BNE) S.y2 = ld16(reinterpret_cast<const bf16*>(p.bb.y) + xo);  // (the epilogue's, in flight)
  };

  f32x4 wacc[4][4];  // dW[ko = 64*wave + 16*mi + 4g + r][ci = 16*ni + i16]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) wacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int rb = wave >> 1, chh = wave & 1;  // dgrad: rows 16*rb .. +15, dx channels 32*chh .. +31
  DgwStage S;
  int t = blockIdx.x;
  if (t < ntiles) load(t, S);
  for (; t < ntiles; t += gridDim.x) {
    // ---- stage dy3 = ca*dm + cb*y + cc (fp32, rounded to bf16; rows past P are zero) and a2 ----
    if (t == (int)blockIdx.x) __syncthreads();  // the constants in LDS (first tile)
    u32x4 y2cur;  // this tile's epilogue BN input (S is refilled with the next tile below)
    if constexpr (BNE) y2cur = S.y2;
    if constexpr (YR) {
      // y[32 x 256] = a2[32 x 64] . W^T: wave w computes channels 64w .. 64w+63 (A from the a2 image, B by
      // transposed reads of the W images: k = input channel j = image row), then writes its bf16 values
      // into the dy3 images, where the apply below reads them as it would have read y
      XA[dgw_pos(tid / 8, xc)] = sel(t * kBr + tid / 8 < p.P, S.x);
      __syncthreads();
      f32x4 yacc[2][4];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) yacc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
      const u32x4* wimg = WD + (wave >> 1) * kImgW;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x4 fa[2], fb[4];
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) fa[mi] = dgw_frag(XA, 16 * mi + i16, 4 * s2 + g);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) fb[ni] = dgw_frag_tr(wimg + 32 * s2 * 16, (wave & 1) * 4 + ni, g, i16);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) Mma<bf16>::run(yacc[mi][ni], fa[mi], fb[ni]);
      }
      bf16* dyh = reinterpret_cast<bf16*>(DY);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int ch = 64 * wave + 16 * ni + i16;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mi + 4 * g + r;
            dyh[((ch >> 7) * kImg + dgw_pos(row, (ch & 127) >> 3)) * 8 + (ch & 7)] = (bf16)yacc[mi][ni][r];
          }
        }
      __syncthreads();
    }
    {
      float ca[8], cb[8], cc[8];  // from LDS: registers go to the accumulators
      BwdEpiAcc<bf16, 3>::ld(ca, cst + ca_c * 8);
      BwdEpiAcc<bf16, 3>::ld(cb, cst + kKo + ca_c * 8);
      BwdEpiAcc<bf16, 3>::ld(cc, cst + 2 * kKo + ca_c * 8);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = tid / 32 + 8 * i;
        float d[8], yv[8];
        unpack(S.dm[i], d);
        if constexpr (YR) unpack(DY[(ca_c >> 4) * kImg + dgw_pos(row, ca_c & 15)], yv);  // recomputed above
        else unpack(S.y[i], yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = fmaf(ca[j], d[j], fmaf(cb[j], yv[j], cc[j]));
        DY[(ca_c >> 4) * kImg + dgw_pos(row, ca_c & 15)] = sel(t * kBr + row < p.P, pack(d));
      }
      if constexpr (!YR) XA[dgw_pos(tid / 8, xc)] = sel(t * kBr + tid / 8 < p.P, S.x);
    }
    __syncthreads();
    if (t + (int)gridDim.x < ntiles) load(t + gridDim.x, S);  // next tile in flight during the MFMAs

    // ---- dgrad: 16 rows x 32 dx channels per wave, K = 256 ----
    f32x4 dacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {  // 32-k steps: 16-byte chunk 4*ks + g of the 256-channel row
      const int ch = 4 * ks + g;
      const u32x4 fa = dgw_frag(DY + (ch >> 4) * kImg, 16 * rb + i16, ch & 15);
#pragma unroll
      for (int ni = 0; ni < 2; ++ni)
        Mma<bf16>::run(dacc[ni], fa, dgw_frag(WD + (ch >> 4) * kImgW, 32 * chh + 16 * ni + i16, ch & 15));
    }
    // ---- wgrad: dW[64*wave .. +63][0..63] += dy3^T . a2 over the tile's 32 rows ----
    {
      u32x4 fa[4], fb[4];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) fa[mi] = dgw_frag_tr(DY + (wave >> 1) * kImg, (wave & 1) * 4 + mi, g, i16);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) fb[ni] = dgw_frag_tr(XA, ni, g, i16);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) Mma<bf16>::run(wacc[mi][ni], fa[mi], fb[ni]);
    }
    __syncthreads();  // the dy3 images become the C tile

    // ---- epilogue: bn2 backward (mask from y2*scale+shift > 0, partial sums), store dm2 ----
    constexpr int LD = kCi + 8;
    bf16* Cs = reinterpret_cast<bf16*>(DY);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(16 * rb + 4 * g + r) * LD + 32 * chh + 16 * ni + i16] = (bf16)dacc[ni][r];
    __syncthreads();
    const int m = t * kBr + tid / 8;
    if (!BNE && m < p.P) {  // plain: the bf16-rounded dx (+ addend), as igemm_kernel's epilogue
      const size_t off = (size_t)m * kCi + xc * 8;
      u32x4 v = *reinterpret_cast<const u32x4*>(Cs + (tid / 8) * LD + xc * 8);
      if (p.addend) {
        float f[8], o[8];
        unpack(v, f);
        unpack(ld16(p.addend + off), o);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += o[j];
        v = pack(f);
      }
      st16_nt(p.out + off, v);
    }
    if (BNE && m < p.P) {  // BwdEpiAcc<bf16, 2>::step with the per-channel constants from LDS
      const size_t off = (size_t)m * kCi + xc * 8;
      float d[8], yv[8], mu[8], is[8], sc[8], sh[8];
      unpack(*reinterpret_cast<const u32x4*>(Cs + (tid / 8) * LD + xc * 8), d);
      unpack(y2cur, yv);
      const float* b2 = cst + 3 * kKo;
      BwdEpiAcc<bf16, 3>::ld(mu, b2 + xc * 8);
      BwdEpiAcc<bf16, 3>::ld(is, b2 + kCi + xc * 8);
      BwdEpiAcc<bf16, 3>::ld(sc, b2 + 2 * kCi + xc * 8);
      BwdEpiAcc<bf16, 3>::ld(sh, b2 + 3 * kCi + xc * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        d[j] = fmaf(yv[j], sc[j], sh[j]) > 0.f ? d[j] : 0.f;
        esum[j] += d[j];
        exs[j] = fmaf(d[j], (yv[j] - mu[j]) * is[j], exs[j]);
      }
      st16_nt(p.out + off, pack(d));
    }
    __syncthreads();  // the C tile area is the next tile's dy3 image
  }

  // ---- this workgroup's weight-gradient partial ----
  float* pw = p.part_w + (size_t)blockIdx.x * kKo * kCi;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) pw[(64 * wave + 16 * mi + 4 * g + r) * kCi + 16 * ni + i16] = wacc[mi][ni][r];

  // ---- bn2 partial row blockIdx.x (+ the folded finalize); scratch: the dy3 + a2 images (24 KB) ----
  if constexpr (!BNE) return;
  BwdEpiAcc<bf16, 2> bwd;  // its fixed-order reduction of the per-thread sums (the constants are unused)
#pragma unroll
  for (int j = 0; j < 8; ++j) { bwd.s[j] = esum[j]; bwd.t[j] = exs[j]; }
  bwd.template reduce<kCi, 256>(p.bb, reinterpret_cast<float2*>(lds), tid / 8, 32, xc, blockIdx.x, kCi, 0);
  if (p.fin.mode) {
    __syncthreads();
    bn_fin_arrive<256, kCi>(p.fin, blockIdx.x, 0, reinterpret_cast<double2*>(lds),
                            reinterpret_cast<int*>(WD));  // flag: a word of the W images (free now)
  }
}

// host ------------------------------------------------------------------------------------------

static int dgw_grid(const argus_conv_desc& d) {
  const long P = (long)d.n * d.ho * d.wo;
  const long tiles = (P + kBr - 1) / kBr;
  return (int)(tiles < 512 ? tiles : 512);  // two workgroups per CU (56 KB LDS each)
}

bool conv_dgw_ok(const argus_conv_desc& d, int dtype) {
  return dtype == ARGUS_BF16 && !d.stem && d.r == 1 && d.s == 1 && d.stride == 1 && d.pad == 0 && d.k == kKo &&
         d.c == kCi && d.h == d.ho && d.w == d.wo && (long)d.n * d.ho * d.wo > 0;
}

size_t conv_dgw_ws_bytes(const argus_conv_desc& d, int dtype) {
  return conv_dgw_ok(d, dtype) ? (size_t)dgw_grid(d) * kKo * kCi * sizeof(float) : 0;
}

int conv_dgw_rows(const argus_conv_desc& d, int dtype) { return conv_dgw_ok(d, dtype) ? dgw_grid(d) : -1; }

int conv_dgw(const argus_conv_desc& d, int dtype, const void* dm, const void* wd, const void* x, void* dx,
             const void* addend, const argus_bn_bwd_epilogue* bn, const argus_bn_bwd_prologue* pro, float* dw,
             void* ws, size_t ws_bytes, hipStream_t st) {
  if (int e = conv_check_desc(d)) return e;
  if (!conv_dgw_ok(d, dtype)) {
    set_error("conv_dgrad_wgrad_bn: only bf16 1x1 stride-1 convs with 64 input and 256 output channels");
    return ARGUS_ERR_SHAPE;
  }
  if (!dm || !wd || !x || !dx || !dw || !pro || !pro->ca || !pro->cb || !pro->cc || pro->dy_out ||
      (bn && (addend || bn->mask_mode != 2 || !bn->y || !bn->mean || !bn->invstd || !bn->scale || !bn->shift ||
              !bn->part || bn->y2 || bn->y == dx))) {
    set_error("conv_dgrad_wgrad_bn: bad arguments (apply prologue without dy_out; a mask-mode-2 epilogue or none, "
              "an addend only without it)");
    return ARGUS_ERR_ARG;
  }
  const int G = dgw_grid(d);
  if (!ws || ws_bytes < (size_t)G * kKo * kCi * sizeof(float)) {
    set_error("conv_dgrad_wgrad_bn: workspace too small");
    return ARGUS_ERR_ARG;
  }
  DgwParams p{};
  p.dm = reinterpret_cast<const bf16*>(dm);
  p.y = reinterpret_cast<const bf16*>(pro->y);
  p.ca = pro->ca; p.cb = pro->cb; p.cc = pro->cc;
  p.wd = reinterpret_cast<const bf16*>(wd);
  p.x = reinterpret_cast<const bf16*>(x);
  p.out = reinterpret_cast<bf16*>(dx);
  p.addend = reinterpret_cast<const bf16*>(addend);
  p.part_w = reinterpret_cast<float*>(ws);
  p.P = d.n * d.ho * d.wo;
  const bool yr = p.y == nullptr;  // y recomputed from x and W (pro->y NULL)
  if (!bn) {
    g_launch_work = (yr ? 3.0 : 2.0) * 2.0 * p.P * kKo * kCi;
    g_launch_bytes = 2.0 * ((double)p.P * ((yr ? 1 : 2) * kKo + (addend ? 3 : 2) * kCi)) + 4.0 * kKo * kCi;
    if (yr) timed_launch("argus::dgw1x1_kernel<false, true>", dgw1x1_kernel<false, true>, dim3(G), dim3(256), st, p);
    else timed_launch("argus::dgw1x1_kernel<false, false>", dgw1x1_kernel<false, false>, dim3(G), dim3(256), st, p);
    if (int e = check_launch("dgw1x1_kernel")) return e;
    return wgrad_reduce_launch(reinterpret_cast<const float*>(ws), G, kKo, kCi, 0, dw, st);
  }
  BnBwdEpi& b = p.bb;
  b.y = bn->y; b.mean = bn->mean; b.invstd = bn->invstd; b.sc = bn->scale; b.sh = bn->shift;
  b.part = reinterpret_cast<float2*>(bn->part); b.mode = 2; b.prow = G;
  if (bn->workspace) {  // the bn2 backward finalize folded into this launch (bnfin.h)
    if (!bn->gamma || !bn->ca || !bn->cb || !bn->cc || kCi / 64 * 65 * 4 > (int)kBnCounterBytes) {
      set_error("conv_dgrad_wgrad_bn: bad finalize arguments");
      return ARGUS_ERR_ARG;
    }
    BnFin& f = p.fin;
    f.mode = 2; f.C = kCi; f.count = (long long)p.P;
    f.cnt = reinterpret_cast<unsigned*>(bn->workspace);
    f.red = reinterpret_cast<double2*>(reinterpret_cast<char*>(bn->workspace) + kBnCounterBytes);
    f.part = reinterpret_cast<const float2*>(bn->part);
    f.gamma = bn->gamma; f.bmean = bn->mean; f.binvstd = bn->invstd;
    f.dgamma = bn->dgamma; f.dbeta = bn->dbeta; f.ca = bn->ca; f.cb = bn->cb; f.cc = bn->cc;
    bn_fin_plan(f, G, 1);
    f.rows = f.T;
  }
  // algorithmic work (ktimer): both GEMMs; bytes: dm, y, a2, y2 read, dx written, dW (fp32) written
  g_launch_work = (yr ? 3.0 : 2.0) * 2.0 * p.P * kKo * kCi;
  g_launch_bytes = 2.0 * ((double)p.P * ((yr ? 1 : 2) * kKo + 3 * kCi)) + 4.0 * kKo * kCi;
  if (yr) timed_launch("argus::dgw1x1_kernel<true, true>", dgw1x1_kernel<true, true>, dim3(G), dim3(256), st, p);
  else timed_launch("argus::dgw1x1_kernel<true, false>", dgw1x1_kernel<true, false>, dim3(G), dim3(256), st, p);
  if (int e = check_launch("dgw1x1_kernel")) return e;
  return wgrad_reduce_launch(reinterpret_cast<const float*>(ws), G, kKo, kCi, 0, dw, st);
}

}  // namespace argus
