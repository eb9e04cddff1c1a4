// BatchNorm2d (train/eval), residual add, ReLU, MaxPool2d(3,2,1), AdaptiveAvgPool2d(1) for the
// ResNet-50 backbone (torchvision, argus/models.py:43,55), NHWC, fp32 statistics.
//
// Train-mode BN is a two-phase dependency: the conv epilogue (conv.hip) emits per-row-tile
// {sum, M2} partials; stats_finalize_kernel (one launch) turns them into mean / invstd and the fused
// coefficients scale/shift that the *consumer* applies (next conv's staging prologue, or
// bn_apply_kernel for block outputs). Backward: bn_bwd_reduce_kernel emits {sum dm, sum dm*xhat}
// partials, bwd_finalize_kernel gives dgamma/dbeta and dy = ca*dm + cb*y + cc coefficients,
// bn_bwd_apply_kernel materialises dy. Every cross-workgroup reduction is a fixed-order two-level
// reduction (deterministic, run-to-run bitwise reproducible).
#include "common.h"
#include "internal.h"
#include "bnfin.h"
#include "ktimer.h"

namespace argus {

// ---- forward statistics: merge of per-tile {sum, M2} partials ------------------------------------
// part float2[rows][C], tile t covers n_t = min(tile_rows, count - t*tile_rows) elements. In fp64:
// S = sum_t sum_t, Q = sum_t (M2_t + sum_t^2 / n_t)  ->  mean = S/n, M2 = Q - S^2/n
// (= sum_t M2_t + sum_t n_t (mean_t - mean)^2, the exact parallel-variance merge; the within-tile
// M2_t carry the large part, so fp64 leaves no cancellation problem).
// Backward partials {sum dm, sum dm*xhat} are plain column sums.
// group count of the finalize merge (fewer, longer groups measured neutral, -1 % and -4.5 % for 1/2,
// 1/4 and 1/8 of these counts)
static int reduce_groups(int rows) {
  return rows < 64 ? 1 : (rows < 512 ? 8 : (rows < 4096 ? 32 : 64));
}

// ---- one-launch statistics merge + finalize ---------------------------------------------------------
// Grid (C/64, G): block (x, g) merges partial rows [g*rpg, (g+1)*rpg) of its 64 channels into
// red[g][c] (fp64) exactly as the two-kernel form did, then takes a ticket on cnt[x]; the block that
// draws G-1 merges the G group results in a fixed order (deterministic) and finalizes its 64 channels.
// Hand-off: write-through (sc1) slab stores, every wave drains, relaxed agent-scope ticket; the
// reducer's agent-scope acquire precedes its plain loads (cdna_hip_programming.md §6 Guideline 16,
// counter form with sc1 stores; correct for any workgroup -> XCD placement). The reducer resets cnt[x], so the
// counters stay zero between calls; they are zeroed once when the workspace is allocated.
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

// a group result, stored write-through (sc1: two 8-byte agent-scope atomic stores), so publishing it
// needs no L2 write-back (release) fence — only the drain in ticket_last
ARGUS_DEV void store_wt(double2* p, double2 v) {
  gu64* q = (gu64*)p;
  __hip_atomic_store(q, (unsigned long long)__double_as_longlong(v.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, (unsigned long long)__double_as_longlong(v.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

ARGUS_DEV bool ticket_last(unsigned* cnt_, int G, int* flag) {
  gu32* cnt = (gu32*)cnt_;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == (unsigned)(G - 1);
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// fixed-order sum over the G group results of this block's 64 channels: kFinLanes row lanes, then the lanes in order
// Finalize blocks: 64 channels x kFinLanes row lanes. 16 lanes (1024 threads: one batch of loads per
// lane per level) measured slower in the step, 0.42 -> 0.57 ms/step of finalize (profiles/
// r04p_timeline.txt): a 16-wave workgroup waits for a CU with 16 free wave slots while the side
// stream's weight gradients hold them (one launch took 68 us).
constexpr int kFinLanes = 4;

ARGUS_DEV double2 merge_groups(const double2* red, int G, int C, int c, double2 (*lds)[64]) {
  const int lane_r = threadIdx.x >> 6, cl = threadIdx.x & 63;
  double S = 0.0, Q = 0.0;
  if (c < C)
    for (int gb = lane_r; gb < G; gb += kFinLanes * kLoadBatch) {  // G <= 64: at most 2 batches
      double2 v[kLoadBatch];
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) v[u] = red[(size_t)min(gb + kFinLanes * u, G - 1) * C + c];
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) {
        const bool ok = gb + kFinLanes * u < G;
        S += ok ? v[u].x : 0.0;
        Q += ok ? v[u].y : 0.0;
      }
    }
  lds[lane_r][cl] = make_double2(S, Q);
  __syncthreads();
  double2 a = lds[0][cl];
  for (int i = 1; i < kFinLanes; ++i) { a.x += lds[i][cl].x; a.y += lds[i][cl].y; }
  return a;
}

struct BnFinArgs {
  const float2* part;
  int rows, C, rpg, tile_rows, G;
  int64_t count;
  double2* red;
  unsigned* cnt;
  const float *gamma, *beta;
  float eps, momentum;
  float *running_mean, *running_var;
  int64_t* nbt;
  float *mean_o, *invstd_o, *scale_o, *shift_o;
};

__global__ __launch_bounds__(64 * kFinLanes) void stats_finalize_kernel(const BnFinArgs a) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lane_r = threadIdx.x >> 6;
  const int g = blockIdx.y;
  const int r0 = g * a.rpg, r1 = min(a.rows, r0 + a.rpg);
  // tile_rows < 0 (ragged producers): row r holds n_r = counts[r] elements, the int32 counts following
  // the float2[rows][C] partials
  const int tr = a.tile_rows < 0 ? -a.tile_rows : a.tile_rows;
  const double inv_full = 1.0 / (double)tr;
  const int* counts = a.tile_rows < 0 ? reinterpret_cast<const int*>(a.part + (size_t)a.rows * a.C) : nullptr;
  double S = 0.0, Q = 0.0;
  if (c < a.C)
    for (int rb = r0 + lane_r; rb < r1; rb += kFinLanes * kLoadBatch) {
      float2 v[kLoadBatch];  // the batch's loads in flight together (clamped rows, masked below)
      int nr[kLoadBatch];
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) v[u] = a.part[(size_t)min(rb + kFinLanes * u, r1 - 1) * a.C + c];
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) nr[u] = counts ? counts[min(rb + kFinLanes * u, r1 - 1)] : tr;
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) {
        const int r = rb + kFinLanes * u;
        const int64_t left = a.count - (int64_t)r * tr;
        const double inv = counts ? (nr[u] > 0 ? 1.0 / (double)nr[u] : 0.0)
                                  : (left >= tr ? inv_full : 1.0 / (double)left);
        const bool ok = r < r1;  // selects, not branches: a branch lets the compiler sink the loads
        S += ok ? (double)v[u].x : 0.0;
        Q += ok ? (double)v[u].y + (double)v[u].x * (double)v[u].x * inv : 0.0;
      }
    }
  __shared__ double2 red[kFinLanes][64];
  __shared__ int flag;
  red[lane_r][threadIdx.x & 63] = make_double2(S, Q);
  __syncthreads();
  if (lane_r == 0 && c < a.C) {
    double2 t = red[0][threadIdx.x];
    for (int i = 1; i < kFinLanes; ++i) { t.x += red[i][threadIdx.x].x; t.y += red[i][threadIdx.x].y; }
    store_wt(a.red + (size_t)g * a.C + c, t);
  }
  if (!ticket_last(a.cnt + blockIdx.x, a.G, &flag)) return;
  __syncthreads();
  const double2 tot = merge_groups(a.red, a.G, a.C, c, red);
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.nbt) a.nbt[0] += 1;
  if (lane_r != 0 || c >= a.C) return;
  const double count = (double)a.count;
  const double mean = tot.x / count;
  double m2 = tot.y - tot.x * mean;
  if (m2 < 0.0) m2 = 0.0;
  const double var = m2 / count;
  const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
  const float sc = a.gamma[c] * invstd;
  if (a.mean_o) a.mean_o[c] = (float)mean;
  if (a.invstd_o) a.invstd_o[c] = invstd;
  if (a.scale_o) a.scale_o[c] = sc;
  if (a.shift_o) a.shift_o[c] = a.beta[c] - (float)mean * sc;
  if (a.running_mean) a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * (float)mean;
  if (a.running_var) {
    const double unbiased = count > 1.0 ? m2 / (count - 1.0) : var;
    a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * (float)unbiased;
  }
}

__global__ void bn_eval_kernel(int C, const float* gamma, const float* beta, const float* rm, const float* rv,
                               float eps, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = 1.f / sqrtf(rv[c] + eps);
  const float sc = gamma[c] * inv;
  scale[c] = sc;
  shift[c] = beta[c] - rm[c] * sc;
}

// ---- elementwise kernels: channel-chunk-stationary threads ---------------------------------------
// Grid x = channel groups of CC chunks, y = pixel blocks; a thread owns one 16-byte channel chunk,
// keeps its per-channel coefficients in registers and walks pixels with stride PL (consecutive
// threads read consecutive chunks of a pixel row: fully coalesced 16-byte accesses).
struct EwGeom {
  int CC, PL, cgroups, rows;
  int64_t ppb;
};
// geometry (measured under the weight-gradient overlap, round 1: backward >= 64 pixels per block and
// <= 1024 blocks per channel group; apply passes target 512 workgroups, >= 16 pixels per thread)
constexpr int kBwdMinPx = 64, kBwdMaxRows = 1024, kEwTarget = 512, kEwMinPpt = 16;

static EwGeom ew_geom(int C, int E, int64_t pixels, int target_blocks) {
  EwGeom g;
  const int chunks = C / E;
  g.CC = chunks < 256 ? chunks : 256;
  g.PL = 256 / g.CC;
  g.cgroups = chunks / g.CC;
  int64_t rows = target_blocks / g.cgroups;
  const int64_t maxrows = (pixels + kEwMinPpt * g.PL - 1) / (kEwMinPpt * g.PL);  // min pixels per thread
  if (rows > maxrows) rows = maxrows;
  if (rows < 1) rows = 1;
  g.ppb = (pixels + rows - 1) / rows;
  g.rows = (int)((pixels + g.ppb - 1) / g.ppb);
  return g;
}

// Every elementwise kernel below walks its pixels U at a time: the U iterations' loads are issued
// before any of their arithmetic or stores, so each thread keeps U x (tensors read) 16-byte loads in
// flight (the memory-level parallelism an HBM stream needs at 4-8 waves per SIMD). U = 8 over 4:
// B=64 13.62-13.66 vs 13.67-13.75 ms in three interleaved rounds, B=256 level (no spills; the bf16
// BN-backward apply at 226 VGPRs, two workgroups per CU as the grid targets; profiles/r05an_*).
// A grid target of 1024 instead of 512 blocks was slower (13.70-13.77 ms, B=256 +0.7 %).
constexpr int kEwU = 8;

// MX-fp8 copy of a stored bf16 chunk (element offset off of a [P][C] tensor): 8 e4m3 bytes at out8 + off
// and, by the first of the 4 lanes of each 32-channel block (chunk cc % 4 == 0), its E8M0 scale at
// out8 + P*C + off / 32 (the x8 layout: argus_conv_fwd_x8)
ARGUS_DEV void st_x8(uint8_t* out8, int64_t pc, int64_t off, u32x4 o, int cc) {
  int e;
  const uint2 q = mx_fp8_quant8(o, e);
  *reinterpret_cast<uint2*>(out8 + off) = q;
  if ((cc & 3) == 0) out8[pc + off / 32] = (uint8_t)(127 + e);
}

template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(int64_t pixels, int C, int CC, int PL, int64_t ppb,
                                                       const T* __restrict__ y, const float* __restrict__ sc,
                                                       const float* __restrict__ sh, const T* __restrict__ res,
                                                       const float* __restrict__ rsc, const float* __restrict__ rsh,
                                                       int relu, T* __restrict__ out, uint8_t* __restrict__ mask_out,
                                                       uint8_t* __restrict__ out8) {
  constexpr int E = Chunk<T>::E;
  const int cc = threadIdx.x % CC, pl = threadIdx.x / CC;
  const int c0 = (blockIdx.x * CC + cc) * E;
  const int64_t p0 = blockIdx.y * ppb, p1 = min(pixels, p0 + ppb);
  float a[E], b[E], ra[E], rb[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    a[j] = sc[c0 + j];
    b[j] = sh[c0 + j];
    ra[j] = rsc ? rsc[c0 + j] : 1.f;
    rb[j] = rsc ? rsh[c0 + j] : 0.f;
  }
  for (int64_t px0 = p0 + pl; px0 < p1; px0 += kEwU * PL) {
    u32x4 yv[kEwU], rv[kEwU];
#pragma unroll
    for (int u = 0; u < kEwU; ++u) {
      const int64_t px = px0 + u * PL;
      const int64_t off = (px < p1 ? px : px0) * C + c0;
      yv[u] = ld16(y + off);
      if (res) rv[u] = ld16(res + off);
    }
#pragma unroll
    for (int u = 0; u < kEwU; ++u) {
      const int64_t px = px0 + u * PL;
      if (px >= p1) break;
      const int64_t off = px * C + c0;
      float f[E], r[E];
      unpack(yv[u], f);
      if (res) unpack(rv[u], r);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        float v = fmaf(f[j], a[j], b[j]);
        if (res) v += fmaf(r[j], ra[j], rb[j]);
        if (relu) v = fmaxf(v, 0.f);
        f[j] = v;
      }
      const u32x4 o = pack(f);
      st16(out + off, o);
      if (mask_out) mask_out[off / E] = chunk_positive_bits<T>(o);
      if constexpr (E == 8) {
        if (out8) st_x8(out8, pixels * C, off, o, cc);
      }
    }
  }
}

// ---- backward reduce ----------------------------------------------------------------------------
// Grid: x = channel groups of CC chunks, y = pixel blocks. Block: CC chunk-columns x PL pixel lanes.
static int bwd_rows(int64_t pixels) {
  int64_t r = (pixels + kBwdMinPx - 1) / kBwdMinPx;  // >= kBwdMinPx pixels per block
  return (int)(r > kBwdMaxRows ? kBwdMaxRows : (r < 1 ? 1 : r));
}
static void bwd_geometry(int C, int E, int64_t pixels, int& CC, int& PL, int& cgroups, int& rows, int64_t& ppb) {
  const int chunks = C / E;
  CC = chunks < 256 ? chunks : 256;
  PL = 256 / CC;
  cgroups = chunks / CC;
  rows = bwd_rows(pixels);
  ppb = (pixels + rows - 1) / rows;
  rows = (int)((pixels + ppb - 1) / ppb);
}

// Mask of the upstream ReLU for one 16-byte chunk (mode 0 none, 1 src>0, 2 y*S+H>0, 3 mask bits).
template <typename T>
ARGUS_DEV void apply_mask(int mode, float (&d)[Chunk<T>::E], const float (&yv)[Chunk<T>::E], const T* __restrict__ msrc,
                          unsigned bits, int64_t off, const float* S, const float* H) {
  constexpr int E = Chunk<T>::E;
  if (mode == 1) {
    float m[E];
    unpack(ld16(msrc + off), m);
#pragma unroll
    for (int j = 0; j < E; ++j) d[j] = m[j] > 0.f ? d[j] : 0.f;
  } else if (mode == 2) {
#pragma unroll
    for (int j = 0; j < E; ++j) d[j] = fmaf(yv[j], S[j], H[j]) > 0.f ? d[j] : 0.f;
  } else if (mode == 3) {  // bits: the chunk's mask byte, loaded with the chunk
#pragma unroll
    for (int j = 0; j < E; ++j) d[j] = (bits >> j) & 1u ? d[j] : 0.f;
  }
}

// Per-block column partials {sum dm, sum dm*xhat} of one (or, DUAL, two BN branches sharing dm:
// bn3 and the downsample BN of a bottleneck both see the gradient of the same block output).
template <typename T, bool DUAL>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(int64_t pixels, int C, int CC, int PL, int64_t ppb,
                                                            const T* __restrict__ dz, int mode,
                                                            const T* __restrict__ mask_src,
                                                            const uint8_t* __restrict__ mbits, const T* __restrict__ y,
                                                            const float* __restrict__ sc, const float* __restrict__ sh,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ invstd, float2* __restrict__ part,
                                                            const T* __restrict__ y2, const float* __restrict__ mean2,
                                                            const float* __restrict__ invstd2,
                                                            float2* __restrict__ part2) {
  constexpr int E = Chunk<T>::E;
  const int cc = threadIdx.x % CC, pl = threadIdx.x / CC;
  const int c0 = (blockIdx.x * CC + cc) * E;
  const int64_t p0 = blockIdx.y * ppb, p1 = min(pixels, p0 + ppb);
  float mu[E], is[E], S[E], H[E], s[E], t[E], mu2[E], is2[E], t2[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    mu[j] = mean[c0 + j];
    is[j] = invstd[c0 + j];
    S[j] = mode == 2 ? sc[c0 + j] : 0.f;
    H[j] = mode == 2 ? sh[c0 + j] : 0.f;
    s[j] = 0.f;
    t[j] = 0.f;
    mu2[j] = DUAL ? mean2[c0 + j] : 0.f;
    is2[j] = DUAL ? invstd2[c0 + j] : 0.f;
    t2[j] = 0.f;
  }
  for (int64_t px0 = p0 + pl; px0 < p1; px0 += kEwU * PL) {
    u32x4 dv[kEwU], yr[kEwU], y2r[kEwU];
    unsigned mb[kEwU];
#pragma unroll
    for (int u = 0; u < kEwU; ++u) {
      const int64_t px = px0 + u * PL;
      const int64_t off = (px < p1 ? px : px0) * C + c0;
      dv[u] = ld16(dz + off);
      yr[u] = ld16(y + off);
      if constexpr (DUAL) y2r[u] = ld16(y2 + off);
      mb[u] = mode == 3 ? mbits[off / E] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kEwU; ++u) {
      const int64_t px = px0 + u * PL;
      if (px >= p1) break;
      const int64_t off = px * C + c0;
      float d[E], yv[E];
      unpack(dv[u], d);
      unpack(yr[u], yv);
      apply_mask<T>(mode, d, yv, mask_src, mb[u], off, S, H);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        s[j] += d[j];
        t[j] = fmaf(d[j], (yv[j] - mu[j]) * is[j], t[j]);
      }
      if constexpr (DUAL) {
        float y2v[E];
        unpack(y2r[u], y2v);
#pragma unroll
        for (int j = 0; j < E; ++j) t2[j] = fmaf(d[j], (y2v[j] - mu2[j]) * is2[j], t2[j]);
      }
    }
  }
  __shared__ float2 red[256 * 8];
  // reduce over pixel lanes: layout red[pl][cc*E + j]
  const int W = CC * E;
#pragma unroll
  for (int br = 0; br < (DUAL ? 2 : 1); ++br) {
#pragma unroll
    for (int j = 0; j < E; ++j) red[pl * W + cc * E + j] = make_float2(s[j], br == 0 ? t[j] : t2[j]);
    __syncthreads();
    float2* out = br == 0 ? part : part2;
    for (int idx = threadIdx.x; idx < W; idx += 256) {
      float2 a = red[idx];
      for (int l = 1; l < PL; ++l) { a.x += red[l * W + idx].x; a.y += red[l * W + idx].y; }
      out[(size_t)blockIdx.y * C + blockIdx.x * W + idx] = a;
    }
    __syncthreads();
  }
}

struct BnBwdFinArgs {
  const float2* part;
  int rows, C, rpg, G;
  double count;
  double2* red;
  unsigned* cnt;
  const float *gamma, *mean, *invstd;
  float *dgamma, *dbeta, *ca, *cb, *cc;
};

// backward column sums + dgamma/dbeta/coefficients in one launch (same ticket hand-off)
__global__ __launch_bounds__(64 * kFinLanes) void bwd_finalize_kernel(const BnBwdFinArgs a) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lane_r = threadIdx.x >> 6;
  const int g = blockIdx.y;
  const int r0 = g * a.rpg, r1 = min(a.rows, r0 + a.rpg);
  double s = 0.0, q = 0.0;
  if (c < a.C)
    for (int rb = r0 + lane_r; rb < r1; rb += kFinLanes * kLoadBatch) {
      float2 v[kLoadBatch];
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) v[u] = a.part[(size_t)min(rb + kFinLanes * u, r1 - 1) * a.C + c];
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) {
        const bool ok = rb + kFinLanes * u < r1;
        s += ok ? (double)v[u].x : 0.0;
        q += ok ? (double)v[u].y : 0.0;
      }
    }
  __shared__ double2 red[kFinLanes][64];
  __shared__ int flag;
  red[lane_r][threadIdx.x & 63] = make_double2(s, q);
  __syncthreads();
  if (lane_r == 0 && c < a.C) {
    double2 t = red[0][threadIdx.x];
    for (int i = 1; i < kFinLanes; ++i) { t.x += red[i][threadIdx.x].x; t.y += red[i][threadIdx.x].y; }
    store_wt(a.red + (size_t)g * a.C + c, t);
  }
  if (!ticket_last(a.cnt + blockIdx.x, a.G, &flag)) return;
  __syncthreads();
  const double2 tot = merge_groups(a.red, a.G, a.C, c, red);
  if (lane_r != 0 || c >= a.C) return;
  const double S = tot.x, Tt = tot.y;
  if (a.dgamma) a.dgamma[c] = (float)Tt;
  if (a.dbeta) a.dbeta[c] = (float)S;
  const double gi = (double)a.gamma[c] * a.invstd[c];
  const double gi2 = gi * a.invstd[c];
  a.ca[c] = (float)gi;
  a.cb[c] = (float)(-gi2 * Tt / a.count);
  a.cc[c] = (float)(-gi * S / a.count + gi2 * Tt / a.count * a.mean[c]);
}

template <typename T, bool DUAL>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(int64_t pixels, int C, int CC, int PL, int64_t ppb,
                                                           const T* __restrict__ dz, int mode,
                                                           const T* __restrict__ mask_src,
                                                           const uint8_t* __restrict__ mbits, const T* __restrict__ y,
                                                           const float* __restrict__ sc, const float* __restrict__ sh,
                                                           const float* __restrict__ ca, const float* __restrict__ cb,
                                                           const float* __restrict__ cc_, T* __restrict__ dy,
                                                           T* __restrict__ dm_out, const T* __restrict__ y2,
                                                           const float* __restrict__ ca2, const float* __restrict__ cb2,
                                                           const float* __restrict__ cc2, T* __restrict__ dy2,
                                                           uint8_t* __restrict__ dy8) {
  constexpr int E = Chunk<T>::E;
  const int cc = threadIdx.x % CC, pl = threadIdx.x / CC;
  const int c0 = (blockIdx.x * CC + cc) * E;
  const int64_t p0 = blockIdx.y * ppb, p1 = min(pixels, p0 + ppb);
  float A[E], Bc[E], Cc[E], S[E], H[E], A2[E], B2[E], C2[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    A[j] = ca[c0 + j];
    Bc[j] = cb[c0 + j];
    Cc[j] = cc_[c0 + j];
    S[j] = mode == 2 ? sc[c0 + j] : 0.f;
    H[j] = mode == 2 ? sh[c0 + j] : 0.f;
    A2[j] = DUAL ? ca2[c0 + j] : 0.f;
    B2[j] = DUAL ? cb2[c0 + j] : 0.f;
    C2[j] = DUAL ? cc2[c0 + j] : 0.f;
  }
  for (int64_t px0 = p0 + pl; px0 < p1; px0 += kEwU * PL) {
    u32x4 dv[kEwU], yr[kEwU], y2r[kEwU];
    unsigned mb[kEwU];
#pragma unroll
    for (int u = 0; u < kEwU; ++u) {
      const int64_t px = px0 + u * PL;
      const int64_t off = (px < p1 ? px : px0) * C + c0;
      dv[u] = ld16(dz + off);
      yr[u] = ld16(y + off);
      if constexpr (DUAL) y2r[u] = ld16(y2 + off);
      mb[u] = mode == 3 ? mbits[off / E] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kEwU; ++u) {
      const int64_t px = px0 + u * PL;
      if (px >= p1) break;
      const int64_t off = px * C + c0;
      float d[E], yv[E];
      unpack(dv[u], d);
      unpack(yr[u], yv);
      apply_mask<T>(mode, d, yv, mask_src, mb[u], off, S, H);
      float o[E];
#pragma unroll
      for (int j = 0; j < E; ++j) o[j] = fmaf(A[j], d[j], fmaf(Bc[j], yv[j], Cc[j]));
      const u32x4 ov = pack(o);
      st16(dy + off, ov);
      if constexpr (E == 8) {
        if (dy8) st_x8(dy8, pixels * C, off, ov, cc);
      }
      if constexpr (DUAL) {
        float y2v[E];
        unpack(y2r[u], y2v);
#pragma unroll
        for (int j = 0; j < E; ++j) o[j] = fmaf(A2[j], d[j], fmaf(B2[j], y2v[j], C2[j]));
        st16(dy2 + off, pack(o));
      }
      if (dm_out) st16(dm_out + off, pack(d));
    }
  }
}

// ---- max pool 3x3/2 p1 fused with the stem BN + ReLU ---------------------------------------------
// One thread per (output pixel, 16-byte channel chunk). 32-bit index math (element counts < 2^31,
// checked on the host); the E argmax bytes of a chunk move as one 8-byte (bf16) / 4-byte (fp32) access.
template <int E> struct AmaxVec;
template <> struct AmaxVec<8> { typedef uint2 type; };
template <> struct AmaxVec<4> { typedef unsigned type; };

template <typename T>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(int n, int H, int W, int C, int Ho, int Wo,
                                                          const T* __restrict__ y, const float* __restrict__ sc,
                                                          const float* __restrict__ sh, T* __restrict__ out,
                                                          uint8_t* __restrict__ amax) {
  constexpr int E = Chunk<T>::E;
  typedef typename AmaxVec<E>::type AV;
  const int CH = C / E;
  const int total = n * Ho * Wo * CH;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = i / CH, ch = i - pix * CH;
    const int q = pix / Wo, ow = pix - q * Wo;
    const int img = q / Ho, oh = q - img * Ho;
    const int c0 = ch * E;
    float s[E], h[E], best[E];
    unsigned idx[E];
#pragma unroll
    for (int j = 0; j < E; ++j) { s[j] = sc[c0 + j]; h[j] = sh[c0 + j]; best[j] = -INFINITY; idx[j] = 0; }
    const T* yb = y + (size_t)img * H * W * C + c0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int ih = 2 * oh - 1 + r;
      if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int iw = 2 * ow - 1 + t;
        if ((unsigned)iw >= (unsigned)W) continue;
        float v[E];
        unpack(ld16(yb + (ih * W + iw) * C), v);
#pragma unroll
        for (int j = 0; j < E; ++j) {
          const float z = fmaxf(fmaf(v[j], s[j], h[j]), 0.f);
          if (z > best[j]) { best[j] = z; idx[j] = (unsigned)(r * 3 + t); }
        }
      }
    }
    st16(out + (size_t)pix * C + c0, pack(best));
    if constexpr (E == 8) {
      const uint2 a = {idx[0] | idx[1] << 8 | idx[2] << 16 | idx[3] << 24, idx[4] | idx[5] << 8 | idx[6] << 16 | idx[7] << 24};
      *reinterpret_cast<AV*>(amax + (size_t)pix * C + c0) = a;
    } else {
      *reinterpret_cast<AV*>(amax + (size_t)pix * C + c0) = idx[0] | idx[1] << 8 | idx[2] << 16 | idx[3] << 24;
    }
  }
}

// Gather form: one thread per (input pixel, 16-byte channel chunk) sums the gradients of the (at most
// 2 x 2) output windows whose argmax is this pixel; the four candidates' loads are issued together.
// BNE: the stem BatchNorm's backward reduction is fused in (the pooled input is relu(bn1(y0))):
// dm = dz * (y0*scale+shift > 0) is stored instead of dz, and each block writes its column partials
// {sum dm, sum dm*(y0-mean)*invstd} (a thread's channel chunk is fixed: the grid stride is a multiple
// of the chunks per pixel) — one partial row per block, the input of argus_bn_bwd_finalize.
// fin.mode: that finalize is folded in (bnfin.h, one producer tile per block, 64-channel column
// tiles): the last blocks to finish merge the rows and write dgamma/dbeta/ca/cb/cc while the pass is
// still resident. A separate finalize launch here is the first main-stream kernel after the pass and
// waits for CUs behind the side stream's layer-1 weight gradients (54 us of 60 in profiles/r04c_timeline.txt).
template <typename T, bool BNE>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(int n, int H, int W, int C, int Ho, int Wo,
                                                          const T* __restrict__ dout, const uint8_t* __restrict__ amax,
                                                          T* __restrict__ dz, const T* __restrict__ y,
                                                          const float* __restrict__ sc, const float* __restrict__ sh,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd, float2* __restrict__ part,
                                                          const BnFin fin) {
  constexpr int E = Chunk<T>::E;
  typedef typename AmaxVec<E>::type AV;
  const int CH = C / E;
  const int total = n * H * W * CH;
  float S[E], Hs[E], mu[E], is[E], s[E], t[E];
  const int ch0 = (int)(threadIdx.x % CH);
  if constexpr (BNE) {
#pragma unroll
    for (int j = 0; j < E; ++j) {
      S[j] = sc[ch0 * E + j]; Hs[j] = sh[ch0 * E + j]; mu[j] = mean[ch0 * E + j]; is[j] = invstd[ch0 * E + j];
      s[j] = 0.f; t[j] = 0.f;
    }
  }
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = i / CH, ch = i - pix * CH;
    const int q = pix / W, iw = pix - q * W;
    const int img = q / H, ih = q - img * H;
    const int c0 = ch * E;
    // output rows/cols whose 3x3/2 window (offset -1) covers this input pixel: oh in {ih/2, (ih+1)/2}
    const int oh0 = ih >> 1, oh1 = (ih + 1) >> 1, ow0 = iw >> 1, ow1 = (iw + 1) >> 1;
    const int ohs[2] = {oh0, oh1}, ows[2] = {ow0, ow1};
    u32x4 g[4];
    AV av[4];
    bool ok[4];
    unsigned want[4];
    const size_t off = (size_t)pix * C + c0;
    u32x4 yraw;
    if constexpr (BNE) yraw = ld16(y + off);  // issued with the gathers below (one memory latency, not two)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int oh = ohs[k >> 1], ow = ows[k & 1];
      const bool dup = ((k >> 1) && oh1 == oh0) || ((k & 1) && ow1 == ow0);
      ok[k] = !dup && oh < Ho && ow < Wo;
      want[k] = (unsigned)((ih - (2 * oh - 1)) * 3 + (iw - (2 * ow - 1)));
      const int o = ok[k] ? ((img * Ho + oh) * Wo + ow) * C + c0 : 0;
      g[k] = ld16(dout + o);
      av[k] = *reinterpret_cast<const AV*>(amax + o);
    }
    float acc[E];
#pragma unroll
    for (int j = 0; j < E; ++j) acc[j] = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!ok[k]) continue;
      float gv[E];
      unpack(g[k], gv);
      unsigned a[E];
      if constexpr (E == 8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { a[j] = (av[k].x >> (8 * j)) & 0xffu; a[4 + j] = (av[k].y >> (8 * j)) & 0xffu; }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = (av[k] >> (8 * j)) & 0xffu;
      }
#pragma unroll
      for (int j = 0; j < E; ++j) acc[j] += a[j] == want[k] ? gv[j] : 0.f;
    }
    if constexpr (BNE) {
      float yv[E];
      unpack(yraw, yv);
      const u32x4 r = pack(acc);  // the dz value as stored by the plain kernel (rounded to T)
      unpack(r, acc);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        const float d = fmaf(yv[j], S[j], Hs[j]) > 0.f ? acc[j] : 0.f;
        acc[j] = d;
        s[j] += d;
        t[j] = fmaf(d, (yv[j] - mu[j]) * is[j], t[j]);
      }
    }
    st16_nt(dz + off, pack(acc));  // 268 MB written once, read by the stem BN backward / wgrad later
  }
  if constexpr (BNE) {
    // element planes red[j][lane row][chunk]: the 8-byte writes of consecutive threads (consecutive
    // chunks) are contiguous (a [lane row][channel] layout put lanes 8 float2 apart: SQ_LDS_BANK_CONFLICT
    // / SQ_LDS_IDX_ACTIVE 0.82 at 376 x 672); the lane rows are summed in order. The summing reads of
    // one wave cover the E planes at the same row: planes kPlanePad float2 (64 bytes) apart beyond their
    // 256 entries, so plane j starts 16 banks after plane j-1 (unpadded, 512 j + 2q put all E planes on
    // the same banks: 0.70 in r04b_376x672_pmc_mfma_summary.txt)
    constexpr int kPlanePad = 8;
    constexpr int PS = 256 + kPlanePad;
    __shared__ __attribute__((aligned(16))) float2 red[PS * E];  // 16-byte: reused as double2 (fin)
    const int lanes = 256 / CH, ln = threadIdx.x / CH;
#pragma unroll
    for (int j = 0; j < E; ++j) red[j * PS + ln * CH + ch0] = make_float2(s[j], t[j]);
    __syncthreads();
    for (int col = threadIdx.x; col < C; col += 256) {
      const float2* plane = red + (col % E) * PS + col / E;  // channel col = chunk * E + j
      float2 a = plane[0];
      for (int l = 1; l < lanes; ++l) { a.x += plane[l * CH].x; a.y += plane[l * CH].y; }
      if (fin.mode) store_part(part + (size_t)blockIdx.x * C + col, a);  // write-through for the merge
      else part[(size_t)blockIdx.x * C + col] = a;
    }
    if (fin.mode) {
      __shared__ int flag;
      // red is free once fin_ticket's barrier has passed (>= 256 * 32 bytes: E >= 4)
      for (int nt = 0; nt < C / 64; ++nt)
        bn_fin_arrive<256, 64>(fin, blockIdx.x, nt, reinterpret_cast<double2*>(red), &flag);
    }
  }
}

// ---- global average pool ------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(int n, int hw, int C, const T* __restrict__ x,
                                                          float* __restrict__ feat) {
  const int64_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)n * C) return;
  const int img = (int)(i / C), c = (int)(i % C);
  float s = 0.f;
  for (int pb = 0; pb < hw; pb += kLoadBatch) {  // kLoadBatch loads in flight (common.h), same order
    float v[kLoadBatch];
#pragma unroll
    for (int u = 0; u < kLoadBatch; ++u) v[u] = to_f32(x[((int64_t)img * hw + min(pb + u, hw - 1)) * C + c]);
#pragma unroll
    for (int u = 0; u < kLoadBatch; ++u) s += pb + u < hw ? v[u] : 0.f;
  }
  feat[i] = s / (float)hw;
}

template <typename T>
__global__ __launch_bounds__(256) void avgpool_bwd_kernel(int64_t nchunks, int hw, int C, const float* __restrict__ dfeat,
                                                          T* __restrict__ dx) {
  constexpr int E = Chunk<T>::E;
  const float inv = 1.f / (float)hw;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < nchunks; i += (int64_t)gridDim.x * 256) {
    const int64_t e = i * E;
    const int c0 = (int)(e % C);
    const int64_t img = e / ((int64_t)hw * C);
    float f[E];
#pragma unroll
    for (int j = 0; j < E; ++j) f[j] = dfeat[img * C + c0 + j] * inv;
    st16(dx + e, pack(f));
  }
}

// demangled kernel names for the kernel timer (ktimer.h), one static string per instantiation
template <typename T> static const char* apply_name() {
  static const std::string s = std::string("argus::bn_apply_kernel<") + type_name<T>() + ">";
  return s.c_str();
}
template <typename T, bool DU> static const char* bred_name() {
  static const std::string s = std::string("argus::bn_bwd_reduce_kernel<") + type_name<T>() + ", " + bool_name(DU) + ">";
  return s.c_str();
}
template <typename T, bool DU> static const char* bapp_name() {
  static const std::string s = std::string("argus::bn_bwd_apply_kernel<") + type_name<T>() + ", " + bool_name(DU) + ">";
  return s.c_str();
}

static int grid_for(int64_t work, int64_t cap = 8192) {
  int64_t b = (work + 255) / 256;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

// maxpool backward with the stem BN reduction fused writes one partial row per block, which the serial
// bwd_finalize at the end of the backward pass merges: 2048 blocks (8 per CU, 32 waves: a full CU) keep
// the gather pass's occupancy and cut the merge to 2 load batches per lane (8192 rows took 4 + ~50 us).
#ifndef ARGUS_MPB_BLOCKS
#define ARGUS_MPB_BLOCKS 2048
#endif
constexpr int64_t kMaxpoolBwdBlocks = ARGUS_MPB_BLOCKS;

}  // namespace argus

using namespace argus;

extern "C" {

// [0, kBnCounterBytes): ticket counters (zero at allocation, kept zero by the kernels): one per
// 64-channel block for the finalize kernels, [column tile][65] for the finalize folded into the conv
// kernels (bnfin.h); then the fp64 group results double2[2 branches][64][channels].
size_t argus_bn_workspace_bytes(int channels) { return kBnCounterBytes + (size_t)2 * 64 * channels * sizeof(double2); }

int argus_bn_finalize(int C, int rows, int tile_rows, const float* part, int64_t count, const float* gamma,
                      const float* beta, float eps, float momentum, float* rm, float* rv, int64_t* nbt, float* mean,
                      float* invstd, float* scale, float* shift, void* ws, argus_stream_t stream) {
  if (C <= 0 || rows <= 0 || tile_rows == 0 || count <= 0 || !part || !gamma || !beta || !ws ||
      (int64_t)rows * (tile_rows < 0 ? -tile_rows : tile_rows) < count) {
    set_error("bn_finalize: bad arguments");
    return ARGUS_ERR_ARG;
  }
  if ((C + 63) / 64 > (int)(kBnCounterBytes / 4)) {
    set_error("bn_finalize: too many channels for the workspace counters");
    return ARGUS_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  BnFinArgs a;
  a.G = reduce_groups(rows);
  a.part = reinterpret_cast<const float2*>(part); a.rows = rows; a.C = C; a.rpg = (rows + a.G - 1) / a.G;
  a.tile_rows = tile_rows; a.count = count;
  a.cnt = reinterpret_cast<unsigned*>(ws);
  a.red = reinterpret_cast<double2*>(reinterpret_cast<char*>(ws) + kBnCounterBytes);
  a.gamma = gamma; a.beta = beta; a.eps = eps; a.momentum = momentum; a.running_mean = rm; a.running_var = rv;
  a.nbt = nbt; a.mean_o = mean; a.invstd_o = invstd; a.scale_o = scale; a.shift_o = shift;
  g_launch_work = 0.0;  // algorithmic bytes: the {sum, M2} partials read
  g_launch_bytes = 8.0 * rows * C;
  timed_launch("argus::stats_finalize_kernel", stats_finalize_kernel, dim3((C + 63) / 64, a.G), dim3(64 * kFinLanes),
               st, a);
  return check_launch("stats_finalize_kernel");
}

int argus_bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                         float* scale, float* shift, argus_stream_t stream) {
  hipLaunchKernelGGL(bn_eval_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, C, gamma, beta, rm,
                     rv, eps, scale, shift);
  return check_launch("bn_eval_kernel");
}

int argus_bn_apply(int dtype, int64_t pixels, int C, const void* y, const float* scale, const float* shift,
                   const void* res, const float* rsc, const float* rsh, int relu, void* out, uint8_t* mask_out,
                   argus_stream_t stream) {
  const int E = dtype == ARGUS_BF16 ? 8 : 4;
  if (C % E || pixels <= 0 || !y || !scale || !shift || !out || ((rsc == nullptr) != (rsh == nullptr)) ||
      (rsc && !res)) {
    set_error("bn_apply: bad arguments");
    return ARGUS_ERR_ARG;
  }
  const EwGeom g = ew_geom(C, E, pixels, kEwTarget);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(g.cgroups, g.rows);
  const double pc = (double)pixels * C;
  g_launch_work = 0.0;  // algorithmic bytes: y, residual, out, mask bits
  g_launch_bytes = (16.0 / E) * pc * (2.0 + (res ? 1.0 : 0.0)) + (mask_out ? pc / E : 0.0);
  if (dtype == ARGUS_BF16)
    timed_launch(apply_name<bf16>(), bn_apply_kernel<bf16>, grid, dim3(256), st, pixels, C, g.CC, g.PL,
                 g.ppb, (const bf16*)y, scale, shift, (const bf16*)res, rsc, rsh, relu, (bf16*)out, mask_out,
                 (uint8_t*)nullptr);
  else
    timed_launch(apply_name<float>(), bn_apply_kernel<float>, grid, dim3(256), st, pixels, C, g.CC,
                 g.PL, g.ppb, (const float*)y, scale, shift, (const float*)res, rsc, rsh, relu, (float*)out, mask_out,
                 (uint8_t*)nullptr);
  return check_launch("bn_apply_kernel");
}

int argus_bn_apply_x8(int64_t pixels, int C, const void* y, const float* scale, const float* shift, const void* res,
                      const float* rsc, const float* rsh, int relu, void* out, uint8_t* mask_out, void* out8,
                      argus_stream_t stream) {
  if (C % 32 || pixels <= 0 || !y || !scale || !shift || !out || !out8 || ((rsc == nullptr) != (rsh == nullptr)) ||
      (rsc && !res)) {
    set_error("bn_apply_x8: bad arguments (bf16, C a multiple of 32, out8 required)");
    return ARGUS_ERR_ARG;
  }
  const EwGeom g = ew_geom(C, 8, pixels, kEwTarget);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(g.cgroups, g.rows);
  const double pc = (double)pixels * C;
  g_launch_work = 0.0;  // algorithmic bytes: y, residual, out, mask bits, the fp8 copy and its scales
  g_launch_bytes = 2.0 * pc * (2.0 + (res ? 1.0 : 0.0)) + (mask_out ? pc / 8 : 0.0) + pc * (1.0 + 1.0 / 32);
  timed_launch("argus::bn_apply_kernel<__bf16, x8>", bn_apply_kernel<bf16>, grid, dim3(256), st, pixels, C, g.CC,
               g.PL, g.ppb, (const bf16*)y, scale, shift, (const bf16*)res, rsc, rsh, relu, (bf16*)out, mask_out,
               (uint8_t*)out8);
  return check_launch("bn_apply_kernel");
}

int argus_bn_bwd_rows(int64_t pixels, int C) {
  (void)C;
  const int r = bwd_rows(pixels);
  const int64_t ppb = (pixels + r - 1) / r;
  return (int)((pixels + ppb - 1) / ppb);
}

int argus_bn_bwd_reduce(int dtype, int64_t pixels, int C, const void* dz, int mode, const void* mask,
                        const void* y, const float* scale, const float* shift, const float* mean,
                        const float* invstd, float* part, const void* y2, const float* mean2, const float* invstd2,
                        float* part2, argus_stream_t stream) {
  const int E = dtype == ARGUS_BF16 ? 8 : 4;
  if (C % E || pixels <= 0) { set_error("bn_bwd_reduce: bad shape"); return ARGUS_ERR_SHAPE; }
  const bool dual = y2 != nullptr;
  if (!dz || !y || !mean || !invstd || !part || mode < 0 || mode > 3 || ((mode == 1 || mode == 3) && !mask) ||
      (mode == 2 && (!scale || !shift)) || (dual && (mode == 2 || !mean2 || !invstd2 || !part2))) {
    set_error("bn_bwd_reduce: bad arguments");
    return ARGUS_ERR_ARG;
  }
  int CC, PL, cg, rows;
  int64_t ppb;
  bwd_geometry(C, E, pixels, CC, PL, cg, rows, ppb);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(cg, rows);
  const uint8_t* mb = mode == 3 ? (const uint8_t*)mask : nullptr;
  {
    const double pc = (double)pixels * C;
    g_launch_work = 0.0;  // algorithmic bytes: dz, y (, y2), mask tensor or bits
    g_launch_bytes = (16.0 / E) * pc * (2.0 + (mode == 1 ? 1.0 : 0.0) + (dual ? 1.0 : 0.0)) + (mode == 3 ? pc / E : 0.0);
  }
#define ARGUS_BWD_REDUCE(TT, DU)                                                                                   \
  timed_launch(bred_name<TT, DU>(), bn_bwd_reduce_kernel<TT, DU>, grid, dim3(256), st,   \
               pixels, C, CC, PL, ppb, (const TT*)dz, mode, mode == 1 ? (const TT*)mask : (const TT*)nullptr, mb,  \
               (const TT*)y, scale, shift, mean, invstd, (float2*)part, (const TT*)y2, mean2, invstd2,            \
               (float2*)part2)
  if (dtype == ARGUS_BF16) {
    if (dual) ARGUS_BWD_REDUCE(bf16, true); else ARGUS_BWD_REDUCE(bf16, false);
  } else {
    if (dual) ARGUS_BWD_REDUCE(float, true); else ARGUS_BWD_REDUCE(float, false);
  }
#undef ARGUS_BWD_REDUCE
  return check_launch("bn_bwd_reduce_kernel");
}

int argus_bn_bwd_finalize(int C, int rows, const float* part, int64_t count, const float* gamma, const float* mean,
                          const float* invstd, float* dgamma, float* dbeta, float* ca, float* cb, float* cc, void* ws,
                          argus_stream_t stream) {
  if (C <= 0 || rows <= 0 || count <= 0 || !part || !gamma || !mean || !invstd || !ca || !cb || !cc || !ws ||
      (C + 63) / 64 > (int)(kBnCounterBytes / 4)) {
    set_error("bn_bwd_finalize: bad arguments");
    return ARGUS_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  BnBwdFinArgs a;
  a.G = reduce_groups(rows);
  a.part = reinterpret_cast<const float2*>(part); a.rows = rows; a.C = C; a.rpg = (rows + a.G - 1) / a.G;
  a.count = (double)count;
  a.cnt = reinterpret_cast<unsigned*>(ws);
  a.red = reinterpret_cast<double2*>(reinterpret_cast<char*>(ws) + kBnCounterBytes);
  a.gamma = gamma; a.mean = mean; a.invstd = invstd; a.dgamma = dgamma; a.dbeta = dbeta; a.ca = ca; a.cb = cb; a.cc = cc;
  hipLaunchKernelGGL(bwd_finalize_kernel, dim3((C + 63) / 64, a.G), dim3(64 * kFinLanes), 0, st, a);
  return check_launch("bwd_finalize_kernel");
}

int argus_bn_bwd_apply(int dtype, int64_t pixels, int C, const void* dz, int mode, const void* mask, const void* y,
                       const float* scale, const float* shift, const float* ca, const float* cb, const float* cc,
                       void* dy, void* dm_out, const void* y2, const float* ca2, const float* cb2, const float* cc2,
                       void* dy2, argus_stream_t stream) {
  const int E = dtype == ARGUS_BF16 ? 8 : 4;
  const bool dual = y2 != nullptr;
  if (C % E || pixels <= 0 || !dz || !y || !ca || !cb || !cc || !dy || mode < 0 || mode > 3 ||
      ((mode == 1 || mode == 3) && !mask) || (mode == 2 && (!scale || !shift)) ||
      (dual && (mode == 2 || !ca2 || !cb2 || !cc2 || !dy2))) {
    set_error("bn_bwd_apply: bad arguments");
    return ARGUS_ERR_ARG;
  }
  const EwGeom g = ew_geom(C, E, pixels, kEwTarget);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(g.cgroups, g.rows);
  const uint8_t* mb = mode == 3 ? (const uint8_t*)mask : nullptr;
  {
    const double pc = (double)pixels * C;
    g_launch_work = 0.0;  // algorithmic bytes: dz, y, dy (, y2, dy2) (, dm), mask tensor or bits
    g_launch_bytes = (16.0 / E) * pc *
                         (3.0 + (mode == 1 ? 1.0 : 0.0) + (dual ? 2.0 : 0.0) + (dm_out ? 1.0 : 0.0)) +
                     (mode == 3 ? pc / E : 0.0);
  }
#define ARGUS_BWD_APPLY(TT, DU)                                                                                    \
  timed_launch(bapp_name<TT, DU>(), bn_bwd_apply_kernel<TT, DU>, grid, dim3(256), st,     \
               pixels, C, g.CC, g.PL, g.ppb, (const TT*)dz, mode, mode == 1 ? (const TT*)mask : (const TT*)nullptr,  \
               mb, (const TT*)y, scale, shift, ca, cb, cc, (TT*)dy, (TT*)dm_out, (const TT*)y2, ca2, cb2, cc2,      \
               (TT*)dy2, (uint8_t*)nullptr)
  if (dtype == ARGUS_BF16) {
    if (dual) ARGUS_BWD_APPLY(bf16, true); else ARGUS_BWD_APPLY(bf16, false);
  } else {
    if (dual) ARGUS_BWD_APPLY(float, true); else ARGUS_BWD_APPLY(float, false);
  }
#undef ARGUS_BWD_APPLY
  return check_launch("bn_bwd_apply_kernel");
}

int argus_bn_bwd_apply_x8(int64_t pixels, int C, const void* dm, const void* y, const float* ca, const float* cb,
                          const float* cc, void* dy, void* dy8, argus_stream_t stream) {
  if (C % 32 || pixels <= 0 || !dm || !y || !ca || !cb || !cc || !dy || !dy8) {
    set_error("bn_bwd_apply_x8: bad arguments (bf16, C a multiple of 32, dy8 required)");
    return ARGUS_ERR_ARG;
  }
  const EwGeom g = ew_geom(C, 8, pixels, kEwTarget);
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(g.cgroups, g.rows);
  const double pc = (double)pixels * C;
  g_launch_work = 0.0;  // algorithmic bytes: dm, y, dy, the fp8 copy and its scales
  g_launch_bytes = 2.0 * pc * 3.0 + pc * (1.0 + 1.0 / 32);
  timed_launch("argus::bn_bwd_apply_kernel<__bf16, false, x8>", bn_bwd_apply_kernel<bf16, false>, grid, dim3(256), st,
               pixels, C, g.CC, g.PL, g.ppb, (const bf16*)dm, 0, (const bf16*)nullptr, (const uint8_t*)nullptr,
               (const bf16*)y, (const float*)nullptr, (const float*)nullptr, ca, cb, cc, (bf16*)dy, (bf16*)nullptr,
               (const bf16*)nullptr, (const float*)nullptr, (const float*)nullptr, (const float*)nullptr,
               (bf16*)nullptr, (uint8_t*)dy8);
  return check_launch("bn_bwd_apply_kernel");
}

int argus_maxpool_fwd(int dtype, int n, int h, int w, int c, const void* y, const float* scale, const float* shift,
                      void* out, uint8_t* amax, argus_stream_t stream) {
  const int E = dtype == ARGUS_BF16 ? 8 : 4;
  if (c % E) { set_error("maxpool_fwd: bad channels"); return ARGUS_ERR_SHAPE; }
  if ((int64_t)n * h * w * c >= (1LL << 31)) { set_error("maxpool_fwd: tensor exceeds 2^31 elements"); return ARGUS_ERR_SHAPE; }
  const int ho = (h + 2 - 3) / 2 + 1, wo = (w + 2 - 3) / 2 + 1;
  const int64_t work = (int64_t)n * ho * wo * (c / E);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ARGUS_BF16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<bf16>, dim3(grid_for(work)), dim3(256), 0, st, n, h, w, c, ho, wo,
                       (const bf16*)y, scale, shift, (bf16*)out, amax);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(grid_for(work)), dim3(256), 0, st, n, h, w, c, ho, wo,
                       (const float*)y, scale, shift, (float*)out, amax);
  return check_launch("maxpool_fwd_kernel");
}

int argus_maxpool_bwd(int dtype, int n, int h, int w, int c, const void* dout, const uint8_t* amax, void* dz,
                      argus_stream_t stream) {
  return argus_maxpool_bwd_bn(dtype, n, h, w, c, dout, amax, dz, nullptr, nullptr, nullptr, nullptr, nullptr,
                              nullptr, stream);
}

int argus_maxpool_bwd_bn_rows(int dtype, int n, int h, int w, int c) {
  const int E = dtype == ARGUS_BF16 ? 8 : 4;
  return c % E ? -1 : grid_for((int64_t)n * h * w * (c / E), kMaxpoolBwdBlocks);
}

int argus_maxpool_bwd_bn(int dtype, int n, int h, int w, int c, const void* dout, const uint8_t* amax, void* dm,
                         const void* y, const float* scale, const float* shift, const float* mean,
                         const float* invstd, float* part, argus_stream_t stream) {
  return argus_maxpool_bwd_bn_fin(dtype, n, h, w, c, dout, amax, dm, y, scale, shift, mean, invstd, part, nullptr,
                                  nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, stream);
}

int argus_maxpool_bwd_bn_fin(int dtype, int n, int h, int w, int c, const void* dout, const uint8_t* amax, void* dm,
                             const void* y, const float* scale, const float* shift, const float* mean,
                             const float* invstd, float* part, const float* gamma, float* dgamma, float* dbeta,
                             float* ca, float* cb, float* cc, void* workspace, argus_stream_t stream) {
  const int E = dtype == ARGUS_BF16 ? 8 : 4;
  if (c % E || 256 % (c / E) || c > 256) { set_error("maxpool_bwd: bad channels"); return ARGUS_ERR_SHAPE; }
  if ((int64_t)n * h * w * c >= (1LL << 31)) { set_error("maxpool_bwd: tensor exceeds 2^31 elements"); return ARGUS_ERR_SHAPE; }
  const bool bne = y != nullptr;
  if (bne && (!scale || !shift || !mean || !invstd || !part)) { set_error("maxpool_bwd_bn: bad arguments"); return ARGUS_ERR_ARG; }
  const int ho = (h + 2 - 3) / 2 + 1, wo = (w + 2 - 3) / 2 + 1;
  const int64_t work = (int64_t)n * h * w * (c / E);
  hipStream_t st = (hipStream_t)stream;
  float2* pt = reinterpret_cast<float2*>(part);
  BnFin f{};
  if (workspace) {  // the finalize folded in
    if (!bne || !gamma || !ca || !cb || !cc || c % 64) {
      set_error("maxpool_bwd_bn_fin: bad finalize arguments (needs y, gamma, ca/cb/cc, channels % 64 == 0)");
      return ARGUS_ERR_ARG;
    }
    f.mode = 2; f.C = c; f.count = (long long)n * h * w;
    bn_fin_plan(f, grid_for(work, kMaxpoolBwdBlocks), 1);
    f.rows = f.T;
    if ((size_t)(c / 64) * (f.ng + 1) * 4 > kBnCounterBytes) { set_error("maxpool_bwd_bn_fin: too many groups"); return ARGUS_ERR_ARG; }
    f.cnt = reinterpret_cast<unsigned*>(workspace);
    f.red = reinterpret_cast<double2*>(reinterpret_cast<char*>(workspace) + kBnCounterBytes);
    f.part = pt;
    f.gamma = gamma; f.bmean = mean; f.binvstd = invstd;
    f.dgamma = dgamma; f.dbeta = dbeta; f.ca = ca; f.cb = cb; f.cc = cc;
  }
#define ARGUS_MPB(TT, B)                                                                                          \
  hipLaunchKernelGGL((maxpool_bwd_kernel<TT, B>), dim3(grid_for(work, kMaxpoolBwdBlocks)), dim3(256), 0, st, n, h, w, c, ho, wo,     \
                     (const TT*)dout, amax, (TT*)dm, (const TT*)y, scale, shift, mean, invstd, pt, f)
  if (dtype == ARGUS_BF16) {
    if (bne) ARGUS_MPB(bf16, true); else ARGUS_MPB(bf16, false);
  } else {
    if (bne) ARGUS_MPB(float, true); else ARGUS_MPB(float, false);
  }
#undef ARGUS_MPB
  return check_launch("maxpool_bwd_kernel");
}

int argus_avgpool_fwd(int dtype, int n, int hw, int c, const void* x, float* feat, argus_stream_t stream) {
  const int64_t work = (int64_t)n * c;
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (int)((work + 255) / 256);
  if (dtype == ARGUS_BF16)
    hipLaunchKernelGGL(avgpool_fwd_kernel<bf16>, dim3(blocks), dim3(256), 0, st, n, hw, c, (const bf16*)x, feat);
  else
    hipLaunchKernelGGL(avgpool_fwd_kernel<float>, dim3(blocks), dim3(256), 0, st, n, hw, c, (const float*)x, feat);
  return check_launch("avgpool_fwd_kernel");
}

int argus_avgpool_bwd(int dtype, int n, int hw, int c, const float* dfeat, void* dx, argus_stream_t stream) {
  const int E = dtype == ARGUS_BF16 ? 8 : 4;
  if (c % E) { set_error("avgpool_bwd: bad channels"); return ARGUS_ERR_SHAPE; }
  const int64_t nch = (int64_t)n * hw * c / E;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == ARGUS_BF16)
    hipLaunchKernelGGL(avgpool_bwd_kernel<bf16>, dim3(grid_for(nch)), dim3(256), 0, st, nch, hw, c, dfeat, (bf16*)dx);
  else
    hipLaunchKernelGGL(avgpool_bwd_kernel<float>, dim3(grid_for(nch)), dim3(256), 0, st, nch, hw, c, dfeat, (float*)dx);
  return check_launch("avgpool_bwd_kernel");
}

}  // extern "C"
