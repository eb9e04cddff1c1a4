// BatchNorm-backward finalize folded into the dgrad that produces its partial sums (the BN-backward
// epilogue's {sum dm, sum dm*xhat} per row tile). Replaces the separate bwd_finalize launch (bn.hip)
// on the critical path. (Folding the forward statistics finalize into the conv measured neutral: the
// forward keeps stats_finalize_kernel.)
//
// Two-level, deterministic, per column tile nt of the producer (COLS channels):
//  1. every workgroup stores its partial row(s) write-through (8-byte agent-scope atomic stores) and
//     takes a ticket on cnt[nt][g], g = its row-tile group (gt tiles); the last arriver of the group
//     merges the group's rows for its COLS channels in fp64, in row order, and publishes the result
//     write-through to red[g][C];
//  2. it then takes a ticket on cnt[nt][ng]; the last group merger sums the ng group results in group
//     order and finalizes those channels: dgamma / dbeta and the apply coefficients ca / cb / cc.
// Hand-off (MI355X_MICROARCH.md §Workgroup dispatch, valid form "sc1 stores + drain + ticket +
// consumer acquire"): every storing wave drains (s_waitcnt vmcnt(0)) before the workgroup barrier,
// one lane takes the agent-scope ticket, the last arriver runs an agent-scope acquire before its plain
// loads. Counters are reset to zero by the workgroup that drew the last ticket, so a workspace is
// reusable by the next launch in the same stream (never by two concurrent launches).
#pragma once
#include "common.h"

namespace argus {

typedef __attribute__((address_space(1))) unsigned long long fin_gu64;
typedef __attribute__((address_space(1))) unsigned fin_gu32;

// one float2 partial / double2 group result, stored write-through (agent-scope 8-byte atomic stores)
ARGUS_DEV void store_part(float2* p, float2 v) {
  __hip_atomic_store((fin_gu64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
ARGUS_DEV void store_wt2(double2* p, double2 v) {
  fin_gu64* q = (fin_gu64*)p;
  __hip_atomic_store(q, (unsigned long long)__double_as_longlong(v.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, (unsigned long long)__double_as_longlong(v.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every thread of the workgroup calls this (uniform). True in the workgroup that drew ticket n-1.
ARGUS_DEV bool fin_ticket(unsigned* cnt_, unsigned n, int* flag) {
  fin_gu32* cnt = (fin_gu32*)cnt_;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its write-through stores
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == n - 1;
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

struct BnFin {
  int mode;        // 0 off, 2 on (plain column sums)
  int T;           // producer row tiles (all dgrad phases); exactly one arrival per (tile, column tile)
  int rpw;         // partial rows per row tile
  int rows;        // valid partial rows
  int gt, ng;      // tiles per group, groups
  int C;           // channels = partial row length
  long long count; // pixels per channel
  unsigned* cnt;   // [C / 64 column tiles][ng + 1] (indexed with the producer's column tile width)
  double2* red;    // [ng][C]; the second branch at red + ng * C
  const float2* part;
  const float2* part2;
  // BN statistics of the forward, outputs (+ the second, downsample branch)
  const float* gamma;
  const float *bmean, *binvstd;
  float *dgamma, *dbeta, *ca, *cb, *cc;
  const float *gamma2, *bmean2, *binvstd2;
  float *dgamma2, *dbeta2, *ca2, *cb2, *cc2;
};

ARGUS_DEV void fin_backward(int c, double2 tot, double count, const float* gamma, const float* mean,
                            const float* invstd, float* dgamma, float* dbeta, float* ca, float* cb, float* cc) {
  const double S = tot.x, Tt = tot.y;
  if (dgamma) dgamma[c] = (float)Tt;
  if (dbeta) dbeta[c] = (float)S;
  const double gi = (double)gamma[c] * invstd[c];
  const double gi2 = gi * invstd[c];
  ca[c] = (float)gi;
  cb[c] = (float)(-gi2 * Tt / count);
  cc[c] = (float)(-gi * S / count + gi2 * Tt / count * mean[c]);
}

// Called by every thread of a producer workgroup after its partial rows are stored (store_part):
// tile t, column tile nt of width COLS. `scratch` = LDS of >= NT * 32 bytes (reused; callers are done
// with it) and an int flag. A thread merges a pair of adjacent columns (16-byte loads of two float2
// partials), 4 rows in flight per batch.
template <int NT, int COLS>
ARGUS_DEV void bn_fin_arrive(const BnFin& f, int t, int nt, double2* scratch, int* flag) {
  constexpr int CP = COLS / 2;   // column pairs
  static_assert(NT % CP == 0, "lanes per column pair");
  constexpr int LR = NT / CP;    // row lanes per column pair
  const int g = t / f.gt;
  const int gsz = min(f.gt, f.T - g * f.gt);
  unsigned* cnt = f.cnt + (size_t)nt * (f.ng + 1);
  if (!fin_ticket(cnt + g, (unsigned)gsz, flag)) return;
  const int cp = threadIdx.x % CP, lr = threadIdx.x / CP;
  const int c = nt * COLS + 2 * cp;
  const bool dual = f.part2 != nullptr;
  // level 1: the group's rows, fixed order (row lanes, then lanes in order)
  const int r0 = g * f.gt * f.rpw, r1 = min(f.rows, (g * f.gt + gsz) * f.rpw);
#pragma unroll
  for (int br = 0; br < 2; ++br) {
    if (br == 1 && !dual) break;
    const float2* part = br == 0 ? f.part : f.part2;
    double S0 = 0.0, Q0 = 0.0, S1 = 0.0, Q1 = 0.0;
    for (int rb = r0 + lr; rb < r1; rb += 4 * LR) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = *reinterpret_cast<const f32x4*>(part + (size_t)min(rb + u * LR, r1 - 1) * f.C + c);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = rb + u * LR < r1;  // selects, not branches (common.h kLoadBatch)
        S0 += ok ? (double)v[u].x : 0.0;
        S1 += ok ? (double)v[u].z : 0.0;
        Q0 += ok ? (double)v[u].y : 0.0;
        Q1 += ok ? (double)v[u].w : 0.0;
      }
    }
    scratch[2 * (lr * CP + cp)] = make_double2(S0, Q0);
    scratch[2 * (lr * CP + cp) + 1] = make_double2(S1, Q1);
    __syncthreads();
    if (lr == 0) {
      double2 a = scratch[2 * cp], b = scratch[2 * cp + 1];
      for (int i = 1; i < LR; ++i) {
        a.x += scratch[2 * (i * CP + cp)].x; a.y += scratch[2 * (i * CP + cp)].y;
        b.x += scratch[2 * (i * CP + cp) + 1].x; b.y += scratch[2 * (i * CP + cp) + 1].y;
      }
      double2* dst = f.red + (size_t)br * f.ng * f.C + (size_t)g * f.C + c;
      store_wt2(dst, a);
      store_wt2(dst + 1, b);
    }
    __syncthreads();
  }
  // level 2: the group results, fixed order
  if (!fin_ticket(cnt + f.ng, (unsigned)f.ng, flag)) return;
#pragma unroll
  for (int br = 0; br < 2; ++br) {
    if (br == 1 && !dual) break;
    const double2* red = f.red + (size_t)br * f.ng * f.C;
    double S0 = 0.0, Q0 = 0.0, S1 = 0.0, Q1 = 0.0;
    for (int qb = lr; qb < f.ng; qb += 4 * LR) {
      double2 a[4], b[4];  // four group results in flight (clamped, masked below: common.h kLoadBatch)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t q = (size_t)min(qb + u * LR, f.ng - 1);
        a[u] = red[q * f.C + c];
        b[u] = red[q * f.C + c + 1];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = qb + u * LR < f.ng;
        S0 += ok ? a[u].x : 0.0; Q0 += ok ? a[u].y : 0.0; S1 += ok ? b[u].x : 0.0; Q1 += ok ? b[u].y : 0.0;
      }
    }
    scratch[2 * (lr * CP + cp)] = make_double2(S0, Q0);
    scratch[2 * (lr * CP + cp) + 1] = make_double2(S1, Q1);
    __syncthreads();
    if (lr == 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double2 a = scratch[2 * cp + h];
        for (int i = 1; i < LR; ++i) { a.x += scratch[2 * (i * CP + cp) + h].x; a.y += scratch[2 * (i * CP + cp) + h].y; }
        if (br == 0) {
          fin_backward(c + h, a, (double)f.count, f.gamma, f.bmean, f.binvstd, f.dgamma, f.dbeta, f.ca, f.cb, f.cc);
        } else {
          fin_backward(c + h, a, (double)f.count, f.gamma2, f.bmean2, f.binvstd2, f.dgamma2, f.dbeta2, f.ca2,
                       f.cb2, f.cc2);
        }
      }
    }
    __syncthreads();
  }
}

// ---- the forward statistics finalize folded into the producing conv (argus_conv_fwd_fin) ----------
// Producer partial rows float2{sum, M2 about the row's own mean}, row r of n_r pixels (tile_rows, the
// last row the remainder; tile_rows < 0: int32 counts[rows] after the partials). The merge repeats
// stats_finalize_kernel (bn.hip) operation for operation, so mean / invstd / scale / shift and the running
// statistics are bit-identical to argus_bn_finalize's: its G = reduce_groups(rows) groups of rpg rows
// (here gt = rpg / rpw producer tiles a group; planned on the host only where rpg % rpw == 0), and in a
// group and over the groups 4 row lanes (lane l: rows / groups l, l + 4, ... in order; lanes added in
// order), every row's contribution S += sum, Q += M2 + sum^2 / n_r in fp64.
struct BnFwdFin {
  int mode;          // 0 off, 1 on
  int T, rpw;        // producer row tiles, partial rows per tile (row of tile t, k = t * rpw + k)
  int rows, C;       // partial rows, channels
  int gt, ng, G;     // tiles per group, groups with rows, stats_finalize_kernel's group count (>= ng)
  int tile_rows;     // pixels per full row (< 0: counts after the partials)
  long long count;   // pixels per channel
  unsigned* cnt;     // [C / 64][ng + 1] tickets (argus_bn_workspace_bytes workspace, zero between calls)
  double2* red;      // [ng][C]
  const float2* part;
  const float *gamma, *beta;
  float eps, momentum;
  float *running_mean, *running_var;
  long long* nbt;
  float *mean_o, *invstd_o, *scale_o, *shift_o;
};

ARGUS_DEV void fin_forward(const BnFwdFin& f, int c, double2 tot) {
  const double count = (double)f.count;
  const double mean = tot.x / count;
  double m2 = tot.y - tot.x * mean;
  if (m2 < 0.0) m2 = 0.0;
  const double var = m2 / count;
  const float invstd = (float)(1.0 / sqrt(var + (double)f.eps));
  const float sc = f.gamma[c] * invstd;
  if (f.mean_o) f.mean_o[c] = (float)mean;
  if (f.invstd_o) f.invstd_o[c] = invstd;
  if (f.scale_o) f.scale_o[c] = sc;
  if (f.shift_o) f.shift_o[c] = f.beta[c] - (float)mean * sc;
  if (f.running_mean) f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * (float)mean;
  if (f.running_var) {
    const double unbiased = count > 1.0 ? m2 / (count - 1.0) : var;
    f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * (float)unbiased;
  }
}

// Called by every thread of a producer workgroup (NT threads) after its partial rows are stored
// write-through (store_part): tile t, column tile nt of width COLS. scratch: LDS of >= 4 * COLS * 16
// bytes (reused; the caller is done with it) and an int flag. 4 * COLS threads take part in the merges.
template <int NT, int COLS>
ARGUS_DEV void bn_fwd_fin_arrive(const BnFwdFin& f, int t, int nt, double2* scratch, int* flag) {
  constexpr int CPT = 4 * COLS / NT < 1 ? 1 : 4 * COLS / NT;  // channels per thread (adjacent)
  constexpr int TC = COLS / CPT;                               // threads per row lane
  static_assert(CPT == 1 || CPT == 2, "one or two channels a thread");
  static_assert(TC * 4 <= NT, "four row lanes per channel");
  const int g = t / f.gt;
  const int gsz = min(f.gt, f.T - g * f.gt);
  unsigned* cnt = f.cnt + (size_t)nt * (f.ng + 1);
  if (!fin_ticket(cnt + g, (unsigned)gsz, flag)) return;
  const int cl = threadIdx.x % TC, lr = threadIdx.x / TC;  // lr < 4: the row lanes
  const int c = nt * COLS + cl * CPT;
  const bool act = lr < 4 && c < f.C;
  const int tr = f.tile_rows < 0 ? -f.tile_rows : f.tile_rows;
  const double inv_full = 1.0 / (double)tr;
  const int* counts = f.tile_rows < 0 ? reinterpret_cast<const int*>(f.part + (size_t)f.rows * f.C) : nullptr;
  // level 1: the group's rows [r0, r1)
  const int r0 = g * f.gt * f.rpw, r1 = min(f.rows, (g * f.gt + gsz) * f.rpw);
  double S[CPT], Q[CPT];
#pragma unroll
  for (int k = 0; k < CPT; ++k) { S[k] = 0.0; Q[k] = 0.0; }
  if (act)
    for (int rb = r0 + lr; rb < r1; rb += 4 * kLoadBatch) {
      float2 v[kLoadBatch][CPT];
      int nr[kLoadBatch];
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) {
        const float2* src = f.part + (size_t)min(rb + 4 * u, r1 - 1) * f.C + c;
        if constexpr (CPT == 2) {
          const f32x4 q4 = *reinterpret_cast<const f32x4*>(src);
          v[u][0] = make_float2(q4.x, q4.y);
          v[u][CPT - 1] = make_float2(q4.z, q4.w);
        } else {
          v[u][0] = *src;
        }
      }
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) nr[u] = counts ? counts[min(rb + 4 * u, r1 - 1)] : tr;
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) {
        const int r = rb + 4 * u;
        const long long left = f.count - (long long)r * tr;
        const double inv = counts ? (nr[u] > 0 ? 1.0 / (double)nr[u] : 0.0)
                                  : (left >= tr ? inv_full : 1.0 / (double)left);
        const bool ok = r < r1;  // selects, not branches (common.h kLoadBatch)
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          S[k] += ok ? (double)v[u][k].x : 0.0;
          Q[k] += ok ? (double)v[u][k].y + (double)v[u][k].x * (double)v[u][k].x * inv : 0.0;
        }
      }
    }
#pragma unroll
  for (int k = 0; k < CPT; ++k)
    if (lr < 4) scratch[lr * COLS + cl * CPT + k] = make_double2(S[k], Q[k]);
  __syncthreads();
  if (lr == 0 && act) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      double2 a = scratch[cl * CPT + k];
      for (int i = 1; i < 4; ++i) { a.x += scratch[i * COLS + cl * CPT + k].x; a.y += scratch[i * COLS + cl * CPT + k].y; }
      store_wt2(f.red + (size_t)g * f.C + c + k, a);
    }
  }
  __syncthreads();
  // level 2: the G group slots in order (those past the ng groups with rows hold zeros in
  // stats_finalize_kernel: the masked +0.0 here)
  if (!fin_ticket(cnt + f.ng, (unsigned)f.ng, flag)) return;
#pragma unroll
  for (int k = 0; k < CPT; ++k) { S[k] = 0.0; Q[k] = 0.0; }
  if (act)
    for (int gb = lr; gb < f.G; gb += 4 * kLoadBatch) {
      double2 v[kLoadBatch][CPT];
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u)
#pragma unroll
        for (int k = 0; k < CPT; ++k) v[u][k] = f.red[(size_t)min(gb + 4 * u, f.ng - 1) * f.C + c + k];
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) {
        const bool ok = gb + 4 * u < f.ng;
#pragma unroll
        for (int k = 0; k < CPT; ++k) {
          S[k] += ok ? v[u][k].x : 0.0;
          Q[k] += ok ? v[u][k].y : 0.0;
        }
      }
    }
#pragma unroll
  for (int k = 0; k < CPT; ++k)
    if (lr < 4) scratch[lr * COLS + cl * CPT + k] = make_double2(S[k], Q[k]);
  __syncthreads();
  if (nt == 0 && threadIdx.x == 0 && f.nbt) f.nbt[0] += 1;
  if (lr == 0 && act) {
#pragma unroll
    for (int k = 0; k < CPT; ++k) {
      double2 a = scratch[cl * CPT + k];
      for (int i = 1; i < 4; ++i) { a.x += scratch[i * COLS + cl * CPT + k].x; a.y += scratch[i * COLS + cl * CPT + k].y; }
      fin_forward(f, c + k, a);
    }
  }
}

// a ragged producer's int32 row count, stored write-through (the fold reads it from another CU)
ARGUS_DEV void store_count(int* p, int n) {
  __hip_atomic_store((__attribute__((address_space(1))) int*)p, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// host: the fold's groups for a producer of T row tiles with rpw partial rows each (rows = its partial
// rows): stats_finalize_kernel's grouping, false where a group boundary would split a producer tile
// (the caller then launches argus_bn_finalize instead)
inline bool bn_fwd_fin_plan(BnFwdFin& f, int T, int rpw, int rows) {
  const int G = rows < 64 ? 1 : (rows < 512 ? 8 : (rows < 4096 ? 32 : 64));  // bn.hip reduce_groups
  const int rpg = (rows + G - 1) / G;
  if (rpg % rpw || (long long)T * rpw < rows) return false;
  f.T = T;
  f.rpw = rpw;
  f.rows = rows;
  f.G = G;
  f.gt = rpg / rpw;
  f.ng = (T + f.gt - 1) / f.gt;
  return f.ng <= G;
}

// host: plan the groups of a producer with T row tiles of rpw partial rows each
inline void bn_fin_plan(BnFin& f, int T, int rpw) {
  f.T = T;
  f.rpw = rpw;
  int gt = 1;  // ~sqrt(T) tiles per group (both merge levels equally short), <= 64 groups
  while (gt * gt < T) ++gt;
  if ((T + gt - 1) / gt > 64) gt = (T + 63) / 64;
  const int minrows = 8;
  if (gt * rpw < minrows) gt = (minrows + rpw - 1) / rpw;
  if (gt > T) gt = T;
  f.gt = gt;
  f.ng = (T + gt - 1) / gt;
}

}  // namespace argus
