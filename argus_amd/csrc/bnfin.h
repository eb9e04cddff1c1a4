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
