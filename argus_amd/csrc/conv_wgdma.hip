// Weight gradient of a 1x1 stride-1 conv with both operands streamed by LDS-DMA (dW[k][c] = sum_p
// dy[p][k] * x[p][c], the BN-backward apply dy = ca*dm + cb*y + cc formed on the MFMA fragments).
//
// Why: the register-staged wgrad_kernel<bf16, 128, 128, ..., FAST, AP> keeps one k-step of operands in
// flight in registers (a two-deep register ring spills at two workgroups per CU), so each 64-pixel
// k-step waits about one HBM latency; in the step it moves ~1.6-2.0 TB/s (bench.py's dominant kernel).
// Here the operands never pass through registers on their way to LDS: a ring of NS stages of 32-pixel
// k-steps is filled by global_load_lds, NS - 1 k-steps ahead of the MFMAs, with counted vmcnt waits.
//
// Layout (as wgrad_kernel's bf16 images): per operand and stage, 32 pixel rows x 256 B (128 channels);
// the 32-byte slot s of row r sits at slot s ^ swz32(r), so the eight rows a 32-lane half touches in
// one ds_read_b64_tr_b16 hit distinct banks. The DMA writes lane-linear 1 KB pieces (4 rows); the
// swizzle is applied to each lane's source address. Rows past the split's range read a zero page: x
// rows are zero, so they add exact zeros whatever the dm / y rows give.
//
// Arithmetic is wgrad_kernel's: the same apply (fp32 FMAs, rounded to bf16) on the same values, the same
// MFMA sequence over 32-pixel K blocks in increasing order, the same split boundaries: the fp32 partials
// are bit-identical.
//
// Reference: the weight gradient of the bottleneck 1x1 convs (torchvision resnet50, argus/models.py:43)
// under loss.backward() (argus/train.py:316).
#include "common.h"
#include "igemm.h"
#include "internal.h"
#include "ktimer.h"

namespace argus {

namespace {
__device__ __attribute__((aligned(64))) u32x4 wgdma_zero_page[4];  // zero-initialised (static storage)

ARGUS_DEV int wg_swz(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }  // = conv.hip's swz32

template <int N> ARGUS_DEV void wg_waitvm() {
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
ARGUS_DEV void wg_gl16(const void* src, uint32_t lds_byte_addr) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(uintptr_t)lds_byte_addr, 16, 0,
                                   0);
}
ARGUS_DEV void wg_bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// Transposed LDS reads as inline asm (as conv_halo.hip's weight gradient): as a builtin the compiler
// assumes it may alias the LDS-DMA stages in flight and drains them (vmcnt(0)) before the first read of
// every k-step. The ring's counted waits and barriers order the reads; wg_tie waits for their data
// (lgkmcnt(0)) with the results tied, so no copy of them moves above the wait.
ARGUS_DEV uint2 wg_tr(uint32_t addr) {
  uint2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr) : "memory");
  return r;
}
// tie the first four results to the wait; the rest follow in volatile asm after it
template <int N> ARGUS_DEV void wg_tie(uint2 (&r)[N]) {
  static_assert(N % 4 == 0, "tie arity");
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]) : : "memory");
#pragma unroll
  for (int i = 4; i < N; i += 4) asm volatile("" : "+v"(r[i]), "+v"(r[i + 1]), "+v"(r[i + 2]), "+v"(r[i + 3]));
}
// wait until at most `after` stages (of D DMAs per wave each) are still in flight; after <= K
template <int K, int D> ARGUS_DEV void wg_wait_after(int after) {
  if constexpr (K == 0) {
    wg_waitvm<0>();
  } else {
    if (after >= K) wg_waitvm<K * D>();
    else wg_wait_after<K - 1, D>(after);
  }
}
typedef __attribute__((address_space(1))) unsigned wg_gu32;
// 16-byte write-through (sc1) store: the slab leaves the writer's L2 for the reducing workgroup
ARGUS_DEV void wg_st16_wt(f32x4* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
}  // namespace

// A tile's split slabs summed by the reducing workgroups of a folded launch (policy key 50). Workgroup
// r (after the compute grid) takes tile r % nwg and part r / nwg of its 128 x BN / 4 float4 fragments;
// it waits for the tile's nsplit arrivals, then sums every fragment over the splits in the order of
// wgrad_reduce_kernel (reduce.hip) for this M x N: lane l of SL sums splits l, l + SL, ... from 0, and
// the SL lane sums are added in lane order - the same fp32 additions, so dW is bit-identical to the
// unfolded launch + wgrad_reduce. The last reducing workgroup of the tile resets its two counters.
template <int NT, int MI, int NI, bool AP, int BN>
ARGUS_DEV void wg_fold_reduce(const WgParams& p, int nwg, int nsplit, int r, f32x4* red) {
  const int tile = r % nwg, part = r / nwg;
  const int ntiles = p.N / BN, mt = tile / ntiles, nt = tile - mt * ntiles;
  constexpr int FR = 128 * BN / 4;  // float4 fragments per tile
  const int SL = p.fold.sl, rpt = p.fold.rpt;
  const int fbeg = (int)((long)FR * part / rpt), fend = (int)((long)FR * (part + 1) / rpt);
  if (threadIdx.x == 0) {
    // poll the tile's arrivals with an atomic read-modify-write (performed at the memory side: a plain
    // or sc1 load may keep returning the XCD's L2 copy); bounded, so a launch can never hang
    wg_gu32* c = (wg_gu32*)(p.fold.cnt + tile);
    int it = 0;
    while (__hip_atomic_fetch_add(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)nsplit) {
      if (++it > (1 << 16)) break;
      __builtin_amdgcn_s_sleep(32);
    }
    if (it > (1 << 16)) __hip_atomic_store((wg_gu32*)(p.fold.cnt + 2 * nwg), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const f32x4* slab0 = reinterpret_cast<const f32x4*>(p.part) + (size_t)tile * nsplit * FR;
  const int t = threadIdx.x, l = t % SL, per = NT / SL;
  for (int f0 = fbeg; f0 < fend; f0 += per) {
    const int f = f0 + t / SL;
    const bool valid = f < fend;
    const int fc = valid ? f : fbeg;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int kb = l; kb < nsplit; kb += SL * kLoadBatch) {
      f32x4 v[kLoadBatch];  // in flight together; clamped, masked below (as wgrad_reduce_kernel)
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) v[u] = slab0[(size_t)min(kb + u * SL, nsplit - 1) * FR + fc];
#pragma unroll
      for (int u = 0; u < kLoadBatch; ++u) s += kb + u * SL < nsplit ? v[u] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    red[t] = s;
    __syncthreads();
    if (l == 0 && valid) {
      for (int j = 1; j < SL; ++j) s += red[t + j];
      // fragment f -> (wave, mi, ni, lane) -> rows m .. m + 3 of column n (the compute epilogue's map)
      const int lane = f & 63, q = f >> 6, ni = q % NI, mi = (q / NI) % MI, wave = q / (NI * MI);
      const int rbase = AP ? 16 * MI * wave : 64 * (wave / (BN / 64));
      const int cbase = AP ? 0 : 64 * (wave % (BN / 64));
      const int n = nt * BN + cbase + 16 * ni + (lane & 15);
      const int m = mt * 128 + rbase + 16 * mi + 4 * (lane >> 4);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) p.fold.dw[(size_t)(m + rr) * p.N + n] = s[rr];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    wg_gu32* c = (wg_gu32*)(p.fold.cnt + tile);
    wg_gu32* dn = (wg_gu32*)(p.fold.cnt + nwg + tile);
    if (__hip_atomic_fetch_add(dn, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)rpt - 1) {
      __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dn, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

constexpr int kWgdBK = 32;  // pixels per k-step

// Tiles of 128 rows (output channels) x BN columns (input channels): BN = 128 with 256 threads, two
// workgroups per CU; BN = 256 with 512 threads, one per CU with the apply, two without (the wider tile reads the A side, dm and
// y, once for 256 columns: 16 instead of 24 KB per 128 x 128 x 32 block with the apply, 12 instead of
// 16 without). Per stage: images A (dm / dy) [, Y] of 32 rows x 256 B and B (x) of 32 rows x 2 BN B.
//
// G (gather, plain form, BN = 128): the x rows of a k-step are gathered per pixel for strided or 3x3
// filters (N = taps x Cin, Cin % 128 == 0: a column tile lies in one tap); rows outside the image
// read the zero page, as the register-staged kernel zeroes them.
template <bool AP, int BN, bool G = false, int NSX = 0>
__global__ __launch_bounds__(2 * BN, BN == 256 && AP ? 1 : 2) void wgrad_dma_kernel(const WgParams p) {
  static_assert(!G || (!AP && BN == 128), "gather: plain 128-wide tiles");
  constexpr int NT = 2 * BN, NW = NT / 64;
  constexpr int AIMG = kWgdBK * 256, BIMG = kWgdBK * BN * 2;
  constexpr int BOFF = AP ? 2 * AIMG : AIMG;   // B image offset in a stage
  constexpr int STAGE = BOFF + BIMG;
  constexpr int APW = 8 / NW;                  // 1 KB A pieces per wave and A image (4 rows each)
  constexpr int BPW = 2;                       // 1 KB B pieces per wave
  constexpr int LPR = BN / 8;                  // lanes per B row (16-byte chunks)
  constexpr int D = APW * (AP ? 2 : 1) + BPW;  // DMAs per wave per stage
  // ring stages: 72 / 64 KB (two workgroups per CU) at BN = 128; 128 KB (one) / 72 KB (two) at BN = 256
  // NSX: the ring depth of the apply / 256-wide form (policy key 48; 5 stages = all 160 KB of LDS)
  constexpr int NS = NSX ? NSX : BN == 256 ? (AP ? 4 : 3) : (AP ? 3 : 4);
  static_assert(NS >= 2 && BPW * NW * 1024 == BIMG && APW * NW * 1024 == AIMG, "wgrad_dma geometry");
  __shared__ __attribute__((aligned(1024))) u32x4 lds[NS * STAGE / 16];
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;

  const int mtiles = p.M / 128, ntiles = p.N / BN;
  const int nwg = mtiles * ntiles;
  const int nsplit = (p.P + p.pps - 1) / p.pps;
  // folded split reduction (p.fold.cnt set, policy key 50): the workgroups past the compute grid sum
  // the split slabs of one tile each (wg_fold_reduce), so no separate wgrad_reduce launch runs
  if (p.fold.cnt && (int)blockIdx.x >= nwg * nsplit) {
    wg_fold_reduce<NT, AP ? 8 / NW : 4, AP ? BN / 16 : 4, AP, BN>(p, nwg, nsplit, (int)blockIdx.x - nwg * nsplit,
                                                                  reinterpret_cast<f32x4*>(lds));
    return;
  }
  int bid, split;
  split_tile(nwg, nsplit, p.group != 0, bid, split);
  const int mt = bid / ntiles, nt = bid - mt * ntiles;
  const int pbeg = split * p.pps;
  const int pend = min(p.P, pbeg + p.pps);
  const int nk = pend > pbeg ? (pend - pbeg + kWgdBK - 1) / kWgdBK : 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // wave tiles: with the apply, NW x 1 waves of 128/NW rows x BN (each A row formed by one wave: the
  // apply is the kernel's VALU work); plain, 2 x BN/64 waves of 64 x 64
  constexpr int MI = AP ? 8 / NW : 4, NI = AP ? BN / 16 : 4;
  const int rbase = AP ? 16 * MI * wave : 64 * (wave / (BN / 64));
  const int cbase = AP ? 0 : 64 * (wave % (BN / 64));
  const bf16* __restrict__ DY = reinterpret_cast<const bf16*>(p.dy);
  const bf16* __restrict__ Y = reinterpret_cast<const bf16*>(p.ap_y);
  const bf16* __restrict__ X = reinterpret_cast<const bf16*>(p.x);

  // this lane's DMA pieces: A rows 4 (APW wave + j) + lane/16, B rows (BPW wave + j) 1024/(2 BN) +
  // lane/LPR; source chunks swizzled so the image holds slot s of row r at s ^ swz(r)
  int arow[APW], ach[APW], brow[BPW], bch[BPW];
#pragma unroll
  for (int j = 0; j < APW; ++j) {
    arow[j] = 4 * (APW * wave + j) + (lane >> 4);
    const int pos = lane & 15;
    ach[j] = ((((pos >> 1) ^ wg_swz(arow[j])) << 1) | (pos & 1)) * 8;
  }
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    brow[j] = (BPW * wave + j) * (1024 / (2 * BN)) + lane / LPR;
    const int pos = lane % LPR;
    bch[j] = ((((pos >> 1) ^ wg_swz(brow[j])) << 1) | (pos & 1)) * 8;
  }
  // rows past the split's range read the zero page: one base pointer per operand plus a selected byte
  // offset (a select between two pointers was lowered to exec-masked branches, i.e. a varying number of
  // DMA instructions per wave, which the counted waits cannot allow)
  const char* zero = reinterpret_cast<const char*>(wgdma_zero_page);
  const long dz = reinterpret_cast<const char*>(DY) - zero, yz = reinterpret_cast<const char*>(Y) - zero,
             xz = reinterpret_cast<const char*>(X) - zero;
  // G: this column tile's tap and first channel
  int tap_r = 0, tap_s = 0, ci0 = nt * BN;
  if constexpr (G) {
    const int t = (nt * BN) / p.Cin;
    ci0 = nt * BN - t * p.Cin;
    tap_r = t / p.S;
    tap_s = t - tap_r * p.S;
  }
  const int HWo = p.Ho * p.Wo;
  auto issue = [&](int kt) {
    const uint32_t sb = lds0 + (kt % NS) * STAGE;
    const int pk = pbeg + kt * kWgdBK;
#pragma unroll
    for (int j = 0; j < APW; ++j) {
      const int pix = pk + arow[j];
      const bool ok = pix < pend;
      const long a_off = 2 * ((long)pix * p.M + mt * 128 + ach[j]);
      const uint32_t la = sb + (APW * wave + j) * 1024;
      wg_gl16(zero + (ok ? dz + a_off : 0), la);
      if constexpr (AP) wg_gl16(zero + (ok ? yz + a_off : 0), la + AIMG);
    }
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      const int pix = pk + brow[j];
      bool ok = pix < pend;
      long x_off;
      if constexpr (G) {
        const int pp = ok ? pix : pbeg;
        const int nimg = fdiv(pp, p.fd_hw);
        const int rem = pp - nimg * HWo;
        const int oh = fdiv(rem, p.fd_w);
        const int ow = rem - oh * p.Wo;
        const int ih = oh * p.stride - p.pad + tap_r, iw = ow * p.stride - p.pad + tap_s;
        ok = ok && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
        x_off = 2 * ((((long)nimg * p.H + ih) * p.W + iw) * p.lda + ci0 + bch[j]);  // 64-bit pixel index
      } else {
        x_off = 2 * ((long)pix * p.lda + ci0 + bch[j]);
      }
      wg_gl16(zero + (ok ? xz + x_off : 0), sb + BOFF + (BPW * wave + j) * 1024);
    }
  };

  const int g = lane >> 4, i16 = lane & 15;
  const int q = i16 >> 2, pq = i16 & 3;
  // apply coefficients of this lane's A rows (channel mt*128 + rbase + 16 mi + i16)
  float ca[AP ? MI : 1], cb[AP ? MI : 1], cc[AP ? MI : 1];
  if constexpr (AP) {
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int m = mt * 128 + rbase + 16 * mi + i16;
      ca[mi] = p.ap_ca[m];
      cb[mi] = p.ap_cb[m];
      cc[mi] = p.ap_cc[m];
    }
  }
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LDS byte offsets of this lane's two transposed-read rows of a 16-channel block (slot)
  auto tr_addr = [&](uint32_t img, int rowbytes, int slot, int h) -> uint32_t {
    const int row = 8 * g + 4 * h + q;
    return img + row * rowbytes + ((slot ^ wg_swz(row)) << 5) + pq * 8;
  };
  auto compute = [&](int kt) {
    const uint32_t base = lds0 + (kt % NS) * STAGE;
    // 64-bit reads, 2 rows per 16-channel block: A (dm) at 0, B (x) at RB, y at RY
    constexpr int RB = 2 * MI, RY = RB + 2 * NI, NR = RY + (AP ? 2 * MI : 0);
    uint2 r[NR];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int slot = (rbase + 16 * mi) >> 4;
        r[2 * mi + h] = wg_tr(tr_addr(base, 256, slot, h));
        if constexpr (AP) r[RY + 2 * mi + h] = wg_tr(tr_addr(base + AIMG, 256, slot, h));
      }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int h = 0; h < 2; ++h) r[RB + 2 * ni + h] = wg_tr(tr_addr(base + BOFF, 2 * BN, (cbase + 16 * ni) >> 4, h));
    wg_tie(r);
    u32x4 fa[MI], fb[NI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      fa[mi] = u32x4{r[2 * mi].x, r[2 * mi].y, r[2 * mi + 1].x, r[2 * mi + 1].y};
      if constexpr (AP) {  // dy = ca*dm + cb*y + cc (wgrad_kernel's fp32 formula, rounded to bf16)
        const u32x4 yv = u32x4{r[RY + 2 * mi].x, r[RY + 2 * mi].y, r[RY + 1 + 2 * mi].x, r[RY + 1 + 2 * mi].y};
        float d[8], yf[8];
        unpack(fa[mi], d);
        unpack(yv, yf);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = fmaf(ca[mi], d[j], fmaf(cb[mi], yf[j], cc[mi]));
        fa[mi] = pack(d);
      }
    }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
      fb[ni] = u32x4{r[RB + 2 * ni].x, r[RB + 2 * ni].y, r[RB + 1 + 2 * ni].x, r[RB + 1 + 2 * ni].y};
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) Mma<bf16>::run(acc[mi][ni], fa[mi], fb[ni]);
  };

  // ring: stages of k-steps kt .. kt + NS - 2 in flight at the wait of step kt (the coefficient loads
  // drained first: the compiler cannot count past the DMAs and would drain the whole prologue for them)
  if constexpr (AP) wg_waitvm<0>();
  for (int kt = 0; kt < NS - 1 && kt < nk; ++kt) issue(kt);
  for (int kt = 0; kt < nk; ++kt) {
    wg_wait_after<NS - 2, D>(min(NS - 2, nk - 1 - kt));  // stages issued after k-step kt's may fly
    wg_bar();  // every wave's pieces of stage kt landed; stage kt - 1 is free
    if (kt + NS - 1 < nk) issue(kt + NS - 1);
    compute(kt);
  }
  wg_waitvm<0>();

  if (p.fold.cnt) {
    // the tile's slab for this split in fragment order (one 16-byte write-through store per fragment),
    // then one arrival on the tile's counter after every wave's stores drained (MI355X_MICROARCH.md
    // hand-off table, row 1: sc1 stores, drained, one agent-scope add per workgroup)
    f32x4* slab = reinterpret_cast<f32x4*>(p.part) + ((size_t)bid * nsplit + split) * (128 * BN / 4);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) wg_st16_wt(slab + ((wave * MI + mi) * NI + ni) * 64 + lane, acc[mi][ni]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add((wg_gu32*)(p.fold.cnt + bid), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  float* out = p.part + (size_t)split * p.M * p.N;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int n = nt * BN + cbase + 16 * ni + i16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 128 + rbase + 16 * mi + 4 * g + r;
        out[(size_t)m * p.N + n] = acc[mi][ni][r];  // cached: the split reduce reads it next
      }
    }
}

// the column-tile width wgrad_dma_launch uses for d under key 45 (0: not served): 256 with the apply
// (key 2) or always (key 3) where Cin % 256 == 0. Measured alone (tools/wgbench.py, B=64, the 12
// 1x1 stride-1 shapes): apply 785 / 815 us (256 / 128 wide), plain 592 / 562 us with the plain
// 256-wide kernel at one workgroup per CU (stalled at its per-k-step barrier with no second workgroup
// to fill it); now two per CU (128 VGPRs, 3 stages) over a grid planned for its tile count
// the strided (1x1 / 3x3 stride 2) weight gradients in the plain form gather their x rows (key 47)
static bool wgrad_dma_gather(const argus_conv_desc& d) { return d.stride != 1 || d.r != 1; }

int wgrad_dma_width(const argus_conv_desc& d, int dtype, int bm, int bn, int key, bool ap, int gather_key) {
  if (!key || dtype != ARGUS_BF16 || d.stem || bm != 128 || bn != 128 || d.k % 128 || d.c % 128) return 0;
  if (wgrad_dma_gather(d)) {  // 3x3 stride 1 stays on the halo / register-staged kernels
    // key 47: 0 off, 1 every size, > 1 at most that many output pixels
    const bool g = gather_key && !ap && d.stride == 2 && d.r == d.s && (d.r == 1 || d.r == 3) &&
                   d.pad == (d.r - 1) / 2 && (gather_key == 1 || (long)d.n * d.ho * d.wo <= gather_key);
    return g ? 128 : 0;
  }
  if (d.pad != 0 || d.h != d.ho || d.w != d.wo) return 0;
  return ((key == 2 && ap) || key >= 3) && d.c % 256 == 0 ? 256 : 128;
}

bool wgrad_dma_ok(const argus_conv_desc& d, int dtype, int bm, int bn, int enabled, bool ap, int gather_key) {
  return wgrad_dma_width(d, dtype, bm, bn, enabled, ap, gather_key) != 0;
}

// grid: the 128 x 128 tiles x splits of the plan; 256-wide tiles take two of its column tiles
// the reducing workgroups of a folded launch: about 128 in all, at least one pass of NT / SL fragments each
static int wgrad_dma_fold_rpt(int nwg, int bn, int sl) {
  const int frag = 128 * bn / 4, per = 2 * bn / sl;
  int rpt = (128 + nwg - 1) / nwg;
  return rpt < 1 ? 1 : (rpt > frag / per ? frag / per : rpt);
}

int wgrad_dma_fold_tiles(const argus_conv_desc& d, int key, int gather_key, bool ap) {
  const int bn = wgrad_dma_width(d, ARGUS_BF16, 128, 128, key, ap, gather_key);
  const int N = d.r * d.s * d.c;
  return bn ? (d.k / 128) * (N / bn) : 0;
}

void wgrad_dma_launch(const argus_conv_desc& d, const WgParams& p_in, int key, int gather_key, int splits, int ns,
                      hipStream_t st) {
  WgParams p = p_in;
  const int bn = wgrad_dma_width(d, ARGUS_BF16, 128, 128, key, p.ap_y != nullptr, gather_key);
  const int nwg = (p.M / 128) * (p.N / bn);
  int grid = nwg * splits;
  if (p.fold.cnt) {
    p.fold.rpt = wgrad_dma_fold_rpt(nwg, bn, p.fold.sl);
    grid += nwg * p.fold.rpt;
  }
  if (wgrad_dma_gather(d)) {
    timed_launch("argus::wgrad_dma_kernel<false, 128, true, 0>", wgrad_dma_kernel<false, 128, true>, dim3(grid),
                 dim3(256), st, p);
  } else if (bn == 256) {
    if (p.ap_y) {
      switch (ns) {
        case 2: timed_launch("argus::wgrad_dma_kernel<true, 256, false, 2>", wgrad_dma_kernel<true, 256, false, 2>,
                             dim3(grid), dim3(512), st, p); break;
        case 3: timed_launch("argus::wgrad_dma_kernel<true, 256, false, 3>", wgrad_dma_kernel<true, 256, false, 3>,
                             dim3(grid), dim3(512), st, p); break;
        case 5: timed_launch("argus::wgrad_dma_kernel<true, 256, false, 5>", wgrad_dma_kernel<true, 256, false, 5>,
                             dim3(grid), dim3(512), st, p); break;
        default: timed_launch("argus::wgrad_dma_kernel<true, 256, false, 0>", wgrad_dma_kernel<true, 256>, dim3(grid),
                              dim3(512), st, p);
      }
    } else
      timed_launch("argus::wgrad_dma_kernel<false, 256, false, 0>", wgrad_dma_kernel<false, 256>, dim3(grid), dim3(512), st, p);
  } else {
    if (p.ap_y)
      timed_launch("argus::wgrad_dma_kernel<true, 128, false, 0>", wgrad_dma_kernel<true, 128>, dim3(grid), dim3(256), st, p);
    else
      timed_launch("argus::wgrad_dma_kernel<false, 128, false, 0>", wgrad_dma_kernel<false, 128>, dim3(grid), dim3(256), st, p);
  }
}

}  // namespace argus
