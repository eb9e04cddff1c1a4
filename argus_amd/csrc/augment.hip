// Photometric training augmentations on the device: the sequence of argus/data.py:41-103
// (random erasing x2 -> Planckian jitter -> ColorJiggle -> Gaussian blur -> motion blur -> plasma
// shadow -> salt-and-pepper) applied to a uint8 batch after the host->device copy, replacing kornia
// on the CPU data-loader workers.
//
// Per-image parameters are sampled on the host (argus_amd/augment.py, seeded torch generator, the
// reference's ranges) and passed as AugParams. The arithmetic restates kornia's published
// definitions (kornia is not installed here, so parity with kornia itself is unpinned; the tests pin
// these kernels to a float64 restatement of the same formulas, tests/aug_reference.py):
//   erasing     pixels of a (y0, x0, h, w) rectangle set to `value` in all channels (RandomErasing;
//               rectangle drawn on the host as kornia's random_rectangles_params_generator)
//   Planckian   per-channel gains of a blackbody white point (mode "blackbody"), clamp [0, 1]
//   brightness  x + (b - 1)                       (kornia adjust_brightness, additive), clamp [0, 1]
//   contrast    x * c                             (adjust_contrast, multiplicative), clamp [0, 1]
//   saturation  HSV s * f, clamp [0, 1]           (adjust_saturation)
//   hue         HSV h + 2*pi*f mod 2*pi           (adjust_hue)
//   blur        5x5 Gaussian, separable, reflect borders
//   motion      3x3 line kernel (host-built from angle / direction), zero borders
//   plasma      x + intensity * [map < quantity], clamp [0, 1]; map = diamond-square plasma fractal
//               (kornia diamond_square): a (2^k + 1)^2 grid, 2^k >= max(H, W) - 1, corners U[0, 1),
//               then per level (step halving) the diamond step (square centres = mean of the 4
//               corners) and the square step (edge midpoints = mean of the in-grid neighbours at
//               +-step/2), each plus (U - 0.5) * roughness^(level + 1); cropped to H x W and min-max
//               normalized to [0, 1]
//   salt/pepper per pixel (all channels): U < amount -> (U' < salt_vs_pepper ? 1 : 0)
// The random numbers of the plasma map and the salt-and-pepper mask are a hash of (image seed,
// stream, index) - reproducible and identical in the restatement.
// Layout: images planar NCHW (n_img, 3, H, W); the 6-channel sample is two such images.
#include "common.h"
#include "internal.h"

namespace argus {

struct AugParams {
  float gain[3];       // Planckian jitter (1, 1, 1 = off)
  float bright, contrast, sat, hue;  // ColorJiggle factors (1, 1, 1, 0 = off); hue in turns
  int order;           // 4 x 2-bit op indices (0 brightness, 1 contrast, 2 saturation, 3 hue), first in bits 0-1
  int jiggle;          // ColorJiggle on
  float blur_w[5];     // normalized 5-tap Gaussian (blur_w[2] == 0 => no blur)
  float motion[9];     // 3x3 motion kernel (all 0 => no motion blur)
  float plasma_int, plasma_q, plasma_rough;  // plasma shadow (intensity 0 => off)
  unsigned seed;       // plasma map seed
  int erase[2][4];     // random erasing rectangles: y0, x0, h, w (h == 0 => off), applied in order
  float erase_val[2];
  float sp_amount, sp_salt;  // salt-and-pepper (amount 0 => off)
  unsigned sp_seed;
};

ARGUS_DEV float clamp01(float x) { return fminf(fmaxf(x, 0.f), 1.f); }

// kornia rgb_to_hsv / hsv_to_rgb (h in radians [0, 2pi), s, v in [0, 1])
ARGUS_DEV void rgb2hsv(float r, float g, float b, float& h, float& s, float& v) {
  const float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b));
  const float d = mx - mn;
  v = mx;
  s = d / (mx + 1e-6f);
  float hh;
  if (d == 0.f) hh = 0.f;
  else if (mx == r) hh = fmodf((g - b) / d, 6.f);
  else if (mx == g) hh = (b - r) / d + 2.f;
  else hh = (r - g) / d + 4.f;
  hh = hh * (2.f * 3.14159265358979f / 6.f);
  if (hh < 0.f) hh += 2.f * 3.14159265358979f;
  h = hh;
}
ARGUS_DEV void hsv2rgb(float h, float s, float v, float& r, float& g, float& b) {
  float hn = h / (2.f * 3.14159265358979f) * 6.f;
  hn = hn - 6.f * floorf(hn / 6.f);
  const float hi = floorf(hn);
  const float f = hn - hi;
  const float p = v * (1.f - s), q = v * (1.f - f * s), t = v * (1.f - (1.f - f) * s);
  switch ((int)hi) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

// one thread per pixel: /255, Planckian gains, ColorJiggle ops in the sampled order -> fp32
__global__ __launch_bounds__(256) void aug_color_kernel(int64_t nimg, int hw, int w, const uint8_t* __restrict__ src,
                                                        float* __restrict__ dst, const AugParams* __restrict__ prm) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nimg * hw) return;
  const int64_t img = i / hw;
  const int64_t px = i - img * hw;
  const AugParams& P = prm[img];
  const uint8_t* s = src + img * 3 * hw + px;
  float c[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) c[k] = (float)s[(int64_t)k * hw] / 255.0f;
  const int py = (int)(px / w), pxx = (int)(px - (int64_t)py * w);
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int* r = P.erase[e];
    if (r[2] > 0 && py >= r[0] && py < r[0] + r[2] && pxx >= r[1] && pxx < r[1] + r[3])
      c[0] = c[1] = c[2] = P.erase_val[e];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) c[k] = clamp01(c[k] * P.gain[k]);
  if (P.jiggle) {
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int op = (P.order >> (2 * o)) & 3;
      if (op == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) c[k] = clamp01(c[k] + (P.bright - 1.f));
      } else if (op == 1) {
#pragma unroll
        for (int k = 0; k < 3; ++k) c[k] = clamp01(c[k] * P.contrast);
      } else {
        float h, sa, v;
        rgb2hsv(c[0], c[1], c[2], h, sa, v);
        if (op == 2) {
          sa = clamp01(sa * P.sat);
        } else {
          const float tp = 2.f * 3.14159265358979f;
          h = fmodf(h + P.hue * tp, tp);
          if (h < 0.f) h += tp;
        }
        hsv2rgb(h, sa, v, c[0], c[1], c[2]);
      }
    }
  }
  float* d = dst + img * 3 * hw + px;
#pragma unroll
  for (int k = 0; k < 3; ++k) d[(int64_t)k * hw] = c[k];
}

ARGUS_DEV int reflect(int i, int n) {  // torch / kornia "reflect": -1 -> 1, n -> n - 2
  if (i < 0) i = -i;
  if (i >= n) i = 2 * n - 2 - i;
  return i < 0 ? 0 : (i >= n ? n - 1 : i);
}

// separable 5-tap Gaussian: pass 0 (rows) x -> tmp, pass 1 (columns) tmp -> x; images without blur
// are skipped (their blur_w[2] is 0)
__global__ __launch_bounds__(256) void aug_blur_kernel(int64_t nimg, int h, int w, float* __restrict__ x,
                                                       float* __restrict__ tmp, const AugParams* __restrict__ prm,
                                                       int pass) {
  const int64_t hw = (int64_t)h * w;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nimg * 3 * hw) return;
  const int64_t plane = i / hw;
  const AugParams& P = prm[plane / 3];
  if (P.blur_w[2] == 0.f) return;
  const int p = (int)(i - plane * hw);
  const int y = p / w, xx = p - y * w;
  const float* src = (pass == 0 ? x : tmp) + plane * hw;
  float acc = 0.f;
#pragma unroll
  for (int t = -2; t <= 2; ++t) {
    const int yy = pass == 0 ? y : reflect(y + t, h);
    const int xs = pass == 0 ? reflect(xx + t, w) : xx;
    acc = fmaf(P.blur_w[t + 2], src[(int64_t)yy * w + xs], acc);
  }
  (pass == 0 ? tmp : x)[plane * hw + p] = acc;
}

// counter-based uniform in [0, 1): hash of (seed, stream, index)
ARGUS_DEV float hash_u01(unsigned seed, unsigned stream, unsigned idx) {
  unsigned h = seed * 0x9E3779B1u ^ stream * 0x85EBCA77u ^ idx * 0xC2B2AE3Du;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// diamond-square grid side: 2^k + 1 with 2^k >= max(h, w) - 1 (k >= 1)
static int ds_side(int h, int w) {
  int k = 1;
  while ((1 << k) < (h > w ? h : w) - 1) ++k;
  return (1 << k) + 1;
}

// corners of every plasma image's grid (stream 0)
__global__ __launch_bounds__(256) void aug_ds_seed_kernel(int64_t nimg, int S, float* __restrict__ map,
                                                          const AugParams* __restrict__ prm) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nimg * 4) return;
  const int64_t img = i >> 2;
  const AugParams& P = prm[img];
  if (P.plasma_int == 0.f) return;
  const int c = (int)(i & 3);
  const int y = (c >> 1) * (S - 1), x = (c & 1) * (S - 1);
  map[img * S * S + (int64_t)y * S + x] = hash_u01(P.seed, 0u, (unsigned)(y * S + x));
}

// one level's diamond (phase 0: square centres) or square (phase 1: edge midpoints) step; step =
// distance between the points already set, m = (S - 1) / step squares per side; stream 1 + 2*level + phase
__global__ __launch_bounds__(256) void aug_ds_step_kernel(int64_t nimg, int S, int level, int step, int phase,
                                                          float* __restrict__ map, const AugParams* __restrict__ prm) {
  const int m = (S - 1) / step, half = step >> 1;
  const int64_t count = phase == 0 ? (int64_t)m * m : 2LL * m * (m + 1);
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nimg * count) return;
  const int64_t img = i / count;
  const AugParams& P = prm[img];
  if (P.plasma_int == 0.f) return;
  const int t = (int)(i - img * count);
  float amp = 1.f;
  for (int l = 0; l <= level; ++l) amp *= P.plasma_rough;
  float* g = map + img * S * S;
  int y, x;
  float mean;
  if (phase == 0) {
    y = (t / m) * step + half;
    x = (t % m) * step + half;
    mean = 0.25f * ((g[(y - half) * S + x - half] + g[(y - half) * S + x + half]) +
                    (g[(y + half) * S + x - half] + g[(y + half) * S + x + half]));
  } else {
    const int mm = m * (m + 1);
    if (t < mm) {  // rows on the coarse grid, midpoints between its columns
      y = (t / m) * step;
      x = (t % m) * step + half;
    } else {       // rows between, on the coarse columns
      y = ((t - mm) / (m + 1)) * step + half;
      x = ((t - mm) % (m + 1)) * step;
    }
    float sum = 0.f;
    int cnt = 0;
    if (y - half >= 0) { sum += g[(y - half) * S + x]; ++cnt; }
    if (y + half < S) { sum += g[(y + half) * S + x]; ++cnt; }
    if (x - half >= 0) { sum += g[y * S + x - half]; ++cnt; }
    if (x + half < S) { sum += g[y * S + x + half]; ++cnt; }
    mean = sum / (float)cnt;
  }
  const float u = hash_u01(P.seed, 1u + 2u * level + phase, (unsigned)(y * S + x));
  g[y * S + x] = fmaf(u - 0.5f, amp, mean);
}

// min and max of each plasma map over its H x W crop (one workgroup per image)
__global__ __launch_bounds__(256) void aug_ds_minmax_kernel(int h, int w, int S, const float* __restrict__ map,
                                                            float2* __restrict__ mm, const AugParams* __restrict__ prm) {
  const int64_t img = blockIdx.x;
  if (prm[img].plasma_int == 0.f) return;
  const float* g = map + img * S * S;
  float lo = 3.4e38f, hi = -3.4e38f;
  for (int i = threadIdx.x; i < h * w; i += 256) {
    const int y = i / w, x = i - y * w;
    const float v = g[y * S + x];
    lo = fminf(lo, v);
    hi = fmaxf(hi, v);
  }
  __shared__ float sl[256], sh[256];
  sl[threadIdx.x] = lo;
  sh[threadIdx.x] = hi;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      sl[threadIdx.x] = fminf(sl[threadIdx.x], sl[threadIdx.x + o]);
      sh[threadIdx.x] = fmaxf(sh[threadIdx.x], sh[threadIdx.x + o]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) mm[img] = make_float2(sl[0], sh[0]);
}

// motion blur (3x3, zero borders) from x into tmp for the images that have it, then plasma shadow
// and the final write: pass 0 = motion into tmp, pass 1 = x <- (motion ? tmp : x) * shade
__global__ __launch_bounds__(256) void aug_motion_plasma_kernel(int64_t nimg, int h, int w, float* __restrict__ x,
                                                                float* __restrict__ tmp, const float* __restrict__ map,
                                                                const float2* __restrict__ mm, int S,
                                                                const AugParams* __restrict__ prm, int pass) {
  const int64_t hw = (int64_t)h * w;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nimg * 3 * hw) return;
  const int64_t plane = i / hw;
  const AugParams& P = prm[plane / 3];
  const bool motion = P.motion[4] != 0.f || P.motion[3] != 0.f || P.motion[5] != 0.f || P.motion[1] != 0.f ||
                      P.motion[7] != 0.f || P.motion[0] != 0.f || P.motion[2] != 0.f || P.motion[6] != 0.f ||
                      P.motion[8] != 0.f;
  const int p = (int)(i - plane * hw);
  const int y = p / w, xx = p - y * w;
  if (pass == 0) {
    if (!motion) return;
    const float* src = x + plane * hw;
    float acc = 0.f;
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx) {
        const int yy = y + dy, xs = xx + dx;
        const bool ok = (unsigned)yy < (unsigned)h && (unsigned)xs < (unsigned)w;
        acc = fmaf(P.motion[(dy + 1) * 3 + dx + 1], ok ? src[(int64_t)yy * w + xs] : 0.f, acc);
      }
    tmp[plane * hw + p] = acc;
    return;
  }
  float v = motion ? tmp[plane * hw + p] : x[plane * hw + p];
  const int64_t img = plane / 3;
  if (P.plasma_int != 0.f) {
    const float2 r = mm[img];
    const float d = r.y - r.x;
    const float n = d > 0.f ? (map[img * S * S + (int64_t)y * S + xx] - r.x) / d : 0.f;
    if (n < P.plasma_q) v += P.plasma_int;
  }
  v = clamp01(v);
  if (P.sp_amount > 0.f) {
    const unsigned idx = (unsigned)p;
    if (hash_u01(P.sp_seed, 0u, idx) < P.sp_amount) v = hash_u01(P.sp_seed, 1u, idx) < P.sp_salt ? 1.f : 0.f;
  }
  x[plane * hw + p] = v;
}

}  // namespace argus

using namespace argus;

extern "C" {

size_t argus_augment_params_bytes(void) { return sizeof(AugParams); }

// scratch layout (floats): blur planes [nimg*3*h*w] | plasma maps [nimg*S*S] | per-image {min, max}
// (float2). The float2 region starts at a 16-byte boundary: the map region is odd-sized (S*S odd), so
// an unrounded offset misaligns the 8-byte accesses whenever nimg*(3hw + S*S) is odd.
static int64_t aug_minmax_offset(int64_t nimg, int64_t hw, int64_t S) {
  return (nimg * 3 * hw + nimg * S * S + 3) & ~(int64_t)3;
}

size_t argus_augment_scratch_bytes(int64_t nimg, int h, int w) {
  if (nimg <= 0 || h <= 0 || w <= 0) return 0;
  const int64_t S = ds_side(h, w);
  return sizeof(float) * (size_t)(aug_minmax_offset(nimg, (int64_t)h * w, S) + 2 * nimg);
}

int argus_augment_photometric(int64_t nimg, int h, int w, const uint8_t* src, float* dst, const void* params,
                              float* scratch, argus_stream_t stream) {
  if (nimg <= 0 || h <= 0 || w <= 0 || !src || !dst || !params || !scratch) {
    set_error("augment_photometric: bad arguments");
    return ARGUS_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  const AugParams* prm = reinterpret_cast<const AugParams*>(params);
  const int64_t hw = (int64_t)h * w;
  const unsigned g1 = (unsigned)((nimg * hw + 255) / 256), g3 = (unsigned)((nimg * 3 * hw + 255) / 256);
  const int S = ds_side(h, w);
  float* map = scratch + nimg * 3 * hw;
  float2* mm = reinterpret_cast<float2*>(scratch + aug_minmax_offset(nimg, hw, S));
  if ((reinterpret_cast<uintptr_t>(scratch) & 15) != 0) {
    set_error("augment_photometric: scratch must be 16-byte aligned");
    return ARGUS_ERR_ARG;
  }
  hipLaunchKernelGGL(aug_color_kernel, dim3(g1), dim3(256), 0, st, nimg, (int)hw, w, src, dst, prm);
  for (int pass = 0; pass < 2; ++pass)
    hipLaunchKernelGGL(aug_blur_kernel, dim3(g3), dim3(256), 0, st, nimg, h, w, dst, scratch, prm, pass);
  // plasma maps: seed the corners, then one launch per level and phase (each reads the previous)
  hipLaunchKernelGGL(aug_ds_seed_kernel, dim3((unsigned)((nimg * 4 + 255) / 256)), dim3(256), 0, st, nimg, S, map, prm);
  for (int step = S - 1, level = 0; step >= 2; step >>= 1, ++level)
    for (int phase = 0; phase < 2; ++phase) {
      const int64_t m = (S - 1) / step;
      const int64_t count = phase == 0 ? m * m : 2 * m * (m + 1);
      hipLaunchKernelGGL(aug_ds_step_kernel, dim3((unsigned)((nimg * count + 255) / 256)), dim3(256), 0, st, nimg,
                         S, level, step, phase, map, prm);
    }
  hipLaunchKernelGGL(aug_ds_minmax_kernel, dim3((unsigned)nimg), dim3(256), 0, st, h, w, S, map, mm, prm);
  for (int pass = 0; pass < 2; ++pass)
    hipLaunchKernelGGL(aug_motion_plasma_kernel, dim3(g3), dim3(256), 0, st, nimg, h, w, dst, scratch, map, mm, S,
                       prm, pass);
  return check_launch("augment_photometric");
}

}  // extern "C"
