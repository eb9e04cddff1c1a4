// Photometric training augmentations on the device: the sequence of argus/data.py:41-103
// (Planckian jitter -> ColorJiggle -> Gaussian blur -> motion blur -> plasma shadow) applied to a
// uint8 batch after the host->device copy, replacing kornia on the CPU data-loader workers.
//
// Per-image parameters are sampled on the host (argus_amd/augment.py, seeded torch generator, the
// reference's ranges) and passed as AugParams. The arithmetic restates kornia's published
// definitions (kornia is not installed here, so parity with kornia itself is unpinned; the tests pin
// these kernels to a torch restatement of the same formulas):
//   brightness  x + (b - 1)                       (kornia adjust_brightness, additive), clamp [0, 1]
//   contrast    x * c                             (adjust_contrast, multiplicative), clamp [0, 1]
//   saturation  HSV s * f, clamp [0, 1]           (adjust_saturation)
//   hue         HSV h + 2*pi*f mod 2*pi           (adjust_hue)
//   Planckian   per-channel gains of a blackbody white point (mode "blackbody")
//   blur        5x5 Gaussian, separable, reflect borders
//   motion      3x3 line kernel (host-built from angle / direction), zero borders
//   plasma      x * (1 + intensity * [noise < quantity]), fractal value noise with amplitude decay
//               `roughness` per octave
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
  unsigned seed;
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
__global__ __launch_bounds__(256) void aug_color_kernel(int64_t nimg, int hw, const uint8_t* __restrict__ src,
                                                        float* __restrict__ dst, const AugParams* __restrict__ prm) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nimg * hw) return;
  const int64_t img = i / hw;
  const int64_t px = i - img * hw;
  const AugParams& P = prm[img];
  const uint8_t* s = src + img * 3 * hw + px;
  float c[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) c[k] = clamp01((float)s[(int64_t)k * hw] / 255.0f * P.gain[k]);
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

// hashed lattice value noise in [0, 1)
ARGUS_DEV float lattice(unsigned seed, int o, int gx, int gy) {
  unsigned hsh = seed * 0x9E3779B1u ^ (unsigned)o * 0x85EBCA77u ^ (unsigned)gx * 0xC2B2AE3Du ^ (unsigned)gy * 0x27D4EB2Fu;
  hsh ^= hsh >> 15; hsh *= 0x2C1B3C6Du; hsh ^= hsh >> 12; hsh *= 0x297A2D39u; hsh ^= hsh >> 15;
  return (float)(hsh >> 8) * (1.0f / 16777216.0f);
}

// plasma-like fractal noise at (y, x): octaves of bilinear value noise, cell size halving, amplitude
// x roughness per octave, normalized to [0, 1)
ARGUS_DEV float plasma(unsigned seed, float rough, int h, int w, int y, int x) {
  float cell = (float)(h > w ? h : w) * 0.5f, amp = 1.f, sum = 0.f, norm = 0.f;
  for (int o = 0; o < 6 && cell >= 1.f; ++o) {
    const float fy = y / cell, fx = x / cell;
    const int gy = (int)floorf(fy), gx = (int)floorf(fx);
    const float ty = fy - gy, tx = fx - gx;
    const float v00 = lattice(seed, o, gx, gy), v01 = lattice(seed, o, gx + 1, gy);
    const float v10 = lattice(seed, o, gx, gy + 1), v11 = lattice(seed, o, gx + 1, gy + 1);
    const float v = (v00 * (1.f - tx) + v01 * tx) * (1.f - ty) + (v10 * (1.f - tx) + v11 * tx) * ty;
    sum = fmaf(amp, v, sum);
    norm += amp;
    amp *= rough;
    cell *= 0.5f;
  }
  return sum / norm;
}

// motion blur (3x3, zero borders) from x into tmp for the images that have it, then plasma shadow
// and the final write: pass 0 = motion into tmp, pass 1 = x <- (motion ? tmp : x) * shade
__global__ __launch_bounds__(256) void aug_motion_plasma_kernel(int64_t nimg, int h, int w, float* __restrict__ x,
                                                                float* __restrict__ tmp,
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
  if (P.plasma_int != 0.f) {
    const float n = plasma(P.seed, P.plasma_rough, h, w, y, xx);
    if (n < P.plasma_q) v *= 1.f + P.plasma_int;
  }
  x[plane * hw + p] = clamp01(v);
}

}  // namespace argus

using namespace argus;

extern "C" {

size_t argus_augment_params_bytes(void) { return sizeof(AugParams); }

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
  hipLaunchKernelGGL(aug_color_kernel, dim3(g1), dim3(256), 0, st, nimg, (int)hw, src, dst, prm);
  for (int pass = 0; pass < 2; ++pass)
    hipLaunchKernelGGL(aug_blur_kernel, dim3(g3), dim3(256), 0, st, nimg, h, w, dst, scratch, prm, pass);
  for (int pass = 0; pass < 2; ++pass)
    hipLaunchKernelGGL(aug_motion_plasma_kernel, dim3(g3), dim3(256), 0, st, nimg, h, w, dst, scratch, prm, pass);
  return check_launch("augment_photometric");
}

}  // extern "C"
