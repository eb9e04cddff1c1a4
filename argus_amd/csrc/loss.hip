// SE(3) geodesic pose loss, forward + backward, one fused kernel.
//
// Reference: geometric_loss_fn (argus/train.py:105-119)
//     torch.sum((pp.se3(pred).Exp() @ target.Inv()).Log() ** 2, axis=-1)
// with pypose's closed forms (se3 = [rho, phi], SE3 = [t, q xyzw]):
//   Exp: q = [sin(th/2)/th phi, cos(th/2)], t = J_l(phi) rho
//   Inv: q^-1 = conj q, t^-1 = -R(q^-1) t;   Mul: (q1 q2, t1 + R(q1) t2)
//   Log: phi = 2 atan(|v|/w)/|v| v (sign-invariant), tau = J_l^-1(phi) t;  loss = |tau|^2 + |phi|^2
// The gradient is the exact derivative of this composite map (= pypose's Lie-Jacobian backward
// 2 xi^T J_l^-1(xi_r) J_l(pred)), obtained by forward-mode dual numbers over the 6 inputs. The
// per-sample arithmetic runs in fp64 (a few hundred flops per sample; the batch is <= 1024).
#include "common.h"
#include "internal.h"

namespace argus {

constexpr double kSmall = 1e-4;  // Taylor-branch threshold (matches oracle/se3.py)

// value + its derivative along kND of the 6 prediction inputs: the loss kernel runs one input
// direction per lane (6 lanes per sample, each with the value chain and one derivative: 2 doubles
// per operation instead of 7 on one lane; the same arithmetic per direction, the same bits)
constexpr int kND = 1;
struct Dual {
  double v;
  double d[kND];
};
ARGUS_DEV Dual cst(double x) { Dual r; r.v = x; for (int i = 0; i < kND; ++i) r.d[i] = 0.0; return r; }
ARGUS_DEV Dual operator+(const Dual& a, const Dual& b) { Dual r; r.v = a.v + b.v; for (int i = 0; i < kND; ++i) r.d[i] = a.d[i] + b.d[i]; return r; }
ARGUS_DEV Dual operator-(const Dual& a, const Dual& b) { Dual r; r.v = a.v - b.v; for (int i = 0; i < kND; ++i) r.d[i] = a.d[i] - b.d[i]; return r; }
ARGUS_DEV Dual operator-(const Dual& a) { Dual r; r.v = -a.v; for (int i = 0; i < kND; ++i) r.d[i] = -a.d[i]; return r; }
ARGUS_DEV Dual operator*(const Dual& a, const Dual& b) { Dual r; r.v = a.v * b.v; for (int i = 0; i < kND; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i]; return r; }
ARGUS_DEV Dual operator*(double s, const Dual& a) { Dual r; r.v = s * a.v; for (int i = 0; i < kND; ++i) r.d[i] = s * a.d[i]; return r; }
ARGUS_DEV Dual operator/(const Dual& a, const Dual& b) {
  Dual r; r.v = a.v / b.v; const double ib = 1.0 / b.v;
  for (int i = 0; i < kND; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) * ib;
  return r;
}
ARGUS_DEV Dual fn(const Dual& a, double f, double df) { Dual r; r.v = f; for (int i = 0; i < kND; ++i) r.d[i] = df * a.d[i]; return r; }
ARGUS_DEV Dual dsqrt(const Dual& a) { const double s = sqrt(a.v); return fn(a, s, s > 0.0 ? 0.5 / s : 0.0); }
ARGUS_DEV Dual dsin(const Dual& a) { return fn(a, sin(a.v), cos(a.v)); }
ARGUS_DEV Dual dcos(const Dual& a) { return fn(a, cos(a.v), -sin(a.v)); }
ARGUS_DEV Dual datan(const Dual& a) { return fn(a, atan(a.v), 1.0 / (1.0 + a.v * a.v)); }

struct V3 { Dual x, y, z; };
ARGUS_DEV V3 cross(const V3& a, const V3& b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
ARGUS_DEV V3 add(const V3& a, const V3& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
ARGUS_DEV V3 sub(const V3& a, const V3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
ARGUS_DEV V3 scale(const Dual& s, const V3& a) { return {s * a.x, s * a.y, s * a.z}; }
ARGUS_DEV Dual dot(const V3& a, const V3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

struct Quat { V3 v; Dual w; };
ARGUS_DEV Quat qmul(const Quat& a, const Quat& b) {
  return {add(add(scale(a.w, b.v), scale(b.w, a.v)), cross(a.v, b.v)), a.w * b.w - dot(a.v, b.v)};
}
ARGUS_DEV V3 qrot(const Quat& q, const V3& p) {
  const V3 t = scale(cst(2.0), cross(q.v, p));
  return add(add(p, scale(q.w, t)), cross(q.v, t));
}

// J_l(phi) x = x + c1 phi x x + c2 phi x (phi x x)
ARGUS_DEV V3 jl_apply(const V3& phi, const V3& x, bool inverse) {
  const Dual th2 = dot(phi, phi);
  const Dual th = dsqrt(th2);
  Dual c1, c2;
  if (!inverse) {
    if (th.v < kSmall) {
      c1 = cst(0.5) - (1.0 / 24) * th2 + (1.0 / 720) * (th2 * th2);
      c2 = cst(1.0 / 6) - (1.0 / 120) * th2 + (1.0 / 5040) * (th2 * th2);
    } else {
      c1 = (cst(1.0) - dcos(th)) / th2;
      c2 = (th - dsin(th)) / (th2 * th);
    }
  } else {
    c1 = cst(-0.5);
    if (th.v < kSmall) {
      c2 = cst(1.0 / 12) + (1.0 / 720) * th2 + (1.0 / 30240) * (th2 * th2);
    } else {
      const Dual half = 0.5 * th;
      c2 = (cst(1.0) - half * dcos(half) / dsin(half)) / th2;
    }
  }
  const V3 k1 = cross(phi, x);
  const V3 k2 = cross(phi, k1);
  return add(add(x, scale(c1, k1)), scale(c2, k2));
}

ARGUS_DEV Dual se3_loss(const Dual (&xi)[6], const double (&T)[7]) {
  // Exp(pred)
  const V3 rho = {xi[0], xi[1], xi[2]};
  const V3 phi = {xi[3], xi[4], xi[5]};
  const Dual th2 = dot(phi, phi);
  const Dual th = dsqrt(th2);
  Dual imag, real;
  if (th.v < kSmall) {
    imag = cst(0.5) - (1.0 / 48) * th2 + (1.0 / 3840) * (th2 * th2);
    real = cst(1.0) - (1.0 / 8) * th2 + (1.0 / 384) * (th2 * th2);
  } else {
    imag = dsin(0.5 * th) / th;
    real = dcos(0.5 * th);
  }
  const Quat qp = {scale(imag, phi), real};
  const V3 tp = jl_apply(phi, rho, false);
  // target^-1
  const Quat qti = {{cst(-T[3]), cst(-T[4]), cst(-T[5])}, cst(T[6])};
  const V3 tt = {cst(T[0]), cst(T[1]), cst(T[2])};
  const V3 tti = scale(cst(-1.0), qrot(qti, tt));
  // Exp(pred) @ target^-1
  const Quat qr = qmul(qp, qti);
  const V3 tr = add(tp, qrot(qp, tti));
  // Log
  const Dual n2 = dot(qr.v, qr.v);
  const Dual n = dsqrt(n2);
  Dual w = qr.w;
  if (w.v == 0.0) w.v = 1e-30;
  Dual factor;
  if (n.v < kSmall) {
    factor = cst(2.0) / w - (2.0 / 3.0) * n2 / (w * w * w);
  } else {
    factor = 2.0 * datan(n / w) / n;
  }
  const V3 phr = scale(factor, qr.v);
  const V3 tau = jl_apply(phr, tr, true);
  return dot(tau, tau) + dot(phr, phr);
}

__global__ void se3_loss_kernel(int B, const float* __restrict__ pred, const float* __restrict__ target,
                                float* __restrict__ loss, float* __restrict__ dpred, float gscale) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = t / 6, dir = t - 6 * b;  // sample, input direction of this lane
  if (b >= B) return;
  Dual xi[6];
  for (int i = 0; i < 6; ++i) xi[i] = cst((double)pred[b * 6 + i]);
  xi[dir].d[0] = 1.0;
  double T[7];
  for (int i = 0; i < 7; ++i) T[i] = (double)target[b * 7 + i];
  const Dual L = se3_loss(xi, T);
  if (dir == 0) loss[b] = (float)L.v;
  if (dpred) dpred[b * 6 + dir] = (float)(gscale * L.d[0]);
}

// se(3) -> SE(3) exponential map (pypose se3.Exp): out[b] = [t (3), q xyzw (4)], w >= 0 canonical
// when `canon` (the data pipeline's quaternion convention).
__global__ void se3_exp_kernel(int B, const float* __restrict__ xi, float* __restrict__ out, int canon) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  Dual x[6];
  for (int i = 0; i < 6; ++i) x[i] = cst((double)xi[b * 6 + i]);
  const V3 rho = {x[0], x[1], x[2]};
  const V3 phi = {x[3], x[4], x[5]};
  const Dual th2 = dot(phi, phi);
  const Dual th = dsqrt(th2);
  Dual imag, real;
  if (th.v < kSmall) {
    imag = cst(0.5) - (1.0 / 48) * th2 + (1.0 / 3840) * (th2 * th2);
    real = cst(1.0) - (1.0 / 8) * th2 + (1.0 / 384) * (th2 * th2);
  } else {
    imag = dsin(0.5 * th) / th;
    real = dcos(0.5 * th);
  }
  const V3 t = jl_apply(phi, rho, false);
  const double sg = (canon && real.v < 0.0) ? -1.0 : 1.0;
  float* o = out + b * 7;
  o[0] = (float)t.x.v; o[1] = (float)t.y.v; o[2] = (float)t.z.v;
  o[3] = (float)(sg * imag.v * phi.x.v); o[4] = (float)(sg * imag.v * phi.y.v);
  o[5] = (float)(sg * imag.v * phi.z.v); o[6] = (float)(sg * real.v);
}

}  // namespace argus

using namespace argus;

extern "C" int argus_se3_exp(int batch, const float* xi, float* out, int canonical_w, argus_stream_t stream) {
  if (batch <= 0 || !xi || !out) {
    set_error("se3_exp: bad arguments");
    return ARGUS_ERR_ARG;
  }
  hipLaunchKernelGGL(se3_exp_kernel, dim3((batch + 63) / 64), dim3(64), 0, (hipStream_t)stream, batch, xi, out,
                     canonical_w);
  return check_launch("se3_exp_kernel");
}

extern "C" int argus_se3_loss(int batch, const float* pred, const float* target, float* loss, float* dpred,
                              float grad_scale, argus_stream_t stream) {
  if (batch <= 0 || !pred || !target || !loss) {
    set_error("se3_loss: bad arguments");
    return ARGUS_ERR_ARG;
  }
  hipLaunchKernelGGL(se3_loss_kernel, dim3((6 * batch + 255) / 256), dim3(256), 0, (hipStream_t)stream, batch, pred, target,
                     loss, dpred, grad_scale);
  return check_launch("se3_loss_kernel");
}
