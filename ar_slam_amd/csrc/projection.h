// projection.h -- device restatement of the reference's residual and its
// analytic Jacobian, shared by the per-capture LM kernels (lm_kernels.hip)
// and the batched localizer (localize.hip).
//
//   projectCorner<T>            ar_slam_util.cpp:131-172
//   ArucoReprojectionError      ar_slam_util.cpp:192-216
//   ceres::AngleAxisRotatePoint Ceres 2.0 rotation.h (incl. the theta^2 <= DBL_EPSILON branch)
//   Jacobian                    SURVEY.md Appendix A
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

namespace arslam {
namespace {

constexpr double kArucoSize = 0.0635;  // ar_slam_util.hpp:319

__device__ __forceinline__ double corner_dx(int i) { return (i == 1 || i == 2) ? 1.0 : -1.0; }
__device__ __forceinline__ double corner_dy(int i) { return (i >= 2) ? 1.0 : -1.0; }

// Angle-axis trigonometry with Ceres' branch (rotation.h AngleAxisRotatePoint).
struct AngleAxis {
  double w[3];
  double th2, th, c, s, ti;
  bool big;
};

// theta^2 exactly as rotation.h evaluates it on x86-64 (three rounded
// products, two rounded sums, no FMA): the branch test theta^2 > DBL_EPSILON
// must pick the same side as the reference for draws within an ulp of it.
__device__ __forceinline__ double aa_theta2(const double *w) {
#pragma clang fp contract(off)
  return w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
}

__device__ __forceinline__ AngleAxis aa_prepare(const double *w) {
  AngleAxis a;
  a.w[0] = w[0]; a.w[1] = w[1]; a.w[2] = w[2];
  a.th2 = aa_theta2(w);
  a.big = a.th2 > DBL_EPSILON;
  if (a.big) {
    a.th = sqrt(a.th2);
    sincos(a.th, &a.s, &a.c);
    a.ti = 1.0 / a.th;
  } else {
    a.th = 0.0; a.s = 0.0; a.c = 1.0; a.ti = 0.0;
  }
  return a;
}

// rotate point p by the angle-axis (Ceres operation order)
__device__ __forceinline__ void aa_rotate(const AngleAxis &a, const double *p, double *out) {
  if (a.big) {
    const double u0 = a.w[0] * a.ti, u1 = a.w[1] * a.ti, u2 = a.w[2] * a.ti;
    const double c0 = u1 * p[2] - u2 * p[1], c1 = u2 * p[0] - u0 * p[2], c2 = u0 * p[1] - u1 * p[0];
    const double tmp = (u0 * p[0] + u1 * p[1] + u2 * p[2]) * (1.0 - a.c);
    out[0] = p[0] * a.c + c0 * a.s + u0 * tmp;
    out[1] = p[1] * a.c + c1 * a.s + u1 * tmp;
    out[2] = p[2] * a.c + c2 * a.s + u2 * tmp;
  } else {
    out[0] = p[0] + (a.w[1] * p[2] - a.w[2] * p[1]);
    out[1] = p[1] + (a.w[2] * p[0] - a.w[0] * p[2]);
    out[2] = p[2] + (a.w[0] * p[1] - a.w[1] * p[0]);
  }
}

// rotation matrix M of the map p -> rotate(p): R(w) or I + [w]x (small branch)
__device__ __forceinline__ void aa_matrix(const AngleAxis &a, double M[9]) {
  if (a.big) {
    const double u0 = a.w[0] * a.ti, u1 = a.w[1] * a.ti, u2 = a.w[2] * a.ti;
    const double omc = 1.0 - a.c;
    M[0] = a.c + omc * u0 * u0;  M[1] = -a.s * u2 + omc * u0 * u1;  M[2] = a.s * u1 + omc * u0 * u2;
    M[3] = a.s * u2 + omc * u1 * u0;  M[4] = a.c + omc * u1 * u1;  M[5] = -a.s * u0 + omc * u1 * u2;
    M[6] = -a.s * u1 + omc * u2 * u0;  M[7] = a.s * u0 + omc * u2 * u1;  M[8] = a.c + omc * u2 * u2;
  } else {
    M[0] = 1.0;     M[1] = -a.w[2]; M[2] = a.w[1];
    M[3] = a.w[2];  M[4] = 1.0;     M[5] = -a.w[0];
    M[6] = -a.w[1]; M[7] = a.w[0];  M[8] = 1.0;
  }
}

// right Jacobian of SO(3): Jr = I - A [w]x + B [w]x^2 (big branch only)
__device__ __forceinline__ void aa_right_jacobian(const AngleAxis &a, double Jr[9]) {
  double A, B;
  if (a.th < 0.5) {
    // A = sum_k (-th2)^k / (2k+2)!, B = sum_k (-th2)^k / (2k+3)!, k < 7 (truncation
    // < 1e-16 relative), by Horner on correctly rounded reciprocal factorials
    // (no double divisions on the device; the oracle sums t / k! directly, the
    // two agree to a few ulps of the Jacobian entries)
    constexpr double ca[7] = {1.0 / 2.0, 1.0 / 24.0, 1.0 / 720.0, 1.0 / 40320.0, 1.0 / 3628800.0,
                              1.0 / 479001600.0, 1.0 / 87178291200.0};
    constexpr double cb[7] = {1.0 / 6.0, 1.0 / 120.0, 1.0 / 5040.0, 1.0 / 362880.0, 1.0 / 39916800.0,
                              1.0 / 6227020800.0, 1.0 / 1307674368000.0};
    const double x = -a.th2;
    A = ca[6];
    B = cb[6];
#pragma unroll
    for (int k = 5; k >= 0; --k) {
      A = A * x + ca[k];
      B = B * x + cb[k];
    }
  } else {
    const double sh = sin(0.5 * a.th);
    A = 2.0 * sh * sh / a.th2;
    B = (a.th - a.s) / (a.th2 * a.th);
  }
  const double w0 = a.w[0], w1 = a.w[1], w2 = a.w[2];
  // [w]x and [w]x^2 = w w^T - th2 I
  Jr[0] = 1.0 + B * (w0 * w0 - a.th2);
  Jr[1] = A * w2 + B * (w0 * w1);
  Jr[2] = -A * w1 + B * (w0 * w2);
  Jr[3] = -A * w2 + B * (w1 * w0);
  Jr[4] = 1.0 + B * (w1 * w1 - a.th2);
  Jr[5] = A * w0 + B * (w1 * w2);
  Jr[6] = A * w1 + B * (w2 * w0);
  Jr[7] = -A * w0 + B * (w2 * w1);
  Jr[8] = 1.0 + B * (w2 * w2 - a.th2);
}

__device__ __forceinline__ void cross3(const double *u, const double *v, double *o) {
  o[0] = u[1] * v[2] - u[2] * v[1];
  o[1] = u[2] * v[0] - u[0] * v[2];
  o[2] = u[0] * v[1] - u[1] * v[0];
}

// row vector (1x3) times 3x3 matrix
__device__ __forceinline__ void vecmat3(const double *v, const double *M, double *o) {
  o[0] = v[0] * M[0] + v[1] * M[3] + v[2] * M[6];
  o[1] = v[0] * M[1] + v[1] * M[4] + v[2] * M[7];
  o[2] = v[0] * M[2] + v[1] * M[5] + v[2] * M[8];
}

// Residual of one row (corner, comp) of ArucoReprojectionError.
__device__ __forceinline__ double residual_row(const AngleAxis &ac, const double *cap,
                                               const AngleAxis &at, const double *tag, double f,
                                               int corner, int comp, double obs, double *a_out,
                                               double *p_out) {
  const double cpt[3] = {0.5 * kArucoSize * corner_dx(corner), 0.5 * kArucoSize * corner_dy(corner), 0.0};
  double a[3], p[3];
  aa_rotate(at, cpt, a);
  a[0] += tag[0]; a[1] += tag[1]; a[2] += tag[2];   // ar_slam_util.cpp:146-148
  a[0] += cap[0]; a[1] += cap[1]; a[2] += cap[2];   // :152-154
  aa_rotate(ac, a, p);                              // :155
  const double xy = (comp == 0 ? p[0] : p[1]) / p[2];
  if (a_out) { a_out[0] = a[0]; a_out[1] = a[1]; a_out[2] = a[2]; }
  if (p_out) { p_out[0] = p[0]; p_out[1] = p[1]; p_out[2] = p[2]; }
  return f * xy - obs;
}

// Residual row and its 13 non-zero Jacobian entries: [f, t_c(3), w_c(3), t_t(3), w_t(3)].
__device__ __forceinline__ double residual_jacobian_row(const double *cam, const double *cap,
                                                        const double *tag, int corner, int comp,
                                                        double obs, double J[13]) {
  const AngleAxis ac = aa_prepare(cap + 3);
  const AngleAxis at = aa_prepare(tag + 3);
  double a[3], p[3];
  const double f = cam[0];
  const double r = residual_row(ac, cap, at, tag, f, corner, comp, obs, a, p);
  const double x = p[0] / p[2], y = p[1] / p[2];
  const double fz = f / p[2];
  const double P[3] = {comp == 0 ? fz : 0.0, comp == 0 ? 0.0 : fz, comp == 0 ? -fz * x : -fz * y};
  double Mc[9];
  aa_matrix(ac, Mc);
  double PM[3];
  vecmat3(P, Mc, PM);
  J[0] = comp == 0 ? x : y;
  J[1] = PM[0]; J[2] = PM[1]; J[3] = PM[2];
  J[7] = PM[0]; J[8] = PM[1]; J[9] = PM[2];
  // d/dw_c = -((P Mc) x a) Jr_c   (small branch: -(P x a))
  double v[3];
  if (ac.big) {
    cross3(PM, a, v);
    double Jr[9], o[3];
    aa_right_jacobian(ac, Jr);
    vecmat3(v, Jr, o);
    J[4] = -o[0]; J[5] = -o[1]; J[6] = -o[2];
  } else {
    cross3(P, a, v);
    J[4] = -v[0]; J[5] = -v[1]; J[6] = -v[2];
  }
  // d/dw_t = -((P Mc Mt) x c) Jr_t   (small branch: -((P Mc) x c))
  const double cpt[3] = {0.5 * kArucoSize * corner_dx(corner), 0.5 * kArucoSize * corner_dy(corner), 0.0};
  if (at.big) {
    double Mt[9], PMM[3], o[3], Jr[9];
    aa_matrix(at, Mt);
    vecmat3(PM, Mt, PMM);
    cross3(PMM, cpt, v);
    aa_right_jacobian(at, Jr);
    vecmat3(v, Jr, o);
    J[10] = -o[0]; J[11] = -o[1]; J[12] = -o[2];
  } else {
    cross3(PM, cpt, v);
    J[10] = -v[0]; J[11] = -v[1]; J[12] = -v[2];
  }
  return r;
}

// Wave-wide reductions without the LDS crossbar (a __shfl_xor is a
// ds_bpermute round trip per 32-bit half and step): DPP inside each 16-lane
// row (xor 1, xor 2, half-row mirror, row mirror), then v_permlane16_swap
// between the rows of a pair and v_permlane32_swap between the halves.
// Every step combines a lane with its partner symmetrically, so all 64
// lanes end with bit-identical results (the LM decisions stay wave-uniform).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xf, 0xf, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// W = 64: the whole wave; W = 32: each half-wave separately (two queries per
// wave in k_localize).
template <int W = 64, class Op>
__device__ __forceinline__ double wave_reduce(double v, Op op) {
  v = op(v, dpp_f64<0xB1>(v));    // quad_perm [1,0,3,2]: lane ^ 1
  v = op(v, dpp_f64<0x4E>(v));    // quad_perm [2,3,0,1]: lane ^ 2
  v = op(v, dpp_f64<0x141>(v));   // row_half_mirror: the other quad of each 8
  v = op(v, dpp_f64<0x140>(v));   // row_mirror: the other 8 of each 16
  unsigned long long u = __double_as_longlong(v);
  const auto a = __builtin_amdgcn_permlane16_swap((unsigned)u, (unsigned)u, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap((unsigned)(u >> 32), (unsigned)(u >> 32), false, false);
  v = op(__longlong_as_double((long long)(((unsigned long long)b[0] << 32) | a[0])),
         __longlong_as_double((long long)(((unsigned long long)b[1] << 32) | a[1])));   // rows 2g, 2g+1
  if (W == 32) return v;
  u = __double_as_longlong(v);
  const auto c = __builtin_amdgcn_permlane32_swap((unsigned)u, (unsigned)u, false, false);
  const auto d = __builtin_amdgcn_permlane32_swap((unsigned)(u >> 32), (unsigned)(u >> 32), false, false);
  return op(__longlong_as_double((long long)(((unsigned long long)d[0] << 32) | c[0])),
            __longlong_as_double((long long)(((unsigned long long)d[1] << 32) | c[1])));   // halves
}

template <int W = 64>
__device__ __forceinline__ double wave_sum(double v) {
  return wave_reduce<W>(v, [](double x, double y) { return x + y; });
}
template <int W = 64>
__device__ __forceinline__ double wave_max(double v) {
  return wave_reduce<W>(v, [](double x, double y) { return fmax(x, y); });
}


}  // namespace
}  // namespace arslam
