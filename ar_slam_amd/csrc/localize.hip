// localize.hip -- batched localizeMany (ar_slam_util.cpp:888-979) on gfx950.
//
// One 64-lane wavefront runs one query's whole ceres::Solve: the capture's
// 6 pose parameters are the only free block (tags :965 and camera :972 are
// constant), so every trust-region step is a 6x6 solve.  Lane l owns
// residual row l (= 8 obs + 2 corner + {x,y}) of each 64-row chunk of the
// query's observations; k = 8 tags per query is exactly one wave.  Per
// iteration the wave forms J'J (21), J'r and the column norms with
// xor-butterfly reductions (identical bits on every lane, so the LM control
// flow is wave-uniform), factors the 6x6 LM system redundantly in every lane,
// evaluates the candidate's cost, and applies Ceres 2.0's step acceptance,
// radius update and termination rules -- no host
// round trip until every query has terminated.  The control flow restates
// the oracle's or_solve (oracle/arslam_oracle.c) for a single free block.
#include "lm_internal.h"
#include "projection.h"
#include "arslam_localize.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

namespace arslam {
namespace {

constexpr int kMaxChunks = ARSLAM_LOC_MAX_OBS * 8 / 64;

struct LocParams {
  int nq, nt;
  const double *cam;           // [3]
  const double *tag;           // [nt*6]
  const unsigned char *tim;    // [nt] or null
  const int *qs;               // [nq+1]
  const int *ot;               // [nb]
  const double *corners;       // [nb*8]
  const double *pose_in;       // [nq*6]
  double *pose_out;            // [nq*6]
  arslam_localize_result *res; // [nq]
  const double *aw;            // [nt*4][4] world points of the (constant) tags' corners
  int init_from_map, max_k;
  int max_iters, max_invalid, jacobi;
  double ftol, gtol, ptol, r0, rmax, rmin, min_rel, dmin, dmax;
};

// ---- initialisers (ar_slam_util.cpp:41-128; Ceres 2.0 rotation.h) ----
__device__ void aa_to_quat(const double aa[3], double q[4]) {
  const double theta_sq = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta_sq > 0.0) {
    const double theta = sqrt(theta_sq);
    const double half = theta * 0.5;
    const double k = sin(half) / theta;
    q[0] = cos(half);
    q[1] = aa[0] * k; q[2] = aa[1] * k; q[3] = aa[2] * k;
  } else {
    q[0] = 1.0;
    q[1] = aa[0] * 0.5; q[2] = aa[1] * 0.5; q[3] = aa[2] * 0.5;
  }
}

__device__ void quat_to_aa(const double q[4], double aa[3]) {
  const double sin_sq = q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  double k = 2.0;
  if (sin_sq > 0.0) {
    const double sin_theta = sqrt(sin_sq), cos_theta = q[0];
    const double two_theta = 2.0 * ((cos_theta < 0.0) ? atan2(-sin_theta, -cos_theta)
                                                       : atan2(sin_theta, cos_theta));
    k = two_theta / sin_theta;
  }
  aa[0] = q[1] * k; aa[1] = q[2] * k; aa[2] = q[3] * k;
}

// composeAxisAngle :41-50
__device__ void compose_axis_angle(const double r1[3], const double r2[3], double out[3]) {
  double a[4], b[4], c[4];
  aa_to_quat(r1, a);
  aa_to_quat(r2, b);
  c[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  c[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  c[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  c[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  quat_to_aa(c, out);
}

__device__ double normalize_angle(double a) {   // ar_slam_util.hpp:348-351
  return fmod(fmod(a, 2 * M_PI) + 3 * M_PI, 2 * M_PI) - M_PI;
}

// calcInitValues :52-95 + initCapturePose :98-115
__device__ void init_capture_pose(const double *corners, const double *camera, const double *ar_pose,
                                  double *inv) {
  const double focal = camera[0];
  double max_dist_sq = 0.0, avg_x = 0.0, avg_y = 0.0;
  for (int i = 0; i < 4; ++i) {
    const double *p1 = corners + 2 * i, *p2 = corners + 2 * ((i + 1) & 3);
    const double dx = p1[0] - p2[0], dy = p1[1] - p2[1];
    const double d = dx * dx + dy * dy;
    max_dist_sq = fmax(d, max_dist_sq);
    avg_x += p1[0];
    avg_y += p1[1];
  }
  avg_x *= 0.25;
  avg_y *= 0.25;
  double avg_angle = 0.0;
  for (int i = 0; i < 4; ++i) {
    const double expected = atan2(corner_dy(i), corner_dx(i));
    const double actual = atan2(corners[2 * i + 1] - avg_y, corners[2 * i] - avg_x);
    const double delta = normalize_angle(actual - expected);
    avg_angle += normalize_angle(delta - avg_angle) / (i + 1);
  }
  const double local_z = focal * kArucoSize / sqrt(max_dist_sq);
  const double local_position[3] = {avg_x * local_z / focal, avg_y * local_z / focal, local_z};
  const double local_rot[3] = {0.0, 0.0, avg_angle};
  const double inv_ar_rot[3] = {-ar_pose[3], -ar_pose[4], -ar_pose[5]};
  compose_axis_angle(local_rot, inv_ar_rot, inv + 3);
  const double cap_rotation[3] = {-inv[3], -inv[4], -inv[5]};
  const AngleAxis cr = aa_prepare(cap_rotation);
  aa_rotate(cr, local_position, inv);
  inv[0] -= ar_pose[0];
  inv[1] -= ar_pose[1];
  inv[2] -= ar_pose[2];
}

// ---- the constant map: tag corners in the world frame ----
// localizeOne holds every tag and the camera constant (ar_slam_util.cpp:965,
// 972), so the first half of projectCorner, a = R(w_t) c_i + t_t (:144-148),
// is the same for every query and iteration: computed once per batch solve.
__global__ void k_tag_corners(int nt, const double *__restrict__ tag, double *__restrict__ aw) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;   // 4 t + corner
  if (e >= 4 * nt) return;
  const double *tg = tag + 6L * (e >> 2);
  const AngleAxis at = aa_prepare(tg + 3);
  const double cpt[3] = {0.5 * kArucoSize * corner_dx(e & 3), 0.5 * kArucoSize * corner_dy(e & 3), 0.0};
  double a[3];
  aa_rotate(at, cpt, a);
  aw[4L * e] = a[0] + tg[0];
  aw[4L * e + 1] = a[1] + tg[1];
  aw[4L * e + 2] = a[2] + tg[2];
  aw[4L * e + 3] = 0.0;
}

// The capture's rotation, its matrix and right Jacobian: the same for every
// row of the query, computed once per evaluation (not per row).
struct CapFrame {
  AngleAxis ac;
  double M[9], Jr[9];
};

__device__ __forceinline__ void cap_frame(const double *x, CapFrame &F, bool jac) {
  F.ac = aa_prepare(x + 3);
  if (!jac) return;
  aa_matrix(F.ac, F.M);
  if (F.ac.big) aa_right_jacobian(F.ac, F.Jr);
}

// Residual row of a corner whose world point is aw: b = aw + t_c, p = R(w_c) b
// (:152-155), r = f p_xy / p_z - obs (:157-162, :198-211); with J6 != null
// also its 6 capture-block Jacobian entries [t_c, w_c].
__device__ __forceinline__ double loc_row(const CapFrame &F, const double *x, const double *aw, double f,
                                          int comp, double obs, double *J6) {
  double b[3] = {aw[0] + x[0], aw[1] + x[1], aw[2] + x[2]}, p[3];
  aa_rotate(F.ac, b, p);
  const double r = f * ((comp == 0 ? p[0] : p[1]) / p[2]) - obs;
  if (J6) {
    const double xx = p[0] / p[2], yy = p[1] / p[2], fz = f / p[2];
    const double P[3] = {comp == 0 ? fz : 0.0, comp == 0 ? 0.0 : fz, comp == 0 ? -fz * xx : -fz * yy};
    double PM[3], v[3];
    vecmat3(P, F.M, PM);
    J6[0] = PM[0]; J6[1] = PM[1]; J6[2] = PM[2];
    if (F.ac.big) {   // d/dw_c = -((P Mc) x b) Jr_c
      double o[3];
      cross3(PM, b, v);
      vecmat3(v, F.Jr, o);
      J6[3] = -o[0]; J6[4] = -o[1]; J6[5] = -o[2];
    } else {          // small branch: -(P x b)
      cross3(P, b, v);
      J6[3] = -v[0]; J6[4] = -v[1]; J6[5] = -v[2];
    }
  }
  return r;
}

// packed upper index of the diagonal entry (j, j) of the 6x6 normal matrix
#define HD(j) ((j) * 6 - ((j) * ((j) - 1)) / 2)

// ---- one query per wavefront ----
template <int NCH>
struct Rows {
  double r[NCH];
  double J[NCH][6];
};

// Residuals and capture-block Jacobian rows at x; wave-reduced cost, J'r,
// column norms and the 21 upper entries of J'J.  Returns false if a residual
// is not finite (uniform).
// Per-query sums of 28 per-lane partials through LDS, instead of 28 butterfly
// reductions (5 dependent DPP/permlane + add steps each, ~15 VALU
// instructions per value): every lane writes its partials, lane v < 28 of the
// query sums value v's LPQ partials by a fixed pairwise tree, and every lane
// reads the 28 sums back -- the same bits on every lane of the query, so its
// control flow stays uniform.  red: this query's [28][LPQ + 2] partials
// (16-byte rows, bank-staggered by the pad) then [28] sums.
template <int LPQ>
__device__ __forceinline__ void query_sums28(double *red, int lane, double c, const double (&gl)[6],
                                             const double (&hl)[21], double &cost) {
  constexpr int P = LPQ + 2;
  red[lane] = c;
#pragma unroll
  for (int e = 0; e < 6; ++e) red[(1 + e) * P + lane] = gl[e];
#pragma unroll
  for (int e = 0; e < 21; ++e) red[(7 + e) * P + lane] = hl[e];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane < 28) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2 *row = reinterpret_cast<const d2 *>(red + lane * P);
    // pairwise: groups of 8 partials (three levels each), then the groups' sums
    double gs[LPQ / 8];
#pragma unroll
    for (int gi = 0; gi < LPQ / 8; ++gi) {
      const d2 a = row[4 * gi], b = row[4 * gi + 1], cc = row[4 * gi + 2], d = row[4 * gi + 3];
      gs[gi] = ((a.x + a.y) + (b.x + b.y)) + ((cc.x + cc.y) + (d.x + d.y));
    }
#pragma unroll
    for (int n = LPQ / 16; n >= 1; n >>= 1)
#pragma unroll
      for (int i = 0; i < n; ++i) gs[i] = gs[2 * i] + gs[2 * i + 1];
    red[28 * P + lane] = gs[0];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  cost = 0.5 * red[28 * P];
  // (J'r and J'J stay in LDS, red + sums_off<LPQ>(): read where they are used,
  // not held in 27 x 2 VGPRs across the LM loop)
}

// offset of query_sums28's sums in a query's LDS region: [0] cost x 2, [1..6] J'r, [7..27] J'J
template <int LPQ>
constexpr int sums_off() { return 28 * (LPQ + 2); }

template <int NCH, int LPQ>
__device__ bool evaluate_jacobian(const LocParams &p, const double *rc, int nrow, const double *x, int lane,
                                  double &cost, double *red,
                                  const AngleAxis *ac_pre = nullptr) {
  double c = 0.0, gl[6] = {0, 0, 0, 0, 0, 0}, hl[21];
#pragma unroll
  for (int e = 0; e < 21; ++e) hl[e] = 0.0;
  bool bad = false;
  CapFrame F;
  if (ac_pre) {   // the accepted candidate's rotation, from its cost evaluation
    F.ac = *ac_pre;
    aa_matrix(F.ac, F.M);
    if (F.ac.big) aa_right_jacobian(F.ac, F.Jr);
  } else {
    cap_frame(x, F, true);
  }
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int R = lane + LPQ * ch;
    if (R < nrow) {
      const double *rr = rc + 4 * R;   // (the row's corner world point and observation, LDS)
      double j6[6];
      const double r = loc_row(F, x, rr, p.cam[0], R & 1, rr[3], j6);
      bad = bad || !isfinite(r);
      c += r * r;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        gl[j] += j6[j] * r;
      }
      int e = 0;
#pragma unroll
      for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = a; b < 6; ++b) hl[e++] += j6[a] * j6[b];
    }
  }
  // the 28 per-lane partials (cost, J'r, J'J) summed per query through LDS
  query_sums28<LPQ>(red, lane, c, gl, hl, cost);
  return wave_max<LPQ>(bad ? 1.0 : 0.0) == 0.0;
}

template <int NCH, int LPQ>
__device__ double evaluate_cost(const LocParams &p, const double *rc, int nrow, const double *x, int lane, bool &finite,
                              CapFrame &F) {
  cap_frame(x, F, false);
  double c = 0.0;
  bool bad = false;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int R = lane + LPQ * ch;
    if (R < nrow) {
      const double *rr = rc + 4 * R;
      const double r = loc_row(F, x, rr, p.cam[0], R & 1, rr[3], nullptr);
      bad = bad || !isfinite(r);
      c += r * r;
    }
  }
  finite = wave_max<LPQ>(bad ? 1.0 : 0.0) == 0.0;
  return 0.5 * wave_sum<LPQ>(c);
}

// LPQ lanes per query (64: one query per wave; 32: two queries per wave, each
// half-wave its own LM -- the 6x6 solves, the LM bookkeeping and the
// capture's rotation then cost half the instructions per query), NCH =
// LPQ-row chunks per query (k <= NCH LPQ / 8 observations).  One wavefront
// per workgroup, so a finished wave's slot is reused at once.
template <int NCH, int LPQ>
__global__ __launch_bounds__(64, 2) void k_localize(LocParams p) {
  const int lane = threadIdx.x & (LPQ - 1);
  const int q = blockIdx.x * (64 / LPQ) + threadIdx.x / LPQ;
  // (query_sums28's partials and sums, one region per query of the wave)
  __shared__ __attribute__((aligned(16))) double red_all[(64 / LPQ) * (28 * (LPQ + 2) + 28)];
  double *red = red_all + (threadIdx.x / LPQ) * (28 * (LPQ + 2) + 28);
  // each row's corner world point and observation, gathered once per query
  // (obs_tag -> the tag's corner points: two dependent global loads per row
  // that every cost and Jacobian evaluation repeated)
  __shared__ __attribute__((aligned(16))) double rc_all[(64 / LPQ) * NCH * LPQ * 4];
  double *rc = rc_all + (threadIdx.x / LPQ) * NCH * LPQ * 4;
  if (q >= p.nq) return;
  const int o0 = p.qs[q], k = p.qs[q + 1] - o0;
  arslam_localize_result res;
  res.status = ARSLAM_LOC_SKIPPED;
  res.rule = ARSLAM_RULE_NONE;
  res.num_iterations = res.num_successful_steps = res.num_unsuccessful_steps = 0;
  res.init_obs = -1;
  res.initial_cost = res.final_cost = 0.0;
  double x[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) x[j] = p.pose_in[6L * q + j];
  // localizeOne :911-933: the first block whose tag is in the map
  for (int j = 0; j < k; ++j)
    if (!p.tim || p.tim[p.ot[o0 + j]]) { res.init_obs = o0 + j; break; }
  const bool skip = k == 0 || (p.init_from_map && res.init_obs < 0);
  if (skip) {
    if (lane == 0) {
      p.res[q] = res;
#pragma unroll
      for (int j = 0; j < 6; ++j) p.pose_out[6L * q + j] = x[j];
    }
    return;
  }
  if (p.init_from_map)
    init_capture_pose(p.corners + 8L * res.init_obs, p.cam, p.tag + 6L * p.ot[res.init_obs], x);
  const int nrow = 8 * k;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int R = lane + LPQ * ch;
    if (R < nrow) {
      const int o = o0 + (R >> 3), row = R & 7;
      const double *a = p.aw + 4L * (4 * p.ot[o] + (row >> 1));
      typedef double d2 __attribute__((ext_vector_type(2)));
      reinterpret_cast<d2 *>(rc + 4 * R)[0] = d2{a[0], a[1]};
      reinterpret_cast<d2 *>(rc + 4 * R)[1] = d2{a[2], p.corners[8L * o + row]};
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // ---- iteration 0 ----
  double cost;
  // J'r and J'J of the last linearization, in LDS (column norms squared = diag(H): HD(j))
  const double *g = red + sums_off<LPQ>() + 1, *H = red + sums_off<LPQ>() + 7;
  double x_norm = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3] + x[4] * x[4] + x[5] * x[5]);
  bool finite = evaluate_jacobian<NCH, LPQ>(p, rc, nrow, x, lane, cost, red);
  res.initial_cost = cost;
  if (!finite) {
    res.status = ARSLAM_FAILURE;
    res.rule = ARSLAM_RULE_EVAL_FAILED;
    res.final_cost = cost;
  } else {
    double scale[6], diag[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) scale[j] = p.jacobi ? 1.0 / (1.0 + sqrt(H[HD(j)])) : 1.0;
    double radius = p.r0, decrease = 2.0;
    bool reuse_diag = false, succ = true;
    int n_invalid = 0, iteration = 0;
    double gmax = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) gmax = fmax(gmax, fabs(g[j]));
    for (;;) {
      // FinalizeIterationAndCheckIfMinimizerCanContinue
      if (succ) res.num_successful_steps += iteration > 0;
      else res.num_unsuccessful_steps++;
      res.num_iterations++;
      if (iteration >= p.max_iters) { res.status = ARSLAM_NO_CONVERGENCE; res.rule = ARSLAM_RULE_MAX_ITERS; break; }
      if (succ && gmax <= p.gtol) { res.status = ARSLAM_CONVERGENCE; res.rule = ARSLAM_RULE_GRADIENT; break; }
      if (radius <= p.rmin) { res.status = ARSLAM_CONVERGENCE; res.rule = ARSLAM_RULE_MIN_RADIUS; break; }
      ++iteration;
      // LevenbergMarquardtStrategy: D^2 = clamp(diag(J~'J~)) / radius
      if (!reuse_diag)
#pragma unroll
        for (int j = 0; j < 6; ++j) diag[j] = fmin(fmax(scale[j] * scale[j] * H[HD(j)], p.dmin), p.dmax);
      reuse_diag = true;
      // (J~'J~ + D^2) y = J~'r, 6x6 Cholesky in every lane
      double A[21], y[6];
      {
        // D^2 = diag / radius by one reciprocal (Ceres forms sqrt(diag / radius)
        // and squares it: the same value to an ulp, twelve fewer sqrt / divide
        // sequences per iteration)
        const double rr = 1.0 / radius;
        int e = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
          for (int b = a; b < 6; ++b) {
            double v = scale[a] * scale[b] * H[e];
            if (a == b) v += diag[a] * rr;
            A[e++] = v;
          }
      }
      // packed upper index of (a,b), a <= b
#define UP(a, b) ((a) * 6 - ((a) * ((a) - 1)) / 2 + ((b) - (a)))
      // in place: L[i][j] (i >= j) overwrites A[UP(j, i)]
      bool lin_ok = true;
      double il[6];
#define L_(i, j) A[UP(j, i)]
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        double s = L_(j, j);
#pragma unroll
        for (int m = 0; m < j; ++m) s -= L_(j, m) * L_(j, m);
        lin_ok = lin_ok && s > 0.0;
        // 1 / L_jj = s^(-1/2): v_rsq_f64 and two Newton steps (the substitutions
        // and the column only multiply by it; L_jj itself is never read)
        double r = __builtin_amdgcn_rsq(s);
        r = r * __builtin_fma(-0.5 * s * r, r, 1.5);
        r = r * __builtin_fma(-0.5 * s * r, r, 1.5);
        il[j] = r;
#pragma unroll
        for (int i = j + 1; i < 6; ++i) {
          double t = L_(i, j);
#pragma unroll
          for (int m = 0; m < j; ++m) t -= L_(i, m) * L_(j, m);
          L_(i, j) = t * il[j];
        }
      }
      if (lin_ok) {
        double z[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          double t = scale[i] * g[i];
#pragma unroll
          for (int m = 0; m < i; ++m) t -= L_(i, m) * z[m];
          z[i] = t * il[i];
        }
#pragma unroll
        for (int i = 5; i >= 0; --i) {
          double t = z[i];
#pragma unroll
          for (int m = i + 1; m < 6; ++m) t -= L_(m, i) * y[m];
          y[i] = t * il[i];
        }
        bool yfin = true;
#pragma unroll
        for (int i = 0; i < 6; ++i) yfin = yfin && isfinite(y[i]);
        lin_ok = yfin;
      }
#undef L_
#undef UP
      // step = -y; model cost change m = -(r'J~ step + step' J~'J~ step / 2),
      // from J'r and J'J (LDS) -- in exact arithmetic the same as Ceres'
      // -sum mr (r + mr/2), mr = J~ step, over the rows, without keeping the
      // rows in registers or reducing over the lanes
      double model = 0.0;
      bool valid = false;
      if (lin_ok) {
        double st[6];
#pragma unroll
        for (int j = 0; j < 6; ++j) st[j] = scale[j] * (-y[j]);   // the unscaled step
        double lin = 0.0, quad = 0.0;
#pragma unroll
        for (int j = 0; j < 6; ++j) lin += g[j] * st[j];
        int e = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
          double row = 0.0;
#pragma unroll
          for (int b = a; b < 6; ++b) row += (b == a ? 0.5 : 1.0) * H[e++] * st[b];
          quad += st[a] * row;
        }
        model = -(lin + quad);
        valid = model > 0.0;
      }
      if (!valid) {
        // Ceres 2.0 HandleInvalidStep: ++num_consecutive_invalid_steps_ >= max -> FAILURE
        if (++n_invalid >= p.max_invalid) { res.status = ARSLAM_FAILURE; res.rule = ARSLAM_RULE_INVALID_STEPS; break; }
        radius = radius / decrease;
        decrease *= 2.0;
        succ = false;
        continue;
      }
      n_invalid = 0;
      double xc[6], sq = 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        xc[j] = x[j] + (-y[j]) * scale[j];
        const double d = x[j] - xc[j];
        sq += d * d;
      }
      bool cfin = true;
      CapFrame Fc;
      double cand = evaluate_cost<NCH, LPQ>(p, rc, nrow, xc, lane, cfin, Fc);
      if (!cfin) cand = DBL_MAX;
      // ParameterToleranceReached / FunctionToleranceReached
      if (sqrt(sq) <= p.ptol * (x_norm + p.ptol)) { res.status = ARSLAM_CONVERGENCE; res.rule = ARSLAM_RULE_PARAMETER; break; }
      const double change = cost - cand;
      if (fabs(change) <= p.ftol * cost) { res.status = ARSLAM_CONVERGENCE; res.rule = ARSLAM_RULE_FUNCTION; break; }
      const double rho = cand >= DBL_MAX ? -DBL_MAX : (cost - cand) / model;
      if (rho > p.min_rel) {
#pragma unroll
        for (int j = 0; j < 6; ++j) x[j] = xc[j];
        x_norm = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3] + x[4] * x[4] + x[5] * x[5]);
        (void)evaluate_jacobian<NCH, LPQ>(p, rc, nrow, x, lane, cost, red, &Fc.ac);
        gmax = 0.0;
#pragma unroll
        for (int j = 0; j < 6; ++j) gmax = fmax(gmax, fabs(g[j]));
        succ = true;
        const double t = 2.0 * rho - 1.0;
        radius = fmin(radius / fmax(1.0 / 3.0, 1.0 - t * t * t), p.rmax);
        decrease = 2.0;
        reuse_diag = false;
      } else {
        succ = false;
        radius = radius / decrease;
        decrease *= 2.0;
      }
    }
    res.final_cost = cost;
  }
  if (lane == 0) {
    p.res[q] = res;
#pragma unroll
    for (int j = 0; j < 6; ++j) p.pose_out[6L * q + j] = x[j];
  }
}

}  // namespace

void launch_localize(const LocParams &p, hipStream_t s);

}  // namespace arslam

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------

namespace {


template <class T>
struct DBuf {
  T *p = nullptr;
  size_t n = 0;
  void alloc(size_t c) {
    release();
    n = c;
    if (c && hipMalloc(&p, c * sizeof(T)) != hipSuccess) {
      p = nullptr;
      throw arslam::ApiError(ARSLAM_E_OUT_OF_MEMORY, "hipMalloc failed");
    }
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  ~DBuf() { release(); }
};

void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess)
    throw arslam::ApiError(e == hipErrorOutOfMemory ? ARSLAM_E_OUT_OF_MEMORY : ARSLAM_E_HIP,
                           std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

struct arslam_localizer {
  arslam_lm_options opt;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  int nq = 0, nt = 0, nb = 0, init_from_map = 0, max_k = 0;
  bool has_tim = false, loaded = false;
  DBuf<double> cam, tag, corners, pose_in, pose_out, aw;
  DBuf<int> qs, ot;
  DBuf<unsigned char> tim;
  DBuf<arslam_localize_result> res;

  ~arslam_localizer() {
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (stream) (void)hipStreamDestroy(stream);
  }

  void ensure_stream() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
      throw arslam::ApiError(ARSLAM_E_NO_DEVICE, "no HIP device");
    int cur = -1;   // (set only when it differs)
    hip_check(hipGetDevice(&cur), "hipGetDevice");
    if (opt.device >= 0 && opt.device != cur) hip_check(hipSetDevice(opt.device), "hipSetDevice");
    if (!stream) {
      hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
      // (timing only: no system-scope fence at the records)
      hip_check(hipEventCreateWithFlags(&ev0, hipEventDisableSystemFence), "hipEventCreate");
      hip_check(hipEventCreateWithFlags(&ev1, hipEventDisableSystemFence), "hipEventCreate");
    }
  }

  void load(const arslam_localize_batch *b) {
    using arslam::api_check;
    api_check(b != nullptr, ARSLAM_E_INVALID_ARG, "null batch");
    api_check(b->n_query >= 0 && b->n_tag >= 0 && b->n_obs >= 0, ARSLAM_E_INVALID_ARG, "negative sizes");
    api_check(b->camera && b->pose && (!b->n_tag || b->tag) && b->query_start, ARSLAM_E_INVALID_ARG,
              "null arrays");
    api_check(!b->n_obs || (b->obs_tag && b->corners), ARSLAM_E_INVALID_ARG, "null observation arrays");
    api_check(b->query_start[0] == 0 && b->query_start[b->n_query] == b->n_obs, ARSLAM_E_INVALID_ARG,
              "query_start must run from 0 to n_obs");
    for (int q = 0; q < b->n_query; ++q) {
      api_check(b->query_start[q + 1] >= b->query_start[q], ARSLAM_E_INVALID_ARG, "query_start not monotone");
      api_check(b->query_start[q + 1] - b->query_start[q] <= ARSLAM_LOC_MAX_OBS, ARSLAM_E_UNSUPPORTED,
                "more than 64 observations in one query");
    }
    for (int o = 0; o < b->n_obs; ++o)
      api_check(b->obs_tag[o] >= 0 && b->obs_tag[o] < b->n_tag, ARSLAM_E_INVALID_ARG, "obs_tag out of range");
    ensure_stream();
    loaded = false;
    nq = b->n_query; nt = b->n_tag; nb = b->n_obs; init_from_map = b->init_from_map != 0;
    max_k = 0;
    for (int q = 0; q < nq; ++q) max_k = std::max(max_k, b->query_start[q + 1] - b->query_start[q]);
    auto up = [&](auto &buf, const auto *src, size_t count) {
      buf.alloc(std::max<size_t>(count, 1));
      if (count)
        hip_check(hipMemcpyAsync(buf.p, src, count * sizeof(*src), hipMemcpyHostToDevice, stream), "upload");
    };
    up(cam, b->camera, 3);
    up(tag, b->tag, 6L * nt);
    up(qs, b->query_start, (size_t)nq + 1);
    up(ot, b->obs_tag, nb);
    up(corners, b->corners, 8L * nb);
    up(pose_in, b->pose, 6L * nq);
    has_tim = b->tag_in_map != nullptr;
    if (has_tim) up(tim, b->tag_in_map, nt);
    pose_out.alloc(std::max(6L * nq, 1L));
    aw.alloc(std::max(16L * nt, 1L));
    res.alloc(std::max(nq, 1));
    hip_check(hipStreamSynchronize(stream), "load sync");
    loaded = true;
  }

  void solve(double *pose_host, arslam_localize_result *res_host, double *kernel_ms) {
    arslam::api_check(loaded, ARSLAM_E_STATE, "no batch loaded");
    arslam::LocParams p{};
    p.nq = nq; p.cam = cam.p; p.tag = tag.p; p.tim = has_tim ? tim.p : nullptr;
    p.qs = qs.p; p.ot = ot.p; p.corners = corners.p; p.pose_in = pose_in.p; p.pose_out = pose_out.p;
    p.res = res.p; p.init_from_map = init_from_map; p.max_k = max_k;
    p.aw = aw.p; p.nt = nt;
    p.max_iters = opt.max_num_iterations; p.max_invalid = opt.max_num_consecutive_invalid_steps;
    p.jacobi = opt.jacobi_scaling;
    p.ftol = opt.function_tolerance; p.gtol = opt.gradient_tolerance; p.ptol = opt.parameter_tolerance;
    p.r0 = opt.initial_trust_region_radius; p.rmax = opt.max_trust_region_radius;
    p.rmin = opt.min_trust_region_radius; p.min_rel = opt.min_relative_decrease;
    p.dmin = opt.min_lm_diagonal; p.dmax = opt.max_lm_diagonal;
    hip_check(hipEventRecord(ev0, stream), "event");
    arslam::launch_localize(p, stream);
    hip_check(hipGetLastError(), "k_localize launch");
    hip_check(hipEventRecord(ev1, stream), "event");
    if (pose_host && nq)
      hip_check(hipMemcpyAsync(pose_host, pose_out.p, 6L * nq * sizeof(double), hipMemcpyDeviceToHost, stream),
                "download");
    if (res_host && nq)
      hip_check(hipMemcpyAsync(res_host, res.p, (size_t)nq * sizeof(arslam_localize_result),
                               hipMemcpyDeviceToHost, stream), "download");
    hip_check(hipStreamSynchronize(stream), "solve sync");
    if (kernel_ms) {
      float ms = 0.0f;
      hip_check(hipEventElapsedTime(&ms, ev0, ev1), "elapsed");
      *kernel_ms = ms;
    }
  }
};

namespace arslam {
void launch_localize(const LocParams &p, hipStream_t s) {
  if (p.nq == 0) return;
  if (p.nt > 0)   // the map's corner points (inside the timed region: one launch per batch solve)
    hipLaunchKernelGGL(k_tag_corners, dim3((unsigned)((4 * p.nt + 255) / 256)), dim3(256), 0, s, p.nt, p.tag,
                       const_cast<double *>(p.aw));
  const dim3 block(64);
  if (p.max_k <= 8)   // (cfg5: k = 8) two queries per wave
    hipLaunchKernelGGL((k_localize<2, 32>), dim3((unsigned)((p.nq + 1) / 2)), block, 0, s, p);
  else if (p.max_k <= 16) hipLaunchKernelGGL((k_localize<2, 64>), dim3((unsigned)p.nq), block, 0, s, p);
  else hipLaunchKernelGGL((k_localize<kMaxChunks, 64>), dim3((unsigned)p.nq), block, 0, s, p);
}
}  // namespace arslam

namespace {
template <class F>
int loc_guarded(F &&f) {
  try {
    f();
    return ARSLAM_OK;
  } catch (const arslam::ApiError &e) {
    arslam::set_last_error(e.what());
    return e.code;
  } catch (const std::bad_alloc &) {
    arslam::set_last_error("host out of memory");
    return ARSLAM_E_OUT_OF_MEMORY;
  } catch (const std::exception &e) {
    arslam::set_last_error(e.what());
    return ARSLAM_E_HIP;
  }
}
}  // namespace

extern "C" {

int arslam_localizer_create(arslam_localizer **out, const arslam_lm_options *opt) {
  if (!out) return ARSLAM_E_INVALID_ARG;
  *out = nullptr;
  return loc_guarded([&] {
    auto *h = new arslam_localizer();
    if (opt) h->opt = *opt; else arslam_lm_options_init(&h->opt);
    *out = h;
  });
}

void arslam_localizer_destroy(arslam_localizer *h) { delete h; }

int arslam_localizer_load(arslam_localizer *h, const arslam_localize_batch *b) {
  if (!h || !b) return ARSLAM_E_INVALID_ARG;
  return loc_guarded([&] { h->load(b); });
}

int arslam_localizer_solve(arslam_localizer *h, double *pose_out, arslam_localize_result *res,
                           double *kernel_ms) {
  if (!h) return ARSLAM_E_INVALID_ARG;
  return loc_guarded([&] { h->solve(pose_out, res, kernel_ms); });
}

int arslam_localize_many(const arslam_localize_batch *b, const arslam_lm_options *opt,
                         arslam_localize_result *res) {
  if (!b) return ARSLAM_E_INVALID_ARG;
  arslam_localizer *h = nullptr;
  int rc = arslam_localizer_create(&h, opt);
  if (rc) return rc;
  rc = arslam_localizer_load(h, b);
  if (!rc) rc = arslam_localizer_solve(h, b->pose, res, nullptr);
  arslam_localizer_destroy(h);
  return rc;
}

}  // extern "C"
