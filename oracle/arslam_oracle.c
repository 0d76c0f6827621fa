/*
 * arslam_oracle.c -- CPU restatement of ar_slam's LM bundle adjustment.
 *
 * TEST INFRASTRUCTURE ONLY (see arslam_oracle.h).  Plain C99 + optional
 * OpenMP; compiled with -ffp-contract=off so every operation rounds as the
 * reference's x86-64 build of Ceres would (no FMA contraction).
 *
 * Citations:
 *   [P]  ar_slam/src/ar_slam_util.cpp  (reference, /root/reference)
 *   [H]  ar_slam/include/ar_slam/ar_slam_util.hpp
 *   [C]  Ceres Solver 2.0.0 (Ubuntu 22.04 libceres-dev, pinned by
 *        .github/workflows/build_and_test.yaml:14; un-vendored): restated
 *        from its published source, see SURVEY.md Appendix B.
 */
#include "arslam_oracle.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* aruco_size [H:319]; ARUCO_DIRECTIONS TL,TR,BR,BL [H:340-345] */
static const double kArucoSize = 0.0635;
static const double kDirs[4][2] = {{-1, -1}, {+1, -1}, {+1, +1}, {-1, +1}};

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

void or_default_options(or_options *o) {
  /* [P:1003-1011] sets max_num_iterations=50 and DENSE_SCHUR; the rest are
   * Ceres 2.0 Solver::Options defaults [C]. */
  o->max_num_iterations = 50;
  o->function_tolerance = 1e-6;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_relative_decrease = 1e-3;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
  o->elimination = OR_ELIM_CAPTURES;
  o->num_threads = 1;
  o->progress = 0;
  o->debug_indefinite_mask = 0;
  o->e_cap = NULL;
  o->e_tag = NULL;
}

/* ---------------------------------------------------------------------- */
/* Residual model                                                          */
/* ---------------------------------------------------------------------- */

/* ceres::AngleAxisRotatePoint [C rotation.h], operation order preserved. */
void or_angle_axis_rotate(const double w[3], const double pt[3], double out[3]) {
  const double theta2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (theta2 > DBL_EPSILON) {
    const double theta = sqrt(theta2);
    const double c = cos(theta), s = sin(theta);
    const double ti = 1.0 / theta;
    const double u[3] = {w[0] * ti, w[1] * ti, w[2] * ti};
    const double cr[3] = {u[1] * pt[2] - u[2] * pt[1], u[2] * pt[0] - u[0] * pt[2],
                          u[0] * pt[1] - u[1] * pt[0]};
    const double tmp = (u[0] * pt[0] + u[1] * pt[1] + u[2] * pt[2]) * (1.0 - c);
    out[0] = pt[0] * c + cr[0] * s + u[0] * tmp;
    out[1] = pt[1] * c + cr[1] * s + u[1] * tmp;
    out[2] = pt[2] * c + cr[2] * s + u[2] * tmp;
  } else {
    const double cr[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2],
                          w[0] * pt[1] - w[1] * pt[0]};
    out[0] = pt[0] + cr[0];
    out[1] = pt[1] + cr[1];
    out[2] = pt[2] + cr[2];
  }
}

/* projectCorner<double> [P:131-172]: tag corner -> world -> camera -> pixel. */
void or_project_corner(const double cam[3], const double cap[6], const double tag[6], int idx,
                       double out[2]) {
  const double corner[3] = {0.5 * kArucoSize * kDirs[idx][0], 0.5 * kArucoSize * kDirs[idx][1],
                            0.0};
  double ctx[3], cc[3];
  or_angle_axis_rotate(&tag[3], corner, ctx);
  ctx[0] += tag[0]; ctx[1] += tag[1]; ctx[2] += tag[2];   /* [P:146-148] */
  ctx[0] += cap[0]; ctx[1] += cap[1]; ctx[2] += cap[2];   /* [P:152-154] */
  or_angle_axis_rotate(&cap[3], ctx, cc);                 /* [P:155] */
  const double x = cc[0] / cc[2], y = cc[1] / cc[2];
  out[0] = cam[0] * x;
  out[1] = cam[0] * y;
}

/* ArucoReprojectionError::operator() [P:198-211] */
void or_residual(const double cam[3], const double cap[6], const double tag[6],
                 const double corners[8], double r[8]) {
  for (int i = 0; i < 4; ++i) {
    double pp[2];
    or_project_corner(cam, cap, tag, i, pp);
    r[2 * i] = pp[0] - corners[2 * i];
    r[2 * i + 1] = pp[1] - corners[2 * i + 1];
  }
}

/* Rotation M (the linear map rotate(w,.) applies) and the helper needed for
 * d rotate(w,x)/dw.  Normal branch: M = R(w), dR x/dw = -R [x]_x Jr(w).
 * Small branch (theta^2 <= eps, Ceres' first-order form x + w x x):
 * M = I + [w]_x, d/dw = -[x]_x. */
typedef struct {
  double M[9];
  double Jr[9];
  int small;
} rot_t;

static void rot_prepare(const double w[3], rot_t *R) {
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (th2 > DBL_EPSILON) {
    R->small = 0;
    const double th = sqrt(th2);
    const double c = cos(th), s = sin(th);
    const double u[3] = {w[0] / th, w[1] / th, w[2] / th};
    /* R = c I + s [u]_x + (1-c) u u^T */
    const double omc = 1.0 - c;
    R->M[0] = c + omc * u[0] * u[0];
    R->M[1] = -s * u[2] + omc * u[0] * u[1];
    R->M[2] = s * u[1] + omc * u[0] * u[2];
    R->M[3] = s * u[2] + omc * u[1] * u[0];
    R->M[4] = c + omc * u[1] * u[1];
    R->M[5] = -s * u[0] + omc * u[1] * u[2];
    R->M[6] = -s * u[1] + omc * u[2] * u[0];
    R->M[7] = s * u[0] + omc * u[2] * u[1];
    R->M[8] = c + omc * u[2] * u[2];
    /* Jr = I - a [w]_x + b [w]_x^2, a = (1-cos)/th^2, b = (th-sin)/th^3 */
    double a, b;
    if (th < 0.5) {
      /* alternating series, 7 terms each (truncation < 1e-16 relative) */
      double t = 1.0, fa = 2.0, fb = 6.0;
      a = 0.0; b = 0.0;
      for (int k = 0; k < 7; ++k) {
        a += t / fa;
        b += t / fb;
        t *= -th2;
        fa *= (double)(2 * k + 3) * (2 * k + 4);
        fb *= (double)(2 * k + 4) * (2 * k + 5);
      }
    } else {
      const double sh = sin(0.5 * th);
      a = 2.0 * sh * sh / th2;
      b = (th - s) / (th2 * th);
    }
    const double W[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double W2[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j)
        W2[3 * i + j] = W[3 * i] * W[j] + W[3 * i + 1] * W[3 + j] + W[3 * i + 2] * W[6 + j];
    for (int i = 0; i < 9; ++i) R->Jr[i] = (i % 4 == 0 ? 1.0 : 0.0) - a * W[i] + b * W2[i];
  } else {
    R->small = 1;
    const double M[9] = {1, -w[2], w[1], w[2], 1, -w[0], -w[1], w[0], 1};
    memcpy(R->M, M, sizeof(M));
    memset(R->Jr, 0, sizeof(R->Jr));
  }
}

/* D = d rotate(w, x) / dw  (3x3 row-major) */
static void rot_dx(const rot_t *R, const double x[3], double D[9]) {
  const double X[9] = {0, -x[2], x[1], x[2], 0, -x[0], -x[1], x[0], 0};
  if (R->small) {
    for (int i = 0; i < 9; ++i) D[i] = -X[i];
    return;
  }
  double T[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      T[3 * i + j] = R->M[3 * i] * X[j] + R->M[3 * i + 1] * X[3 + j] + R->M[3 * i + 2] * X[6 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      D[3 * i + j] = -(T[3 * i] * R->Jr[j] + T[3 * i + 1] * R->Jr[3 + j] + T[3 * i + 2] * R->Jr[6 + j]);
}

void or_residual_jacobian(const double cam[3], const double cap[6], const double tag[6],
                          const double corners[8], double r[8], double J[120]) {
  rot_t Rc, Rt;
  rot_prepare(&cap[3], &Rc);
  rot_prepare(&tag[3], &Rt);
  memset(J, 0, 120 * sizeof(double));
  for (int i = 0; i < 4; ++i) {
    const double corner[3] = {0.5 * kArucoSize * kDirs[i][0], 0.5 * kArucoSize * kDirs[i][1], 0.0};
    double a[3], p[3];
    or_angle_axis_rotate(&tag[3], corner, a);
    a[0] += tag[0]; a[1] += tag[1]; a[2] += tag[2];
    a[0] += cap[0]; a[1] += cap[1]; a[2] += cap[2];   /* a is now b = R_t c + t_t + t_c */
    or_angle_axis_rotate(&cap[3], a, p);
    const double x = p[0] / p[2], y = p[1] / p[2];
    r[2 * i] = cam[0] * x - corners[2 * i];
    r[2 * i + 1] = cam[0] * y - corners[2 * i + 1];
    /* P = (f/pz) [[1,0,-x],[0,1,-y]] */
    const double fz = cam[0] / p[2];
    const double P[6] = {fz, 0, -fz * x, 0, fz, -fz * y};
    double Dc[9], Dt[9], PM[6], PDc[6], PMDt[6];
    rot_dx(&Rc, a, Dc);
    rot_dx(&Rt, corner, Dt);
    for (int k = 0; k < 2; ++k)
      for (int j = 0; j < 3; ++j) {
        PM[3 * k + j] = P[3 * k] * Rc.M[j] + P[3 * k + 1] * Rc.M[3 + j] + P[3 * k + 2] * Rc.M[6 + j];
        PDc[3 * k + j] = P[3 * k] * Dc[j] + P[3 * k + 1] * Dc[3 + j] + P[3 * k + 2] * Dc[6 + j];
      }
    for (int k = 0; k < 2; ++k)
      for (int j = 0; j < 3; ++j)
        PMDt[3 * k + j] = PM[3 * k] * Dt[j] + PM[3 * k + 1] * Dt[3 + j] + PM[3 * k + 2] * Dt[6 + j];
    for (int k = 0; k < 2; ++k) {
      double *row = &J[(2 * i + k) * 15];
      row[0] = (k == 0) ? x : y;           /* d/df */
      /* row[1], row[2] = d/dl1, d/dl2 = 0 (distortion commented out [P:164-171]) */
      for (int j = 0; j < 3; ++j) {
        row[3 + j] = PM[3 * k + j];        /* d/dt_c */
        row[6 + j] = PDc[3 * k + j];       /* d/dw_c */
        row[9 + j] = PM[3 * k + j];        /* d/dt_t */
        row[12 + j] = PMDt[3 * k + j];     /* d/dw_t */
      }
    }
  }
}

/* ---------------------------------------------------------------------- */
/* Dense Cholesky (restates Eigen::LLT used by DenseSchurComplementSolver)  */
/* ---------------------------------------------------------------------- */

static double dot(const double *a, const double *b, long n) {
  double s = 0.0;
  for (long i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

int or_llt_lower(double *A, long n, long ld, int num_threads) {
  const long NB = 64;
  (void)num_threads;
  for (long k0 = 0; k0 < n; k0 += NB) {
    const long kb = (n - k0 < NB) ? n - k0 : NB;
    /* diagonal block, unblocked (pivots checked as Eigen's llt_inplace) */
    for (long j = k0; j < k0 + kb; ++j) {
      double *Aj = A + j * ld;
      double x = Aj[j] - dot(Aj + k0, Aj + k0, j - k0);
      if (!(x > 0.0)) return (int)(j + 1);
      const double d = sqrt(x);
      Aj[j] = d;
      for (long i = j + 1; i < k0 + kb; ++i) {
        double *Ai = A + i * ld;
        Ai[j] = (Ai[j] - dot(Ai + k0, Aj + k0, j - k0)) / d;
      }
    }
    /* panel below the diagonal block (TRSM) */
#pragma omp parallel for schedule(static) num_threads(num_threads > 0 ? num_threads : 1)
    for (long i = k0 + kb; i < n; ++i) {
      double *Ai = A + i * ld;
      for (long j = k0; j < k0 + kb; ++j) {
        const double *Aj = A + j * ld;
        Ai[j] = (Ai[j] - dot(Ai + k0, Aj + k0, j - k0)) / Aj[j];
      }
    }
    /* trailing update A[i][j] -= L[i][k0:k0+kb] . L[j][k0:k0+kb], j <= i */
#pragma omp parallel for schedule(dynamic, 16) num_threads(num_threads > 0 ? num_threads : 1)
    for (long i = k0 + kb; i < n; ++i) {
      double *Ai = A + i * ld;
      const double *Li = Ai + k0;
      for (long j = k0 + kb; j <= i; ++j) Ai[j] -= dot(Li, A + j * ld + k0, kb);
    }
  }
  return 0;
}

/* y = L^{-T} L^{-1} b, in place on b (row-major lower L) */
static void llt_solve(const double *L, long n, long ld, double *b) {
  for (long i = 0; i < n; ++i) b[i] = (b[i] - dot(L + i * ld, b, i)) / L[i * ld + i];
  for (long i = n - 1; i >= 0; --i) {
    const double yi = b[i] / L[i * ld + i];
    b[i] = yi;
    for (long k = 0; k < i; ++k) b[k] -= L[i * ld + k] * yi;
  }
}

/* 6x6 SPD inverse via LLT solve against the identity, as Ceres'
 * InvertPSDMatrix<kFullRank=true> [C schur_eliminator_impl.h]. */
static void inv6(const double U[36], double Ui[36]) {
  double L[36];
  memcpy(L, U, sizeof(L));
  for (int j = 0; j < 6; ++j) {
    double x = L[6 * j + j];
    for (int p = 0; p < j; ++p) x -= L[6 * j + p] * L[6 * j + p];
    const double d = sqrt(x);   /* no pivot test: NaN propagates as in Eigen */
    L[6 * j + j] = d;
    for (int i = j + 1; i < 6; ++i) {
      double v = L[6 * i + j];
      for (int p = 0; p < j; ++p) v -= L[6 * i + p] * L[6 * j + p];
      L[6 * i + j] = v / d;
    }
  }
  for (int c = 0; c < 6; ++c) {
    double e[6] = {0, 0, 0, 0, 0, 0};
    e[c] = 1.0;
    llt_solve(L, 6, 6, e);
    for (int i = 0; i < 6; ++i) Ui[6 * i + c] = e[i];
  }
}

/* ---------------------------------------------------------------------- */
/* LM / trust region                                                       */
/* ---------------------------------------------------------------------- */

typedef struct {
  const or_problem *p;
  const or_comm *comm;
  int nc, nt, nb;
  long n;             /* 3 + 6 nc + 6 nt parameter slots */
  long nF;            /* 6 nt + 3 reduced (f-side) size, camera last */
  int *cap_start;     /* CSR by capture */
  int *cap_obs;
  unsigned char *free_;   /* per parameter slot */
  unsigned char *obs_active;
  double *x, *xc;     /* current and candidate parameters (slot layout) */
  double *g, *colnorm, *scale, *diag;
  double *r;          /* residuals at x, [nb*8] */
  double *J;          /* Jacobian at x (unscaled), [nb*120] */
  double *S, *rhs;    /* reduced system (elim) or full system */
  double *y;          /* solution of (Jt'Jt + D^2) y = Jt' r */
  double *delta;
  int nthreads;
  int dbg_indefinite;   /* test hook for this linear solve (or_options.debug_indefinite_mask) */
  /* OR_ELIM_MIXED: the e-set, the reduced index of each slot (-1: an e-block's
   * slot), and the observations by tag */
  const unsigned char *e_cap, *e_tag;
  long *fidx;
  int *tag_start, *tag_obs;
} lm_t;

static inline long slot_cam(void) { return 0; }
static inline long slot_cap(const lm_t *L, int c) { (void)L; return 3 + 6L * c; }
static inline long slot_tag(const lm_t *L, int t) { return 3 + 6L * L->nc + 6L * t; }
static inline long fidx_tag(int t) { return 6L * t; }
static inline long fidx_cam(const lm_t *L) { return 6L * L->nt; }

static void unpack(const lm_t *L, const double *x, const double **cam, const double **cap,
                   const double **tag, int o) {
  *cam = x + slot_cam();
  *cap = x + slot_cap(L, L->p->obs_cap[o]);
  *tag = x + slot_tag(L, L->p->obs_tag[o]);
}

static void allreduce_sum(const lm_t *L, double *buf, long n) {
  if (L->comm && L->comm->allreduce_sum) L->comm->allreduce_sum(L->comm->ctx, buf, n);
}
static void allreduce_max(const lm_t *L, double *buf, long n) {
  if (L->comm && L->comm->allreduce_max) L->comm->allreduce_max(L->comm->ctx, buf, n);
}
static int is_root(const lm_t *L) { return !L->comm || L->comm->rank == 0; }

/* cost of active observations at x; *finite = 0 if any residual is not finite */
static double eval_cost(const lm_t *L, const double *x, int *finite, double *fixed_cost) {
  double cost = 0.0, fixed = 0.0;
  int ok = 1;
  for (int o = 0; o < L->nb; ++o) {
    const double *cam, *cap, *tag;
    unpack(L, x, &cam, &cap, &tag, o);
    double r[8];
    or_residual(cam, cap, tag, L->p->corners + 8L * o, r);
    double sq = 0.0;
    for (int i = 0; i < 8; ++i) {
      if (!isfinite(r[i])) ok = 0;
      sq += r[i] * r[i];
    }
    if (L->obs_active[o]) cost += 0.5 * sq; else fixed += 0.5 * sq;
  }
  double red[3] = {cost, fixed, ok ? 0.0 : 1.0};
  allreduce_sum(L, red, 2);
  allreduce_max(L, red + 2, 1);
  *finite = red[2] == 0.0;
  if (fixed_cost) *fixed_cost = red[1];
  return red[0];
}

/* residuals, Jacobian, cost, unscaled gradient and column norms at L->x */
static double evaluate_jacobian(lm_t *L, int *finite) {
  double cost = 0.0;
  int ok = 1;
  memset(L->g, 0, L->n * sizeof(double));
  memset(L->colnorm, 0, L->n * sizeof(double));
  for (int o = 0; o < L->nb; ++o) {
    const double *cam, *cap, *tag;
    unpack(L, L->x, &cam, &cap, &tag, o);
    double *r = L->r + 8L * o, *J = L->J + 120L * o;
    or_residual_jacobian(cam, cap, tag, L->p->corners + 8L * o, r, J);
    double sq = 0.0;
    for (int i = 0; i < 8; ++i) {
      if (!isfinite(r[i])) ok = 0;
      sq += r[i] * r[i];
    }
    if (!L->obs_active[o]) continue;
    cost += 0.5 * sq;
    const long base[3] = {slot_cam(), slot_cap(L, L->p->obs_cap[o]), slot_tag(L, L->p->obs_tag[o])};
    const int off[3] = {0, 3, 9}, len[3] = {3, 6, 6};
    for (int b = 0; b < 3; ++b)
      for (int j = 0; j < len[b]; ++j) {
        const long s = base[b] + j;
        if (!L->free_[s]) continue;
        double gs = 0.0, cs = 0.0;
        for (int i = 0; i < 8; ++i) {
          const double v = J[15 * i + off[b] + j];
          gs += v * r[i];
          cs += v * v;
        }
        L->g[s] += gs;
        L->colnorm[s] += cs;
      }
  }
  /* tag + camera slots are shared across ranks; capture slots are local */
  const long shared0 = slot_tag(L, 0);
  allreduce_sum(L, L->g + shared0, L->n - shared0);
  allreduce_sum(L, L->g, 3);
  allreduce_sum(L, L->colnorm + shared0, L->n - shared0);
  allreduce_sum(L, L->colnorm, 3);
  double red[2] = {cost, ok ? 0.0 : 1.0};
  allreduce_sum(L, red, 1);
  allreduce_max(L, red + 1, 1);
  *finite = red[1] == 0.0;
  return red[0];
}

static void grad_norms(const lm_t *L, double *gmax, double *gnorm) {
  double mx = 0.0, sq = 0.0;
  const long shared0 = slot_tag(L, 0);
  for (long s = 0; s < L->n; ++s) {
    if (!L->free_[s]) continue;
    const double a = fabs(L->g[s]);
    if (a > mx) mx = a;
    const int shared = (s < 3) || (s >= shared0);
    if (!shared || is_root(L)) sq += L->g[s] * L->g[s];
  }
  allreduce_max(L, &mx, 1);
  allreduce_sum(L, &sq, 1);
  *gmax = mx;
  *gnorm = sqrt(sq);
}

static double norm_free(const lm_t *L, const double *v) {
  double sq = 0.0;
  const long shared0 = slot_tag(L, 0);
  for (long s = 0; s < L->n; ++s) {
    if (!L->free_[s]) continue;
    const int shared = (s < 3) || (s >= shared0);
    if (!shared || is_root(L)) sq += v[s] * v[s];
  }
  allreduce_sum(L, &sq, 1);
  return sqrt(sq);
}

/* Scaled Jacobian row (15 cols) of observation o, row i. */
static inline void scaled_row(const lm_t *L, int o, int i, double out[15]) {
  const double *J = L->J + 120L * o + 15 * i;
  const long base[3] = {slot_cam(), slot_cap(L, L->p->obs_cap[o]), slot_tag(L, L->p->obs_tag[o])};
  const int off[3] = {0, 3, 9}, len[3] = {3, 6, 6};
  for (int b = 0; b < 3; ++b)
    for (int j = 0; j < len[b]; ++j) out[off[b] + j] = J[off[b] + j] * L->scale[base[b] + j];
}

/* DENSE_SCHUR linear solve with captures as e-blocks.  Returns 0 ok, 1 on
 * Cholesky failure of the reduced system. Writes L->y. */
static int solve_schur(lm_t *L, const double *D2) {
  const long nF = L->nF, ld = nF;
  memset(L->S, 0, (size_t)nF * nF * sizeof(double));
  memset(L->rhs, 0, nF * sizeof(double));
  int maxk = 0;
  for (int c = 0; c < L->nc; ++c) {
    const int k = L->cap_start[c + 1] - L->cap_start[c];
    if (k > maxk) maxk = k;
  }
  const int mmax = 3 + 6 * maxk;
  double *W = malloc(sizeof(double) * 6 * mmax);
  double *FtF = malloc(sizeof(double) * mmax * mmax);
  double *Ftr = malloc(sizeof(double) * mmax);
  double *Z = malloc(sizeof(double) * 6 * mmax);
  long *gidx = malloc(sizeof(long) * mmax);
  int *lblk = malloc(sizeof(int) * (maxk + 1));
  int *btag = malloc(sizeof(int) * (maxk + 1));

  for (int c = 0; c < L->nc; ++c) {
    const int o0 = L->cap_start[c], o1 = L->cap_start[c + 1];
    const int k = o1 - o0;
    if (k == 0) continue;
    /* local f-blocks: 0 = camera (3 cols), then distinct tags (6 cols) */
    int nblk = 1;
    for (int q = 0; q < k; ++q) {
      const int o = L->cap_obs[o0 + q];
      const int t = L->p->obs_tag[o];
      int b = -1;
      for (int u = 1; u < nblk; ++u)
        if (btag[u] == t) { b = u; break; }
      if (b < 0) { b = nblk++; btag[b] = t; }
      lblk[q] = b;
    }
    const int m = 3 + 6 * (nblk - 1);
    for (int j = 0; j < 3; ++j) gidx[j] = fidx_cam(L) + j;
    for (int u = 1; u < nblk; ++u)
      for (int j = 0; j < 6; ++j) gidx[3 + 6 * (u - 1) + j] = fidx_tag(btag[u]) + j;

    double U[36] = {0}, Etr[6] = {0};
    memset(W, 0, sizeof(double) * 6 * m);
    memset(FtF, 0, sizeof(double) * m * m);
    memset(Ftr, 0, sizeof(double) * m);
    for (int q = 0; q < k; ++q) {
      const int o = L->cap_obs[o0 + q];
      const double *r = L->r + 8L * o;
      const int fo = 3 + 6 * (lblk[q] - 1);
      for (int i = 0; i < 8; ++i) {
        double row[15];
        scaled_row(L, o, i, row);
        const double *E = row + 3;
        /* F columns of this row: camera (local 0..2), tag (local fo..fo+5) */
        double Fv[9];
        long fl[9];
        for (int j = 0; j < 3; ++j) { Fv[j] = row[j]; fl[j] = j; }
        for (int j = 0; j < 6; ++j) { Fv[3 + j] = row[9 + j]; fl[3 + j] = fo + j; }
        for (int a = 0; a < 6; ++a) {
          Etr[a] += E[a] * r[i];
          for (int b = 0; b < 6; ++b) U[6 * a + b] += E[a] * E[b];
          for (int j = 0; j < 9; ++j) W[a * m + fl[j]] += E[a] * Fv[j];
        }
        for (int j = 0; j < 9; ++j) {
          Ftr[fl[j]] += Fv[j] * r[i];
          for (int jj = 0; jj < 9; ++jj) FtF[fl[j] * m + fl[jj]] += Fv[j] * Fv[jj];
        }
      }
    }
    const long sc = slot_cap(L, c);
    for (int a = 0; a < 6; ++a) U[6 * a + a] += D2[sc + a];
    double Ui[36];
    inv6(U, Ui);
    /* Z = Ui W ; S_c = FtF - W^T Z ; rhs_c = Ftr - W^T (Ui Etr) */
    for (int a = 0; a < 6; ++a)
      for (int j = 0; j < m; ++j) {
        double s = 0.0;
        for (int b = 0; b < 6; ++b) s += Ui[6 * a + b] * W[b * m + j];
        Z[a * m + j] = s;
      }
    double UiE[6];
    for (int a = 0; a < 6; ++a) {
      double s = 0.0;
      for (int b = 0; b < 6; ++b) s += Ui[6 * a + b] * Etr[b];
      UiE[a] = s;
    }
    for (int i = 0; i < m; ++i) {
      double s = 0.0;
      for (int a = 0; a < 6; ++a) s += W[a * m + i] * UiE[a];
      L->rhs[gidx[i]] += Ftr[i] - s;
      for (int j = 0; j < m; ++j) {
        const long gi = gidx[i], gj = gidx[j];
        if (gj > gi) continue;   /* lower triangle only */
        double t = 0.0;
        for (int a = 0; a < 6; ++a) t += W[a * m + i] * Z[a * m + j];
        L->S[gi * ld + gj] += FtF[i * m + j] - t;
      }
    }
  }
  free(W); free(FtF); free(Ftr); free(Z); free(gidx); free(lblk); free(btag);

  allreduce_sum(L, L->S, nF * nF);
  allreduce_sum(L, L->rhs, nF);
  /* S += D_f^2 */
  for (int t = 0; t < L->nt; ++t)
    for (int j = 0; j < 6; ++j) L->S[(fidx_tag(t) + j) * (ld + 1)] += D2[slot_tag(L, t) + j];
  for (int j = 0; j < 3; ++j) L->S[(fidx_cam(L) + j) * (ld + 1)] += D2[slot_cam() + j];
  if (L->dbg_indefinite) L->S[fidx_cam(L) * (ld + 1)] = -1.0;   /* test hook */

  if (or_llt_lower(L->S, nF, ld, L->nthreads) != 0) return 1;
  double *yF = malloc(sizeof(double) * nF);
  memcpy(yF, L->rhs, nF * sizeof(double));
  llt_solve(L->S, nF, ld, yF);
  for (int t = 0; t < L->nt; ++t)
    for (int j = 0; j < 6; ++j) L->y[slot_tag(L, t) + j] = yF[fidx_tag(t) + j];
  for (int j = 0; j < 3; ++j) L->y[slot_cam() + j] = yF[fidx_cam(L) + j];

  /* back substitution: y_c = (E'E + D^2)^{-1} E'(r - F y_F) */
  for (int c = 0; c < L->nc; ++c) {
    const int o0 = L->cap_start[c], o1 = L->cap_start[c + 1];
    const long sc = slot_cap(L, c);
    if (o1 == o0) { for (int a = 0; a < 6; ++a) L->y[sc + a] = 0.0; continue; }
    double U[36] = {0}, v[6] = {0};
    for (int q = o0; q < o1; ++q) {
      const int o = L->cap_obs[q];
      const double *r = L->r + 8L * o;
      const long st = slot_tag(L, L->p->obs_tag[o]);
      for (int i = 0; i < 8; ++i) {
        double row[15];
        scaled_row(L, o, i, row);
        double fz = 0.0;
        for (int j = 0; j < 3; ++j) fz += row[j] * L->y[slot_cam() + j];
        for (int j = 0; j < 6; ++j) fz += row[9 + j] * L->y[st + j];
        const double sj = r[i] - fz;
        for (int a = 0; a < 6; ++a) {
          v[a] += row[3 + a] * sj;
          for (int b = 0; b < 6; ++b) U[6 * a + b] += row[3 + a] * row[3 + b];
        }
      }
    }
    for (int a = 0; a < 6; ++a) U[6 * a + a] += D2[sc + a];
    double Ui[36];
    inv6(U, Ui);
    for (int a = 0; a < 6; ++a) {
      double s = 0.0;
      for (int b = 0; b < 6; ++b) s += Ui[6 * a + b] * v[b];
      L->y[sc + a] = s;
    }
  }
  free(yF);
  return 0;
}

/* DENSE_SCHUR over an arbitrary independent e-block set (OR_ELIM_MIXED): the
 * set Ceres 2.0 itself takes with no linear_solver_ordering ([P:1011];
 * ReorderProgramForSchurTypeLinearSolver -> ComputeStableSchurOrdering [C]),
 * which mixes captures and tags.  Each e-block (an eliminated capture or tag)
 * is eliminated from its own residuals exactly as in solve_schur, with the
 * other pose block of each residual on the reduced side; residuals touching
 * no e-block add their normal-equation blocks to the reduced system directly
 * (SchurEliminator's rows without an e-block [C schur_eliminator_impl.h
 * NoEBlockRowsUpdate]).  Reduced rows: every non-e capture and tag (L->fidx),
 * the camera last.  Returns 0 ok, 1 on Cholesky failure; writes L->y. */
static int solve_schur_mixed(lm_t *L, const double *D2) {
  const long nF = L->nF, ld = nF;
  memset(L->S, 0, (size_t)nF * nF * sizeof(double));
  memset(L->rhs, 0, nF * sizeof(double));
  int maxk = 0;
  for (int c = 0; c < L->nc; ++c)
    if (L->e_cap[c] && L->cap_start[c + 1] - L->cap_start[c] > maxk) maxk = L->cap_start[c + 1] - L->cap_start[c];
  for (int t = 0; t < L->nt; ++t)
    if (L->e_tag[t] && L->tag_start[t + 1] - L->tag_start[t] > maxk) maxk = L->tag_start[t + 1] - L->tag_start[t];
  const int mmax = 3 + 6 * maxk;
  double *W = malloc(sizeof(double) * 6 * mmax);
  double *FtF = malloc(sizeof(double) * mmax * mmax);
  double *Ftr = malloc(sizeof(double) * mmax);
  double *Z = malloc(sizeof(double) * 6 * mmax);
  long *gidx = malloc(sizeof(long) * mmax);
  int *lblk = malloc(sizeof(int) * (maxk + 1));
  long *bslot = malloc(sizeof(long) * (maxk + 1));
  const int n_eb = L->nc + L->nt;
  /* e-block eb < nc: capture eb; else tag eb - nc.  eoff / foff: its own and
   * the other pose's columns in the 15-column Jacobian row */
  for (int eb = 0; eb < n_eb; ++eb) {
    const int is_cap = eb < L->nc, id = is_cap ? eb : eb - L->nc;
    if (is_cap ? !L->e_cap[id] : !L->e_tag[id]) continue;
    const int *olist = is_cap ? L->cap_obs + L->cap_start[id] : L->tag_obs + L->tag_start[id];
    const int k = is_cap ? L->cap_start[id + 1] - L->cap_start[id] : L->tag_start[id + 1] - L->tag_start[id];
    const long se = is_cap ? slot_cap(L, id) : slot_tag(L, id);
    const int eoff = is_cap ? 3 : 9, foff = is_cap ? 9 : 3;
    if (k == 0) continue;
    int nblk = 1;
    for (int q = 0; q < k; ++q) {
      const int o = olist[q];
      const long sf = is_cap ? slot_tag(L, L->p->obs_tag[o]) : slot_cap(L, L->p->obs_cap[o]);
      int b = -1;
      for (int u = 1; u < nblk; ++u)
        if (bslot[u] == sf) { b = u; break; }
      if (b < 0) { b = nblk++; bslot[b] = sf; }
      lblk[q] = b;
    }
    const int m = 3 + 6 * (nblk - 1);
    for (int j = 0; j < 3; ++j) gidx[j] = L->fidx[slot_cam() + j];
    for (int u = 1; u < nblk; ++u)
      for (int j = 0; j < 6; ++j) gidx[3 + 6 * (u - 1) + j] = L->fidx[bslot[u] + j];
    double U[36] = {0}, Etr[6] = {0};
    memset(W, 0, sizeof(double) * 6 * m);
    memset(FtF, 0, sizeof(double) * m * m);
    memset(Ftr, 0, sizeof(double) * m);
    for (int q = 0; q < k; ++q) {
      const int o = olist[q];
      const double *r = L->r + 8L * o;
      const int fo = 3 + 6 * (lblk[q] - 1);
      for (int i = 0; i < 8; ++i) {
        double row[15];
        scaled_row(L, o, i, row);
        const double *E = row + eoff;
        double Fv[9];
        long fl[9];
        for (int j = 0; j < 3; ++j) { Fv[j] = row[j]; fl[j] = j; }
        for (int j = 0; j < 6; ++j) { Fv[3 + j] = row[foff + j]; fl[3 + j] = fo + j; }
        for (int a = 0; a < 6; ++a) {
          Etr[a] += E[a] * r[i];
          for (int b = 0; b < 6; ++b) U[6 * a + b] += E[a] * E[b];
          for (int j = 0; j < 9; ++j) W[a * m + fl[j]] += E[a] * Fv[j];
        }
        for (int j = 0; j < 9; ++j) {
          Ftr[fl[j]] += Fv[j] * r[i];
          for (int jj = 0; jj < 9; ++jj) FtF[fl[j] * m + fl[jj]] += Fv[j] * Fv[jj];
        }
      }
    }
    for (int a = 0; a < 6; ++a) U[6 * a + a] += D2[se + a];
    double Ui[36];
    inv6(U, Ui);
    for (int a = 0; a < 6; ++a)
      for (int j = 0; j < m; ++j) {
        double s = 0.0;
        for (int b = 0; b < 6; ++b) s += Ui[6 * a + b] * W[b * m + j];
        Z[a * m + j] = s;
      }
    double UiE[6];
    for (int a = 0; a < 6; ++a) {
      double s = 0.0;
      for (int b = 0; b < 6; ++b) s += Ui[6 * a + b] * Etr[b];
      UiE[a] = s;
    }
    for (int i = 0; i < m; ++i) {
      double s = 0.0;
      for (int a = 0; a < 6; ++a) s += W[a * m + i] * UiE[a];
      L->rhs[gidx[i]] += Ftr[i] - s;
      for (int j = 0; j < m; ++j) {
        const long gi = gidx[i], gj = gidx[j];
        if (gj > gi) continue;
        double t = 0.0;
        for (int a = 0; a < 6; ++a) t += W[a * m + i] * Z[a * m + j];
        L->S[gi * ld + gj] += FtF[i * m + j] - t;
      }
    }
  }
  /* residuals with no e-block: their J'J and J'r straight into the reduced system */
  for (int o = 0; o < L->nb; ++o) {
    if (L->e_cap[L->p->obs_cap[o]] || L->e_tag[L->p->obs_tag[o]]) continue;
    const long base[3] = {slot_cam(), slot_cap(L, L->p->obs_cap[o]), slot_tag(L, L->p->obs_tag[o])};
    long gi[15];
    for (int j = 0; j < 3; ++j) gi[j] = L->fidx[base[0] + j];
    for (int j = 0; j < 6; ++j) { gi[3 + j] = L->fidx[base[1] + j]; gi[9 + j] = L->fidx[base[2] + j]; }
    for (int i = 0; i < 8; ++i) {
      double row[15];
      scaled_row(L, o, i, row);
      for (int a = 0; a < 15; ++a) {
        L->rhs[gi[a]] += row[a] * L->r[8L * o + i];
        for (int b = 0; b < 15; ++b)
          if (gi[b] <= gi[a]) L->S[gi[a] * ld + gi[b]] += row[a] * row[b];
      }
    }
  }
  free(W); free(FtF); free(Ftr); free(Z); free(gidx); free(lblk); free(bslot);
  for (long sl = 0; sl < L->n; ++sl)
    if (L->fidx[sl] >= 0) L->S[L->fidx[sl] * (ld + 1)] += D2[sl];
  if (L->dbg_indefinite) L->S[L->fidx[slot_cam()] * (ld + 1)] = -1.0;   /* test hook */
  if (or_llt_lower(L->S, nF, ld, L->nthreads) != 0) return 1;
  double *yF = malloc(sizeof(double) * nF);
  memcpy(yF, L->rhs, nF * sizeof(double));
  llt_solve(L->S, nF, ld, yF);
  for (long sl = 0; sl < L->n; ++sl)
    if (L->fidx[sl] >= 0) L->y[sl] = yF[L->fidx[sl]];
  /* back substitution per e-block: y_e = (E'E + D^2)^{-1} E'(r - F y_F) */
  for (int eb = 0; eb < n_eb; ++eb) {
    const int is_cap = eb < L->nc, id = is_cap ? eb : eb - L->nc;
    if (is_cap ? !L->e_cap[id] : !L->e_tag[id]) continue;
    const int *olist = is_cap ? L->cap_obs + L->cap_start[id] : L->tag_obs + L->tag_start[id];
    const int k = is_cap ? L->cap_start[id + 1] - L->cap_start[id] : L->tag_start[id + 1] - L->tag_start[id];
    const long se = is_cap ? slot_cap(L, id) : slot_tag(L, id);
    const int eoff = is_cap ? 3 : 9, foff = is_cap ? 9 : 3;
    if (k == 0) { for (int a = 0; a < 6; ++a) L->y[se + a] = 0.0; continue; }
    double U[36] = {0}, v[6] = {0};
    for (int q = 0; q < k; ++q) {
      const int o = olist[q];
      const double *r = L->r + 8L * o;
      const long sf = is_cap ? slot_tag(L, L->p->obs_tag[o]) : slot_cap(L, L->p->obs_cap[o]);
      for (int i = 0; i < 8; ++i) {
        double row[15];
        scaled_row(L, o, i, row);
        double fz = 0.0;
        for (int j = 0; j < 3; ++j) fz += row[j] * L->y[slot_cam() + j];
        for (int j = 0; j < 6; ++j) fz += row[foff + j] * L->y[sf + j];
        const double sj = r[i] - fz;
        for (int a = 0; a < 6; ++a) {
          v[a] += row[eoff + a] * sj;
          for (int b = 0; b < 6; ++b) U[6 * a + b] += row[eoff + a] * row[eoff + b];
        }
      }
    }
    for (int a = 0; a < 6; ++a) U[6 * a + a] += D2[se + a];
    double Ui[36];
    inv6(U, Ui);
    for (int a = 0; a < 6; ++a) {
      double s = 0.0;
      for (int b = 0; b < 6; ++b) s += Ui[6 * a + b] * v[b];
      L->y[se + a] = s;
    }
  }
  free(yF);
  return 0;
}

/* DENSE_QR-free reference: full normal equations over every slot. */
static int solve_full(lm_t *L, const double *D2) {
  const long n = L->n;
  memset(L->S, 0, (size_t)n * n * sizeof(double));
  memset(L->rhs, 0, n * sizeof(double));
  for (int o = 0; o < L->nb; ++o) {
    if (!L->obs_active[o]) continue;
    const long base[3] = {slot_cam(), slot_cap(L, L->p->obs_cap[o]), slot_tag(L, L->p->obs_tag[o])};
    long gi[15];
    for (int j = 0; j < 3; ++j) gi[j] = base[0] + j;
    for (int j = 0; j < 6; ++j) { gi[3 + j] = base[1] + j; gi[9 + j] = base[2] + j; }
    for (int i = 0; i < 8; ++i) {
      double row[15];
      scaled_row(L, o, i, row);
      for (int a = 0; a < 15; ++a) {
        L->rhs[gi[a]] += row[a] * L->r[8L * o + i];
        for (int b = 0; b < 15; ++b)
          if (gi[b] <= gi[a]) L->S[gi[a] * n + gi[b]] += row[a] * row[b];
      }
    }
  }
  for (long s = 0; s < n; ++s) L->S[s * (n + 1)] += D2[s];
  if (L->dbg_indefinite) L->S[slot_cam() * (n + 1)] = -1.0;   /* test hook */
  if (or_llt_lower(L->S, n, n, L->nthreads) != 0) return 1;
  memcpy(L->y, L->rhs, n * sizeof(double));
  llt_solve(L->S, n, n, L->y);
  return 0;
}

static void print_header(void) {
  printf("iter      cost      cost_change  |gradient|   |step|    tr_ratio  tr_radius  ls_iter  iter_time  total_time\n");
}
static void print_row(const or_iter *it) {
  printf("% 4d % 8e   % 3.2e   % 3.2e  % 3.2e  % 3.2e % 3.2e     % 4d   % 3.2e   % 3.2e\n",
         it->iteration, it->cost, it->cost_change, it->gradient_max_norm, it->step_norm,
         it->relative_decrease, it->trust_region_radius, 0, it->iteration_time,
         it->cumulative_time);
  fflush(stdout);
}

int or_solve(or_problem *p, const or_options *o, or_summary *s, const or_comm *comm) {
  const double t_start = now_s();
  lm_t L;
  memset(&L, 0, sizeof(L));
  memset(s, 0, sizeof(*s));
  L.p = p;
  L.comm = comm;
  L.nthreads = o->num_threads;
  L.nc = p->n_cap; L.nt = p->n_tag; L.nb = p->n_obs;
  L.n = 3 + 6L * L.nc + 6L * L.nt;
  L.nF = 6L * L.nt + 3;
  const int mixed = o->elimination == OR_ELIM_MIXED;
  if (mixed) {
    if (comm || !o->e_cap || !o->e_tag) return -1;   /* single process, both sets given */
    L.e_cap = o->e_cap;
    L.e_tag = o->e_tag;
    for (int b = 0; b < L.nb; ++b)
      if (L.e_cap[p->obs_cap[b]] && L.e_tag[p->obs_tag[b]]) return -1;   /* not an independent set */
    /* reduced rows: the non-e captures, then the non-e tags, then the camera */
    L.fidx = malloc(sizeof(long) * L.n);
    long f = 0;
    for (int c = 0; c < L.nc; ++c)
      for (int j = 0; j < 6; ++j) L.fidx[3 + 6L * c + j] = L.e_cap[c] ? -1 : f++;
    for (int t = 0; t < L.nt; ++t)
      for (int j = 0; j < 6; ++j) L.fidx[3 + 6L * L.nc + 6L * t + j] = L.e_tag[t] ? -1 : f++;
    for (int j = 0; j < 3; ++j) L.fidx[j] = f++;
    L.nF = f;
    /* observations by tag (stable) */
    L.tag_start = calloc(L.nt + 1, sizeof(int));
    L.tag_obs = malloc(sizeof(int) * (L.nb > 0 ? L.nb : 1));
    for (int b = 0; b < L.nb; ++b) L.tag_start[p->obs_tag[b] + 1]++;
    for (int t = 0; t < L.nt; ++t) L.tag_start[t + 1] += L.tag_start[t];
    int *fill = malloc(sizeof(int) * (L.nt + 1));
    memcpy(fill, L.tag_start, sizeof(int) * (L.nt + 1));
    for (int b = 0; b < L.nb; ++b) L.tag_obs[fill[p->obs_tag[b]]++] = b;
    free(fill);
  }

  /* CSR by capture (stable) */
  L.cap_start = calloc(L.nc + 1, sizeof(int));
  L.cap_obs = malloc(sizeof(int) * (L.nb > 0 ? L.nb : 1));
  for (int b = 0; b < L.nb; ++b) L.cap_start[p->obs_cap[b] + 1]++;
  for (int c = 0; c < L.nc; ++c) L.cap_start[c + 1] += L.cap_start[c];
  {
    int *fill = malloc(sizeof(int) * (L.nc + 1));
    memcpy(fill, L.cap_start, sizeof(int) * (L.nc + 1));
    for (int b = 0; b < L.nb; ++b) L.cap_obs[fill[p->obs_cap[b]]++] = b;
    free(fill);
  }
  /* free slots: a block is a parameter iff it appears in a residual and is
   * not held constant (Ceres drops unused and constant blocks). */
  L.free_ = calloc(L.n, 1);
  L.obs_active = calloc(L.nb > 0 ? L.nb : 1, 1);
  {
    int *deg_t = calloc(L.nt > 0 ? L.nt : 1, sizeof(int));
    for (int b = 0; b < L.nb; ++b) deg_t[p->obs_tag[b]]++;
    /* tag usage is global: a shard may see a tag only through other ranks */
    double *dt = malloc(sizeof(double) * (L.nt > 0 ? L.nt : 1));
    for (int t = 0; t < L.nt; ++t) dt[t] = deg_t[t];
    double nb_all = L.nb;
    allreduce_sum(&L, dt, L.nt);
    allreduce_sum(&L, &nb_all, 1);
    const int cam_free = !p->camera_const && nb_all > 0;
    for (int j = 0; j < 3; ++j) L.free_[j] = (unsigned char)cam_free;
    for (int c = 0; c < L.nc; ++c) {
      const int f = (L.cap_start[c + 1] > L.cap_start[c]) && !(p->cap_const && p->cap_const[c]);
      for (int j = 0; j < 6; ++j) L.free_[slot_cap(&L, c) + j] = (unsigned char)f;
    }
    for (int t = 0; t < L.nt; ++t) {
      const int f = dt[t] > 0 && !(p->tag_const && p->tag_const[t]);
      for (int j = 0; j < 6; ++j) L.free_[slot_tag(&L, t) + j] = (unsigned char)f;
    }
    for (int b = 0; b < L.nb; ++b)
      L.obs_active[b] = (unsigned char)(L.free_[0] || L.free_[slot_cap(&L, p->obs_cap[b])] ||
                                        L.free_[slot_tag(&L, p->obs_tag[b])]);
    free(deg_t);
    free(dt);
  }

  L.x = malloc(sizeof(double) * L.n);
  L.xc = malloc(sizeof(double) * L.n);
  L.g = calloc(L.n, sizeof(double));
  L.colnorm = calloc(L.n, sizeof(double));
  L.scale = calloc(L.n, sizeof(double));
  L.diag = calloc(L.n, sizeof(double));
  L.y = calloc(L.n, sizeof(double));
  L.delta = calloc(L.n, sizeof(double));
  double *D2 = calloc(L.n, sizeof(double));
  L.r = malloc(sizeof(double) * 8 * (L.nb > 0 ? L.nb : 1));
  L.J = malloc(sizeof(double) * 120 * (L.nb > 0 ? L.nb : 1));
  const long nsys = (o->elimination == OR_ELIM_NONE) ? L.n : L.nF;
  L.S = malloc(sizeof(double) * nsys * nsys);
  L.rhs = malloc(sizeof(double) * nsys);

  memcpy(L.x, p->camera, 3 * sizeof(double));
  memcpy(L.x + 3, p->cap, 6L * L.nc * sizeof(double));
  memcpy(L.x + slot_tag(&L, 0), p->tag, 6L * L.nt * sizeof(double));

  if (o->progress) print_header();

  /* ---- iteration 0 [C trust_region_minimizer.cc IterationZero] ---- */
  double x_norm = norm_free(&L, L.x);
  int finite = 1;
  double x_cost = evaluate_jacobian(&L, &finite);
  {
    int ok = 1;
    (void)eval_cost(&L, L.x, &ok, &s->fixed_cost);
  }
  s->initial_cost = x_cost + s->fixed_cost;
  if (!finite) {
    s->termination = OR_FAILURE;
    s->rule = OR_RULE_EVAL_FAILED;
    s->final_cost = s->initial_cost;
    goto done;
  }
  for (long k = 0; k < L.n; ++k)
    L.scale[k] = L.free_[k] ? (o->jacobi_scaling ? 1.0 / (1.0 + sqrt(L.colnorm[k])) : 1.0) : 0.0;

  double radius = o->initial_trust_region_radius, decrease_factor = 2.0;
  int reuse_diag = 0, n_invalid = 0;
  double minimum_cost = x_cost;
  or_iter it;
  memset(&it, 0, sizeof(it));
  it.iteration = 0;
  it.cost = x_cost + s->fixed_cost;
  grad_norms(&L, &it.gradient_max_norm, &it.gradient_norm);
  it.step_is_valid = 1;
  it.step_is_successful = 1;
  it.trust_region_radius = radius;
  double t_iter = t_start;

  for (;;) {
    /* ---- FinalizeIterationAndCheckIfMinimizerCanContinue ---- */
    if (it.step_is_successful) {
      s->num_successful_steps += (it.iteration > 0);
      if (x_cost < minimum_cost || it.iteration == 0) {
        minimum_cost = x_cost;
        memcpy(p->camera, L.x, 3 * sizeof(double));
        memcpy(p->cap, L.x + 3, 6L * L.nc * sizeof(double));
        memcpy(p->tag, L.x + slot_tag(&L, 0), 6L * L.nt * sizeof(double));
      }
    } else {
      s->num_unsuccessful_steps++;
    }
    it.trust_region_radius = radius;
    const double tn = now_s();
    it.iteration_time = tn - t_iter;
    it.cumulative_time = tn - t_start;
    t_iter = tn;
    if (s->n_iters <= OR_MAX_ITERS) s->iters[s->n_iters++] = it;
    if (o->progress && is_root(&L)) print_row(&it);
    if (it.iteration >= o->max_num_iterations) {
      s->termination = OR_NO_CONVERGENCE; s->rule = OR_RULE_MAX_ITERS; break;
    }
    if (it.step_is_successful && it.gradient_max_norm <= o->gradient_tolerance) {
      s->termination = OR_CONVERGENCE; s->rule = OR_RULE_GRADIENT; break;
    }
    if (radius <= o->min_trust_region_radius) {
      s->termination = OR_CONVERGENCE; s->rule = OR_RULE_MIN_RADIUS; break;
    }

    const double prev_gmax = it.gradient_max_norm, prev_gnorm = it.gradient_norm;
    memset(&it, 0, sizeof(it));
    it.iteration = s->iters[s->n_iters - 1].iteration + 1;

    /* ---- ComputeTrustRegionStep [C] + LevenbergMarquardtStrategy ---- */
    if (!reuse_diag) {
      for (long k = 0; k < L.n; ++k) {
        double d = L.scale[k] * L.scale[k] * L.colnorm[k];
        if (d < o->min_lm_diagonal) d = o->min_lm_diagonal;
        if (d > o->max_lm_diagonal) d = o->max_lm_diagonal;
        L.diag[k] = d;
      }
    }
    for (long k = 0; k < L.n; ++k) {
      const double dk = sqrt(L.diag[k] / radius);
      D2[k] = dk * dk;
    }
    s->num_linear_solves++;
    L.dbg_indefinite = (int)((o->debug_indefinite_mask >> (s->num_linear_solves - 1 < 63 ? s->num_linear_solves - 1 : 63)) & 1ull);
    int lin_fail = (o->elimination == OR_ELIM_NONE) ? solve_full(&L, D2)
                   : mixed ? solve_schur_mixed(&L, D2) : solve_schur(&L, D2);
    reuse_diag = 1;
    double model_cost_change = 0.0;
    int valid = 0;
    if (!lin_fail) {
      double bad = 0.0;
      for (long k = 0; k < L.n; ++k)
        if (!isfinite(L.y[k])) bad = 1.0;
      allreduce_max(&L, &bad, 1);
      if (bad == 0.0) {
        /* step = -y ; model_residuals = Jt step ; m = -mr.(r + mr/2) */
        for (long k = 0; k < L.n; ++k) L.delta[k] = -L.y[k];
        double mcc = 0.0;
        for (int ob = 0; ob < L.nb; ++ob) {
          if (!L.obs_active[ob]) continue;
          const long base[3] = {slot_cam(), slot_cap(&L, p->obs_cap[ob]), slot_tag(&L, p->obs_tag[ob])};
          for (int i = 0; i < 8; ++i) {
            double row[15];
            scaled_row(&L, ob, i, row);
            double mr = 0.0;
            for (int j = 0; j < 3; ++j) mr += row[j] * L.delta[base[0] + j];
            for (int j = 0; j < 6; ++j) mr += row[3 + j] * L.delta[base[1] + j];
            for (int j = 0; j < 6; ++j) mr += row[9 + j] * L.delta[base[2] + j];
            mcc += mr * (L.r[8L * ob + i] + mr / 2.0);
          }
        }
        allreduce_sum(&L, &mcc, 1);
        model_cost_change = -mcc;
        valid = model_cost_change > 0.0;
        if (valid)
          for (long k = 0; k < L.n; ++k) L.delta[k] = L.delta[k] * L.scale[k];
      }
    }
    if (!valid) {
      /* Ceres 2.0 TrustRegionMinimizer::HandleInvalidStep (trust_region_minimizer.cc):
       *   if (++num_consecutive_invalid_steps_ >= options_.max_num_consecutive_invalid_steps)
       *     { termination_type = FAILURE; return false; }
       * i.e. the 5th consecutive invalid step (default 5) ends the solve, unrecorded
       * (its message reads "more than", the test is >=).  Restated from the upstream
       * source as recalled (Ceres is not in this image); round 2 had `>` here. */
      if (++n_invalid >= o->max_num_consecutive_invalid_steps) {
        s->termination = OR_FAILURE; s->rule = OR_RULE_INVALID_STEPS; break;
      }
      radius = radius / decrease_factor;   /* StepIsInvalid == StepRejected */
      decrease_factor *= 2.0;
      reuse_diag = 1;
      it.cost = x_cost + s->fixed_cost;
      it.cost_change = 0.0;
      it.gradient_max_norm = prev_gmax;
      it.gradient_norm = prev_gnorm;
      it.step_norm = 0.0;
      it.relative_decrease = 0.0;
      it.step_is_valid = 0;
      it.step_is_successful = 0;
      continue;
    }
    n_invalid = 0;
    it.step_is_valid = 1;

    /* ---- ComputeCandidatePointAndEvaluateCost ---- */
    for (long k = 0; k < L.n; ++k) L.xc[k] = L.x[k] + L.delta[k];
    int cfin = 1;
    double candidate_cost = eval_cost(&L, L.xc, &cfin, NULL);
    if (!cfin) candidate_cost = DBL_MAX;

    /* ---- ParameterToleranceReached ---- */
    {
      double sq = 0.0;
      const long shared0 = slot_tag(&L, 0);
      for (long k = 0; k < L.n; ++k) {
        if (!L.free_[k]) continue;
        const int shared = (k < 3) || (k >= shared0);
        const double d = L.x[k] - L.xc[k];
        if (!shared || is_root(&L)) sq += d * d;
      }
      allreduce_sum(&L, &sq, 1);
      it.step_norm = sqrt(sq);
    }
    if (it.step_norm <= o->parameter_tolerance * (x_norm + o->parameter_tolerance)) {
      s->termination = OR_CONVERGENCE; s->rule = OR_RULE_PARAMETER;
      break;
    }
    /* ---- FunctionToleranceReached ---- */
    it.cost_change = x_cost - candidate_cost;
    if (fabs(it.cost_change) <= o->function_tolerance * x_cost) {
      s->termination = OR_CONVERGENCE; s->rule = OR_RULE_FUNCTION;
      break;
    }
    /* ---- IsStepSuccessful (monotonic TrustRegionStepEvaluator) ---- */
    it.relative_decrease = (candidate_cost >= DBL_MAX) ? -DBL_MAX
                                                       : (x_cost - candidate_cost) / model_cost_change;
    if (it.relative_decrease > o->min_relative_decrease) {
      /* HandleSuccessfulStep */
      double *tmp = L.x; L.x = L.xc; L.xc = tmp;
      x_norm = norm_free(&L, L.x);
      int fin = 1;
      x_cost = evaluate_jacobian(&L, &fin);
      it.cost = x_cost + s->fixed_cost;
      grad_norms(&L, &it.gradient_max_norm, &it.gradient_norm);
      it.step_is_successful = 1;
      const double q = 2.0 * it.relative_decrease - 1.0;
      double f = 1.0 - q * q * q;
      if (f < 1.0 / 3.0) f = 1.0 / 3.0;
      radius = radius / f;
      if (radius > o->max_trust_region_radius) radius = o->max_trust_region_radius;
      decrease_factor = 2.0;
      reuse_diag = 0;
    } else {
      /* HandleUnsuccessfulStep */
      it.step_is_successful = 0;
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      reuse_diag = 1;
      it.cost = candidate_cost + s->fixed_cost;
      it.gradient_max_norm = prev_gmax;
      it.gradient_norm = prev_gnorm;
    }
  }
  s->final_cost = minimum_cost + s->fixed_cost;
done:
  free(L.cap_start); free(L.cap_obs); free(L.free_); free(L.obs_active);
  free(L.x); free(L.xc); free(L.g); free(L.colnorm); free(L.scale); free(L.diag);
  free(L.y); free(L.delta); free(D2); free(L.r); free(L.J); free(L.S); free(L.rhs);
  free(L.fidx); free(L.tag_start); free(L.tag_obs);
  return s->termination;
}

double or_cost(const or_problem *p) {
  double cost = 0.0;
  for (int o = 0; o < p->n_obs; ++o) {
    double r[8];
    or_residual(p->camera, p->cap + 6L * p->obs_cap[o], p->tag + 6L * p->obs_tag[o],
                p->corners + 8L * o, r);
    double sq = 0.0;
    for (int i = 0; i < 8; ++i) sq += r[i] * r[i];
    cost += 0.5 * sq;
  }
  return cost;
}

/* ------------------------------------------------------------------------ */
/* initialisers (ar_slam_util.cpp:41-128) and localize (:888-979)            */
/* ------------------------------------------------------------------------ */

/* Ceres 2.0 rotation.h */
static void aa_to_quat(const double aa[3], double q[4]) {
  const double theta_sq = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta_sq > 0.0) {
    const double theta = sqrt(theta_sq);
    const double half = theta * 0.5;
    const double k = sin(half) / theta;
    q[0] = cos(half);
    q[1] = aa[0] * k; q[2] = aa[1] * k; q[3] = aa[2] * k;
  } else {
    const double k = 0.5;
    q[0] = 1.0;
    q[1] = aa[0] * k; q[2] = aa[1] * k; q[3] = aa[2] * k;
  }
}

static void quat_product(const double z[4], const double w[4], double zw[4]) {
  zw[0] = z[0] * w[0] - z[1] * w[1] - z[2] * w[2] - z[3] * w[3];
  zw[1] = z[0] * w[1] + z[1] * w[0] + z[2] * w[3] - z[3] * w[2];
  zw[2] = z[0] * w[2] - z[1] * w[3] + z[2] * w[0] + z[3] * w[1];
  zw[3] = z[0] * w[3] + z[1] * w[2] - z[2] * w[1] + z[3] * w[0];
}

static void quat_to_aa(const double q[4], double aa[3]) {
  const double q1 = q[1], q2 = q[2], q3 = q[3];
  const double sin_sq = q1 * q1 + q2 * q2 + q3 * q3;
  double k;
  if (sin_sq > 0.0) {
    const double sin_theta = sqrt(sin_sq);
    const double cos_theta = q[0];
    const double two_theta = 2.0 * ((cos_theta < 0.0) ? atan2(-sin_theta, -cos_theta)
                                                       : atan2(sin_theta, cos_theta));
    k = two_theta / sin_theta;
  } else {
    k = 2.0;
  }
  aa[0] = q1 * k; aa[1] = q2 * k; aa[2] = q3 * k;
}

void or_compose_axis_angle(const double rot1[3], const double rot2[3], double out[3]) {
  double q1[4], q2[4], q3[4];
  aa_to_quat(rot1, q1);
  aa_to_quat(rot2, q2);
  quat_product(q1, q2, q3);
  quat_to_aa(q3, out);
}

static double normalize_angle(double a) {   /* ar_slam_util.hpp:348-351 */
  return fmod(fmod(a, 2 * M_PI) + 3 * M_PI, 2 * M_PI) - M_PI;
}

void or_calc_init_values(const double corners[8], double focal, double out[4]) {
  static const double dir[4][2] = {{-1, -1}, {1, -1}, {1, 1}, {-1, 1}};   /* ar_slam_util.hpp:340-345 */
  double max_dist_sq = 0.0, avg_x = 0.0, avg_y = 0.0;
  for (int i = 0; i < 4; ++i) {
    const double *p1 = corners + 2 * i, *p2 = corners + 2 * ((i + 1) & 3);
    const double d = pow(p1[0] - p2[0], 2) + pow(p1[1] - p2[1], 2);
    if (d > max_dist_sq) max_dist_sq = d;
    avg_x += p1[0];
    avg_y += p1[1];
  }
  avg_x *= 0.25;
  avg_y *= 0.25;
  double avg_angle = 0.0;
  for (int i = 0; i < 4; ++i) {
    const double expected = atan2(dir[i][1], dir[i][0]);
    const double actual = atan2(corners[2 * i + 1] - avg_y, corners[2 * i] - avg_x);
    const double delta = normalize_angle(actual - expected);
    avg_angle += normalize_angle(delta - avg_angle) / (i + 1);
  }
  const double local_z = focal * kArucoSize / sqrt(max_dist_sq);
  out[0] = avg_x * local_z / focal;
  out[1] = avg_y * local_z / focal;
  out[2] = local_z;
  out[3] = avg_angle;
}

void or_init_capture_pose(const double corners[8], const double camera[3], const double ar_pose[6],
                          double inv_cap_pose[6]) {
  double v[4];
  or_calc_init_values(corners, camera[0], v);
  const double local_position[3] = {v[0], v[1], v[2]};
  const double local_rot[3] = {0.0, 0.0, v[3]};
  const double inv_ar_rot[3] = {-ar_pose[3], -ar_pose[4], -ar_pose[5]};
  or_compose_axis_angle(local_rot, inv_ar_rot, inv_cap_pose + 3);
  const double cap_rotation[3] = {-inv_cap_pose[3], -inv_cap_pose[4], -inv_cap_pose[5]};
  or_angle_axis_rotate(cap_rotation, local_position, inv_cap_pose);
  inv_cap_pose[0] -= ar_pose[0];
  inv_cap_pose[1] -= ar_pose[1];
  inv_cap_pose[2] -= ar_pose[2];
}

void or_init_ar_pose(const double corners[8], const double camera[3], const double inv_cap_pose[6],
                     double ar_pose[6]) {
  double v[4];
  or_calc_init_values(corners, camera[0], v);
  const double local_position[3] = {v[0], v[1], v[2]};
  const double cap_rotation[3] = {-inv_cap_pose[3], -inv_cap_pose[4], -inv_cap_pose[5]};
  or_angle_axis_rotate(cap_rotation, local_position, ar_pose);
  ar_pose[0] -= inv_cap_pose[0];
  ar_pose[1] -= inv_cap_pose[1];
  ar_pose[2] -= inv_cap_pose[2];
  const double local_rot[3] = {0.0, 0.0, v[3]};
  const double cap_rot[3] = {-inv_cap_pose[3], -inv_cap_pose[4], -inv_cap_pose[5]};
  or_compose_axis_angle(cap_rot, local_rot, ar_pose + 3);
}

int or_localize_many(int n_query, const int *q_start, const int *obs_tag, const double *corners,
                     const double camera[3], const double *tag, int n_tag,
                     const unsigned char *tag_in_map, int init_from_map, double *pose,
                     const or_options *o, int *status, or_summary *summaries) {
  int n_done = 0;
  for (int q = 0; q < n_query; ++q) {
    const int o0 = q_start[q], k = q_start[q + 1] - o0;
    double *x = pose + 6L * q;
    int init = -1;
    for (int j = 0; j < k; ++j)
      if (!tag_in_map || tag_in_map[obs_tag[o0 + j]]) { init = o0 + j; break; }
    if (init < 0 && init_from_map) { status[q] = -1; continue; }   /* :929-933 */
    if (k == 0) { status[q] = -1; continue; }
    if (init_from_map) or_init_capture_pose(corners + 8L * init, camera, tag + 6L * obs_tag[init], x);
    /* one capture, its blocks' tags and the camera constant: :956-972.  The
     * problem holds only this capture's tags (compact local indices). */
    double cam[3] = {camera[0], camera[1], camera[2]};
    int *oc = calloc(k, sizeof(int)), *ot = malloc(sizeof(int) * k), *loc = malloc(sizeof(int) * k);
    int nl = 0;
    for (int j = 0; j < k; ++j) {
      const int t = obs_tag[o0 + j];
      int u = -1;
      for (int i = 0; i < nl; ++i)
        if (loc[i] == t) { u = i; break; }
      if (u < 0) { u = nl; loc[nl++] = t; }
      ot[j] = u;
    }
    (void)n_tag;
    unsigned char *tc = malloc(nl);
    memset(tc, 1, nl);
    double *tg = malloc(sizeof(double) * 6 * nl);
    for (int i = 0; i < nl; ++i) memcpy(tg + 6L * i, tag + 6L * loc[i], 6 * sizeof(double));
    or_problem pr = {1, nl, k, cam, x, tg, oc, ot, corners + 8L * o0, 1, NULL, tc};
    or_summary s;
    status[q] = or_solve(&pr, o, &s, NULL);
    if (summaries) summaries[q] = s;
    free(oc); free(ot); free(loc); free(tc); free(tg);
    ++n_done;
  }
  return n_done;
}
