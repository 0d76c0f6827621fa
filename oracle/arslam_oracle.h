/*
 * arslam_oracle.h -- CPU restatement of ar_slam's bundle-adjustment hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library; the product path
 * (ar_slam_amd/, libarslam_lm.so) never links or calls it.
 *
 * What it restates:
 *   - projectCorner / ArucoReprojectionError   ar_slam_util.cpp:131-172, 192-216
 *   - ceres::AngleAxisRotatePoint              Ceres 2.0 include/ceres/rotation.h
 *   - ceres::Solve(DENSE_SCHUR, LM, 50 iters)  ar_slam_util.cpp:1001-1018 and the
 *     Ceres 2.0 TrustRegionMinimizer / LevenbergMarquardtStrategy /
 *     SchurEliminator / DenseSchurComplementSolver.
 *
 * Parity status: the reference cannot be built here (Ceres, Eigen, OpenCV
 * and ROS are absent) and its only test pins nothing on this
 * path, so the restatement is pinned by (1) torch-fp64 autograd and central
 * differences for the Jacobian, (2) scipy.optimize.least_squares for the
 * converged cost, (3) noise-free graphs converging to the truth modulo
 * gauge, and (4) the Schur step equalling the full normal-equation step.
 * Against Ceres itself it is "parity unpinned".
 */
#ifndef ARSLAM_ORACLE_H
#define ARSLAM_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAX_ITERS 1024

/* Problem in SoA form.  Parameters are updated in place by or_solve. */
typedef struct {
  int n_cap, n_tag, n_obs;
  double *camera;                 /* [3]        f, l1, l2                */
  double *cap;                    /* [n_cap*6]  inv_pose t_c, w_c        */
  double *tag;                    /* [n_tag*6]  pose t_t, w_t            */
  const int *obs_cap;             /* [n_obs]                             */
  const int *obs_tag;             /* [n_obs]                             */
  const double *corners;          /* [n_obs*8] x0,y0,..,x3,y3            */
  int camera_const;               /* SetParameterBlockConstant(camera)   */
  const unsigned char *cap_const; /* [n_cap] or NULL                     */
  const unsigned char *tag_const; /* [n_tag] or NULL                     */
} or_problem;

/* OR_ELIM_MIXED: the e-blocks are exactly the captures with e_cap[c] != 0 and
 * the tags with e_tag[t] != 0 (an independent set: no residual joins two of
 * them) -- Ceres' own ComputeStableSchurOrdering set, which mixes the two
 * kinds (ar_slam_util.cpp:1011 sets no ordering).  Single process only. */
enum { OR_ELIM_CAPTURES = 0, OR_ELIM_NONE = 1, OR_ELIM_MIXED = 2 };

typedef struct {
  int max_num_iterations;              /* 50 (ar_slam_util.cpp:1004) */
  double function_tolerance;           /* 1e-6  */
  double gradient_tolerance;           /* 1e-10 */
  double parameter_tolerance;          /* 1e-8  */
  double initial_trust_region_radius;  /* 1e4   */
  double max_trust_region_radius;      /* 1e16  */
  double min_trust_region_radius;      /* 1e-32 */
  double min_relative_decrease;        /* 1e-3  */
  double min_lm_diagonal;              /* 1e-6  */
  double max_lm_diagonal;              /* 1e32  */
  int max_num_consecutive_invalid_steps; /* 5 */
  int jacobi_scaling;                  /* 1 */
  int elimination;                     /* OR_ELIM_CAPTURES | OR_ELIM_NONE | OR_ELIM_MIXED */
  int num_threads;                     /* OpenMP threads for the dense LLT (1 = reference) */
  int progress;                        /* print the Ceres progress table */
  /* test hook (not a Ceres option): at linear solve i (0-based) with bit
   * min(i,63) set, the reduced system's first camera row gets diagonal -1
   * after D_f^2 is added, so its LLT fails and the step is invalid -- the
   * same hook as the device's arslam_lm_debug_force_indefinite. */
  unsigned long long debug_indefinite_mask;
  const unsigned char *e_cap;          /* OR_ELIM_MIXED: [n_cap] eliminated captures */
  const unsigned char *e_tag;          /* OR_ELIM_MIXED: [n_tag] eliminated tags */
} or_options;

typedef struct {
  int iteration;
  double cost, cost_change, gradient_max_norm, gradient_norm, step_norm;
  double relative_decrease, trust_region_radius;
  int step_is_valid, step_is_successful;
  double iteration_time, cumulative_time;
} or_iter;

enum { OR_CONVERGENCE = 0, OR_NO_CONVERGENCE = 1, OR_FAILURE = 2 };
enum { OR_RULE_NONE = 0, OR_RULE_GRADIENT = 1, OR_RULE_PARAMETER = 2, OR_RULE_FUNCTION = 3,
       OR_RULE_MIN_RADIUS = 4, OR_RULE_MAX_ITERS = 5, OR_RULE_INVALID_STEPS = 6,
       OR_RULE_EVAL_FAILED = 7 };

typedef struct {
  int termination;        /* OR_CONVERGENCE / OR_NO_CONVERGENCE / OR_FAILURE */
  int rule;               /* which test fired */
  int num_successful_steps, num_unsuccessful_steps;
  int num_linear_solves;  /* trust-region step computations (the LM iteration count of the metric) */
  double initial_cost, final_cost, fixed_cost;
  int n_iters;            /* number of entries in iters[] (iteration 0 included) */
  or_iter iters[OR_MAX_ITERS + 1];
} or_summary;

/* Reduction hooks for the capture-sharded (multi-rank) restatement.  Each
 * rank holds every tag and the camera plus its own captures/observations;
 * the hooks all-reduce in place.  NULL comm = single process. */
typedef struct {
  void *ctx;
  int rank;
  void (*allreduce_sum)(void *ctx, double *buf, long n);
  void (*allreduce_max)(void *ctx, double *buf, long n);
} or_comm;

void or_default_options(or_options *o);

/* ceres::AngleAxisRotatePoint */
void or_angle_axis_rotate(const double w[3], const double x[3], double out[3]);

/* projectCorner<double> (ar_slam_util.cpp:131-172) */
void or_project_corner(const double cam[3], const double cap[6], const double tag[6],
                       int idx, double out[2]);

/* ArucoReprojectionError::operator() (ar_slam_util.cpp:198-211) */
void or_residual(const double cam[3], const double cap[6], const double tag[6],
                 const double corners[8], double r[8]);

/* Residual and analytic Jacobian, J row-major [8][15]: cols cam(3), cap(6), tag(6). */
void or_residual_jacobian(const double cam[3], const double cap[6], const double tag[6],
                          const double corners[8], double r[8], double J[120]);

/* Sum over observations of 0.5*|r|^2 (the Ceres cost). */
double or_cost(const or_problem *p);

/* Solve in place; returns termination type. comm may be NULL. */
int or_solve(or_problem *p, const or_options *o, or_summary *s, const or_comm *comm);

/* Dense lower Cholesky in place (row-major, ld), returns 0 on success,
 * k+1 if the pivot of column k is not positive.  Exposed for tests and the
 * CPU baseline. */
int or_llt_lower(double *A, long n, long ld, int num_threads);

/* ---- initialisers (ar_slam_util.cpp:41-128) ---- */
/* composeAxisAngle :41-50 (Ceres AngleAxisToQuaternion / QuaternionProduct /
 * QuaternionToAngleAxis) */
void or_compose_axis_angle(const double rot1[3], const double rot2[3], double out[3]);
/* calcInitValues :52-95: (local_x, local_y, local_z, rot_z) of a tag seen in a rect */
void or_calc_init_values(const double corners[8], double focal, double out[4]);
/* initCapturePose :98-115 / initArPose :118-128 */
void or_init_capture_pose(const double corners[8], const double camera[3], const double ar_pose[6],
                          double inv_cap_pose[6]);
void or_init_ar_pose(const double corners[8], const double camera[3], const double inv_cap_pose[6],
                     double ar_pose[6]);

/* ---- localizeMany / localizeOne (ar_slam_util.cpp:888-979) ----
 * Query q owns observations [q_start[q], q_start[q+1]) in block order.  With
 * init_from_map, the pose is initialised by initCapturePose from the first
 * block whose tag is in the map (tag_in_map; NULL = all) and the query is
 * skipped (status -1, pose untouched) when there is none (:929-933);
 * otherwise pose[] is the initial value.  Each query is then one ceres::Solve
 * with its tags and the camera constant (:965, :972).  status[q] = Ceres
 * termination type, or -1 if skipped; summaries[q] optional. */
int or_localize_many(int n_query, const int *q_start, const int *obs_tag, const double *corners,
                     const double camera[3], const double *tag, int n_tag,
                     const unsigned char *tag_in_map, int init_from_map, double *pose,
                     const or_options *o, int *status, or_summary *summaries);

#ifdef __cplusplus
}
#endif
#endif
