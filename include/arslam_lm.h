/*
 * arslam_lm.h -- C-ABI of the MI355X-native Levenberg-Marquardt bundle
 * adjuster that replaces ar_slam's ceres::Solve call.
 *
 * Drop-in boundary.  The reference builds a ceres::Problem
 * and hands it to ceres::Solve:
 *
 *   AddResidualBlock(AutoDiff<ArucoReprojectionError,8,3,6,6>, nullptr,
 *                    camera, capture.inv_pose, aruco.pose)
 *        ar_slam_util.cpp:720-727, 829-836, 956-963
 *   SetParameterBlockConstant(block)       ar_slam_util.cpp:965, 972
 *   ceres::Solve(options, &problem_, &s)   ar_slam_util.cpp:1001-1018
 *   resetProblem()                         ar_slam_util.cpp:1021-1025
 *
 * Each entry point below replaces one of those calls with the same argument
 * meaning: parameter blocks are caller-owned double arrays keyed by their
 * address (camera[3] = f,l1,l2; capture[6] = inv_pose t,w; tag[6] = pose
 * t,w), observations are copied (as the functor copies its ArucoRect,
 * ar_slam_util.cpp:194-196), and results are written back into the caller's
 * arrays when the solve ends (Ceres' default; update_state_every_iteration
 * writes them after every improving step).
 *
 * Conventions: every function returns 0 (ARSLAM_OK) or a negative
 * ARSLAM_E_* code; no C++ exception crosses the ABI; a handle is not
 * thread-safe.  arslam_lm_last_error() returns the message of the most
 * recent failure on the calling thread.
 */
#ifndef ARSLAM_LM_H
#define ARSLAM_LM_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ARSLAM_LM_MAX_ITERS 1024
#define ARSLAM_COMM_ID_BYTES 128

enum {
  ARSLAM_OK = 0,
  ARSLAM_E_INVALID_ARG = -1,
  ARSLAM_E_UNSUPPORTED = -2,
  ARSLAM_E_NO_DEVICE = -3,
  ARSLAM_E_HIP = -4,
  ARSLAM_E_OUT_OF_MEMORY = -5,
  ARSLAM_E_COMM = -6,
  ARSLAM_E_STATE = -7,
  ARSLAM_E_DEVICE = -8          /* a device executor fault (a dependency wait that never completed) */
};

/* Which side of the capture/tag graph the Schur complement eliminates
 * (DENSE_SCHUR's e-blocks, ar_slam_util.cpp:1011).  AUTO follows Ceres 2.0's
 * own choice (ReorderProgramForSchurTypeLinearSolver -> ComputeStableSchurOrdering:
 * the stable greedy independent set of the Hessian graph in ascending degree,
 * blocks in program order): the side that holds the majority of that set is
 * eliminated (Ceres may mix the two sides; the step is the same exact solve of
 * the same system, only the rounding differs).  MIXED eliminates exactly
 * Ceres' set -- captures and tags together when it mixes them (residuals
 * joining two reduced-side blocks then go straight into the reduced system, as
 * in Ceres' SchurEliminator); summary.elimination_used then reports MIXED, or
 * the side when the set is one whole side.  Multi-rank solves always
 * eliminate captures (the shards are capture ranges); MIXED is single-rank. */
enum { ARSLAM_ELIM_AUTO = 0, ARSLAM_ELIM_CAPTURES = 1, ARSLAM_ELIM_TAGS = 2, ARSLAM_ELIM_MIXED = 3 };

/* Ceres termination types (ceres::TerminationType) */
enum { ARSLAM_CONVERGENCE = 0, ARSLAM_NO_CONVERGENCE = 1, ARSLAM_FAILURE = 2, ARSLAM_USER_SUCCESS = 3,
       ARSLAM_USER_FAILURE = 4 };

/* summary.setup_kind: a full load (structure, elimination order, plan), the
 * loaded problem with new values only, or an appended problem whose new
 * residual blocks fit the loaded tile pattern (order and plan kept) */
enum { ARSLAM_SETUP_LOAD = 0, ARSLAM_SETUP_VALUES = 1, ARSLAM_SETUP_APPEND = 2 };

/* which termination test fired */
enum {
  ARSLAM_RULE_NONE = 0, ARSLAM_RULE_GRADIENT = 1, ARSLAM_RULE_PARAMETER = 2,
  ARSLAM_RULE_FUNCTION = 3, ARSLAM_RULE_MIN_RADIUS = 4, ARSLAM_RULE_MAX_ITERS = 5,
  ARSLAM_RULE_INVALID_STEPS = 6, ARSLAM_RULE_EVAL_FAILED = 7, ARSLAM_RULE_USER_CALLBACK = 8
};

/* ceres::Solver::Options subset used by ArSlamSolver::optimize
 * (ar_slam_util.cpp:1003-1012); defaults from arslam_lm_options_init are
 * the reference's values (max_num_iterations = 50, DENSE_SCHUR) plus Ceres
 * 2.0 defaults for everything it leaves unset. */
typedef struct {
  int max_num_iterations;
  double function_tolerance;
  double gradient_tolerance;
  double parameter_tolerance;
  double initial_trust_region_radius;
  double max_trust_region_radius;
  double min_trust_region_radius;
  double min_relative_decrease;
  double min_lm_diagonal;
  double max_lm_diagonal;
  int max_num_consecutive_invalid_steps;
  int jacobi_scaling;
  int elimination;                   /* ARSLAM_ELIM_* */
  int minimizer_progress_to_stdout;  /* Ceres progress table */
  int update_state_every_iteration;  /* write improving iterates back */
  int device;                        /* HIP device ordinal, -1 = current */
  int cholesky_skip_zero_tiles;      /* 1: skip structurally-zero tiles of the reduced system */
  int reduced_ordering;              /* tags in the reduced system: 0 natural, 1 reverse
                                        Cuthill-McKee, 2 nested dissection (default) */
  int kernel_timing;                 /* 1: HIP events around every launch of the dominant kernel */
  int factor_executor;               /* reduced-system Cholesky: 0 two launches per elimination-tree
                                        level, 1 one persistent task-graph launch (default) */
  int phase_timing;                  /* 1: HIP events around each phase of the step (summary
                                        t_*_ms; host loop only); 0 (default): none (each event
                                        record costs a few microseconds of GPU time) */
} arslam_lm_options;

/* ceres::IterationSummary subset */
typedef struct {
  int iteration;
  double cost, cost_change, gradient_max_norm, gradient_norm, step_norm;
  double relative_decrease, trust_region_radius;
  int step_is_valid, step_is_successful;
  double iteration_time, cumulative_time;
} arslam_lm_iteration;

/* ceres::Solver::Summary subset plus per-phase device timings */
typedef struct {
  int termination;              /* ARSLAM_CONVERGENCE ... */
  int rule;                     /* ARSLAM_RULE_* */
  int num_successful_steps, num_unsuccessful_steps;
  int num_linear_solves;        /* trust-region step computations = LM iterations of the metric */
  double initial_cost, final_cost, fixed_cost;
  double final_rms_px;          /* sqrt(2 final_cost / (4 n_obs)) */
  int n_obs, n_reduced;         /* residual blocks; size of the reduced (tag+camera) system */
  double setup_time_s;          /* host assembly + upload */
  int setup_kind;               /* ARSLAM_SETUP_*: how the problem reached the device for this solve */
  double minimizer_time_s;      /* first evaluation to termination */
  double total_time_s;
  /* accumulated device time per phase (ms), from HIP events */
  double t_linearize_ms, t_schur_ms, t_cholesky_ms, t_solve_ms, t_backsub_ms, t_cost_ms;
  /* dominant kernel (reduced-system trailing update on MFMA), kernel_timing = 1 only */
  double t_dominant_ms;         /* sum of its launch durations */
  double dominant_flops;        /* algorithmic flops of those launches */
  long n_dominant_launches;
  /* reduced-system tile plan (per factorization) */
  long n_factor_tiles;          /* 64x64 tiles of the factor that exist */
  int n_levels;                 /* levels of the tile elimination tree (launch pairs) */
  long n_update_tiles;          /* tile updates (MFMA work items) */
  double factor_update_flops;   /* useful flops of the trailing updates */
  double factor_scalar_flops;   /* flops of the scalar Cholesky of the real rows (the algorithmic count:
                                   no padding rows, no zeros inside fill tiles) per factorization */
  double comm_bytes;            /* multi-rank: bytes this rank all-reduced during the solve */
  int elimination_used;         /* ARSLAM_ELIM_CAPTURES, _TAGS or _MIXED (Ceres' set, both kinds) */
  int ceres_e_captures;         /* Ceres 2.0's e-block set for this problem (ComputeStableSchurOrdering): */
  int ceres_e_tags;             /*   captures and tags in it (the camera joins it only in degenerate graphs) */
  /* several ranks (subtree-to-rank split of the reduced system's elimination tree) */
  int n_ranks;
  int n_owned_captures;         /* captures this rank owns (every capture on one rank) */
  long n_top_tiles;             /* tiles of the replicated top columns: the per-step exchange is these */
  double split_top_work;        /* tile tasks of the top columns (replicated on every rank) */
  double split_max_rank_work;   /* tile tasks of the busiest rank's subtrees */
  double split_total_work;      /* tile tasks of the whole factorization */
  double t_factor_own_ms;       /* device time of the factorization's phase 0 (own subtrees) and */
  double t_factor_top_ms;       /*   phase 1 (the top), summed over the solve (phase_timing = 1) */
  int n_iters;                  /* entries in iters[], iteration 0 included */
  arslam_lm_iteration iters[ARSLAM_LM_MAX_ITERS + 1];
  double setup_phase_s[5];      /* the last full load (ARSLAM_SETUP_LOAD): problem structure (Ceres'
                                   e-block rule + host problem), elimination order (reduced layout; several
                                   ranks: + the split), tile plan + task graph, Schur gather plan + upload,
                                   the rest (stream, co-visibility bookkeeping) */
  long comm_calls;              /* multi-rank: collectives this rank made during the solve */
  int n_active_ranks;           /* ranks that own subtrees of the split (the others own only captures that
                                   see top tags alone); 1 on one rank */
  int order_reused;             /* the last full load kept the earlier elimination order (an incremental
                                   reload: 1) or computed a fresh one (0) */
} arslam_lm_summary;

/* Whole problem in struct-of-arrays form (bulk / benchmark path). */
typedef struct {
  int n_cap, n_tag, n_obs;
  double *camera;                  /* [3], updated in place */
  double *cap;                     /* [n_cap*6], updated in place */
  double *tag;                     /* [n_tag*6], updated in place */
  const int *obs_cap;              /* [n_obs] */
  const int *obs_tag;              /* [n_obs] */
  const double *corners;           /* [n_obs*8] centred pixels x0,y0..x3,y3 */
  int camera_const;
  const unsigned char *cap_const;  /* [n_cap] or NULL */
  const unsigned char *tag_const;  /* [n_tag] or NULL */
} arslam_soa_problem;

typedef struct arslam_lm arslam_lm;

/* Fill *opt with the reference's solver options. */
int arslam_lm_options_init(arslam_lm_options *opt);

/* new ceres::Problem (ArSlamSolver::problem_, ar_slam_util.hpp:473) */
int arslam_lm_create(arslam_lm **out, const arslam_lm_options *opt);
void arslam_lm_destroy(arslam_lm *h);

/* Per-solve options (the Solver::Options ArSlamSolver::optimize builds on
 * every call, ar_slam_util.cpp:1003-1012).  Changing device, reduced_ordering
 * or cholesky_skip_zero_tiles drops a problem loaded by arslam_lm_load_soa
 * (load again); the pointer-keyed problem is unaffected. */
int arslam_lm_set_options(arslam_lm *h, const arslam_lm_options *opt);
int arslam_lm_get_options(const arslam_lm *h, arslam_lm_options *opt);

/* problem_.AddResidualBlock(new AutoDiffCostFunction<ArucoReprojectionError,
 * 8,3,6,6>(new ArucoReprojectionError(rect)), nullptr, camera, capture, tag)
 * -- ar_slam_util.cpp:720-727.  corners = ArucoRect x0,y0,..,x3,y3. */
int arslam_lm_add_residual_block(arslam_lm *h, const double corners[8], double *camera,
                                 double *capture, double *tag);

/* problem_.SetParameterBlockConstant(block) -- ar_slam_util.cpp:965, 972 */
int arslam_lm_set_parameter_block_constant(arslam_lm *h, double *block);
int arslam_lm_set_parameter_block_variable(arslam_lm *h, double *block);

/* ceres::Solve(options, &problem_, &summary) -- ar_slam_util.cpp:1015 */
int arslam_lm_solve(arslam_lm *h, arslam_lm_summary *summary);

/* ArSlamSolver::resetProblem -- ar_slam_util.cpp:1021-1025 */
int arslam_lm_reset(arslam_lm *h);

int arslam_lm_num_residual_blocks(const arslam_lm *h);

/* Bulk path: load an SoA problem into device memory once (HBM-resident), then
 * solve it any number of times from the loaded initial state; results are
 * written to the SoA arrays given at load time. */
int arslam_lm_load_soa(arslam_lm *h, const arslam_soa_problem *p);
int arslam_lm_solve_loaded(arslam_lm *h, arslam_lm_summary *summary);

/* One-shot bulk solve. */
int arslam_lm_solve_soa(arslam_soa_problem *p, const arslam_lm_options *opt,
                        arslam_lm_summary *summary);

/* Multi-GPU (one process per GPU): every rank loads the WHOLE problem (the
 * same arslam_soa_problem / the same residual blocks) and the solver splits
 * it: the elimination tree of the reduced tag+camera system is cut below its
 * top separators, each rank owns some of the subtrees below the cut and the
 * captures whose tags lie in them, factors those columns, and the ranks then
 * sum only the top columns' tiles over RCCL before factoring the top
 * (replicated).  Results are written back for the rank's own captures
 * (arslam_lm_owned_captures) and for the camera and every tag. */
int arslam_comm_unique_id(unsigned char id[ARSLAM_COMM_ID_BYTES]);
int arslam_lm_set_comm(arslam_lm *h, int rank, int nranks,
                       const unsigned char id[ARSLAM_COMM_ID_BYTES]);

/* The same exchange through a caller-supplied host all-reduce (MPI, gloo,
 * ...): the solver stages each device buffer to host memory, calls
 * fn(ctx, buf, count, dtype, op) -- reduce `count` elements of `buf` in
 * place over all ranks, return 0 on success -- and copies the result back.
 * For ranks that share one GPU (RCCL needs one GPU per rank) and for tests.
 * Like arslam_lm_set_comm, this drops a loaded problem (load again). */
enum { ARSLAM_DT_F64 = 0, ARSLAM_DT_U8 = 1 };
enum { ARSLAM_OP_SUM = 0, ARSLAM_OP_MAX = 1 };
typedef int (*arslam_allreduce_fn)(void *ctx, void *buf, size_t count, int dtype, int op);
int arslam_lm_set_comm_callback(arslam_lm *h, int rank, int nranks, arslam_allreduce_fn fn, void *ctx);

/* The captures (indices into the loaded problem) this rank owns, ascending;
 * *n = their count (writes <= cap).  One rank owns every capture. */
int arslam_lm_owned_captures(const arslam_lm *h, int *out, int cap, int *n);

/* ceres::IterationCallback (Solver::Options::callbacks; the reference installs
 * one for its debug display, ar_slam_util.cpp:982-998, 1006-1009): called
 * after every iteration is recorded (iteration 0 included), before the
 * termination tests, with the parameter blocks already written back when
 * update_state_every_iteration is set.  Return ARSLAM_SOLVER_CONTINUE,
 * ARSLAM_SOLVER_ABORT (termination ARSLAM_USER_FAILURE) or
 * ARSLAM_SOLVER_TERMINATE_SUCCESSFULLY (ARSLAM_USER_SUCCESS).  fn = NULL
 * removes it.  Runs on the calling thread, inside arslam_lm_solve*. */
enum { ARSLAM_SOLVER_CONTINUE = 0, ARSLAM_SOLVER_ABORT = 1, ARSLAM_SOLVER_TERMINATE_SUCCESSFULLY = 2 };
typedef int (*arslam_iteration_callback)(void *ctx, const arslam_lm_iteration *it);
int arslam_lm_set_iteration_callback(arslam_lm *h, arslam_iteration_callback fn, void *ctx);

/* Diagnostics */
int arslam_device_count(void);
const char *arslam_lm_last_error(void);
const char *arslam_lm_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ARSLAM_LM_H */
