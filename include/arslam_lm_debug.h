/*
 * arslam_lm_debug.h -- component entry points of libarslam_lm.so used by the
 * parity tests to check one device stage at a time against the CPU oracle.
 * Not part of the drop-in boundary (arslam_lm.h); same error conventions.
 */
#ifndef ARSLAM_LM_DEBUG_H
#define ARSLAM_LM_DEBUG_H

#include "arslam_lm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Residuals and Jacobians of n independent observations on the device.
 * cam [n*3], cap [n*6], tag [n*6], corners [n*8] -> r [n*8],
 * J [n*8*15] row-major with columns cam(3) cap(6) tag(6), as ceres'
 * AutoDiffCostFunction<ArucoReprojectionError,8,3,6,6> would produce. */
int arslam_debug_residual_jacobian(int n, const double *cam, const double *cap, const double *tag,
                                   const double *corners, double *r, double *J);

/* ceres::AngleAxisRotatePoint (rotation.h; called at ar_slam_util.cpp:145,155)
 * of n points p[n*3] by angle-axis w[n*3] on the device -> out[n*3], and the
 * branch each took: branch[i] = 1 if theta^2 > DBL_EPSILON (Rodrigues), 0 for
 * the first-order form x + w x p. */
int arslam_debug_angle_axis_rotate(int n, const double *w, const double *p, double *out, int *branch);

/* Dense reduced-system solve on the device: factor the lower triangle of the
 * n x n row-major SPD matrix A (in place: on return A holds L) and solve
 * A y = b.  *info = 0 on success, k+1 if pivot k was not positive. */
int arslam_debug_dense_llt(long n, double *A, const double *b, double *y, int *info);
/* the same with the factorization executor chosen (0 level launches, 1 persistent task graph);
 * info < 0 reports a task-graph wait that timed out */
int arslam_debug_dense_llt_ex(long n, double *A, const double *b, double *y, int *info, int executor);

/* Host-only symbolic analysis of the reduced system (no device needed): the
 * row layout arslam_lm_load_soa would choose for problem p under the given
 * ordering (0 natural, 1 RCM, 2 nested dissection) and tile pattern
 * (skip_zero_tiles), its tile Cholesky plan, and optionally the first row of
 * each tag (tag_row[n_tag], -1 if the tag is not a parameter). */
typedef struct {
  long n_reduced;          /* rows of the reduced system (6 per free tag + 3 camera) */
  long n_padded;           /* tiles_per_side * 64 */
  long pad_rows;           /* alignment padding rows among the tag rows */
  int tiles_per_side;
  int n_parts;             /* ordering parts (ND leaves + separators) */
  int camera_row;          /* -1 if the camera is constant */
  int n_levels;            /* height of the tile elimination tree */
  long n_assembled_tiles;  /* tiles the Schur assembly writes */
  long n_factor_tiles;     /* after symbolic fill */
  long n_update_tiles;     /* (target, column) tile products per factorization */
  long n_update_items;     /* update work items (after splitting long k-lists) */
  long n_split_targets;
  double update_flops;     /* algorithmic flops of the trailing updates per factorization */
  long n_dag_tasks;        /* tasks of the persistent executor's graph */
  int dag_valid;           /* 1: run one at a time in ticket order, every wait is already met, and
                              every simulated interleaving finishes (grids 1..512 and the small-graph
                              grid, random and adversarial policies); -(grid * 16 + policy) of the
                              first simulated deadlock */
  double factor_flops;     /* flops of the tile plan per factorization (POTRF, TRSM, updates, inverses) */
  double scalar_flops;     /* flops of the scalar Cholesky of the real rows in this order (no padding,
                              no structurally zero entries inside tiles) */
  int fill_first_ok;       /* 1: every fill tile's first application is an unfolded update item, so the
                              solver leaves fill tiles uncleared and that update stores 0 - acc */
} arslam_plan_info;

/* diagnostic builds only (-DARSLAM_SCHUR_STAMPS): per-phase cycles of the
 * Schur kernel accumulated over all its waves (zeros otherwise) */
int arslam_debug_schur_stamps(unsigned long long out[16]);

/* Test hooks on a solver handle.
 * force_indefinite: at every linear solve i (0-based) whose bit
 * min(i, 63) is set in step_mask, the reduced system's first camera row
 * (the last row if the camera is constant) gets diagonal -1 after the LM
 * diagonal is added, so the Cholesky reports a failed pivot and the LM step
 * is invalid (Ceres' LinearSolver FAILURE path).  0 turns it off.
 * break_dependency: on a problem loaded by arslam_lm_load_soa with the
 * persistent executor, raise the first wait of the first task at or after
 * `ticket` that has one beyond any count it can reach; the next solve must
 * then fail with ARSLAM_E_DEVICE.  *broken = the task changed.  Load again
 * to repair. */
int arslam_lm_debug_force_indefinite(arslam_lm *h, unsigned long long step_mask);
int arslam_lm_debug_break_dependency(arslam_lm *h, long ticket, long *broken);
/* force_multirank: on = 1 makes the handle take the multi-rank path with one
 * rank -- the subtree split (the two-rank split's replicated top, everything
 * below it this rank's), the two-phase factorization and every collective of
 * a multi-rank solve -- so that arslam_lm_set_comm(h, 0, 1, id) creates a
 * one-rank RCCL communicator and the solver issues its real ncclAllReduce
 * calls (f64 SUM / MAX, u8 MAX) on its stream on a one-GPU box.  Resets the
 * communicator (set it again after this call); 0 restores the one-rank path. */
int arslam_lm_debug_force_multirank(arslam_lm *h, int on);
/* tag_pair_tile: on a pointer-keyed problem loaded with capture elimination
 * on one rank, where the coupling of tag blocks a and b (and the pair's
 * mirror) falls in the reduced system: *status = 2 a tile assembled at the
 * load, 1 a fill tile of the loaded factor (an appended capture coupling them
 * keeps the plan: the gather writes into the fill tile), 0 no tile of the
 * factor (an append reloads), -1 a or b is not a free tag of the loaded
 * problem. */
int arslam_lm_debug_tag_pair_tile(arslam_lm *h, const double *tag_a, const double *tag_b, int *status);

/* Ceres 2.0's DENSE_SCHUR e-block set for problem p (ComputeStableSchurOrdering,
 * the rule ARSLAM_ELIM_AUTO follows), host only: out = {captures, tags,
 * camera (0/1) in the set, most observations of one tag}. */
int arslam_debug_ceres_e_blocks(const arslam_soa_problem *p, int out[4]);

/* Host only: the set itself (e_cap[n_cap], e_tag[n_tag]: 1 = eliminated) and the
 * ARSLAM_ELIM_MIXED device problem built from it: out = {groups (eliminated
 * captures + eliminated tags + direct groups), reduced-side blocks, direct
 * groups, most local blocks of one group}. */
int arslam_debug_mixed_groups(const arslam_soa_problem *p, int out[4], unsigned char *e_cap, unsigned char *e_tag);

int arslam_debug_reduced_plan(const arslam_soa_problem *p, int ordering, int skip_zero_tiles,
                              arslam_plan_info *info, int *tag_row);
/* Host only: the reduced layout (nested dissection, sparse tiles) and tile plan
 * of p's device problem under elimination (ARSLAM_ELIM_CAPTURES, _TAGS or
 * _MIXED: Ceres' set), built as a fresh one-rank load builds it.  Returns the
 * side used (MIXED falls back to a whole side as the load does) or an error. */
int arslam_debug_reduced_plan_side(const arslam_soa_problem *p, int elimination, arslam_plan_info *info);

/* Host only: one simulated interleaving of n_workers workgroups running the
 * persistent executor's protocol on the one-rank plan of p (policy 0 random,
 * 1-3 adversarial orders; + 16 drops the cap on claimed continuations in
 * flight, which the protocol relies on).  *ok = 1 if every task finished, 0 on
 * a deadlock. */
int arslam_debug_dag_simulate(const arslam_soa_problem *p, int n_workers, unsigned seed, int policy, int *ok);
/* The same with only n_started of the grid's n_workers workgroups ever
 * starting (each when the schedule picks it): fewer workgroups resident than
 * the grid.  The executor caps claimed continuations at half the workgroups
 * started so far; policy + 32 simulates round 5's cap (half the grid), which
 * such schedules deadlock. */
int arslam_debug_dag_simulate_started(const arslam_soa_problem *p, int n_workers, int n_started, unsigned seed,
                                      int policy, int *ok);
/* Process-wide: every later k_factor_dag launch lets only its first k
 * workgroups start (the others return at once), as if only k were resident;
 * k <= 0 restores the whole grid.  The factorization's result does not depend
 * on it (fixed summation order). */
int arslam_debug_dag_workgroup_limit(int k);

/* Host only: the message an executor fault carries for the one-rank plan of p
 * (nested dissection, sparse tiles) and a fault record rec[9] = {ticket, kind
 * (1 dependency wait, 2 in-order application, 3 late wait), counter, value
 * seen, value awaited, tickets drawn, claimed continuations in flight,
 * workgroup, INT_MAX - the smallest ticket whose wait ran out of time (0:
 * none)}: the task, the counter, the tickets that advance it.  Writes at most
 * len bytes (NUL-terminated) to buf. */
int arslam_debug_dag_fault_detail(const arslam_soa_problem *p, const int rec[9], char *buf, int len);

/* The memory round trips of the persistent executor's hand-offs on this
 * device, measured in a few milliseconds (one lane each): out = {never-matching
 * CAS poll (ns, dependent chain), agent-scope sc1 load (ns, dependent chain),
 * write-through store + its acknowledgement (ns each), workgroup ping-pong
 * through agent-scope flags (ns per round trip, -1 if it timed out), the two
 * workgroups' XCC ids}.  device < 0: the current device. */
int arslam_debug_box_fingerprint(int device, double out[6]);

/* Host only: the multi-rank split arslam_lm_load_soa makes for rank `rank` of
 * `nranks` (nested dissection, sparse tiles) -- its two-phase tile plan, and
 * every capture's owning rank (cap_owner[n_cap], may be NULL). */
typedef struct {
  int tiles_per_side;
  int n_top_cols;           /* tile columns replicated on every rank */
  int n_own_cols;           /* tile columns of this rank's subtrees */
  long n_top_tiles;         /* tiles of the top columns (the per-step exchange) */
  long n_tiles;             /* tiles stored on this rank (top + own) */
  long n_dag_tasks, phase_split;   /* tasks of the plan; [0, phase_split) run before the exchange */
  int dag_valid;            /* 1: ticket order valid and the randomised interleavings finish */
  int n_owned_captures;
  double top_work, max_rank_work, total_work;   /* tile-task counts (RankSplit) */
  int n_active;             /* ranks owning subtrees (the others own top-only captures) */
} arslam_split_info;
int arslam_debug_rank_split(const arslam_soa_problem *p, int nranks, int rank, arslam_split_info *info,
                            int *cap_owner);
/* Host-only: the Schur gather plan of p's first c0 captures (their residual
 * blocks, p's order), extended by captures c0.. (schur_gather_extend, the
 * appended-problem path), against the plan built afresh for all of p with the
 * same layout.  *identical = 1 when every array agrees; *n_dest the
 * destinations of the full plan. */
int arslam_debug_gather_extend(const arslam_soa_problem *p, int c0, int *identical, int *n_dest);

#ifdef __cplusplus
}
#endif
#endif
