/*
 * arslam_localize.h -- C-ABI of the batched localizer: the reference's
 * ArSlamSolver::localizeMany (ar_slam_util.cpp:888-979) run for thousands of
 * queries at once on the device.
 *
 * Per query (localizeOne, :903-979):
 *   - find the first block of the capture whose tag was seen by a mapping
 *     capture (:911-927); none -> the query is skipped, pose untouched
 *     (:929-933);
 *   - initialise the capture pose from that block (initCapturePose, :943-947;
 *     ar_slam_util.cpp:98-115);
 *   - add every block of the capture as a residual with its tag held
 *     constant (:949-966) and the camera constant (:972);
 *   - ceres::Solve with the reference's options (optimize, :1001-1018): an
 *     independent Levenberg-Marquardt over the capture's 6 parameters, with
 *     its own trust region and termination.
 * With init_from_map = 0 the given pose is the initial value and no block is
 * required to be in the map (the plain optimize of a fixed map).
 *
 * Same conventions as arslam_lm.h: 0 or a negative ARSLAM_E_* code, no
 * exceptions across the ABI, handles not thread-safe.
 */
#ifndef ARSLAM_LOCALIZE_H
#define ARSLAM_LOCALIZE_H

#include "arslam_lm.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ARSLAM_LOC_SKIPPED (-1)
#define ARSLAM_LOC_MAX_OBS 64   /* observations per query */

typedef struct {
  int n_query, n_tag, n_obs;
  const double *camera;               /* [3] intrinsics, constant (:972) */
  const double *tag;                  /* [n_tag*6] map tag poses, constant (:965) */
  const unsigned char *tag_in_map;    /* [n_tag] 1 if a mapping capture saw the tag; NULL = all */
  const int *query_start;             /* [n_query+1] observations of query q, in block order */
  const int *obs_tag;                 /* [n_obs] */
  const double *corners;              /* [n_obs*8] ArucoRect x0,y0,..,x3,y3 (centred px) */
  double *pose;                       /* [n_query*6] inv_pose t_c, w_c: in (init_from_map = 0), out */
  int init_from_map;                  /* 1: localizeOne's initialisation and skip rule */
} arslam_localize_batch;

typedef struct {
  int status;                  /* ARSLAM_CONVERGENCE / _NO_CONVERGENCE / _FAILURE or ARSLAM_LOC_SKIPPED */
  int rule;                    /* ARSLAM_RULE_* */
  int num_iterations;          /* Ceres summary.iterations.size() (iteration 0 included) */
  int num_successful_steps;
  int num_unsuccessful_steps;
  int init_obs;                /* observation used by initCapturePose, -1 if none */
  double initial_cost;
  double final_cost;
} arslam_localize_result;

/* One-shot: upload, solve every query, write poses back into b->pose and
 * one result per query into res (nullable). */
int arslam_localize_many(const arslam_localize_batch *b, const arslam_lm_options *opt,
                         arslam_localize_result *res);

/* Resident form (benchmarks, repeated localisation against one map). */
typedef struct arslam_localizer arslam_localizer;
int arslam_localizer_create(arslam_localizer **out, const arslam_lm_options *opt);
void arslam_localizer_destroy(arslam_localizer *h);
/* upload a batch (the map, the queries and their initial poses) */
int arslam_localizer_load(arslam_localizer *h, const arslam_localize_batch *b);
/* solve every loaded query from the loaded initial state; pose_out [n_query*6]
 * and res [n_query] are nullable (skip the download).  *kernel_ms (nullable)
 * receives the device time of the solve kernel. */
int arslam_localizer_solve(arslam_localizer *h, double *pose_out, arslam_localize_result *res,
                           double *kernel_ms);

#ifdef __cplusplus
}
#endif
#endif
