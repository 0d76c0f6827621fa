/*
 * arslam_slam.h -- C-ABI over the C++ ArSlamSolver mirror
 * (ar_slam_amd/host/ar_slam_solver.hpp), for FFI hosts and the tests.
 *
 * The reference's host surface (ar_slam/include/ar_slam/ar_slam_util.hpp:
 * 361-497) with strings for capture uids / aruco ids and indices for handles:
 *   loadYaml / saveYaml              :374-376
 *   addDetections                    :394-395  (Detections.msg without header/image)
 *   solve / solveIncremental         :384-386
 *   localizeMany                     :392
 *   getTransforms / getCameraInfo    :397-400
 *   at(handle) accessors             :409-416
 * Same conventions as arslam_lm.h (0 / negative ARSLAM_E_*, message in
 * arslam_lm_last_error; a handle is not thread-safe).  Reference methods that
 * throw std::runtime_error return ARSLAM_E_STATE here.
 */
#ifndef ARSLAM_SLAM_H
#define ARSLAM_SLAM_H

#include "arslam_lm.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct arslam_slam arslam_slam;

typedef struct {
  char child_frame_id[128];   /* aruco id or capture uid (truncated); frame_id is "world" */
  double translation[3];
  double rotation[4];         /* w, x, y, z */
} arslam_transform;

int arslam_slam_create(arslam_slam **out, const arslam_lm_options *opt);
void arslam_slam_destroy(arslam_slam *h);
int arslam_slam_set_verbose(arslam_slam *h, int verbose);

int arslam_slam_load_yaml(arslam_slam *h, const char *path);
int arslam_slam_load_yaml_string(arslam_slam *h, const char *text);
int arslam_slam_save_yaml(const arslam_slam *h, const char *path);

/* Detections.msg: n detections, ids[n], corners[n*8] (x0,y0,..,x3,y3, centred
 * pixels).  *capture_idx = the new capture's index, or -1 when the message is
 * ignored (no detections, or an image size different from the map's). */
int arslam_slam_add_detections(arslam_slam *h, const char *capture_uid, int image_width, int image_height,
                               const char *image_path, int n, const char *const *ids,
                               const double *corners, int *capture_idx);

int arslam_slam_solve(arslam_slam *h);
int arslam_slam_solve_incremental(arslam_slam *h);
int arslam_slam_localize_many(arslam_slam *h, int first_loc_cap_idx);

int arslam_slam_num_captures(const arslam_slam *h);
int arslam_slam_num_arucos(const arslam_slam *h);
int arslam_slam_num_blocks(const arslam_slam *h);
int arslam_slam_num_solves(const arslam_slam *h);   /* optimize() calls so far */
int arslam_slam_last_summary(const arslam_slam *h, arslam_lm_summary *s);
/* the summary of optimize() call i (0 <= i < arslam_slam_num_solves) */
int arslam_slam_solve_summary(const arslam_slam *h, int i, arslam_lm_summary *s);

/* the capture whose optimize() was call i (the visiting order of solve /
 * solveIncremental) */
int arslam_slam_solve_capture(const arslam_slam *h, int i, int *capture_idx);
/* the unsolved captures (std::unordered_set<CaptureHandle>, ar_slam_util.hpp:492)
 * in the set's iteration order, begin() first; *n = count (writes <= cap) */
int arslam_slam_unsolved_captures(const arslam_slam *h, int *out, int cap, int *n);

/* capture c: uid (copied, NUL-terminated, truncated to cap), inv_pose[6] */
int arslam_slam_capture(const arslam_slam *h, int c, char *uid, int cap, double inv_pose[6]);
int arslam_slam_set_capture_pose(arslam_slam *h, int c, const double inv_pose[6]);
int arslam_slam_aruco(const arslam_slam *h, int a, char *id, int cap, double pose[6], int *initialized);
int arslam_slam_set_aruco_pose(arslam_slam *h, int a, const double pose[6]);
/* block b: its capture and aruco indices, rect[8], added flag */
int arslam_slam_block(const arslam_slam *h, int b, int *capture, int *aruco, double rect[8], int *added);
int arslam_slam_camera(const arslam_slam *h, double params[3], int *width, int *height);
int arslam_slam_set_camera(arslam_slam *h, const double params[3]);

/* getTransforms: arucos first, then captures; *n = count written (<= cap) */
int arslam_slam_get_transforms(const arslam_slam *h, arslam_transform *out, int cap, int *n);
/* getCameraInfo: K (3x3), P (3x4), row-major; needs a known image size */
int arslam_slam_camera_info(const arslam_slam *h, double k[9], double p[12]);

#ifdef __cplusplus
}
#endif
#endif
