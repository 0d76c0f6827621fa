// slam_capi.cpp -- include/arslam_slam.h over arslam::ArSlamSolver.
#include "arslam_slam.h"

#include "ar_slam_solver.hpp"

#include <cstring>
#include <fstream>
#include <new>
#include <stdexcept>
#include <string>

namespace arslam {
void set_last_error(const std::string &msg);   // lm_solver.hip
}

struct arslam_slam {
  explicit arslam_slam(const arslam_lm_options *o) : s(o) {}
  arslam::ArSlamSolver s;
};

namespace {

template <class F>
int slam_guarded(F &&f) {
  try {
    f();
    return ARSLAM_OK;
  } catch (const std::bad_alloc &) {
    arslam::set_last_error("host out of memory");
    return ARSLAM_E_OUT_OF_MEMORY;
  } catch (const std::out_of_range &e) {
    arslam::set_last_error(std::string("out of range: ") + e.what());
    return ARSLAM_E_INVALID_ARG;
  } catch (const std::exception &e) {
    arslam::set_last_error(e.what());
    return ARSLAM_E_STATE;
  }
}

void copy_str(const std::string &s, char *dst, int cap) {
  if (!dst || cap <= 0) return;
  const size_t n = std::min<size_t>(s.size(), (size_t)cap - 1);
  std::memcpy(dst, s.data(), n);
  dst[n] = '\0';
}

}  // namespace

extern "C" {

int arslam_slam_create(arslam_slam **out, const arslam_lm_options *opt) {
  if (!out) return ARSLAM_E_INVALID_ARG;
  *out = nullptr;
  return slam_guarded([&] { *out = new arslam_slam(opt); });
}

void arslam_slam_destroy(arslam_slam *h) { delete h; }

int arslam_slam_set_verbose(arslam_slam *h, int v) {
  if (!h) return ARSLAM_E_INVALID_ARG;
  h->s.setVerbose(v != 0);
  return ARSLAM_OK;
}

int arslam_slam_load_yaml(arslam_slam *h, const char *path) {
  if (!h || !path) return ARSLAM_E_INVALID_ARG;
  return slam_guarded([&] { h->s.loadYaml(path); });
}

int arslam_slam_load_yaml_string(arslam_slam *h, const char *text) {
  if (!h || !text) return ARSLAM_E_INVALID_ARG;
  return slam_guarded([&] { h->s.loadYamlString(text); });
}

int arslam_slam_save_yaml(const arslam_slam *h, const char *path) {
  if (!h || !path) return ARSLAM_E_INVALID_ARG;
  return slam_guarded([&] {
    std::ofstream f(path);
    if (!f) throw std::runtime_error(std::string("cannot write ") + path);
    h->s.saveYaml(f);
  });
}

int arslam_slam_add_detections(arslam_slam *h, const char *capture_uid, int image_width, int image_height,
                               const char *image_path, int n, const char *const *ids,
                               const double *corners, int *capture_idx) {
  if (!h || !capture_uid || n < 0 || (n && (!ids || !corners)) || image_width < 0 || image_height < 0)
    return ARSLAM_E_INVALID_ARG;
  return slam_guarded([&] {
    arslam::Detections d;
    d.capture_uid = capture_uid;
    d.image_width = (uint32_t)image_width;
    d.image_height = (uint32_t)image_height;
    d.image_path = image_path ? image_path : "";
    for (int i = 0; i < n; ++i) {
      arslam::Detection det;
      det.id = ids[i];
      for (int c = 0; c < 4; ++c) det.corners[c] = arslam::Point{corners[8L * i + 2 * c], corners[8L * i + 2 * c + 1]};
      d.detections.push_back(det);
    }
    auto hnd = h->s.addDetections(d);
    if (capture_idx) *capture_idx = hnd ? (int)hnd->idx : -1;
  });
}

int arslam_slam_solve(arslam_slam *h) {
  if (!h) return ARSLAM_E_INVALID_ARG;
  return slam_guarded([&] { h->s.solve(); });
}

int arslam_slam_solve_incremental(arslam_slam *h) {
  if (!h) return ARSLAM_E_INVALID_ARG;
  return slam_guarded([&] { h->s.solveIncremental(); });
}

int arslam_slam_localize_many(arslam_slam *h, int first) {
  if (!h || first < 0) return ARSLAM_E_INVALID_ARG;
  return slam_guarded([&] { h->s.localizeMany((unsigned)first); });
}

int arslam_slam_num_captures(const arslam_slam *h) { return h ? (int)h->s.numCaptures() : 0; }
int arslam_slam_num_arucos(const arslam_slam *h) { return h ? (int)h->s.numArucos() : 0; }
int arslam_slam_num_blocks(const arslam_slam *h) { return h ? (int)h->s.numBlocks() : 0; }
int arslam_slam_num_solves(const arslam_slam *h) { return h ? (int)h->s.solveLog().size() : 0; }

int arslam_slam_last_summary(const arslam_slam *h, arslam_lm_summary *s) {
  if (!h || !s) return ARSLAM_E_INVALID_ARG;
  if (h->s.solveLog().empty()) return ARSLAM_E_STATE;
  *s = h->s.solveLog().back().summary;
  return ARSLAM_OK;
}

int arslam_slam_solve_summary(const arslam_slam *h, int i, arslam_lm_summary *s) {
  if (!h || !s || i < 0 || i >= (int)h->s.solveLog().size()) return ARSLAM_E_INVALID_ARG;
  *s = h->s.solveLog()[i].summary;
  return ARSLAM_OK;
}

int arslam_slam_solve_capture(const arslam_slam *h, int i, int *capture_idx) {
  if (!h || !capture_idx || i < 0 || i >= (int)h->s.solveLog().size()) return ARSLAM_E_INVALID_ARG;
  *capture_idx = (int)h->s.solveLog()[i].capture_idx;
  return ARSLAM_OK;
}

int arslam_slam_unsolved_captures(const arslam_slam *h, int *out, int cap, int *n) {
  if (!h || !n || (cap > 0 && !out)) return ARSLAM_E_INVALID_ARG;
  int k = 0;
  for (const arslam::CaptureHandle &ch : h->s.unsolvedCaptures()) {
    if (k < cap) out[k] = (int)ch.idx;
    ++k;
  }
  *n = k;
  return ARSLAM_OK;
}

int arslam_slam_capture(const arslam_slam *h, int c, char *uid, int cap, double inv_pose[6]) {
  if (!h || c < 0 || c >= (int)h->s.numCaptures()) return ARSLAM_E_INVALID_ARG;
  const arslam::Capture &cp = h->s.at(arslam::CaptureHandle{(unsigned)c});
  copy_str(cp.uid, uid, cap);
  if (inv_pose) std::memcpy(inv_pose, cp.data(), 6 * sizeof(double));
  return ARSLAM_OK;
}

int arslam_slam_set_capture_pose(arslam_slam *h, int c, const double inv_pose[6]) {
  if (!h || !inv_pose || c < 0 || c >= (int)h->s.numCaptures()) return ARSLAM_E_INVALID_ARG;
  std::memcpy(h->s.at(arslam::CaptureHandle{(unsigned)c}).data(), inv_pose, 6 * sizeof(double));
  return ARSLAM_OK;
}

int arslam_slam_aruco(const arslam_slam *h, int a, char *id, int cap, double pose[6], int *initialized) {
  if (!h || a < 0 || a >= (int)h->s.numArucos()) return ARSLAM_E_INVALID_ARG;
  const arslam::Aruco &ar = h->s.at(arslam::ArucoHandle{(unsigned)a});
  copy_str(ar.id, id, cap);
  if (pose) std::memcpy(pose, ar.data(), 6 * sizeof(double));
  if (initialized) *initialized = ar.initialized ? 1 : 0;
  return ARSLAM_OK;
}

int arslam_slam_set_aruco_pose(arslam_slam *h, int a, const double pose[6]) {
  if (!h || !pose || a < 0 || a >= (int)h->s.numArucos()) return ARSLAM_E_INVALID_ARG;
  std::memcpy(h->s.at(arslam::ArucoHandle{(unsigned)a}).data(), pose, 6 * sizeof(double));
  return ARSLAM_OK;
}

int arslam_slam_block(const arslam_slam *h, int b, int *capture, int *aruco, double rect[8], int *added) {
  if (!h || b < 0 || b >= (int)h->s.numBlocks()) return ARSLAM_E_INVALID_ARG;
  const arslam::Block &bl = h->s.at(arslam::BlockHandle{(unsigned)b});
  if (capture) *capture = (int)bl.capture.idx;
  if (aruco) *aruco = (int)bl.aruco.idx;
  if (rect)
    for (int i = 0; i < 4; ++i) { rect[2 * i] = bl.aruco_rect.corners[i].x; rect[2 * i + 1] = bl.aruco_rect.corners[i].y; }
  if (added) *added = bl.added ? 1 : 0;
  return ARSLAM_OK;
}

int arslam_slam_camera(const arslam_slam *h, double params[3], int *width, int *height) {
  if (!h) return ARSLAM_E_INVALID_ARG;
  const arslam::CameraParams &c = h->s.camera();
  if (params) std::memcpy(params, c.params.data(), 3 * sizeof(double));
  if (width) *width = c.size ? c.size->width : -1;
  if (height) *height = c.size ? c.size->height : -1;
  return ARSLAM_OK;
}

int arslam_slam_set_camera(arslam_slam *h, const double params[3]) {
  if (!h || !params) return ARSLAM_E_INVALID_ARG;
  std::memcpy(h->s.camera().params.data(), params, 3 * sizeof(double));
  return ARSLAM_OK;
}

int arslam_slam_get_transforms(const arslam_slam *h, arslam_transform *out, int cap, int *n) {
  if (!h || !n || cap < 0 || (cap && !out)) return ARSLAM_E_INVALID_ARG;
  return slam_guarded([&] {
    const auto ts = h->s.getTransforms();
    const int m = std::min<int>(cap, (int)ts.size());
    for (int i = 0; i < m; ++i) {
      copy_str(ts[i].child_frame_id, out[i].child_frame_id, (int)sizeof(out[i].child_frame_id));
      std::memcpy(out[i].translation, ts[i].translation, sizeof(ts[i].translation));
      std::memcpy(out[i].rotation, ts[i].rotation, sizeof(ts[i].rotation));
    }
    *n = (int)ts.size();
  });
}

int arslam_slam_camera_info(const arslam_slam *h, double k[9], double p[12]) {
  if (!h || !k || !p) return ARSLAM_E_INVALID_ARG;
  return slam_guarded([&] {
    const auto info = h->s.getCameraInfo();
    std::memcpy(k, info.k.data(), 9 * sizeof(double));
    std::memcpy(p, info.p.data(), 12 * sizeof(double));
  });
}

}  // extern "C"
