// ar_slam_solver.hpp -- C++ host mirror of ar_slam's ArSlamSolver
// (ar_slam/include/ar_slam/ar_slam_util.hpp:361-497) with the MI355X solver
// behind it: the same data store (captures, arucos, blocks, handles, uid
// maps), the same incremental / BFS / localize drivers and initialisers, the
// same YAML map format, and ceres::Problem replaced by the C-ABI of
// include/arslam_lm.h (pointer-keyed residual blocks) and the batched
// localizer of include/arslam_localize.h.
//
// Not mirrored (out of scope): image loading / ArUco
// detection (loadImages, needs OpenCV), the debug display, ROS message types
// (Detections / TransformStamped / CameraInfo are plain structs here).
#pragma once

#include "arslam_lm.h"
#include "arslam_localize.h"

#include <array>
#include <cstdint>
#include <deque>
#include <memory>
#include <optional>
#include <ostream>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace arslam {

struct Point {   // ar_slam_util.hpp:56-63
  double x = 0.0;
  double y = 0.0;
};

struct ImageSize {
  int width = 0;
  int height = 0;
  bool operator==(const ImageSize &o) const { return width == o.width && height == o.height; }
  bool operator!=(const ImageSize &o) const { return !(*this == o); }
};

struct CameraParams {   // :66-78
  std::array<double, 3> params{3000.0, 0.0, 0.0};   // focal, l1, l2 (non-zero initial focal)
  std::optional<ImageSize> size;
};

struct PoseParams {   // :81-94 -- translation then angle-axis
  std::array<double, 6> params{0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
};

struct CaptureHandle {
  unsigned idx = ~0u;
  bool operator==(const CaptureHandle &o) const { return idx == o.idx; }
};
struct CaptureHandleHash {   // std::hash<CaptureHandle>, ar_slam_util.hpp:140-145
  size_t operator()(const CaptureHandle &h) const { return h.idx; }
};
struct ArucoHandle { unsigned idx = ~0u; };
struct BlockHandle { unsigned idx = ~0u; };

struct ArucoRect {   // :265-293, centred pixel coordinates, TL TR BR BL
  std::array<Point, 4> corners;
};

struct Capture {   // :196-227
  std::string uid;
  CaptureHandle handle;
  std::string img_fn;
  std::vector<BlockHandle> blocks;
  std::optional<BlockHandle> init_block;
  PoseParams inv_pose;
  double *data() { return inv_pose.params.data(); }
  const double *data() const { return inv_pose.params.data(); }
};

struct Aruco {   // :229-240
  std::string id;
  ArucoHandle handle;
  bool initialized = false;
  std::vector<BlockHandle> blocks;
  PoseParams pose;
  double *data() { return pose.params.data(); }
  const double *data() const { return pose.params.data(); }
};

struct Block {   // :296-315
  BlockHandle handle;
  ArucoRect aruco_rect;
  CaptureHandle capture;
  ArucoHandle aruco;
  bool added = false;
};

// ar_slam_interfaces/msg/Detection(s).msg without the ROS header and image
struct Detection {
  std::array<Point, 4> corners;
  std::string id;
};
struct Detections {
  std::string capture_uid;
  uint32_t image_height = 0;
  uint32_t image_width = 0;
  std::string image_path;
  std::vector<Detection> detections;
};

// geometry_msgs/TransformStamped subset (getTransforms, :1028-1075)
struct Transform {
  std::string frame_id, child_frame_id;
  double translation[3];
  double rotation[4];   // w, x, y, z
};

// sensor_msgs/CameraInfo subset (getCameraInfo, :1077-1110)
struct CameraInfo {
  uint32_t width = 0, height = 0;
  std::string distortion_model;
  std::array<double, 5> d{};
  std::array<double, 9> k{}, r{};
  std::array<double, 12> p{};
};

// Ceres summary of the last optimize() (the reference prints progress only)
struct SolveRecord {
  std::string capture_uid;
  unsigned capture_idx = ~0u;
  arslam_lm_summary summary;
};

class ArSlamSolver {
 public:
  explicit ArSlamSolver(const arslam_lm_options *opt = nullptr);
  ~ArSlamSolver();
  ArSlamSolver(const ArSlamSolver &) = delete;
  ArSlamSolver &operator=(const ArSlamSolver &) = delete;

  void loadYaml(const std::string &fn);                 // :304-384
  void loadYamlString(const std::string &text);
  void saveYaml(std::ostream &output) const;            // :387-465

  void solve();                                         // BFS from the best capture, :744-866
  void solveIncremental();                              // :629-678
  void localizeMany(unsigned first_loc_cap_idx);        // :888-901 (batched on the device)

  std::string genUniqueCaptureUid() const;              // :286-300
  unsigned getNextCaptureIndex() const { return (unsigned)captures_.size(); }

  std::optional<CaptureHandle> addDetections(const Detections &detections);   // :591-627
  std::vector<Transform> getTransforms() const;         // :1028-1075
  CameraInfo getCameraInfo() const;                     // :1077-1110

  Capture &at(CaptureHandle h) { return captures_.at(h.idx); }
  const Capture &at(CaptureHandle h) const { return captures_.at(h.idx); }
  Aruco &at(ArucoHandle h) { return arucos_.at(h.idx); }
  const Aruco &at(ArucoHandle h) const { return arucos_.at(h.idx); }
  Block &at(BlockHandle h) { return blocks_.at(h.idx); }
  const Block &at(BlockHandle h) const { return blocks_.at(h.idx); }

  size_t numCaptures() const { return captures_.size(); }
  size_t numArucos() const { return arucos_.size(); }
  size_t numBlocks() const { return blocks_.size(); }
  CameraParams &camera() { return camera_; }
  const CameraParams &camera() const { return camera_; }
  std::optional<CaptureHandle> findCapture(const std::string &uid) const;
  std::optional<ArucoHandle> findAruco(const std::string &id) const;
  const std::deque<SolveRecord> &solveLog() const { return solve_log_; }
  const std::unordered_set<CaptureHandle, CaptureHandleHash> &unsolvedCaptures() const { return unsolved_captures_; }
  void setVerbose(bool v) { verbose_ = v; }

  // data-store builders (protected in the reference; public here so a host
  // or test can assemble a problem without ROS messages)
  Capture &addCapture(const std::string &cap_uid, const std::string &fn);   // :419-428
  Aruco &addAruco(const std::string &ar_id);                               // :430-436
  Aruco &getOrAddAruco(const std::string &ar_id);                          // :438-445
  Block &addBlock(const ArucoRect &rect, CaptureHandle cap, ArucoHandle ar);   // :447-457

 protected:
  void localizeOne(Capture &capture, unsigned first_loc_cap_idx);
  void addConnectedCaptures(const Capture &base, std::deque<CaptureHandle> &open);   // :868-886
  void solveCapture(Capture &capture, std::optional<BlockHandle> init_block);    // :680-742
  void addCaptureBlocks(Capture &capture);
  void optimize(const Capture &capture);                                         // :1001-1018
  void resetProblem();                                                           // :1021-1025

  arslam_lm_options options_;
  arslam_lm *problem_ = nullptr;   // was: ceres::Problem problem_ (:473)
  CameraParams camera_;
  std::deque<Capture> captures_;   // stable addresses: the solver keys blocks by pointer
  std::deque<Aruco> arucos_;
  std::vector<Block> blocks_;
  std::unordered_map<std::string, unsigned> capture_map_;
  std::unordered_map<std::string, unsigned> aruco_map_;
  // the reference's container and hash (ar_slam_util.hpp:140-145, 492): solveIncremental
  // visits the unsolved captures in its iteration (bucket) order
  std::unordered_set<CaptureHandle, CaptureHandleHash> unsolved_captures_;
  std::deque<SolveRecord> solve_log_;   // (records are ~90 KB: no reallocation copies)
  bool verbose_ = false;
};

// initialisers (ar_slam_util.cpp:41-128)
void composeAxisAngle(const double *rot1, const double *rot2, double *out);
void calcInitValues(const ArucoRect &rect, double focal, double out[4]);
void initCapturePose(const ArucoRect &rect, const double *camera, const double *ar_pose, double *inv_cap_pose);
void initArPose(const ArucoRect &rect, const double *camera, const double *inv_cap_pose, double *ar_pose);

}  // namespace arslam
