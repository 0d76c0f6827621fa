// ar_slam_solver.cpp -- see ar_slam_solver.hpp.  Each method cites the
// reference function it restates (ar_slam/src/ar_slam_util.cpp).
#include "ar_slam_solver.hpp"

#include "yaml_lite.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>

namespace arslam {

namespace {

constexpr double kArucoSize = 0.0635;   // ar_slam_util.hpp:319
constexpr double kDirections[4][2] = {{-1.0, -1.0}, {1.0, -1.0}, {1.0, 1.0}, {-1.0, 1.0}};   // :340-345

void check(int rc) {
  if (rc < 0) throw std::runtime_error(std::string("arslam_lm: ") + arslam_lm_last_error());
}

double normalize_angle(double a) {   // ar_slam_util.hpp:348-351
  return std::fmod(std::fmod(a, 2 * M_PI) + 3 * M_PI, 2 * M_PI) - M_PI;
}

// Ceres 2.0 rotation.h
void aa_to_quat(const double aa[3], double q[4]) {
  const double theta_sq = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta_sq > 0.0) {
    const double theta = std::sqrt(theta_sq), half = theta * 0.5, k = std::sin(half) / theta;
    q[0] = std::cos(half);
    q[1] = aa[0] * k; q[2] = aa[1] * k; q[3] = aa[2] * k;
  } else {
    q[0] = 1.0;
    q[1] = aa[0] * 0.5; q[2] = aa[1] * 0.5; q[3] = aa[2] * 0.5;
  }
}

void quat_to_aa(const double q[4], double aa[3]) {
  const double sin_sq = q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  double k = 2.0;
  if (sin_sq > 0.0) {
    const double s = std::sqrt(sin_sq), c = q[0];
    const double two_theta = 2.0 * ((c < 0.0) ? std::atan2(-s, -c) : std::atan2(s, c));
    k = two_theta / s;
  }
  aa[0] = q[1] * k; aa[1] = q[2] * k; aa[2] = q[3] * k;
}

void angle_axis_rotate(const double w[3], const double p[3], double out[3]) {
  const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  if (th2 > 2.220446049250313e-16) {   // DBL_EPSILON branch of AngleAxisRotatePoint
    const double th = std::sqrt(th2), c = std::cos(th), s = std::sin(th), ti = 1.0 / th;
    const double u[3] = {w[0] * ti, w[1] * ti, w[2] * ti};
    const double cr[3] = {u[1] * p[2] - u[2] * p[1], u[2] * p[0] - u[0] * p[2], u[0] * p[1] - u[1] * p[0]};
    const double tmp = (u[0] * p[0] + u[1] * p[1] + u[2] * p[2]) * (1.0 - c);
    for (int i = 0; i < 3; ++i) out[i] = p[i] * c + cr[i] * s + u[i] * tmp;
  } else {
    const double cr[3] = {w[1] * p[2] - w[2] * p[1], w[2] * p[0] - w[0] * p[2], w[0] * p[1] - w[1] * p[0]};
    for (int i = 0; i < 3; ++i) out[i] = p[i] + cr[i];
  }
}

}  // namespace

// ---- initialisers, ar_slam_util.cpp:41-128 ----

void composeAxisAngle(const double *rot1, const double *rot2, double *out) {   // :41-50
  double q1[4], q2[4], q3[4];
  aa_to_quat(rot1, q1);
  aa_to_quat(rot2, q2);
  q3[0] = q1[0] * q2[0] - q1[1] * q2[1] - q1[2] * q2[2] - q1[3] * q2[3];
  q3[1] = q1[0] * q2[1] + q1[1] * q2[0] + q1[2] * q2[3] - q1[3] * q2[2];
  q3[2] = q1[0] * q2[2] - q1[1] * q2[3] + q1[2] * q2[0] + q1[3] * q2[1];
  q3[3] = q1[0] * q2[3] + q1[1] * q2[2] - q1[2] * q2[1] + q1[3] * q2[0];
  quat_to_aa(q3, out);
}

void calcInitValues(const ArucoRect &rect, double focal, double out[4]) {   // :52-95
  double max_dist_sq = 0.0, avg_x = 0.0, avg_y = 0.0;
  for (unsigned i = 0; i < 4; ++i) {
    const Point &p1 = rect.corners[i], &p2 = rect.corners[(i + 1) & 3];
    const double d = std::pow(p1.x - p2.x, 2) + std::pow(p1.y - p2.y, 2);
    max_dist_sq = std::max(d, max_dist_sq);
    avg_x += p1.x;
    avg_y += p1.y;
  }
  avg_x *= 0.25;
  avg_y *= 0.25;
  double avg_angle = 0.0;
  for (unsigned i = 0; i < 4; ++i) {
    const Point &pt = rect.corners[i];
    const double expected = std::atan2(kDirections[i][1], kDirections[i][0]);
    const double actual = std::atan2(pt.y - avg_y, pt.x - avg_x);
    const double delta = normalize_angle(actual - expected);
    avg_angle += normalize_angle(delta - avg_angle) / (i + 1);
  }
  const double local_z = focal * kArucoSize / std::sqrt(max_dist_sq);
  out[0] = avg_x * local_z / focal;
  out[1] = avg_y * local_z / focal;
  out[2] = local_z;
  out[3] = avg_angle;
}

void initCapturePose(const ArucoRect &rect, const double *camera, const double *ar_pose,
                     double *inv) {   // :98-115
  double v[4];
  calcInitValues(rect, camera[0], v);
  const double local_position[3] = {v[0], v[1], v[2]};
  const double local_rot[3] = {0.0, 0.0, v[3]};
  const double inv_ar_rot[3] = {-ar_pose[3], -ar_pose[4], -ar_pose[5]};
  composeAxisAngle(local_rot, inv_ar_rot, inv + 3);
  const double cap_rotation[3] = {-inv[3], -inv[4], -inv[5]};
  angle_axis_rotate(cap_rotation, local_position, inv);
  inv[0] -= ar_pose[0];
  inv[1] -= ar_pose[1];
  inv[2] -= ar_pose[2];
}

void initArPose(const ArucoRect &rect, const double *camera, const double *inv,
                double *ar_pose) {   // :118-128
  double v[4];
  calcInitValues(rect, camera[0], v);
  const double local_position[3] = {v[0], v[1], v[2]};
  const double cap_rotation[3] = {-inv[3], -inv[4], -inv[5]};
  angle_axis_rotate(cap_rotation, local_position, ar_pose);
  ar_pose[0] -= inv[0];
  ar_pose[1] -= inv[1];
  ar_pose[2] -= inv[2];
  const double local_rot[3] = {0.0, 0.0, v[3]};
  const double cap_rot[3] = {-inv[3], -inv[4], -inv[5]};
  composeAxisAngle(cap_rot, local_rot, ar_pose + 3);
}

// ---- ArSlamSolver ----

ArSlamSolver::ArSlamSolver(const arslam_lm_options *opt) {
  if (opt) options_ = *opt;
  else arslam_lm_options_init(&options_);
  check(arslam_lm_create(&problem_, &options_));
}

ArSlamSolver::~ArSlamSolver() { arslam_lm_destroy(problem_); }

Capture &ArSlamSolver::addCapture(const std::string &cap_uid, const std::string &fn) {   // :419-428
  const unsigned idx = (unsigned)captures_.size();
  if (!capture_map_.emplace(cap_uid, idx).second) throw std::runtime_error("Capture with uid already added");
  captures_.emplace_back();
  Capture &c = captures_.back();
  c.uid = cap_uid;
  c.handle = CaptureHandle{idx};
  c.img_fn = fn;
  return c;
}

Aruco &ArSlamSolver::addAruco(const std::string &ar_id) {   // :430-436
  const unsigned idx = (unsigned)arucos_.size();
  aruco_map_.emplace(ar_id, idx);
  arucos_.emplace_back();
  Aruco &a = arucos_.back();
  a.id = ar_id;
  a.handle = ArucoHandle{idx};
  return a;
}

Aruco &ArSlamSolver::getOrAddAruco(const std::string &ar_id) {   // :438-445
  auto it = aruco_map_.find(ar_id);
  if (it == aruco_map_.end()) return addAruco(ar_id);
  return arucos_[it->second];
}

Block &ArSlamSolver::addBlock(const ArucoRect &rect, CaptureHandle cap, ArucoHandle ar) {   // :447-457
  const BlockHandle h{(unsigned)blocks_.size()};
  blocks_.push_back(Block{h, rect, cap, ar, false});
  at(cap).blocks.push_back(h);
  at(ar).blocks.push_back(h);
  return blocks_.back();
}

std::optional<CaptureHandle> ArSlamSolver::findCapture(const std::string &uid) const {
  auto it = capture_map_.find(uid);
  if (it == capture_map_.end()) return std::nullopt;
  return CaptureHandle{it->second};
}

std::optional<ArucoHandle> ArSlamSolver::findAruco(const std::string &id) const {
  auto it = aruco_map_.find(id);
  if (it == aruco_map_.end()) return std::nullopt;
  return ArucoHandle{it->second};
}

std::string ArSlamSolver::genUniqueCaptureUid() const {   // :286-300
  const std::string base = "cap_" + std::to_string(captures_.size());
  if (!capture_map_.count(base)) return base;
  for (unsigned idx = 0; idx < 1000; ++idx) {
    const std::string uid = base + "_" + std::to_string(idx);
    if (!capture_map_.count(uid)) return uid;
  }
  throw std::runtime_error("cannot generate unique id");
}

void ArSlamSolver::loadYaml(const std::string &fn) {
  std::ifstream f(fn);
  if (!f) throw std::runtime_error("cannot open " + fn);
  std::stringstream ss;
  ss << f.rdbuf();
  loadYamlString(ss.str());
}

void ArSlamSolver::loadYamlString(const std::string &text) {   // :304-384
  const yaml::Node doc = yaml::parse(text);
  if (const yaml::Node *caps = doc.find("captures")) {
    for (const auto &kv : caps->map) {
      if (capture_map_.count(kv.first))
        throw std::runtime_error("capture with id CaptureUid:" + kv.first + " already exists");
      Capture &capture = addCapture(kv.first, kv.second["img_fn"].as_string());
      const yaml::Node &ip = kv.second["inv_pose"];
      for (size_t i = 0; i < capture.inv_pose.params.size(); ++i) capture.inv_pose.params[i] = ip[i].as_double();
    }
  }
  if (const yaml::Node *ars = doc.find("arucos")) {
    for (const auto &kv : ars->map) {
      Aruco &aruco = addAruco(kv.first);
      const yaml::Node &pd = kv.second["pose"];
      for (size_t i = 0; i < aruco.pose.params.size(); ++i) aruco.pose.params[i] = pd[i].as_double();
    }
  }
  if (const yaml::Node *blocks = doc.find("blocks")) {
    for (const yaml::Node &bd : blocks->seq) {
      auto ci = capture_map_.find(bd["capture"].as_string());
      auto ai = aruco_map_.find(bd["aruco"].as_string());
      if (ci == capture_map_.end() || ai == aruco_map_.end()) throw std::out_of_range("unordered_map::at");
      const yaml::Node &rd = bd["aruco_rect"];
      ArucoRect rect;
      if (rd.size() != 2 * rect.corners.size()) throw std::runtime_error("aruco_rect has wrong number of values");
      for (unsigned i = 0; i < rect.corners.size(); ++i) {
        rect.corners[i].x = rd[2 * i].as_double();
        rect.corners[i].y = rd[2 * i + 1].as_double();
      }
      addBlock(rect, CaptureHandle{ci->second}, ArucoHandle{ai->second});
    }
  }
  {
    const yaml::Node &cam = doc["camera"];
    camera_.size = ImageSize{(int)cam["width"].as_long(), (int)cam["height"].as_long()};
    const yaml::Node &cp = cam["params"];
    for (size_t i = 0; i < cp.size(); ++i) camera_.params.at(i) = cp[i].as_double();
  }
}

void ArSlamSolver::saveYaml(std::ostream &y) const {   // :387-465 (yaml-cpp emitter layout)
  using yaml::format_double;
  using yaml::quote_if_needed;
  auto flow = [&](const double *v, size_t n) {
    y << "[";
    for (size_t i = 0; i < n; ++i) y << (i ? ", " : "") << format_double(v[i]);
    y << "]";
  };
  y << "blocks:";
  if (blocks_.empty()) y << " []";
  y << "\n";
  for (const Block &b : blocks_) {
    y << "  - capture: " << quote_if_needed(at(b.capture).uid) << "\n";
    y << "    aruco: " << quote_if_needed(at(b.aruco).id) << "\n";
    double xy[8];
    for (int i = 0; i < 4; ++i) { xy[2 * i] = b.aruco_rect.corners[i].x; xy[2 * i + 1] = b.aruco_rect.corners[i].y; }
    y << "    aruco_rect: ";
    flow(xy, 8);
    y << "\n";
  }
  y << "captures:";
  if (captures_.empty()) y << " {}";
  y << "\n";
  for (const Capture &c : captures_) {
    y << "  " << quote_if_needed(c.uid) << ":\n    inv_pose: ";
    flow(c.inv_pose.params.data(), 6);
    y << "\n    img_fn: " << (c.img_fn.empty() ? std::string("\"\"") : quote_if_needed(c.img_fn)) << "\n";
  }
  y << "arucos:";
  if (arucos_.empty()) y << " {}";
  y << "\n";
  for (const Aruco &a : arucos_) {
    y << "  " << quote_if_needed(a.id) << ":\n    pose: ";
    flow(a.pose.params.data(), 6);
    y << "\n";
  }
  y << "camera:\n  params: ";
  flow(camera_.params.data(), 3);
  y << "\n";
  if (camera_.size) y << "  width: " << camera_.size->width << "\n  height: " << camera_.size->height << "\n";
  y << std::endl;
}

std::optional<CaptureHandle> ArSlamSolver::addDetections(const Detections &d) {   // :591-627
  if (d.detections.empty()) return std::nullopt;
  const ImageSize image_size{(int)d.image_width, (int)d.image_height};
  if (camera_.size) {
    if (*camera_.size != image_size) {
      std::cerr << "WARN Mismatched image size" << std::endl;
      return std::nullopt;
    }
  } else {
    camera_.size = image_size;
  }
  Capture &capture = addCapture(d.capture_uid, d.image_path);   // duplicate uid throws (:419-428)
  for (const Detection &det : d.detections) {
    Aruco &aruco = getOrAddAruco(det.id);
    ArucoRect rect;
    rect.corners = det.corners;
    addBlock(rect, capture.handle, aruco.handle);
  }
  unsolved_captures_.insert(capture.handle);
  return capture.handle;
}

void ArSlamSolver::solveIncremental() {   // :629-678
  // make sure at least one capture is solved: the seed is the set's begin()
  // (libstdc++ bucket order, as in the reference)
  if (!unsolved_captures_.empty() && unsolved_captures_.size() == captures_.size()) {
    const CaptureHandle ch = *unsolved_captures_.begin();
    unsolved_captures_.erase(ch);
    solveCapture(at(ch), std::nullopt);
  }
  bool repeat_solve;
  do {
    repeat_solve = false;
    for (auto itr = unsolved_captures_.begin(); itr != unsolved_captures_.end(); ++itr) {
      Capture &capture = at(*itr);
      for (BlockHandle bh : capture.blocks) {
        if (at(at(bh).aruco).initialized) {
          repeat_solve = true;
          itr = unsolved_captures_.erase(itr);
          solveCapture(capture, bh);
          break;
        }
      }
      // as in the reference, the element after an erased one is skipped by
      // the loop increment (it is revisited on the next pass)
      if (itr == unsolved_captures_.end()) break;
    }
  } while (repeat_solve);
}

void ArSlamSolver::addCaptureBlocks(Capture &capture) {   // block loop of :704-735 / :826-843
  for (BlockHandle bh : capture.blocks) {
    Block &block = at(bh);
    Aruco &aruco = at(block.aruco);
    if (!aruco.initialized) {
      aruco.initialized = true;
      initArPose(block.aruco_rect, camera_.params.data(), capture.data(), aruco.data());
    }
    if (block.added) throw std::runtime_error("block for capture was somehow already added?");
    block.added = true;
    double xy[8];
    for (int i = 0; i < 4; ++i) { xy[2 * i] = block.aruco_rect.corners[i].x; xy[2 * i + 1] = block.aruco_rect.corners[i].y; }
    // was: problem_.AddResidualBlock(AutoDiffCostFunction<ArucoReprojectionError,8,3,6,6>, nullptr, ...)
    check(arslam_lm_add_residual_block(problem_, xy, camera_.params.data(), capture.data(), aruco.data()));
  }
}

void ArSlamSolver::solveCapture(Capture &capture, std::optional<BlockHandle> init_block) {   // :680-742
  if (init_block) {
    const Block &block = at(*init_block);
    initCapturePose(block.aruco_rect, camera_.params.data(), at(block.aruco).data(), capture.data());
  }
  addCaptureBlocks(capture);
  optimize(capture);
}

void ArSlamSolver::solve() {   // :744-866
  if (captures_.empty()) return;
  std::deque<CaptureHandle> open_captures;
  unsigned best_cap_idx = 0;
  {
    size_t best = captures_.front().blocks.size();
    for (unsigned i = 1; i < captures_.size(); ++i)
      if (captures_[i].blocks.size() > best) { best = captures_[i].blocks.size(); best_cap_idx = i; }
  }
  Capture &best_capture = captures_[best_cap_idx];
  best_capture.init_block = BlockHandle{~0u};   // prevents the capture from being added again
  open_captures.push_back(best_capture.handle);
  while (!open_captures.empty()) {
    const CaptureHandle ch = open_captures.front();
    open_captures.pop_front();
    Capture &capture = at(ch);
    if (ch.idx != best_cap_idx) {
      const Block &block = at(*capture.init_block);
      initCapturePose(block.aruco_rect, camera_.params.data(), at(block.aruco).data(), at(block.capture).data());
    }
    addCaptureBlocks(capture);
    optimize(capture);
    addConnectedCaptures(capture, open_captures);
  }
}

void ArSlamSolver::addConnectedCaptures(const Capture &base, std::deque<CaptureHandle> &open) {   // :868-886
  for (BlockHandle bbh : base.blocks) {
    const Aruco &base_aruco = at(at(bbh).aruco);
    for (BlockHandle bh : base_aruco.blocks) {
      Capture &capture = at(at(bh).capture);
      if (!capture.init_block) {
        capture.init_block = bh;
        open.push_back(capture.handle);
      }
    }
  }
}

void ArSlamSolver::localizeMany(unsigned first_loc_cap_idx) {   // :888-901, each query as localizeOne :903-979
  // Every localizeOne resets the problem and holds the tags and the camera
  // constant, so the queries are independent: they run as one device batch.
  const unsigned n = (unsigned)captures_.size();
  if (first_loc_cap_idx >= n) return;
  std::vector<unsigned char> in_map(arucos_.size(), 0);
  for (const Aruco &a : arucos_)
    for (BlockHandle bh : a.blocks)
      if (at(bh).capture.idx < first_loc_cap_idx) { in_map[a.handle.idx] = 1; break; }
  std::vector<double> tags(6 * std::max<size_t>(arucos_.size(), 1));
  for (const Aruco &a : arucos_) std::copy(a.pose.params.begin(), a.pose.params.end(), tags.begin() + 6 * a.handle.idx);
  std::vector<int> q_start{0}, obs_tag;
  std::vector<double> corners, pose;
  std::vector<unsigned> qcap;
  for (unsigned ci = first_loc_cap_idx; ci < n; ++ci) {
    Capture &capture = captures_[ci];
    for (BlockHandle bh : capture.blocks) {
      Block &block = at(bh);
      if (block.added) throw std::runtime_error("block for capture was somehow already added?");
      obs_tag.push_back((int)block.aruco.idx);
      for (const Point &p : block.aruco_rect.corners) { corners.push_back(p.x); corners.push_back(p.y); }
    }
    q_start.push_back((int)obs_tag.size());
    pose.insert(pose.end(), capture.inv_pose.params.begin(), capture.inv_pose.params.end());
    qcap.push_back(ci);
  }
  arslam_localize_batch b{};
  b.n_query = (int)qcap.size();
  b.n_tag = (int)arucos_.size();
  b.n_obs = (int)obs_tag.size();
  b.camera = camera_.params.data();
  b.tag = tags.data();
  b.tag_in_map = in_map.data();
  b.query_start = q_start.data();
  b.obs_tag = obs_tag.data();
  b.corners = corners.data();
  b.pose = pose.data();
  b.init_from_map = 1;
  std::vector<arslam_localize_result> res(std::max<size_t>(qcap.size(), 1));
  check(arslam_localize_many(&b, &options_, res.data()));
  for (size_t q = 0; q < qcap.size(); ++q) {
    Capture &capture = captures_[qcap[q]];
    if (res[q].status == ARSLAM_LOC_SKIPPED) {
      if (verbose_) std::cout << "WARNING : Cannot find connected ar tags for capture " << qcap[q] << std::endl;
      continue;
    }
    for (BlockHandle bh : capture.blocks) at(bh).added = true;
    std::copy(pose.begin() + 6 * q, pose.begin() + 6 * q + 6, capture.inv_pose.params.begin());
  }
}

void ArSlamSolver::optimize(const Capture &capture) {   // :1001-1018
  arslam_lm_options o = options_;
  o.max_num_iterations = 50;                      // :1004
  // DENSE_SCHUR (:1011) eliminates Ceres' own e-block set: ARSLAM_ELIM_MIXED
  // unless the caller asked for a side (round 6: a grown problem whose new
  // captures see only reduced tags appends to the set, and a reload keeps the
  // earlier order by block -- the cfg2 flow 1.16x the all-captures one,
  // DESIGN.md §2, §7b)
  if (o.elimination == ARSLAM_ELIM_AUTO) o.elimination = ARSLAM_ELIM_MIXED;
  o.minimizer_progress_to_stdout = verbose_ ? 1 : 0;
  check(arslam_lm_set_options(problem_, &o));
  SolveRecord rec;
  rec.capture_uid = capture.uid;
  rec.capture_idx = capture.handle.idx;
  check(arslam_lm_solve(problem_, &rec.summary));
  solve_log_.push_back(std::move(rec));
}

void ArSlamSolver::resetProblem() { check(arslam_lm_reset(problem_)); }   // :1021-1025

std::vector<Transform> ArSlamSolver::getTransforms() const {   // :1028-1075
  std::vector<Transform> out;
  out.reserve(captures_.size() + arucos_.size());
  for (const Aruco &a : arucos_) {
    Transform t{};
    t.frame_id = "world";
    t.child_frame_id = a.id;
    for (int i = 0; i < 3; ++i) t.translation[i] = a.pose.params[i];
    aa_to_quat(&a.pose.params[3], t.rotation);
    out.push_back(t);
  }
  for (const Capture &c : captures_) {
    Transform t{};
    t.frame_id = "world";
    t.child_frame_id = c.uid;
    const double rot[3] = {-c.inv_pose.params[3], -c.inv_pose.params[4], -c.inv_pose.params[5]};
    aa_to_quat(rot, t.rotation);
    for (int i = 0; i < 3; ++i) t.translation[i] = -c.inv_pose.params[i];
    out.push_back(t);
  }
  return out;
}

CameraInfo ArSlamSolver::getCameraInfo() const {   // :1077-1126
  if (!camera_.size) throw std::bad_optional_access();
  CameraInfo info;
  info.distortion_model = "plumb_bob";
  const double fx = camera_.params[0], fy = camera_.params[0];
  const double cx = camera_.size->width * 0.5, cy = camera_.size->height * 0.5;
  info.k = {fx, 0.0, cx, 0.0, fy, cy, 0.0, 0.0, 1.0};
  info.r = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0};
  info.p = {fx, 0.0, cx, 0.0, 0.0, fy, cy, 0.0, 0.0, 0.0, 1.0, 0.0};
  return info;
}

}  // namespace arslam
