// yaml_lite.hpp -- the YAML subset of ar_slam's map files (ArSlamSolver::
// loadYaml / saveYaml, ar_slam_util.cpp:304-465): block mappings and
// sequences, flow sequences of scalars, plain / quoted scalars, comments.
// yaml-cpp is not part of this build; this reader accepts what yaml-cpp's
// emitter writes for that schema (and hand-written equivalents), and the
// writer emits the same layout.
#pragma once

#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace arslam {
namespace yaml {

struct Node {
  enum Kind { Null, Scalar, Seq, Map } kind = Null;
  std::string scalar;
  std::vector<Node> seq;
  std::vector<std::pair<std::string, Node>> map;   // insertion order kept

  bool is_null() const { return kind == Null; }
  // map lookup; throws if missing
  const Node &operator[](const std::string &key) const;
  const Node *find(const std::string &key) const;
  const Node &operator[](size_t i) const;
  size_t size() const { return kind == Seq ? seq.size() : kind == Map ? map.size() : 0; }
  double as_double() const;
  long as_long() const;
  const std::string &as_string() const;
};

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

Node parse(const std::string &text);
Node parse_file(const std::string &path);

// Emitter state for the map-file layout: 2-space indentation, flow
// sequences for numeric arrays, %.17g doubles (round-trip exact).
std::string format_double(double v);
std::string quote_if_needed(const std::string &s);

}  // namespace yaml
}  // namespace arslam
