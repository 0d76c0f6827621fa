// stl_uset.cpp -- the reference's unsolved-capture container, for the oracle
// driver (TEST INFRASTRUCTURE ONLY; loaded by oracle/driver.py).
//
// ArSlamSolver keeps unsolved captures in std::unordered_set<CaptureHandle>
// (ar_slam_util.hpp:492) whose hash is the handle's index (:140-145), and
// solveIncremental (ar_slam_util.cpp:643, 657-676) visits them in that set's
// iteration order.  The order is libstdc++'s bucket/list order, which a
// restatement can only reproduce by using the same container: this file is
// that container behind a C-ABI (g++ 11's libstdc++, the one Ubuntu 22.04 /
// ros:iron-perception-jammy ships).
#include <unordered_set>
#include <cstddef>

namespace {
struct Handle {   // CaptureHandle (ar_slam_util.hpp)
  unsigned idx;
  bool operator==(const Handle &o) const { return idx == o.idx; }
};
struct HandleHash {   // std::hash<CaptureHandle>, ar_slam_util.hpp:140-145
  size_t operator()(const Handle &h) const { return h.idx; }
};
using Set = std::unordered_set<Handle, HandleHash>;
}  // namespace

extern "C" {
void *or_uset_new() { return new Set(); }
void or_uset_free(void *s) { delete static_cast<Set *>(s); }
void or_uset_insert(void *s, unsigned idx) { static_cast<Set *>(s)->insert(Handle{idx}); }
int or_uset_erase(void *s, unsigned idx) { return (int)static_cast<Set *>(s)->erase(Handle{idx}); }
int or_uset_size(void *s) { return (int)static_cast<Set *>(s)->size(); }
// the elements in iteration order (begin() first); returns the count
int or_uset_list(void *s, unsigned *out) {
  int n = 0;
  for (const Handle &h : *static_cast<Set *>(s)) out[n++] = h.idx;
  return n;
}
}
