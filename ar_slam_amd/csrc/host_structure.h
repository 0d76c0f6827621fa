// host_structure.h -- host-only structure of a loaded problem (no HIP):
// capture-major observation CSR, parameter freedom, and the layout + tile
// pattern of the reduced (tag + camera) system.  Used by the solver's load
// and by arslam_debug_reduced_plan (CPU-testable).
#pragma once

#include "arslam_lm.h"

#include <cstdint>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

namespace arslam {

constexpr int kTileRows = 64;
// the most distinct f-blocks (tags; captures under tag elimination) one
// eliminated block may couple: its k_schur wave holds the local system in LDS
// (lm_internal.h schur_lds_bytes; every ArUco dictionary the reference
// supports has at most 250 ids, aruco_detector.cpp:146-150)
constexpr int kMaxSchurBlocks = 256;

// An error with the C-ABI code it maps to.
struct ApiError : std::runtime_error {
  int code;
  ApiError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

// message returned by arslam_lm_last_error() on the calling thread
void set_last_error(const std::string &msg);

inline void api_check(bool ok, int code, const char *msg) {
  if (!ok) throw ApiError(code, msg);
}

// In-place all-reduce hooks of the capture-sharded path (null: one rank).
using ReduceSumF64 = std::function<void(std::vector<double> &)>;
using ReduceMaxU8 = std::function<void(std::vector<uint8_t> &)>;

// Capture-major observation order and parameter freedom.  A block is a
// parameter iff some residual uses it and it is not held constant (Ceres
// removes unused and constant blocks; ar_slam_util.cpp:965,972).  Tag use and
// the observation count are global over ranks (tag_deg_sum).
struct HostProblem {
  int nc = 0, nt = 0, nb = 0;
  long n = 0;                       // 3 + 6 nc + 6 nt parameter slots
  int maxk = 0;                     // most observations in one capture
  int maxblk = 0;                   // most distinct tags of one capture
  std::vector<int> cap_start;       // [nc+1] observations of capture c (capture-major)
  std::vector<int> obs_tag;         // [nb]
  std::vector<int> obs_lblk;        // [nb] 1 + local tag block of the observation in its capture
  std::vector<int> cap_blk_start;   // [nc+1] distinct tags of capture c
  std::vector<int> blk_tag;         // tag of each (capture, local block)
  std::vector<int> tag_start;       // [nt+1] tag CSR over the capture-major order
  std::vector<int> tag_obs;         // [nb]
  std::vector<int> obs_tpos;        // [nb] position of observation q in the tag CSR (tag_obs[obs_tpos[q]] = q)
  std::vector<double> corners;      // [8 nb] capture-major
  std::vector<unsigned char> slot_free, obs_active;
  std::vector<double> x0;           // [n] initial slots
  long nb_global = 0;
  // [3 nt] the reduced blocks' places for the geometric separators (empty: the
  // tag translations in x0); a mixed set's reduced captures sit at the mean of
  // the tags they see (a capture's translation slot is minus its centre)
  std::vector<double> nd_xyz;
};

// Reverse Cuthill-McKee order of an undirected graph (adjacency lists).
std::vector<int> rcm_order(int n, const std::vector<std::vector<int>> &adj);
// Nested-dissection parts (leaves and separators) in elimination order.
// xyz (optional, 3 per node): an embedding for geometric separators; the
// smaller of the geometric and the BFS-level separator is used.
// (fast: components of up to 512 tags try a quarter of the geometric cuts --
// for the reorders of a growing incremental problem)
std::vector<std::vector<int>> nd_parts(int n, const std::vector<std::vector<int>> &adj, int leaf,
                                       const std::vector<double> &xyz = {}, bool fast = false);

HostProblem host_problem(const arslam_soa_problem *p, const ReduceSumF64 &tag_deg_sum);

// Ceres 2.0's e-block set for DENSE_SCHUR with no user ordering
// (ReorderProgramForSchurTypeLinearSolver -> ComputeStableSchurOrdering ->
// StableIndependentSetOrdering), counted by kind; max_tag_obs = most
// observations of one tag; max_cap_blk / max_tag_blk = most distinct tags of
// one capture / captures of one tag (kMaxSchurBlocks bounds the eliminated side's).
struct SchurSide {
  int e_cap = 0, e_tag = 0, e_cam = 0;
  int max_tag_obs = 0;
  int max_cap_blk = 0, max_tag_blk = 0;
};
// (e_cap / e_tag: also the set itself, 1 per eliminated capture / tag)
SchurSide ceres_schur_side(const arslam_soa_problem *p, std::vector<uint8_t> *e_cap = nullptr,
                           std::vector<uint8_t> *e_tag = nullptr);
// the same problem with the roles of captures and tags exchanged (pointers only)
arslam_soa_problem swap_roles(const arslam_soa_problem &p);

// Ceres' exact e-block set when it mixes captures and tags (ARSLAM_ELIM_MIXED),
// as a device problem the per-e-block kernels run unchanged per group:
//   "captures" (groups, the kernels' e-slots): the eliminated captures (kind
//     kMixCap), the eliminated tags (kind kMixTag: roles swapped, as under tag
//     elimination) and, per capture on the reduced side that has residuals
//     with no e-block (both poses on the reduced side), one direct group (kind
//     kMixDirect) holding those residuals -- its own pose is not eliminated:
//     its k_schur wave stores the plain normal-equation blocks, its own pose
//     included as one more local f-block (appended last, mixed_patch);
//   "tags" (f-blocks, the reduced side): every tag and capture outside the
//     set (tags first, then captures).
// A direct group's slot is a copy of its capture's f-block slot: the same
// values, scale and step, summed into the f-block's gradient / column norm
// (f_alias) and left out of the norms (DevProblem::f_own).
enum MixKind : unsigned char { kMixCap = 0, kMixTag = 1, kMixDirect = 2 };
struct MixedProblem {
  arslam_soa_problem soa{};               // the device problem (points into the arrays below)
  std::vector<double> cap, tag;
  std::vector<int> obs_cap, obs_tag;
  std::vector<unsigned char> cap_const, tag_const;
  std::vector<unsigned char> kind;        // [groups]
  std::vector<int> group_src;             // [groups] original capture (kMixCap, kMixDirect) or tag (kMixTag)
  std::vector<int> f_src;                 // [f-blocks] original tag or capture
  std::vector<unsigned char> f_is_cap;    // [f-blocks]
  std::vector<int> f_alias;               // [f-blocks] the direct group copying it, -1
  int n_direct = 0;
  int src_n_cap = 0, src_n_tag = 0;       // the original problem's block counts (reload guard)
};
// p's observations regrouped by the e-set (e_cap / e_tag from ceres_schur_side)
MixedProblem mixed_problem(const arslam_soa_problem &p, const std::vector<uint8_t> &e_cap,
                           const std::vector<uint8_t> &e_tag);
// host_problem(&m.soa) patched: each direct group's own f-block appended to its
// block list, and every f-block free iff its original block is
void mixed_patch(HostProblem &h, const MixedProblem &m, const arslam_soa_problem &p);
// the parameter vector of the mixed device problem from the original blocks
void mixed_values(const MixedProblem &m, const arslam_soa_problem &p, double *x);

// Row layout of the reduced system and its tile pattern (before fill).
//   ordering 0 natural, 1 reverse Cuthill-McKee, 2 nested dissection (parts
//   aligned to 64-row tiles); the camera's 3 rows come last; the rhs is row nR.
struct ReducedLayout {
  std::vector<int> tag_row;         // [nt] first row of tag t, -1 if not a parameter
  std::vector<int> row_slot;        // [nR] parameter slot of each row, -1 for padding
  int cam_row = -1;
  long nR = 0, N = 0;               // rows; N = round_up(nR + 1, 64)
  int T = 0;                        // tiles per side
  std::vector<uint8_t> pattern;     // [T*T] lower tile pattern of the assembled system
  int n_parts = 0;                  // ordering parts (ND: leaves + separators)
  long pad_rows = 0;                // alignment padding rows among the tag rows
  double scalar_flops = 0.0;        // flops of the scalar Cholesky of the real rows in this order
  long n_edges = 0;                 // co-visibility edges (directed) among the free tags
  long order_edges = 0;             // edges when the tag order was computed (n_edges unless reused)
  bool order_reused = false;        // the tag order is the caller's earlier one
};

// Flops of the scalar (row-level) Cholesky of the reduced system in the row
// order tag_row gives, padding excluded: sum over columns of c (c + 1) + c + 1
// with c the column's below-diagonal count from the symbolic factorization of
// the tag co-visibility graph (6x6 dense blocks) plus the dense camera border.
double scalar_cholesky_flops(const std::vector<std::vector<int>> &adj, const std::vector<int> &tag_row,
                             bool camera);

// reuse_tag_row: the tag rows of an earlier layout of the same problem family,
// made when the co-visibility graph had reuse_edges edges; used as is (no new
// ordering) when the set of free tags is unchanged and the graph has grown by
// at most a tenth since -- an incremental solve that only added captures
// keeps its elimination order until the fill it was made for is outdated.
// reuse_by_identity: reuse_tag_row has one entry per tag of h (the earlier
// row of the same block, -1 for a block new to the reduced side) -- a mixed
// set re-chosen on a grown graph (ARSLAM_ELIM_MIXED), whose reduced blocks are
// renumbered; earlier rows of blocks gone from the reduced side stay padding,
// the new blocks go to the end of the last part.
ReducedLayout reduced_layout(const HostProblem &h, int ordering, bool sparse, const ReduceMaxU8 &adj_max,
                             const ReduceMaxU8 &pattern_max,
                             const std::vector<int> *reuse_tag_row = nullptr, long reuse_edges = 0,
                             bool fast_order = false, bool reuse_by_identity = false);

// Deterministic Schur assembly.  k_schur stores capture c's local reduced
// system at slab + cap_off[c] block-packed: local blocks U = 0 (f, 1 row),
// 1..nblk (a tag, 6 rows), nblk+1 (the rhs row); the lower block pairs
// (U >= V) in row-block order, each block contiguous and row-major, so the
// gather of one destination block reads one contiguous run per capture
// (schur_block_off).  k_schur_gather sums, for every destination block of the
// reduced system (global first rows rX >= rY; 1 row for f and the rhs, 6 for
// a tag), the contributing captures' blocks in capture order and stores the
// sum -- plain stores, no atomics, bitwise reproducible.
#if defined(__HIPCC__)
#define ARSLAM_HD __host__ __device__
#else
#define ARSLAM_HD
#endif
struct SchurContrib {
  long off;     // first element of the contributing local block in the slab
  int tr, ld;   // tr: the block is stored transposed (local U < V); ld: its row length
};
// local block of local column x (m = 1 + 6 nblk: the rhs row)
ARSLAM_HD inline int schur_blk(int x, int m) { return x == 0 ? 0 : (x == m ? 1 + (m - 1) / 6 : 1 + (x - 1) / 6); }
ARSLAM_HD inline int schur_blk_size(int U, int nblk) { return (U == 0 || U == nblk + 1) ? 1 : 6; }
ARSLAM_HD inline int schur_blk_start(int U, int nblk) { return U == 0 ? 0 : (U <= nblk ? 1 + 6 * (U - 1) : 1 + 6 * nblk); }
// first element of block (U, V), U >= V: row blocks before U, then the blocks
// (U, V') with V' < V (their columns = the local start of V)
ARSLAM_HD inline long schur_block_off(int U, int V, int nblk) {
  const long R = U == 0 ? 0 : 1 + 6L * (U - 1) + 18L * U * (U - 1);
  return R + (long)schur_blk_size(U, nblk) * schur_blk_start(V, nblk);
}
ARSLAM_HD inline long schur_slab_size(int nblk) { return 3 + 12L * nblk + 18L * nblk * (nblk + 1); }
// A destination with more than kSchurChunk contributions per lane group of its
// k_schur_gather wave (gather_partition) is summed in pieces
// (work items writing partial sums, then one combine per split destination
// adding the pieces in order), so no wave walks a long list serially.
constexpr int kSchurChunk = 64;
struct SchurGather {
  std::vector<long> cap_off;          // [nc+1]
  std::vector<int> dest_row;          // [2 nd] rX, rY
  std::vector<int> dest_start;        // [nd+1] contributions of each destination
  std::vector<SchurContrib> contrib;
  std::vector<int> items;             // [4 ni] {destination, first, end contribution, partial slot or -1}
  std::vector<int> splits;            // [4 ns] {destination, first partial slot, pieces, 0}
  int n_pslots = 0;
  int max_contrib = 0;
};
SchurGather schur_gather_plan(const HostProblem &h, const ReducedLayout &L);
// the same plan, updated for a problem grown by captures [c0, nc) (the captures below c0 unchanged)
void schur_gather_extend(SchurGather &G, const HostProblem &h, const ReducedLayout &L, int c0);

}  // namespace arslam
