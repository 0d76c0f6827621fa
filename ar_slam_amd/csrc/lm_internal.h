// lm_internal.h -- device problem layout and kernel launch wrappers shared by
// the LM driver (lm_solver.hip), the per-capture kernels (lm_kernels.hip) and
// the reduced-system Cholesky (dense_llt.hip).
//
// Parameter slots (one contiguous f64 vector, x):
//   [0,3)                camera  f, l1, l2
//   [3 + 6c, 9 + 6c)     capture c inv_pose  t_c, w_c
//   [3 + 6Nc + 6t, ...)  tag t pose  t_t, w_t
// Reduced (f-side) rows: tag t -> tag_row[t] + a, camera -> cam_row + b, in an
// ordering chosen on the host (llt_plan.cpp); the camera comes last, so the
// reduced matrix is an arrow-head (sparse tag block + one dense border).
#pragma once
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "host_structure.h"

namespace arslam {
constexpr int kCuFlags = 2048;   // k_factor_dag's per-CU flags: 8 XCCs x 256 (SE, SH, CU) ids
// dag_counters after ready[n_tiles] | applied[n_tiles] (offsets from
// 2 n_tiles): the phase-0 ticket, the claimed-continuation count, the per-CU
// flags, the phase-1 ticket, and the fault record of a timed-out wait
// (kDagFault*: written once, by the workgroup whose fault code won the flag)
constexpr int kDagOffTicket0 = 0;
constexpr int kDagOffInflight = 1;
constexpr int kDagOffCuFlags = 2;
constexpr int kDagOffTicket1 = 2 + kCuFlags;
constexpr int kDagOffFault = 3 + kCuFlags;
enum DagFaultField {
  kFaultTicket = 0,   // the stuck ticket
  kFaultKind = 1,     // 1 dependency (early) wait, 2 in-order application, 3 late wait
  kFaultCounter = 2,  // the awaited counter: ready[c] (c < n_tiles) or applied[c - n_tiles]
  kFaultSeen = 3,     // its value when the wait gave up
  kFaultNeed = 4,     // the value it waited for
  kFaultDrawn = 5,    // tickets drawn by then (the launch's ticket counter)
  kFaultInflight = 6, // claimed continuations in flight
  kFaultBlock = 7,    // the workgroup
  kFaultFirstStuck = 8,   // INT_MAX - the smallest ticket whose wait ran out of time (0: none)
  kDagFaultSlots = 9
};
// workgroups of the phase-0 / phase-1 launch that have started (k_factor_dag's
// claim cap is half of these, not half the grid: DESIGN §8b)
constexpr int kDagOffStarted0 = kDagOffFault + kDagFaultSlots;
constexpr int kDagOffStarted1 = kDagOffStarted0 + 1;
constexpr int kDagCounterExtra = kDagOffStarted1 + 1;
// k_factor_dag workgroups resident per CU (its launch bounds; 73 KB of LDS
// each): a launch never asks for more than this times the CU count
constexpr int kDagWorkgroupsPerCu = 2;

constexpr int kWave = 64;
constexpr int kTile = 64;          // reduced-system Cholesky tile
constexpr int kRowStride = 14;     // LDS row: 13 Jacobian entries + residual
// The stored copy of a row (DevProblem::jrows): 11 values.  The capture- and
// tag-translation columns of a row are the same three numbers (d/dt_c =
// d/dt_t = P M_c: the point is R_t corner + t_t + t_c), so columns 7..9 are
// not stored; column j of the row is stored column jrow_col(j).
constexpr int kJStored = 11;
__host__ __device__ constexpr int jrow_col(int j) {
  return j <= 6 ? j : j <= 9 ? j - 6 : j <= 12 ? j - 3 : 10;
}
// The per-capture kernels take a capture's observations through LDS in
// chunks of kObsChunk (8 observations = one wave's 64 residual rows), so
// k_linearize, k_backsub and the cost take any number of observations per
// capture.  k_schur keeps the capture's local system over its distinct tags
// in LDS: up to kSchurMfmaBlocks tags (m + 1 <= 64 local rows) it forms it as
// one MFMA product in the main launch; captures with more tags run in a second
// launch sized for them, up to kMaxSchurBlocks distinct tags (its LDS at
// schur_lds_bytes(kMaxSchurBlocks) <= 160 KiB, the CU's LDS).
constexpr int kObsChunk = 8;
constexpr int kSchurMfmaBlocks = 10;
// k_schur's dynamic LDS for captures of at most nblk distinct tags (the
// layout at the top of k_schur)
constexpr size_t schur_lds_bytes(int nblk) {
  // stage 6 min(m + 1, 64) | tscale 6 kObsChunk | U 36 | Ui 36 | Etr 8 | W 6 m | Ftr m (+1) | FF 28 nblk |
  // lblk (ints, kObsChunk + 2) | ff00
  return sizeof(double) * (6 * ((6 * nblk + 2) < 64 ? (6 * nblk + 2) : 64) + 6 * kObsChunk + 36 + 36 + 8 +
                           7 * (6 * nblk + 1) + 2 + 28 * nblk) +
         sizeof(int) * (kObsChunk + 2) + 2 * sizeof(double) + 64;
}
static_assert(schur_lds_bytes(kMaxSchurBlocks) <= 160 * 1024, "k_schur's LDS at kMaxSchurBlocks");

// number of per-capture partial sums written by the per-capture kernels
enum PartIdx {
  P_COST = 0,        // sum 0.5|r|^2 over active observations
  P_FIXED = 1,       // same, observations whose blocks are all constant
  P_GF = 2,          // camera-f gradient partial
  P_CF = 3,          // camera-f squared column norm partial
  P_MODEL = 4,       // model cost change partial  p.(r - p/2)
  P_STEP2 = 5,       // squared step norm (capture slots)
  P_YBAD = 6,        // non-finite step flag (max)
  P_CBAD = 7,        // non-finite candidate residual flag (max)
  NPART = 8
};

struct DevProblem {
  int nc, nt, nb;
  long n;              // number of parameter slots 3 + 6nc + 6nt
  long nR;             // rows of the reduced system (tags + camera + alignment padding); row nR = rhs
  long N;              // padded matrix size (multiple of kTile, > nR)
  long lda;            // leading dimension of S
  int max_obs_per_cap;
  int max_blk_per_cap;       // most distinct tags (f-blocks) of one capture
  // captures with more than kSchurMfmaBlocks distinct tags (k_schur's second
  // launch); null when there are none
  const int *big_caps = nullptr;
  int n_big_caps = 0;
  // captures with more than kObsChunk observations (the chunked launches of
  // k_linearize, k_cost and k_backsub); null when there are none
  const int *chunk_caps = nullptr;
  int n_chunk_caps = 0;
  // 1: the e-blocks (the "capture" slots, CSR cap_start) are the problem's tags
  // and the f-blocks (the "tag" slots) its captures -- ARSLAM_ELIM_TAGS: the
  // residual is then evaluated with the two pose arguments exchanged and the
  // two 6-column halves of its Jacobian row swapped back into e|f order
  int swap_roles;
  // ARSLAM_ELIM_MIXED (MixedProblem): each group's kind (kMixCap, kMixTag --
  // roles swapped for that group -- or kMixDirect), and per f-block the direct
  // group whose slot copies it, -1; null otherwise (swap_roles holds for all)
  const unsigned char *cap_kind = nullptr;
  const int *f_alias = nullptr;
  int nf;                    // f-side parameter slots: camera 3 + 6 nt
  const int *fslot_row;      // [nf]    reduced row of f-side slot j (camera j < 3, tag slot 3 + 6 t + a), -1 if none
  int cam_row;               // first reduced row of the camera block, -1 if the camera is not free
  const int *cap_start;      // [nc+1]  CSR of observations by capture
  const int *obs_tag;        // [nb]
  const int *obs_lblk;       // [nb]    local f-block (1..) of the observation's tag in its capture
  const int *cap_blk_start;  // [nc+1]  CSR of distinct tags per capture
  const int *blk_tag;        // [sum]   tag of each local block
  const unsigned char *obs_active;   // [nb]
  const unsigned char *slot_free;    // [n]
  const int *tag_start;      // [nt+1]  CSR of observations by tag (capture-major order inside)
  const int *obs_tpos;       // [nb]    position of each observation in that CSR: k_linearize's per-observation
                             //         tag sums are stored tag-major (obs_tg), so a tag's are contiguous
  const double *corners;     // [nb*8]
  const int *tag_row;        // [nt]    first reduced row of tag t (6 rows), -1 if not free
  const int *row_slot;       // [nR]    parameter slot of a reduced row, -1 for padding rows
  const int *tile_id;        // [T*T]   compact tile index of the reduced system (see LltPlan)
  int T;                     // tiles per side
  // deterministic Schur assembly (SchurGather): packed local systems + gather lists
  const long *cap_off;       // [nc+1]
  double *slab;              // [cap_off[nc]]
  const int2 *dest_row;      // [n_dest] first rows (rX, rY) of each destination block
  const int *dest_start;     // [n_dest+1]
  const SchurContrib *contrib;
  int n_dest;
  const int4 *gather_items;  // [n_items] {destination, first, end contribution, partial slot or -1}
  const int4 *gather_splits; // [n_splits] {destination, first partial slot, pieces, 0}
  double *gather_part;       // [n_pslots * 36]
  int n_items, n_splits;
  // multi-rank: class of each tile column (0 this rank's subtree, 1 the
  // replicated top, 2 another rank's; LltPlan::tile_class), null on one rank
  const signed char *tile_class;
  // several ranks: the f-side slots whose values this rank holds (its own
  // subtree's tags; the replicated top's tags, the camera and the constant
  // tags on rank 0 only), null on one rank: the sums over f-side slots
  // (x^2, the f-side step) count each slot on one rank, and the final tag
  // values are gathered from these
  const unsigned char *f_own = nullptr;
  double *jrows;             // [8 nb kJStored] unscaled Jacobian rows + residual at the linearization point
                             // (column-major per capture: (row, jrow_col(j)) at 8 o0 kJStored + jrow_col(j) 8k + row)
  double *cap_ui;            // [36 nc] (U_c + D_c^2)^{-1} of the current step (k_schur -> k_backsub)
};

// element (r, c), r >= c, of the compact-tiled reduced system
__device__ inline double *reduced_elem(double *S, const DevProblem &P, long r, long c) {
  return S + (long)P.tile_id[(r >> 6) * P.T + (c >> 6)] * 4096 + (r & 63) * 64 + (c & 63);
}

// k_slot_norms' blocks (each one's six partials are reduced by the last to finish)
#ifndef ARSLAM_NORM_BLOCKS
#define ARSLAM_NORM_BLOCKS 64
#endif
constexpr int kNormBlocks = ARSLAM_NORM_BLOCKS;
static_assert(kNormBlocks <= 256 && (kNormBlocks & (kNormBlocks - 1)) == 0, "k_slot_norms: one 256-thread tree");

// Fields of a ticket's record (LltPlan::dag_rec, 32 ints).  -1 where absent.
enum DagRecField {
  kRecType = 0, kRecY, kRecZ, kRecW,           // the task (type, y, z, w)
  kRecSub, kRecLate, kRecWait0, kRecWait1,     // fused TRSM tile, start of the late waits, the wait list
  kRecCont, kRecContAkk, kRecMaxdep,           // continuation target, its A_kk tile, own maxdep
  kRecContMaxdep, kRecContWait0, kRecContLate, // the target's maxdep and early-wait range
  kRecQ0 = 16, kRecQ1,                         // POTRF fold / update item: columns [q0, q1) of ks
  kRecFoldK0, kRecFoldTile0,                   // POTRF: ks[q0] and tid(k, ks[q0])
  kRecSid = 18, kRecTi, kRecTj,                // update item: split slot, target tile (ti, tj)
  kRecSplitN, kRecSplitP,                      // update item of a split target: pieces, first partial slot
  kRecTile0I, kRecTile0J,                      // update item: its first column's operand tile ids
  kDagRecInts = 32
};

// Tile plan of the reduced-system Cholesky (dense_llt.hip), level-scheduled
// over the tile elimination tree.  Device arrays, host per-level offsets.
struct LltPlan {
  // every device array of the plan lives in one grow-only arena (one
  // allocation and one host->device copy per load; kept across re-plans)
  char *arena = nullptr;
  size_t arena_bytes = 0;
  int T = 0;
  long lda = 0;
  int nlev = 0;
  int2 *panel = nullptr;        // (i,k) factor tasks; i == k is the diagonal tile
  int2 *upd_targets = nullptr;  // (i,j) tiles updated by a level
  int *upd_kstart = nullptr;    // CSR over targets of the contributing columns k
  int *upd_ks = nullptr;
  // work items of the update launches: {target, q0, q1, split} -- a target with
  // a long k-list is split into chunks whose partial products go to upd_part
  // and are summed in chunk order by the last-arriving chunk (deterministic)
  int4 *upd_items = nullptr;
  int2 *upd_split = nullptr;    // [n_split] {n_chunks, first partial slot}
  int *upd_cnt = nullptr;       // [n_split] arrival counters (zeroed per factorization)
  double *upd_part = nullptr;   // [n_part * 4096]
  long n_split = 0, n_part = 0;
  std::vector<int> h_item_off;      // [nlev+1]
  int *bs_cols = nullptr;       // backward-solve columns, root level first
  int2 *bs_gather = nullptr;    // (i,k) tiles gathered by each backward level, root level first
  int *bs_gbeg = nullptr;       // [ncols+1] gather range of each backward column (bs_cols order)
  double *bs_part = nullptr;    // [n_gather*64] per-gather partial sums L_ik^T y_i (summed in order)
  int *bs_counters = nullptr;   // [T+1] persistent backward solve: done[column] | ticket
  int *tile_id = nullptr;       // [T*T] compact index of tile (i,j), -1 if structurally zero
  std::vector<int> h_tile_id;
  long n_tiles = 0;             // tiles of the factor (compact storage = n_tiles * 4096 doubles)
  long n_assembled = 0;         // tiles the Schur assembly writes (numbered first; multi-rank: = n_top_tiles)
  bool fill_first_ok = false;   // every fill tile's first application is an unfolded update item (dag_build)
  // multi-rank plans (llt_plan_symbolic with column classes): phase 0 factors
  // this rank's subtree columns, phase 1 the replicated top columns after the
  // exchange of the top tiles (numbered first: tiles [0, n_top_tiles))
  int n_phases = 1;
  long phase_split = 0;         // tickets [0, phase_split) are phase 0
  long n_top_tiles = 0;
  std::vector<int> h_col_class; // [T] 0 own subtree, 1 top, 2 another rank's (not stored)
  std::vector<int> h_dag_phase; // [n_dag_tasks]
  signed char *tile_class = nullptr;   // [T] device copy of h_col_class
  double *ldiag = nullptr;      // 2T x 64 x 64: diagonal factors L_kk, then their inverses (row-major)
  std::vector<int> h_panel_off;     // [nlev+1]
  std::vector<int> h_upd_off;       // [nlev+1]
  std::vector<int> h_bs_off;        // [nlev+1], in backward (root-first) order
  std::vector<int> h_bsg_off;       // [nlev+1], gather tasks per backward level
  std::vector<double> h_upd_flops;  // useful flops of each level's update
  // persistent task-graph executor (launch_dense_llt_dag), host side: tasks
  // in ticket order {type, a, b, c} (0 POTRF k; 1 TRSM i,k; 2 update item a,
  // level sequence b, target tile c), each with a list of {counter, value}
  // waits (h_dag_wait_off); counters = [ready(n_tiles) | applied(n_tiles) |
  // ticket].  h_dag_sub[t] = {tile id of the TRSM fused into POTRF task t or
  // -1, index in the waits where that TRSM's late waits begin}.
  // h_dag_cont[t]: the POTRF task the workgroup finishing POTRF task t may run
  // next (the parent column, whose fold is exactly the tile t solved) or -1;
  // h_dag_maxdep[t]: for such targets the largest ticket t waits on, else -1;
  // h_dag_cont_akk[t]: the storage index of the target's A_kk when the target
  // folds task t's column alone (its A_kk is then all it loads, and task t's
  // workgroup prefetches it beside the fused solve), else -1.
  // dag_claimed[t] (device): taken by the predecessor's workgroup or by the drawer.
  std::vector<int2> h_dag_sub;
  int *dag_claimed = nullptr;
  std::vector<int> h_dag_cont, h_dag_maxdep, h_dag_cont_akk;
  // dag_rec[32 t ..]: every field the executor reads about ticket t, in one
  // 128-byte record (kDagRec* offsets), fetched with two scalar loads -- the
  // separate arrays were a chain of dependent loads (task -> item -> column
  // -> tile id), each a memory round trip under the factorization's traffic.
  // dag_ks_tiles[q]: the operand tile ids {tid(ti, ks[q]), tid(tj, ks[q])} of
  // column q of an update item with target (ti, tj).
  int *dag_rec = nullptr;
  int2 *dag_ks_tiles = nullptr;
  std::vector<int> h_dag_rec;
  std::vector<int2> h_dag_ks_tiles;
  // (dag_counters = [ready | applied | ticket | inflight | kCuFlags per-CU flags | phase-1 ticket |
  //  fault record], kDagOff*)
  int2 *dag_waits = nullptr;
  int *dag_counters = nullptr;
  long n_dag_tasks = 0;
  std::vector<int4> h_dag_tasks;
  std::vector<int> h_dag_wait_off;
  std::vector<int2> h_dag_waits;
  // host copies of the device lists (llt_plan_symbolic)
  std::vector<int2> h_panel, h_targets, h_gather, h_split;
  std::vector<int> h_kstart, h_ks, h_bcols, h_gbeg;
  std::vector<int4> h_items;
  double total_upd_flops = 0.0;
  double total_factor_flops = 0.0;   // updates + POTRF (+ inverse) + TRSM of the task graph
  long total_upd_tiles = 0;
};

// Symbolic tile fill of the lower pattern (T*T bytes, in/out) and the host
// task lists (no HIP calls: usable without a device).
// (col_class: null = one rank; else per tile column 0 this rank's subtree,
// 1 the replicated top, 2 another rank's -- a two-phase plan, see LltPlan)
void llt_plan_symbolic(LltPlan &plan, int T, long lda, std::vector<uint8_t> &pattern,
                       const std::vector<int> *col_class = nullptr);
// symbolic tile-level Cholesky fill (in place) and the tile elimination tree
void tile_fill(int T, std::vector<uint8_t> &pattern, std::vector<int> &parent);
// Subtree-to-rank split of the tile elimination tree (multi-GPU): the top of
// the tree (the upper nested-dissection separators, the camera and the rhs)
// is replicated, the subtrees below it are dealt to the ranks, and every
// capture goes to the rank owning the lowest tile column of its tags (its
// columns lie on one root path: they are pairwise coupled), or, if its tags
// are all in the top, to the rank with the fewest observations so far.
struct RankSplit {
  std::vector<int> col_owner;   // [T] owning rank, -1 = top (replicated)
  std::vector<int> cap_owner;   // [nc]
  int n_top_cols = 0;
  int n_active = 0;             // ranks owning subtrees (the others own top-only captures)
  double top_work = 0.0, max_rank_work = 0.0, total_work = 0.0;   // tile-task counts
  std::vector<int> col_class(int rank) const {   // llt_plan_symbolic's classes
    std::vector<int> c(col_owner.size());
    for (size_t k = 0; k < c.size(); ++k) c[k] = col_owner[k] < 0 ? 1 : (col_owner[k] == rank ? 0 : 2);
    return c;
  }
};
RankSplit rank_split(const HostProblem &h, const ReducedLayout &L, int nranks);
// Ticket-order check of the task graph: executing the tasks one at a time in
// ticket order, is every wait already satisfied when its task runs?
bool dag_check(const LltPlan &plan);
// Randomised (policy 0) or adversarial interleavings of n_workers workgroups
// running k_factor_dag's protocol; false on a reachable deadlock (dag_simulate
// in llt_plan.cpp lists the policies).
// n_started >= 0: only that many of the n_workers workgroups ever start, one
// at a time as the schedule picks them (fewer resident than the grid).
bool dag_simulate(const LltPlan &plan, int n_workers, unsigned seed, int policy = 0, int n_started = -1);
constexpr int kDagSimPolicies = 4;
constexpr int kDagSimNoCap = 16;
constexpr int kDagSimGridCap = 32;   // (tests) round 5's cap: half the grid, not half the started workgroups
// The fault record of a timed-out executor wait (kDagFault*) in words: the
// stuck task, the awaited counter, its producers and how far the launch drew.
std::string dag_fault_detail(const LltPlan &plan, const int *rec);
// Upload the host lists and allocate the plan's device buffers.
void llt_plan_upload(LltPlan &plan, hipStream_t s);
// llt_plan_symbolic + llt_plan_upload
void llt_plan_build(LltPlan &plan, int T, long lda, std::vector<uint8_t> &pattern, hipStream_t s,
                    const std::vector<int> *col_class = nullptr);
void llt_plan_free(LltPlan &plan);                 // device arrays and the arena
void llt_plan_reset(LltPlan &plan);                // host side only; the arena is kept for the next plan


// ---- lm_kernels.hip ----
struct ExecReset;   // (dense_llt section below)
void launch_linearize(const DevProblem &P, const double *x, double *g, double *colnorm,
                      double *obs_tg, double *parts, hipStream_t s);
// k_linearize's reductions in one launch: the per-capture partials into
// out[0..NPART+1] (launch_reduce_parts without fparts) and the tag slots' g and colnorm
// (save: also the cost and fixed cost, out[P_COST], out[P_FIXED], into save[0..1])
void launch_lin_reduce(const DevProblem &P, const double *obs_tg, double *g, double *colnorm,
                       const double *parts, double *out, hipStream_t s, double *hout = nullptr,
                       double *save = nullptr);
struct LmDiagArgs;
// (ld: also the LM diagonal from the new scale, ld->diag / dmin / dmax)
void launch_scale(const DevProblem &P, const double *colnorm, int jacobi, double *scale,
                  hipStream_t s, const LmDiagArgs *ld = nullptr);
void launch_lm_diag(const DevProblem &P, const double *scale, const double *colnorm, double dmin,
                    double dmax, double *diag, hipStream_t s);
// (prep = true: k_prep_reduced's diagonal work is done by the gather itself --
// single rank only, where the gathered S is final)
// (zero_tiles: the first zero_tiles 64x64 tiles of S are cleared by extra
// k_schur blocks before the gather writes S)
// (er: the persistent executors' reset rides along in k_schur's blocks past
// the tiles; only with P.nc > 0)
// k_schur<true>'s dynamic-LDS attribute on the current device (once per device)
void set_schur_big_lds_attribute();
void launch_schur(const DevProblem &P, const double *x, const double *scale, const double *diag,
                  double radius, double *S, hipStream_t s, bool prep = false, long zero_tiles = 0,
                  const ExecReset *er = nullptr);
// (which: -1 every row; 0 / 1 only the rows of tile columns of that class)
void launch_prep_reduced(const DevProblem &P, const double *diag, double radius, double *S,
                         hipStream_t s, int which = -1);
// multi-rank: the backward solve's y before its all-reduce: this rank's
// subtree rows kept, the top rows kept on rank 0 only, every other row 0
// (keep_top: the top rows kept on every rank -- every rank holds the top's y)
void launch_mask_y(const DevProblem &P, double *yF, int rank, hipStream_t s, bool keep_top = false);
// dst[i] = f_own[first + i] ? src[i] : 0 for i < count (several ranks: the values this rank holds)
void launch_own_copy(const DevProblem &P, long first, long count, const double *src, double *dst, hipStream_t s);
void launch_backsub(const DevProblem &P, const double *x, const double *scale, const double *diag,
                    double radius, const double *yF, double *xc, double *parts, hipStream_t s,
                    bool reuse_ui = false, bool with_cost = false);
// candidate f-side slots: xc = x - s yF on reduced rows, xc = x elsewhere (every
// f-side slot is written); fparts: 2 per 256 reduced rows
void launch_update_f(const DevProblem &P, const double *x, const double *scale, const double *yF,
                     double *xc, double *fparts, hipStream_t s);
void launch_cost(const DevProblem &P, const double *x, double *parts, hipStream_t s);
// reduce per-capture partials [NPART][nc] (+ f-slot partials) into out[NPART]
// (flag: also out[NPART + 2] = indefinite (flag > 0), out[NPART + 3] = executor
// fault (flag < 0), out[NPART + 4] = the raw flag)
// (seq_done, seq > 0: with hout, the last block to finish also stores seq into
// hout[kHostSeq] after every block's host words -- the LM loop's host polls that
// word instead of an event; seq_done: a zeroed device int, left zero again)
// x[0..n) into the page-locked dst; the last block stores seq into *word (page-locked,
// after the data; seq_done: a zeroed device int, left zero again)
void launch_copy_out(const double *src, long n, double *dst, int *seq_done, double *word, double seq, hipStream_t s);
void launch_reduce_parts(const double *parts, int nc, const double *fparts, int nfparts,
                         double *out, hipStream_t s, const int *flag = nullptr,
                         double *hout = nullptr, int *seq_done = nullptr, double seq = 0.0);
void debug_set_reduced_diag(const DevProblem &P, double *S, long row, double v, hipStream_t s);
// multi-rank exchange buffers: up to 4 segments packed at offsets off[] of one buffer
struct PackSegs {
  int n = 0;
  double *p[4] = {nullptr, nullptr, nullptr, nullptr};
  long len[4] = {0, 0, 0, 0}, off[4] = {0, 0, 0, 0};
  void add(double *ptr, long count) {
    p[n] = ptr;
    len[n] = count;
    off[n] = n ? off[n - 1] + len[n - 1] : 0;
    ++n;
  }
  long total() const { return n ? off[n - 1] + len[n - 1] : 0; }
};
void launch_pack(const PackSegs &sg, double *buf, bool unpack, hipStream_t s);
// tail[0..m) = g[idx], tail[m..2m) = cn[idx], tail[2m..2m+2) = red[P_GF], red[P_CF] (unpack: the reverse):
// the top tags' linearization sums riding in front of the top tiles' all-reduce
void launch_top_tail(const int *idx, int m, double *g, double *cn, double *red, double *tail, bool unpack,
                     hipStream_t s);
// all-gather of up to kAgFields scalars src[idx[f]] through one SUM all-reduce of
// ag[nranks][kAgFields] (launch_ag_put), combined in rank order by sum, or max
// where bit f of `max` is set (launch_ag_reduce, into dst[idx[f]])
constexpr int kAgFields = 32;
struct AgFields {
  int n = 0;
  int idx[kAgFields] = {};
  unsigned max = 0;
  void add(int i, bool is_max) {
    if (n >= kAgFields) throw std::logic_error("AgFields: more than kAgFields scalars");
    if (is_max) max |= 1u << n;
    idx[n++] = i;
  }
};
void launch_ag_put(const double *src, const AgFields &fl, double *ag, int nranks, int rank, hipStream_t s);
// (several ranks) device ranges stored into page-locked host words by the
// all-gather's combining launch itself, then the sequence number the host
// polls (as one rank's reductions do): no copy launches, no event
struct HostOut {
  const double *src[3] = {};
  double *dst[3] = {};
  int len[3] = {};
  int n = 0;
  double *seq_word = nullptr;
  double seq = 0.0;
  void add(const double *s, double *d, int l) {
    if (n >= 3) throw std::logic_error("HostOut: more than 3 ranges");
    src[n] = s;
    dst[n] = d;
    len[n++] = l;
  }
};
void launch_ag_reduce(const double *ag, const AgFields &fl, double *dst, int nranks, hipStream_t s,
                      const HostOut *ho = nullptr);
// The camera slots of g and colnorm from the reduced partials red (P_GF, P_CF),
// then the norms over free parameter slots: out[0..2] = max|g|, sum g^2, sum x^2
// over capture slots, out[3..5] the same over camera + tag slots.  out[7] is
// the launch's block count (must be zero before the first launch), out[8..]
// its per-block partials.
// (ld: also the LM diagonal clamp(s^2 colnorm) of every slot from ld->scale, into ld->diag)
// (seq > 0: with hout, the last block stores seq into hout[kHostSeq] after the results)
void launch_slot_norms(const DevProblem &P, const double *red, double *g, double *colnorm, const double *x,
                       double *out, hipStream_t s, double *hout = nullptr, const LmDiagArgs *ld = nullptr,
                       double seq = 0.0);
// (hout, in the three launchers above: page-locked host words that also receive
// the results, so a single-rank solve needs no device-to-host copy for them;
// each writer releases them at system scope)
// hout[kHostSeq]: the launch's sequence number, stored last (a host-memory flag:
// a ~8 us kernel-to-host round trip against ~13 us for an event query on
// MI355X, tools/sync_bench.hip)
constexpr int kHostSeq = 15;

// Optional per-launch event pairs around the dominant kernel (trailing update).
struct LaunchTiming {
  hipEvent_t *ev = nullptr;   // 2 * cap events
  int cap = 0;
  int used = 0;
  double flops = 0.0;         // algorithmic flops of the recorded launches
};

// ---- dense_llt.hip ----
// Cholesky of the lower triangle of S (row-major, lda) over the plan's tiles,
// in place.  Row nR carries the right-hand side, so on exit row nR =
// (L^{-1} b)^T.  *flag is set non-zero if a pivot is not positive.  Then
// y = L^{-T} z into yF[0..nR).
void launch_dense_llt(const LltPlan &P, double *S, int *flag, hipStream_t s,
                      LaunchTiming *timing = nullptr);
// The same factorization as one persistent launch over the plan's task graph
// (tickets in a topological order, dependency counters in global memory).
// (reset = false: the counters were zeroed by launch_exec_reset)
// (phase: -1 every task; 0 / 1 one phase of a multi-rank plan, LltPlan)
// (first_store: the tiles from first_store on are fill tiles the Schur gather
// does not write and S is not cleared for -- their first update stores
// instead of reading the tile; LONG_MAX: none)
// debug: only the first k workgroups of every k_factor_dag launch start (the
// others return at once; k <= 0 restores all), process-wide
void set_dag_workgroup_limit(int k);
void launch_dense_llt_dag(const LltPlan &P, double *S, int *flag, hipStream_t s, int n_workgroups,
                          int *progress = nullptr, unsigned long long *trace = nullptr, bool reset = true,
                          int phase = -1, long first_store = LONG_MAX);
// the LM diagonal clamp(s^2 colnorm, dmin, dmax) over n slots (k_lm_diag)
struct LmDiagArgs {
  long n;
  const double *scale, *colnorm;
  double dmin, dmax;
  double *diag;
  double *ysent = nullptr;   // (also: the backward solve's y, nys rows, to kYSentinel)
  long nys = 0;
};
// k_bsolve_dag's "not solved yet" value of a y entry: a signalling-NaN bit
// pattern no arithmetic produces (those NaNs are quiet)
constexpr unsigned long long kYSentinel = 0x7ff47ff47ff47ff4ull;
// *flag and every counter of the two persistent executors to zero, one launch
// (with ld: the LM diagonal in the same launch)
void launch_exec_reset(const LltPlan &P, int *flag, hipStream_t s, const LmDiagArgs *ld = nullptr);
// The same reset as element-wise work another launch can carry (k_schur's
// blocks past the captures and tiles, when the diagonal needs no update):
// element e < n() zeroes one counter / writes one y sentinel; e == 0 also the flag.
struct ExecReset {
  int *flag = nullptr;
  int *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
  long na = 0, nb = 0, nc = 0, nd = 0;
  double *ysent = nullptr;
  long nys = 0;
  __host__ __device__ long n() const { return na + nb + nc + nd > nys ? na + nb + nc + nd : nys; }
};
ExecReset exec_reset_args(const LltPlan &P, int *flag, double *ysent, long nys);
__device__ __forceinline__ void exec_reset_elem(const ExecReset &r, long e) {
  if (e < r.nys) r.ysent[e] = __longlong_as_double((long long)kYSentinel);
  if (e < r.na) r.a[e] = 0;
  else if (e < r.na + r.nb) r.b[e - r.na] = 0;
  else if (e < r.na + r.nb + r.nc) r.c[e - r.na - r.nb] = 0;
  else if (e < r.na + r.nb + r.nc + r.nd) r.d[e - r.na - r.nb - r.nc] = 0;
  if (e == 0 && r.flag) *r.flag = 0;
}
void launch_dense_back_solve(const LltPlan &P, const double *S, long nR, double *z, double *yF,
                             const int *flag, hipStream_t s);
// The same backward solve as one persistent launch (columns in root-first
// ticket order, per-column completion counters).
void launch_dense_back_solve_dag(const LltPlan &P, const double *S, long nR, double *yF, int *flag,
                                 hipStream_t s, int n_workgroups, bool reset = true);
void launch_zero_tiles(const LltPlan &P, double *S, hipStream_t s);
// copy the diagonal factors L_kk into S (tests only: S then holds the whole factor)
void launch_scatter_diag(const LltPlan &P, double *S, hipStream_t s);

}  // namespace arslam
