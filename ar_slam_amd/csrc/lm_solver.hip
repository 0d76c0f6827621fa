// lm_solver.hip -- host side of the MI355X LM bundle adjuster and its C-ABI
// (include/arslam_lm.h).
//
// The trust-region loop restates Ceres 2.0's TrustRegionMinimizer +
// LevenbergMarquardtStrategy as configured by ArSlamSolver::optimize
// (ar_slam_util.cpp:1001-1018).  Only scalars cross
// PCIe per step (cost, model cost change, norms, the Cholesky flag); the
// problem, the parameters and the reduced system stay resident in HBM.
#include "host_threads.h"
#include "lm_internal.h"
#include "arslam_lm.h"
#include "arslam_lm_debug.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <thread>
#include <unordered_set>
#include <vector>

namespace {

thread_local std::string g_last_error;

using Error = arslam::ApiError;

#define HIP_CHECK(expr)                                                                      \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess)                                                                    \
      throw Error(_e == hipErrorOutOfMemory ? ARSLAM_E_OUT_OF_MEMORY : ARSLAM_E_HIP,         \
                  std::string(#expr) + ": " + hipGetErrorString(_e));                       \
  } while (0)

#define NCCL_CHECK(expr)                                                                     \
  do {                                                                                       \
    ncclResult_t _r = (expr);                                                                \
    if (_r != ncclSuccess)                                                                   \
      throw Error(ARSLAM_E_COMM, std::string(#expr) + ": " + ncclGetErrorString(_r));       \
  } while (0)

void fail_if(bool cond, int code, const std::string &msg) {
  if (cond) throw Error(code, msg);
}

// decode the persistent executors' negative flags (dense_llt.hip)
std::string executor_fault_message(int code, int rank, int iteration) {
  std::string what;
  const int c = -code;
  if (code == 0) what = "on another rank";
  else if (c >= 4000000) what = "backward-solve column " + std::to_string(c - 4000000) + ": dependency wait timed out";
  else if (c >= 3000000) what = "ticket " + std::to_string(c - 3000000) + ": late wait (fused TRSM / folded TRSM's L_kk) timed out";
  else if (c >= 2000000) what = "ticket " + std::to_string(c - 2000000) + ": in-order update wait timed out";
  else if (c >= 1000000) what = "ticket " + std::to_string(c - 1000000) + ": dependency wait timed out";
  else what = "code " + std::to_string(code);
  return "reduced-system executor fault (rank " + std::to_string(rank) + ", LM iteration " +
         std::to_string(iteration) + "): " + what;
}

// ... and, for a timed-out wait of k_factor_dag, what its fault record says:
// the awaited counter, the tickets that advance it, how far the launch drew
// (read after the step's stream sync; the record is reset with the counters)
std::string executor_fault_message(int code, int rank, int iteration, const arslam::LltPlan &plan,
                                   hipStream_t s) {
  std::string m = executor_fault_message(code, rank, iteration);
  if (code > -1000000 || code <= -4000000 || !plan.dag_counters) return m;
  int rec[arslam::kDagFaultSlots];
  if (hipMemcpyAsync(rec, plan.dag_counters + 2 * plan.n_tiles + arslam::kDagOffFault, sizeof(rec),
                     hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess || rec[arslam::kFaultTicket] != (-code) % 1000000)
    return m;
  return m + " -- " + arslam::dag_fault_detail(plan, rec);
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Device buffer; grow-only, so reloading a problem of the same or a smaller
// size (every optimize() of an incremental solve) does no hipMalloc/hipFree.
template <class T>
struct DevBuf {
  T *p = nullptr;
  size_t n = 0, cap = 0;
  void alloc(size_t count) {   // grows by half again (a growing incremental problem reallocates rarely)
    n = count;
    if (count <= cap) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = cap == 0 && count <= 16 ? count : count + count / 2;
    HIP_CHECK(hipMalloc(&p, want * sizeof(T)));
    cap = want;
  }
  void upload(const T *h, size_t count, hipStream_t s) {
    if (count) HIP_CHECK(hipMemcpyAsync(p, h, count * sizeof(T), hipMemcpyHostToDevice, s));
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = cap = 0;
  }
  ~DevBuf() { release(); }
};

// page-locked host words: a D2H copy into them stays asynchronous
struct PinnedBuf {
  double *p = nullptr;
  size_t cap = 0;
  void alloc(size_t count) {   // grows only (by half again: page-locking is slow); kept across solves
    if (count <= cap) return;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = count + count / 2;
    HIP_CHECK(hipHostMalloc(&p, want * sizeof(double), hipHostMallocDefault));
    cap = want;
  }
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
};

// The problem's uploaded arrays: one grow-only device allocation, one
// page-locked host image, one host->device copy per load (instead of a
// pageable copy and a driver staging pass per array).
struct UploadArena {
  char *dev = nullptr, *host = nullptr;
  size_t dev_cap = 0, host_cap = 0;
  struct Piece { void **dst; const void *src; size_t bytes, off; };
  std::vector<Piece> pieces;
  hipEvent_t copied = nullptr;   // the last commit's transfer has read the host image
  template <class T>
  void add(T **dst, const T *src, size_t count) { pieces.push_back({reinterpret_cast<void **>(dst), src, count * sizeof(T), 0}); }
  // lay the pieces out, copy them into the host image and enqueue the one
  // transfer; the sources may go out of scope once this returns, the image
  // stays untouched until the caller's next stream sync
  void commit(hipStream_t s) {
    // the previous transfer may still be reading the image (a load with no
    // reduced system has no stream sync before the next upload)
    if (copied) HIP_CHECK(hipEventSynchronize(copied));
    size_t used = 0;
    for (Piece &p : pieces) {
      p.off = used;
      used += (std::max<size_t>(p.bytes, 1) + 255) & ~size_t(255);
    }
    if (used > host_cap) {
      if (host) (void)hipHostFree(host);
      host = nullptr;
      host_cap = 0;
      HIP_CHECK(hipHostMalloc(&host, used + used / 2, hipHostMallocDefault));
      host_cap = used + used / 2;
    }
    if (used > dev_cap) {
      if (dev) (void)hipFree(dev);
      dev = nullptr;
      dev_cap = 0;
      HIP_CHECK(hipMalloc(&dev, used + used / 2));
      dev_cap = used + used / 2;
    }
    for (Piece &p : pieces) {
      if (p.bytes) std::memcpy(host + p.off, p.src, p.bytes);
      *p.dst = dev + p.off;
    }
    if (used) {
      HIP_CHECK(hipMemcpyAsync(dev, host, used, hipMemcpyHostToDevice, s));
      if (!copied) HIP_CHECK(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
      HIP_CHECK(hipEventRecord(copied, s));
    }
    pieces.clear();
  }
  ~UploadArena() {
    if (copied) (void)hipEventDestroy(copied);
    if (dev) (void)hipFree(dev);
    if (host) (void)hipHostFree(host);
  }
};

struct Timer {
  hipEvent_t a = nullptr, b = nullptr;
  double acc_ms = 0.0;
  bool pending = false;
  bool on = true;   // options.phase_timing
  void init() {
    if (!a) {
      // timing only (read after the stream's sync): no system-scope fence at
      // the record -- its cache writeback and invalidation sat between the
      // kernels it brackets (~6 us each side of the factorization)
      HIP_CHECK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
      HIP_CHECK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
    }
  }
  void start(hipStream_t s) {
    if (on) HIP_CHECK(hipEventRecord(a, s));
  }
  void stop(hipStream_t s) {
    if (!on) return;
    HIP_CHECK(hipEventRecord(b, s));
    pending = true;
  }
  void collect() {  // call after the stream was synchronized (or its flag seen: b may still be pending)
    if (!pending) return;
    float ms = 0.f;
    HIP_CHECK(hipEventSynchronize(b));
    HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    acc_ms += ms;
    pending = false;
  }
  void destroy() {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    a = b = nullptr;
  }
};

enum { PH_LIN, PH_SCHUR, PH_CHOL, PH_SOLVE, PH_BACK, PH_COST, PH_FAC0, PH_FAC1, PH_N };

}  // namespace

struct arslam_lm {
  arslam_lm_options opt;

  // ---- pointer-keyed problem (Ceres API mirror) ----
  double *camera_ptr = nullptr;
  std::unordered_map<double *, int> cap_of, tag_of;
  std::vector<double *> cap_ptrs, tag_ptrs;
  std::vector<int> pk_obs_cap, pk_obs_tag;
  std::vector<double> pk_corners;
  std::unordered_set<double *> constant;
  // The pointer-keyed structure (blocks, residuals, constants) changed since
  // the last load: arslam_lm_solve reloads; otherwise it reuses the resident
  // problem, plan and buffers and uploads only the parameter values.
  bool pk_dirty = true;

  // ---- loaded problem ----
  bool loaded = false;
  arslam_soa_problem soa{};
  int nc = 0, nt = 0, nb = 0;
  long n = 0, nR = 0, N = 0;
  bool has_f = false;
  std::vector<unsigned char> slot_free;
  std::vector<double> x0;   // initial slots
  long nb_global = 0;       // observations over all ranks
  double setup_s = 0.0;     // host structure + ordering + plan + upload of the last load (or value reload)
  double setup_phase[5] = {0, 0, 0, 0, 0};   // the last full load's phases (summary.setup_phase_s)
  double comm_bytes = 0.0;  // bytes this rank all-reduced (RCCL or the host callback) since the count was reset
  long comm_calls = 0;      // ... and the collectives that carried them
  arslam::DevProblem P{};
  hipStream_t stream = nullptr;
  int device = 0;

  // uploaded arrays (pointers into `upload`, re-laid out by every load)
  UploadArena upload;
  int *u_cap_start = nullptr, *u_obs_tag = nullptr, *u_obs_lblk = nullptr, *u_cap_blk_start = nullptr,
      *u_blk_tag = nullptr, *u_tag_start = nullptr, *u_obs_tpos = nullptr, *u_tag_row = nullptr,
      *u_row_slot = nullptr, *u_fslot_row = nullptr, *u_dest_start = nullptr, *u_big_caps = nullptr;
  unsigned char *u_f_own = nullptr;
  unsigned char *u_cap_kind = nullptr;   // ARSLAM_ELIM_MIXED: DevProblem::cap_kind, f_alias
  int *u_f_alias = nullptr;
  std::vector<unsigned char> f_own;   // several ranks: DevProblem::f_own
  std::vector<int> big_caps;   // captures with more than kSchurMfmaBlocks distinct tags (k_schur's second launch)
  std::vector<int> chunk_caps;   // captures with more than kObsChunk observations (the chunked launches)
  int *u_chunk_caps = nullptr;
  unsigned char *u_obs_active = nullptr, *u_slot_free = nullptr;
  double *u_corners = nullptr, *u_x0 = nullptr;
  long *u_cap_off = nullptr;
  int2 *u_dest_row = nullptr;
  int4 *u_gather_items = nullptr, *u_gather_splits = nullptr;
  arslam::SchurContrib *u_contrib = nullptr;
  // One rank, persistent executor: the fill tiles (numbered after the
  // assembled ones) are never cleared -- their first update stores.  n_clear:
  // the tiles k_schur clears (the assembled ones; every tile when an appended
  // problem's gather writes into a fill tile: then no first-update store)
  long n_clear = 0;
  DevBuf<double> d_xa, d_xb, d_xbest, d_g, d_colnorm, d_scale, d_diag;
  DevBuf<double> d_obs_tg, d_parts, d_fparts, d_red, d_S, d_z, d_yF;
  // the reduced system's tiles: Sp = d_S.p + s_pre.  Several ranks: the top
  // tags' linearization sums (top_tail_len doubles) ride in the prefix, just in
  // front of the top tiles, in the step's one bulk all-reduce
  double *Sp = nullptr;
  long s_pre = 0;
  int *u_top_slots = nullptr;
  int n_top_slots = 0;
  long top_tail_len() const { return 2L * n_top_slots + 2; }
  double *d_norms_p = nullptr;   // inside d_red
  DevBuf<int> d_flag;
  DevBuf<double> d_slab, d_jrows, d_cap_ui;
  DevBuf<double> d_gather_part;
  arslam::LltPlan plan;
  // x: the current point, xc: the candidate, xbest: the best point so far --
  // three of d_xa / d_xb / d_xbest by pointer, xc never aliasing the other two
  double *x = nullptr, *xc = nullptr, *xbest = nullptr;
  unsigned long long dbg_indefinite_mask = 0;   // arslam_lm_debug_force_indefinite
  arslam_iteration_callback iter_cb = nullptr;  // arslam_lm_set_iteration_callback
  void *iter_cb_ctx = nullptr;
  int n_fparts = 0;

  Timer timers[PH_N];
  arslam::LaunchTiming upd_timing;
  std::vector<hipEvent_t> upd_events;
  double dom_ms = 0.0, dom_flops = 0.0;
  double scalar_flops = 0.0;   // scalar Cholesky flops of the reduced system's real rows (ReducedLayout)
  long dom_launches = 0;

  void timing_begin() {
    if (!opt.kernel_timing || !has_f) return;
    const int need = plan.nlev + 1;
    if ((int)upd_events.size() < 2 * need) {
      for (auto e : upd_events) (void)hipEventDestroy(e);
      upd_events.assign(2 * need, nullptr);
      for (auto &e : upd_events) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));   // (as Timer)
    }
    upd_timing.ev = upd_events.data();
    upd_timing.cap = need;
    upd_timing.used = 0;
    upd_timing.flops = 0.0;
  }
  void timing_collect() {   // after a stream synchronize
    if (!opt.kernel_timing || !has_f) return;
    for (int i = 0; i < upd_timing.used; ++i) {
      float ms = 0.f;
      HIP_CHECK(hipEventSynchronize(upd_events[2 * i + 1]));
      HIP_CHECK(hipEventElapsedTime(&ms, upd_events[2 * i], upd_events[2 * i + 1]));
      dom_ms += ms;
    }
    dom_launches += upd_timing.used;
    dom_flops += upd_timing.flops;
    upd_timing.used = 0;
    upd_timing.flops = 0.0;
  }

  // ---- multi-GPU ----
  int rank = 0, nranks = 1;
  ncclComm_t comm = nullptr;
  // debug (arslam_debug_force_multirank): take the multi-rank path -- the
  // split, the two-phase factorization and every collective -- with one rank,
  // so its RCCL calls run on a one-GPU box
  bool force_multi = false;
  bool multi() const { return nranks > 1 || force_multi; }

  ~arslam_lm() {
    for (auto &t : timers) t.destroy();
    for (auto e : upd_events) (void)hipEventDestroy(e);
    if (ev_sync) (void)hipEventDestroy(ev_sync);
    arslam::llt_plan_free(plan);
    if (comm) (void)ncclCommDestroy(comm);
    if (stream) (void)hipStreamDestroy(stream);
  }

  // host-callback transport (arslam_lm_set_comm_callback): stage through host memory
  arslam_allreduce_fn comm_cb = nullptr;
  void *comm_cb_ctx = nullptr;
  std::vector<unsigned char> comm_stage;

  // In-place all-reduce of a device buffer over the ranks (RCCL, or the
  // caller's callback).  Every rank issues the same sequence of calls.
  void allreduce_any(void *buf, size_t count, int dtype, int op) {
    if (!multi() || count == 0) return;
    const size_t bytes = count * (dtype == ARSLAM_DT_F64 ? sizeof(double) : 1);
    comm_bytes += (double)bytes;
    ++comm_calls;
    if (comm_cb) {
      comm_stage.resize(bytes);
      HIP_CHECK(hipMemcpyAsync(comm_stage.data(), buf, bytes, hipMemcpyDeviceToHost, stream));
      HIP_CHECK(hipStreamSynchronize(stream));
      fail_if(comm_cb(comm_cb_ctx, comm_stage.data(), count, dtype, op) != 0, ARSLAM_E_COMM,
              "all-reduce callback failed");
      HIP_CHECK(hipMemcpyAsync(buf, comm_stage.data(), bytes, hipMemcpyHostToDevice, stream));
      HIP_CHECK(hipStreamSynchronize(stream));
      return;
    }
    fail_if(!comm, ARSLAM_E_STATE, "the multi-rank path without a communicator");
    NCCL_CHECK(ncclAllReduce(buf, buf, count, dtype == ARSLAM_DT_F64 ? ncclDouble : ncclUint8,
                             op == ARSLAM_OP_SUM ? ncclSum : ncclMax, comm, stream));
  }
  void allreduce(double *buf, size_t count, int op) { allreduce_any(buf, count, ARSLAM_DT_F64, op); }

  // Every rank derives the split itself (no structure is exchanged), so ranks
  // that disagree -- a rank-dependent environment, a different problem --
  // would issue mismatched collectives and hang.  One all-reduce (MAX of h and
  // of -h, 52-bit hash of the owner maps) proves they agree before the first step.
  DevBuf<double> d_split_hash;
  void check_same_split(const arslam::RankSplit &sp) {
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](long v) { h = (h ^ (unsigned long long)v) * 1099511628211ull; };
    for (int v : sp.col_owner) mix(v);
    for (int v : sp.cap_owner) mix(v);
    mix(sp.n_active);
    const double hv[2] = {(double)(h >> 12), -(double)(h >> 12)};   // exact in a double
    ensure_stream();
    d_split_hash.alloc(2);
    HIP_CHECK(hipMemcpyAsync(d_split_hash.p, hv, sizeof(hv), hipMemcpyHostToDevice, stream));
    allreduce(d_split_hash.p, 2, ARSLAM_OP_MAX);
    double got[2];
    HIP_CHECK(hipMemcpyAsync(got, d_split_hash.p, sizeof(got), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    fail_if(got[0] != -got[1], ARSLAM_E_COMM,
            "the ranks derived different capture / tile-column splits (same problem and options on every rank, "
            "no rank-dependent ARSLAM_* environment)");
  }

  int dag_workgroups = 512;
  static inline bool dag_traced = false;   // debug trace: one per process
  static inline int dag_trace_seen = 0;

  int cus_device = -1, cus = 0;   // the CU count, queried once per device
  // The thread and options device the handle's stream was last made ready
  // for: a later load from the same thread with the same options, while the
  // thread's current device is still the handle's, makes one hipGetDevice (a
  // thread-local read) and nothing else.  The current-device check matters
  // when one thread drives handles on several devices: another handle's load
  // may have switched it, and this handle's allocations must land on its own
  // device.
  std::thread::id ready_thread{};
  int ready_opt_device = -2;
  void ensure_stream() {
    int cur = -1;
    HIP_CHECK(hipGetDevice(&cur));
    if (stream && ready_thread == std::this_thread::get_id() && ready_opt_device == opt.device && cur == device) {
      return;
    }
    // the handle's device: the options device, else the one its stream lives on, else the current one
    const int want = opt.device >= 0 ? opt.device : (stream ? device : cur);
    fail_if(stream && want != device, ARSLAM_E_STATE,
            "the handle's device changed after its stream was created (set options.device before the first load)");
    if (want != cur) HIP_CHECK(hipSetDevice(want));   // (set only when it differs)
    device = want;
    if (cus_device != device) {
      cus = 0;
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 0;
      cus_device = device;
      arslam::set_schur_big_lds_attribute();   // (k_schur's big-capture launch: once per device)
    }
    // 1.75 persistent workgroups per CU (73 KB of LDS each: two fit): 448 on
    // the MI355X's 256 CUs.  cfg3 k_factor_dag 663.1 -> 655.7 us and
    // 597.6 -> 593.0 us against 512 (same-box A/B, tools/ab.py): fewer
    // co-resident update workgroups beside the chain's POTRF tasks
    if (cus > 0) dag_workgroups = 7 * cus / 4;
    if (const char *g = std::getenv("ARSLAM_DAG_GRID")) dag_workgroups = std::max(1, std::atoi(g));   // debug
    // never more than can be resident at once (the claim cap is half the grid)
    if (cus > 0) dag_workgroups = std::min(dag_workgroups, arslam::kDagWorkgroupsPerCu * cus);
    if (!stream) HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    for (auto &t : timers) t.init();
    ready_thread = std::this_thread::get_id();
    ready_opt_device = opt.device;
  }

  void load(const arslam_soa_problem *p);
  // (extend_from >= 0: captures [extend_from, nc) were appended to the loaded
  // problem, the others unchanged: the gather plan is extended, not rebuilt)
  void upload_problem(const arslam::HostProblem &h, const arslam::ReducedLayout &L, int extend_from = -1);
  arslam::SchurGather sg;   // the loaded problem's Schur gather plan
  bool sg_ready = false;    // load(): sg was built beside the tile plan (upload_problem keeps it)
  bool try_extend(const arslam_soa_problem *p);
  bool try_extend_mixed(const arslam_soa_problem *p);
  arslam::ReducedLayout lay;      // the loaded layout (one rank), kept for try_extend
  bool pk_appended_only = false;  // since the last load only residual blocks of known tags were added
  int setup_kind = ARSLAM_SETUP_LOAD;
  int elim_used = ARSLAM_ELIM_CAPTURES;   // the side load() eliminates (the device problem is role-swapped for TAGS)
  arslam::MixedProblem mx;                // ARSLAM_ELIM_MIXED: the regrouped device problem (host_structure.h)
  int ceres_e_cap = 0, ceres_e_tag = 0;   // Ceres 2.0's e-block set of the loaded problem, by kind
  void reload_values(const arslam_soa_problem *p);
  bool pk_loaded = false;   // the resident problem came from the pointer-keyed API
  // several ranks: the whole problem's capture count, this rank's captures
  // (ascending; the loaded problem's capture c is own_caps[c]) and its local arrays
  int nc_full = 0;
  int nc_user = 0;   // the caller's capture count (the device problem's "captures" are tags or groups under TAGS / MIXED)
  std::vector<int> own_caps;
  std::vector<double> loc_cap, loc_corners;
  std::vector<int> loc_obs_cap, loc_obs_tag;
  std::vector<unsigned char> loc_cap_const;
  double split_top_work = 0.0, split_max_rank_work = 0.0, split_total_work = 0.0;
  int split_active = 1;   // ranks owning subtrees (RankSplit::n_active)
  // co-visibility of the free tags (a bit matrix, directed edge count as
  // ReducedLayout::n_edges), kept up to date through appends: an appended
  // problem whose graph outgrew the one its elimination order was computed
  // for by more than a tenth reloads with a fresh order (a stale order on the
  // incremental cfg2 flow: 18 elimination-tree levels and 358 us per
  // factorization against 10 and 217 us fresh)
  std::vector<uint64_t> covis;
  long covis_nt = 0, covis_edges = 0;
  void covis_build(const arslam::HostProblem &h, const arslam::ReducedLayout &L) {
    covis_nt = h.nt <= 16384 ? h.nt : 0;
    covis_edges = 0;
    covis.assign(((size_t)covis_nt * covis_nt + 63) / 64, 0);
    for (int c = 0; c < h.nc && covis_nt; ++c) covis_add(h, L, c);
  }
  void covis_add(const arslam::HostProblem &h, const arslam::ReducedLayout &L, int c) {
    if (!covis_nt) return;
    for (int a = h.cap_blk_start[c]; a < h.cap_blk_start[c + 1]; ++a)
      for (int b = h.cap_blk_start[c]; b < h.cap_blk_start[c + 1]; ++b) {
        const int ta = h.blk_tag[a], tb = h.blk_tag[b];
        if (ta == tb || L.tag_row[ta] < 0 || L.tag_row[tb] < 0) continue;
        const size_t bit = (size_t)ta * covis_nt + tb;
        if (!(covis[bit >> 6] >> (bit & 63) & 1)) {
          covis[bit >> 6] |= 1ull << (bit & 63);
          ++covis_edges;
        }
      }
  }
  bool reuse_order = false;  // load(): keep the previous tag order when the free tags are unchanged
  std::vector<int> prev_tag_row;
  // ARSLAM_ELIM_MIXED: the rows of the last layout by original block (tag /
  // capture id, -1 off the reduced side), for a reload whose re-chosen set
  // renumbers the reduced blocks (reduced_layout by identity)
  std::vector<int> prev_mx_tag_row, prev_mx_cap_row;
  int prev_ordering = -1, prev_skip = -1;
  long prev_order_edges = 0;
  // the capture count the order was computed at: nested dissection cuts along
  // the tags' positions, which the first solves of an incremental flow only
  // roughly know, so a grown problem (by a quarter) gets a fresh order even if
  // its co-visibility graph barely changed (incremental cfg2: an order kept
  // from the first load gave 18 elimination-tree levels, a fresh one 10)
  int prev_order_nc = 0;
  bool last_order_reused = false;   // summary.order_reused
  int prev_order_height = 0;   // tile elimination-tree height of the layout the order was computed for
  static int etree_height(const arslam::ReducedLayout &L) {
    std::vector<uint8_t> P = L.pattern;
    std::vector<int> parent;
    arslam::tile_fill(L.T, P, parent);
    std::vector<int> lev(L.T, 1);
    int h = 0;
    for (int k = 0; k < L.T; ++k) {   // (parents have larger indices)
      if (parent[k] >= 0) lev[parent[k]] = std::max(lev[parent[k]], lev[k] + 1);
      h = std::max(h, lev[k]);
    }
    return h;
  }
  void linearize(double *x_cost, double *fixed_cost, double *gmax, double *gnorm, double *xnorm);
  // linearize split at the host read: enqueue (results copied to h_lin), collect after a sync
  void linearize_launch();
  void linearize_collect(double *x_cost, double *fixed_cost, double *gmax, double *gnorm, double *xnorm);
  // Several ranks: a linearization's sums over the ranks are not collectives
  // of their own.  Its tag slots' gradient and column norms and the camera's
  // f partials (lin_xpending) ride in front of the top tiles in the next
  // step's bulk all-reduce (or one packed all-reduce, complete_pending_lin,
  // when no step follows); its cost and norms (norms_pending) ride with the
  // step's scalars (exchange_scalars; exchange_norms when no step follows).
  bool lin_xpending = false, norms_pending = false;
  DevBuf<double> d_lx, d_ag;   // the packed exchange; the all-gathered scalars
  static constexpr int kLinSave = 16 + 8 + 6 * arslam::kNormBlocks;   // d_red[kLinSave..+1]: the linearization's cost, fixed
  void complete_pending_lin();
  void lin_norms();   // k_slot_norms once the linearization's sums are final
  void exchange_scalars(arslam::AgFields fl, arslam::HostOut *ho = nullptr);   // (+ the pending norms), into d_red
  void exchange_norms() {
    if (norms_pending) exchange_scalars(arslam::AgFields{});
  }
  PinnedBuf h_lin;   // [0..3] cost, fixed, g_f, col_f; [16..21] slot norms; [16 + kHostSeq] lin_seq
  double lin_seq = 0.0;   // (one rank) the last linearization's sequence number
  void lin_sync() {   // the linearization's host words (one rank: its flag; several: after the copies)
    if (!multi() && lin_seq > 0.0) flag_sync(h_lin.p + 16 + arslam::kHostSeq, lin_seq);
    else spin_sync();
  }
  // host LM loop: the Jacobi scale of this solve is set, so each later
  // linearization also forms the LM diagonal (k_slot_norms) and the step's
  // executor reset rides in k_schur's launch
  bool diag_in_lin = false;
  PinnedBuf h_x;     // [n] parameter download (write_back)
  PinnedBuf h_step;  // [0..NPART+1] the step's reduced scalars, [NPART+2..4] the factorization flags
  hipEvent_t ev_sync = nullptr;
  // Wait for the stream by polling an event: the LM loop's one host round
  // trip per step, without the blocking-sync wake-up latency.
  void spin_sync() {
    if (!ev_sync) HIP_CHECK(hipEventCreateWithFlags(&ev_sync, hipEventDisableTiming));
    HIP_CHECK(hipEventRecord(ev_sync, stream));
    hipError_t e;
    while ((e = hipEventQuery(ev_sync)) == hipErrorNotReady) {
    }
    HIP_CHECK(e);
  }
  // One rank: the LM loop's host reads wait for the kernel that stores their
  // page-locked words to store its sequence number last (hout[kHostSeq]),
  // instead of an event behind it: ~8 against ~13 us per round trip on
  // MI355X (tools/sync_bench.hip), ~7 round trips per cfg3 solve and ~7,000
  // in the incremental cfg2 flow.  The stream is queried now and then so a
  // launch that never stores it (an error) is reported, not waited for.
  double host_seq = 0.0;
  DevBuf<int> d_seq_done;   // k_reduce_parts' finished blocks (zero between launches)
  double next_seq(double *word) {
    *(volatile double *)word = -1.0;   // (before the launch: the kernel's store lands after it)
    return host_seq += 1.0;
  }
  void flag_sync(const double *word, double seq) {
    for (long k = 1;; ++k) {
      if (*(const volatile double *)word == seq) break;
      if ((k & 4095) == 0) {
        const hipError_t e = hipStreamQuery(stream);
        if (e == hipErrorNotReady) continue;
        HIP_CHECK(e);
        if (*(const volatile double *)word == seq) break;
        throw Error(ARSLAM_E_DEVICE, "the stream finished without storing the host sequence word");
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  void solve(arslam_lm_summary *s);
  void write_back(const double *d_src);
  // the pointer-keyed solve in progress: its (unswapped) staging problem, whose
  // arrays soa aliases; write_back also scatters them into the caller's blocks
  const arslam_soa_problem *pk_stage = nullptr;
  void scatter_to_blocks();
  // arslam_lm_debug_break_dependency: the patched wait entry, restored after the next solve
  int dbg_patched_wait = -1;
  void restore_patched_wait();
  // multi-rank: does any rank have an iteration callback (agreed once per solve)
  bool any_iter_cb = false;
  DevBuf<double> d_cb;
  int agree_callback(int r);
};

namespace {

long round_up(long v, long m) { return (v + m - 1) / m * m; }

}  // namespace

void arslam_lm::load(const arslam_soa_problem *p_in) {
  const double t_load = now_s();
  loaded = false;
  // (the process's first HIP call starts the runtime, 0.02-0.2 s: the first
  // load of a process pays it here, in summary.setup_phase_s[0] -- round 4's
  // "1.2 ms per full load" was that one start averaged over 179 loads)
  ensure_stream();
  // the e-block side (ARSLAM_ELIM_*): Ceres' own independent set decides AUTO;
  // tag elimination runs the same kernels on the role-swapped problem
  std::vector<uint8_t> e_cap, e_tag;
  const bool want_set = opt.elimination == ARSLAM_ELIM_MIXED;
  const arslam::SchurSide cs =
      arslam::ceres_schur_side(p_in, want_set ? &e_cap : nullptr, want_set ? &e_tag : nullptr);
  ceres_e_cap = cs.e_cap;
  ceres_e_tag = cs.e_tag;
  // (an eliminated block's local system over its distinct f-blocks lives in
  // one wave's LDS: at most kMaxSchurBlocks of them)
  const bool tags_fit = cs.max_tag_blk <= arslam::kMaxSchurBlocks, caps_fit = cs.max_cap_blk <= arslam::kMaxSchurBlocks;
  int side = opt.elimination;
  if (side == ARSLAM_ELIM_AUTO)
    side = (!multi() && tags_fit && (cs.e_tag > cs.e_cap || !caps_fit)) ? ARSLAM_ELIM_TAGS : ARSLAM_ELIM_CAPTURES;
  if (side == ARSLAM_ELIM_MIXED) {
    // Ceres' exact set: a whole side when it holds one kind only (then it is
    // every free block of that kind), the mixed device problem otherwise; the
    // camera joins it only in degenerate graphs (one residual), where the
    // device eliminates the captures instead
    fail_if(multi(), ARSLAM_E_UNSUPPORTED, "the mixed e-block set is single-rank only (the ranks own captures)");
    if (cs.e_cam || cs.e_tag == 0) side = ARSLAM_ELIM_CAPTURES;
    else if (cs.e_cap == 0) side = ARSLAM_ELIM_TAGS;
  }
  fail_if(side == ARSLAM_ELIM_TAGS && multi(), ARSLAM_E_UNSUPPORTED,
          "tag elimination is single-rank only (the ranks own captures)");
  fail_if(multi() && opt.factor_executor != 1, ARSLAM_E_UNSUPPORTED,
          "several ranks need the persistent executor (factor_executor = 1)");
  fail_if(side == ARSLAM_ELIM_TAGS && !tags_fit, ARSLAM_E_UNSUPPORTED,
          "tag elimination: a tag seen by more than 256 distinct captures");
  fail_if(side == ARSLAM_ELIM_CAPTURES && !caps_fit, ARSLAM_E_UNSUPPORTED,
          "capture elimination: a capture sees more than 256 distinct tags");
  // (the f-side changed, or is a mixed set of its own: no order to reuse by
  // index; a mixed set after a mixed set maps the earlier rows by block)
  const bool was_mixed = elim_used == ARSLAM_ELIM_MIXED;
  if (side != elim_used || side == ARSLAM_ELIM_MIXED) prev_tag_row.clear();
  elim_used = side;
  const arslam_soa_problem swapped = arslam::swap_roles(*p_in);
  if (side == ARSLAM_ELIM_MIXED) mx = arslam::mixed_problem(*p_in, e_cap, e_tag);
  else mx = arslam::MixedProblem{};
  static const bool mx_fresh = std::getenv("ARSLAM_MIXED_FRESH_ORDER") != nullptr;   // debug A/B: round 6's first cut
  const bool by_identity = side == ARSLAM_ELIM_MIXED && was_mixed && reuse_order && !mx_fresh && !mx.f_src.empty() &&
                           (!prev_mx_tag_row.empty() || !prev_mx_cap_row.empty());
  if (by_identity) {
    prev_tag_row.assign(mx.f_src.size(), -1);
    for (size_t f = 0; f < mx.f_src.size(); ++f) {
      const std::vector<int> &m = mx.f_is_cap[f] ? prev_mx_cap_row : prev_mx_tag_row;
      if (mx.f_src[f] < (int)m.size()) prev_tag_row[f] = m[mx.f_src[f]];
    }
  }
  const arslam_soa_problem *p = side == ARSLAM_ELIM_TAGS ? &swapped : side == ARSLAM_ELIM_MIXED ? &mx.soa : p_in;
  static const bool prof = std::getenv("ARSLAM_SETUP_PROFILE") != nullptr;   // debug: setup phases
  double tp[6] = {now_s(), 0, 0, 0, 0, 0};
  double t_host = tp[0];   // (one rank: after host_problem)
  // an incremental re-load (pointer-keyed path, same options) whose free tags
  // are unchanged keeps the previous elimination order: the ordering (nested
  // dissection) is the largest part of the host setup
  const bool can_reuse = reuse_order && !prev_tag_row.empty() && prev_ordering == opt.reduced_ordering &&
                         prev_skip == opt.cholesky_skip_zero_tiles && 4L * p->n_cap <= 5L * prev_order_nc;
  arslam::HostProblem h;
  arslam::ReducedLayout L;
  std::vector<int> col_class;
  own_caps.clear();
  nc_full = p->n_cap;
  nc_user = p_in->n_cap;
  if (multi()) {
    // Several ranks: every rank holds the whole problem and computes the same
    // structure (deterministic host code, no exchange): the reduced layout,
    // then the subtree-to-rank split of the tile elimination tree, which
    // gives this rank its captures and tile columns (arslam::rank_split).
    const arslam::HostProblem hf = arslam::host_problem(p, nullptr);   // validates p
    L = arslam::reduced_layout(hf, opt.reduced_ordering, opt.cholesky_skip_zero_tiles != 0, nullptr, nullptr,
                               can_reuse ? &prev_tag_row : nullptr, prev_order_edges);
    arslam::RankSplit split = arslam::rank_split(hf, L, std::max(nranks, 2));
    if (nranks == 1) {
      // (forced multi-rank path on one rank: the two-rank split's replicated
      // top, everything below it this rank's -- the exchange then carries the
      // top tiles, as it would between ranks)
      for (int &o : split.col_owner) o = o < 0 ? -1 : 0;
      for (int &o : split.cap_owner) o = 0;
      split.n_active = 1;
    }
    col_class = split.col_class(rank);
    split_top_work = split.top_work;
    split_max_rank_work = split.max_rank_work;
    split_total_work = split.total_work;
    split_active = split.n_active;
    check_same_split(split);
    for (int c = 0; c < p->n_cap; ++c)
      if (split.cap_owner[c] == rank) own_caps.push_back(c);
    // this rank's problem: its captures (ascending), their observations, every tag
    std::vector<int> loc_of(p->n_cap, -1);
    loc_cap.resize(6 * own_caps.size());
    loc_cap_const.assign(own_caps.size(), 0);
    for (size_t c = 0; c < own_caps.size(); ++c) {
      loc_of[own_caps[c]] = (int)c;
      std::memcpy(&loc_cap[6 * c], p->cap + 6L * own_caps[c], 6 * sizeof(double));
      if (p->cap_const) loc_cap_const[c] = p->cap_const[own_caps[c]];
    }
    loc_obs_cap.clear(); loc_obs_tag.clear(); loc_corners.clear();
    for (int b = 0; b < p->n_obs; ++b) {
      const int lc = loc_of[p->obs_cap[b]];
      if (lc < 0) continue;
      loc_obs_cap.push_back(lc);
      loc_obs_tag.push_back(p->obs_tag[b]);
      loc_corners.insert(loc_corners.end(), p->corners + 8L * b, p->corners + 8L * b + 8);
    }
    arslam_soa_problem pl = *p;
    pl.n_cap = (int)own_caps.size();
    pl.n_obs = (int)loc_obs_cap.size();
    pl.cap = loc_cap.data();
    pl.obs_cap = loc_obs_cap.data();
    pl.obs_tag = loc_obs_tag.data();
    pl.corners = loc_corners.data();
    pl.cap_const = p->cap_const ? loc_cap_const.data() : nullptr;
    // the tags' use (freedom) and the observation count are the whole problem's
    const arslam::ReduceSumF64 global_deg = [&](std::vector<double> &deg) {
      std::fill(deg.begin(), deg.end(), 0.0);
      for (int b = 0; b < p->n_obs; ++b) deg[p->obs_tag[b]] += 1.0;
      deg[p->n_tag] = p->n_obs;
    };
    h = arslam::host_problem(&pl, global_deg);
    // the layout's tag slots are the whole problem's (3 + 6 nc_full + 6 t + a):
    // renumber them for this rank's parameter vector (3 + 6 nc_own + 6 t + a)
    const long shift = 6L * (p->n_cap - (long)own_caps.size());
    for (int &sl : L.row_slot)
      if (sl >= 3) sl -= (int)shift;
  } else {
    h = arslam::host_problem(p, nullptr);   // validates p
    if (side == ARSLAM_ELIM_MIXED) arslam::mixed_patch(h, mx, *p_in);
    t_host = now_s();
    // (a grown pointer-keyed problem: a fresh order takes the faster separator search)
    L = arslam::reduced_layout(h, opt.reduced_ordering, opt.cholesky_skip_zero_tiles != 0, nullptr, nullptr,
                               can_reuse ? &prev_tag_row : nullptr, prev_order_edges, reuse_order, by_identity);
    // A kept order whose tile elimination tree grew taller than the fresh
    // order's by more than a level (new co-visibility across its separators:
    // 10 -> 14 -> 20 levels within a few loads of the incremental cfg2 flow)
    // is recomputed: the factorization is chain-bound, the order ~3 ms.
    if (L.order_reused && L.nR > 0 && etree_height(L) > prev_order_height + 1)
      L = arslam::reduced_layout(h, opt.reduced_ordering, opt.cholesky_skip_zero_tiles != 0, nullptr, nullptr,
                                 nullptr, 0, true);
  }
  tp[1] = now_s();
  soa = *p;   // (several ranks: the whole problem; write_back maps this rank's captures)
  nc = h.nc;
  nt = h.nt;
  nb = h.nb;
  n = h.n;
  nb_global = h.nb_global;
  slot_free = h.slot_free;
  x0 = h.x0;
  last_order_reused = L.order_reused;
  if (!L.order_reused) {
    prev_order_nc = h.nc;
    prev_order_height = L.nR > 0 ? etree_height(L) : 0;
  }
  prev_tag_row = L.tag_row;
  prev_order_edges = L.order_edges;
  prev_mx_tag_row.clear();
  prev_mx_cap_row.clear();
  if (side == ARSLAM_ELIM_MIXED) {
    prev_mx_tag_row.assign(p_in->n_tag, -1);
    prev_mx_cap_row.assign(p_in->n_cap, -1);
    for (size_t f = 0; f < mx.f_src.size(); ++f)
      (mx.f_is_cap[f] ? prev_mx_cap_row : prev_mx_tag_row)[mx.f_src[f]] = L.tag_row[f];
  }
  prev_ordering = opt.reduced_ordering;
  prev_skip = opt.cholesky_skip_zero_tiles;
  tp[2] = now_s();
  scalar_flops = L.scalar_flops;
  nR = L.nR;
  has_f = nR > 0;
  sg_ready = false;
  if (has_f && !multi()) {
    // the Schur gather plan (host only, from h and L) on a second thread while
    // this one builds and uploads the tile plan (its HIP calls stay on the
    // thread whose device is current) and does the co-visibility bookkeeping
    N = L.N;
    arslam::SchurGather sg_new;
    arslam::host_fork2(
        true, [&] { sg_new = arslam::schur_gather_plan(h, L); },
        [&] {
          arslam::llt_plan_build(plan, L.T, N, L.pattern, stream, nullptr);
          covis_build(h, L);
        });
    sg = std::move(sg_new);
    sg_ready = true;
  } else if (has_f) {
    N = L.N;
    arslam::llt_plan_build(plan, L.T, N, L.pattern, stream, multi() ? &col_class : nullptr);
  } else {
    if (!multi()) covis_build(h, L);
    N = 0;
    arslam::llt_plan_free(plan);
  }
  tp[3] = now_s();
  tp[4] = now_s();
  upload_problem(h, L);
  tp[5] = now_s();
  if (!multi()) lay = std::move(L);   // (try_extend: an appended problem keeps this layout and plan)
  setup_kind = ARSLAM_SETUP_LOAD;
  soa = side == ARSLAM_ELIM_MIXED ? *p_in : *p;   // (mixed: write_back maps the device slots to p_in's blocks)
  loaded = true;
  pk_appended_only = true;
  const double t_end = now_s();
  setup_s = t_end - t_load;
  // summary.setup_phase_s: structure (side rule + host problem), elimination
  // order (reduced layout; several ranks: + the split), tile plan + task graph,
  // gather plan + upload, the rest
  setup_phase[0] = (tp[0] - t_load) + (t_host - tp[0]);
  setup_phase[1] = tp[1] - t_host;
  setup_phase[2] = tp[3] - tp[2];
  setup_phase[3] = tp[5] - tp[4];
  setup_phase[4] = setup_s - setup_phase[0] - setup_phase[1] - setup_phase[2] - setup_phase[3];
  if (prof)
    std::fprintf(stderr, "arslam setup: nc %d nt %d side %.3f host+layout %.3f covis %.3f plan %.3f gather+upload %.3f tail %.3f total %.3f ms (order %s, %d levels, %ld tiles)\n",
                 nc, nt, 1e3 * (tp[0] - t_load), 1e3 * (tp[1] - tp[0]), 1e3 * (tp[2] - tp[1]), 1e3 * (tp[3] - tp[2]),
                 1e3 * (tp[5] - tp[4]), 1e3 * (t_end - tp[5]), 1e3 * setup_s,
                 prev_order_nc == nc ? "fresh" : "kept", plan.nlev, (long)plan.n_tiles);
}

// Everything the device needs from the host structure, the layout and the
// Schur gather plan, in one upload (UploadArena), plus the scratch buffers
// sized for the problem.  Ends with the load's one stream sync.
void arslam_lm::upload_problem(const arslam::HostProblem &h, const arslam::ReducedLayout &L, int extend_from) {
  const int maxk = h.maxk;
  const std::vector<int> &row_slot = L.row_slot;
  // f-side slot -> reduced row (camera slots 0..2, then the tag slots)
  std::vector<int> fslot_row(3 + 6L * nt, -1);
  for (size_t r = 0; r < row_slot.size(); ++r) {
    const long sl = row_slot[r];
    if (sl < 0) continue;
    if (sl < 3) fslot_row[sl] = (int)r;
    else if (sl >= 3 + 6L * nc) fslot_row[sl - 6L * nc] = (int)r;
  }
  static const bool prof = std::getenv("ARSLAM_SETUP_PROFILE") != nullptr;   // debug: setup phases
  const double tu0 = prof ? now_s() : 0.0;
  if (!has_f) sg = arslam::SchurGather{};
  else if (sg_ready) {}   // (load: built beside the tile plan)
  else if (extend_from >= 0 && (int)sg.cap_off.size() == extend_from + 1) arslam::schur_gather_extend(sg, h, L, extend_from);
  else sg = arslam::schur_gather_plan(h, L);
  sg_ready = false;
  const double tu1 = prof ? now_s() : 0.0;
  const int n_dest = has_f ? (int)sg.dest_start.size() - 1 : 0;
  const int n_items = (int)sg.items.size() / 4, n_splits = (int)sg.splits.size() / 4;
  upload.add(&u_cap_start, h.cap_start.data(), nc + 1);
  upload.add(&u_obs_tag, h.obs_tag.data(), nb);
  upload.add(&u_obs_lblk, h.obs_lblk.data(), nb);
  upload.add(&u_cap_blk_start, h.cap_blk_start.data(), nc + 1);
  upload.add(&u_blk_tag, h.blk_tag.data(), h.blk_tag.size());
  upload.add(&u_tag_start, h.tag_start.data(), nt + 1);
  upload.add(&u_obs_tpos, h.obs_tpos.data(), nb);
  upload.add(&u_obs_active, h.obs_active.data(), nb);
  upload.add(&u_slot_free, h.slot_free.data(), n);
  upload.add(&u_corners, h.corners.data(), 8L * nb);
  upload.add(&u_x0, x0.data(), n);
  upload.add(&u_tag_row, L.tag_row.data(), L.tag_row.size());
  upload.add(&u_row_slot, row_slot.data(), row_slot.size());
  upload.add(&u_fslot_row, fslot_row.data(), fslot_row.size());
  // several ranks: the top tags' slots (their linearization sums ride with the top tiles)
  std::vector<int> top_slots;
  if (multi() && has_f)
    for (long sl = 3 + 6L * nc; sl < n; ++sl) {
      const int r = fslot_row[sl - 6L * nc];
      if (r >= 0 && plan.h_col_class[r / arslam::kTile] == 1) top_slots.push_back((int)sl);
    }
  n_top_slots = (int)top_slots.size();
  if (n_top_slots) upload.add(&u_top_slots, top_slots.data(), top_slots.size());
  // several ranks: the f-side slots this rank holds -- its own subtree's tag
  // rows; the top's rows, the camera and the tags outside the reduced system
  // on rank 0 (every rank holds the top, one counts it); capture slots all
  f_own.clear();
  if (multi()) {
    f_own.assign(n, 0);
    for (long sl = 3; sl < 3 + 6L * nc; ++sl) f_own[sl] = 1;
    for (long sl = 0; sl < n; ++sl) {
      if (sl >= 3 && sl < 3 + 6L * nc) continue;
      const int r = fslot_row[sl < 3 ? sl : sl - 6L * nc];
      const int cls = r >= 0 && has_f ? plan.h_col_class[r / arslam::kTile] : 1;
      f_own[sl] = cls == 0 || (cls == 1 && rank == 0);
    }
    upload.add(&u_f_own, f_own.data(), f_own.size());
  }
  const bool mixed = elim_used == ARSLAM_ELIM_MIXED;
  if (mixed) {
    // the direct groups' slots copy f-block slots: counted once, on the f-block
    f_own.assign(n, 1);
    for (int g = 0; g < nc; ++g)
      if (mx.kind[g] == arslam::kMixDirect) std::fill(f_own.begin() + 3 + 6L * g, f_own.begin() + 9 + 6L * g, 0);
    upload.add(&u_f_own, f_own.data(), f_own.size());
    upload.add(&u_cap_kind, mx.kind.data(), mx.kind.size());
    upload.add(&u_f_alias, mx.f_alias.data(), mx.f_alias.size());
  }
  big_caps.clear();
  for (int c = 0; c < nc; ++c)
    if (h.cap_blk_start[c + 1] - h.cap_blk_start[c] > arslam::kSchurMfmaBlocks) big_caps.push_back(c);
  if (!big_caps.empty()) upload.add(&u_big_caps, big_caps.data(), big_caps.size());
  chunk_caps.clear();
  for (int c = 0; c < nc; ++c)
    if (h.cap_start[c + 1] - h.cap_start[c] > arslam::kObsChunk) chunk_caps.push_back(c);
  if (!chunk_caps.empty()) upload.add(&u_chunk_caps, chunk_caps.data(), chunk_caps.size());
  if (has_f) {
    upload.add(&u_cap_off, sg.cap_off.data(), nc + 1);
    upload.add(&u_dest_row, reinterpret_cast<const int2 *>(sg.dest_row.data()), n_dest);
    upload.add(&u_dest_start, sg.dest_start.data(), n_dest + 1);
    upload.add(&u_contrib, sg.contrib.data(), sg.contrib.size());
    upload.add(&u_gather_items, reinterpret_cast<const int4 *>(sg.items.data()), n_items);
    upload.add(&u_gather_splits, reinterpret_cast<const int4 *>(sg.splits.data()), n_splits);
  }
  n_clear = has_f ? plan.n_tiles : 0;
  if (has_f && !multi()) {
    // does the gather write into a fill tile (an appended problem's new
    // coupling; the plan is kept)?
    const int T = plan.T;
    bool fill_gathered = false;
    for (int d = 0; d < n_dest && !fill_gathered; ++d) {
      const int rX = sg.dest_row[2L * d], rY = sg.dest_row[2L * d + 1];
      const int sx = (rX == nR || rX == L.cam_row) ? 1 : 6, sy = rY == L.cam_row ? 1 : 6;
      for (int I = rX >> 6; I <= (rX + sx - 1) >> 6; ++I)
        for (int J = rY >> 6; J <= (rY + sy - 1) >> 6 && J <= I; ++J)
          fill_gathered = fill_gathered || plan.h_tile_id[(long)I * T + J] >= plan.n_assembled;
    }
    if (!fill_gathered && plan.fill_first_ok) n_clear = plan.n_assembled;
  }
  upload.commit(stream);
  d_xa.alloc(n); d_xb.alloc(n); d_xbest.alloc(n);
  d_g.alloc(n); d_colnorm.alloc(n); d_scale.alloc(n); d_diag.alloc(n);
  d_obs_tg.alloc(std::max(12L * nb, 1L));
  d_jrows.alloc(std::max(8L * arslam::kJStored * nb, 1L));
  d_cap_ui.alloc(std::max(36L * nc, 1L));
  d_parts.alloc((size_t)arslam::NPART * std::max(nc, 1));
  n_fparts = (int)((std::max(nR, 1L) + 255) / 256);
  d_fparts.alloc(2L * std::max(n_fparts, 1));
  // stays zero when there are no reduced rows (k_update_f is then not launched)
  if (!has_f) HIP_CHECK(hipMemsetAsync(d_fparts.p, 0, d_fparts.n * sizeof(double), stream));
  const double *red_prev = d_red.p;
  d_red.alloc(kLinSave + 8);   // LM scalars | slot norms: results, block count, k_slot_norms block partials | saved
  d_norms_p = d_red.p + 16;       // (one D2H carries both after a linearization)
  if (d_red.p != red_prev) HIP_CHECK(hipMemsetAsync(d_norms_p + 7, 0, sizeof(double), stream));   // the count
  d_flag.alloc(1);
  const int *seq_prev = d_seq_done.p;
  d_seq_done.alloc(1);
  if (d_seq_done.p != seq_prev) HIP_CHECK(hipMemsetAsync(d_seq_done.p, 0, sizeof(int), stream));
  if (has_f) {
    d_slab.alloc(std::max(sg.cap_off[nc], 1L));
    d_gather_part.alloc(36L * std::max(sg.n_pslots, 1));
    s_pre = multi() ? round_up(top_tail_len(), 512) : 0;
    d_S.alloc((size_t)s_pre + (size_t)plan.n_tiles * 4096);   // (cleared by k_schur's extra blocks every step)
    Sp = d_S.p + s_pre;
    d_z.alloc(N);
    d_yF.alloc(N);
  } else {
    d_S.release();
    Sp = nullptr;
    s_pre = 0;
    d_z.release();
    d_yF.alloc(1);
  }
  HIP_CHECK(hipMemsetAsync(d_parts.p, 0, d_parts.n * sizeof(double), stream));

  P.nc = nc; P.nt = nt; P.nb = nb; P.n = n; P.nR = nR; P.N = N; P.lda = N; P.cam_row = L.cam_row;
  P.max_obs_per_cap = std::max(maxk, 1);
  P.max_blk_per_cap = h.maxblk;
  P.big_caps = big_caps.empty() ? nullptr : u_big_caps;
  P.n_big_caps = (int)big_caps.size();
  P.chunk_caps = chunk_caps.empty() ? nullptr : u_chunk_caps;
  P.n_chunk_caps = (int)chunk_caps.size();
  P.swap_roles = elim_used == ARSLAM_ELIM_TAGS ? 1 : 0;
  P.nf = 3 + 6 * nt;
  P.fslot_row = u_fslot_row;
  P.cap_start = u_cap_start; P.obs_tag = u_obs_tag; P.obs_lblk = u_obs_lblk;
  P.cap_blk_start = u_cap_blk_start; P.blk_tag = u_blk_tag;
  P.obs_active = u_obs_active; P.slot_free = u_slot_free;
  P.tag_start = u_tag_start; P.obs_tpos = u_obs_tpos; P.corners = u_corners;
  P.tag_row = u_tag_row; P.row_slot = u_row_slot;
  P.tile_id = plan.tile_id; P.T = plan.T;
  P.tile_class = multi() && has_f ? plan.tile_class : nullptr;
  P.f_own = multi() || mixed ? u_f_own : nullptr;
  P.cap_kind = mixed ? u_cap_kind : nullptr;
  P.f_alias = mixed ? u_f_alias : nullptr;
  P.cap_off = u_cap_off; P.slab = d_slab.p; P.dest_row = u_dest_row; P.dest_start = u_dest_start;
  P.contrib = u_contrib; P.n_dest = n_dest; P.jrows = d_jrows.p; P.cap_ui = d_cap_ui.p;
  P.gather_items = u_gather_items; P.gather_splits = u_gather_splits; P.gather_part = d_gather_part.p;
  P.n_items = n_items; P.n_splits = n_splits;
  const double tu2 = prof ? now_s() : 0.0;
  // (no sync: the copy reads the arena's page-locked image, which stays
  // untouched until the next upload -- after this solve's syncs)
  if (prof)
    std::fprintf(stderr, "arslam upload: gather plan %.3f arena+allocs %.3f sync %.3f ms\n", 1e3 * (tu1 - tu0),
                 1e3 * (tu2 - tu1), 1e3 * (now_s() - tu2));
}

// An appended problem (arslam_lm_solve after AddResidualBlock only, no new
// tag, no constant changed): if every capture's tile pairs are tiles of the
// loaded factor (assembled or fill: k_schur clears every tile of S each step
// and the gather addresses any of them), the reduced layout, the elimination
// order and the whole factorization plan stay as they are -- only the capture
// side, the gather plan and the values are rebuilt and uploaded.  false:
// load() instead.  (summary.factor_scalar_flops keeps the loaded problem's
// count: a new coupling inside a fill tile changes the scalar structure.)
bool arslam_lm::try_extend(const arslam_soa_problem *p) {
  // (ARSLAM_ELIM_MIXED whose set was every capture: new captures join it, as in try_extend_mixed)
  if (!loaded || multi() || elim_used != ARSLAM_ELIM_CAPTURES || !has_f ||
      (opt.elimination != ARSLAM_ELIM_AUTO && opt.elimination != ARSLAM_ELIM_CAPTURES &&
       opt.elimination != ARSLAM_ELIM_MIXED))
    return false;
  const double t0 = now_s();
  if (opt.elimination == ARSLAM_ELIM_AUTO) {   // the side Ceres would eliminate may change as the graph grows
    const arslam::SchurSide cs = arslam::ceres_schur_side(p);
    if (cs.max_tag_blk <= arslam::kMaxSchurBlocks && (cs.e_tag > cs.e_cap || cs.max_cap_blk > arslam::kMaxSchurBlocks))
      return false;
    ceres_e_cap = cs.e_cap;
    ceres_e_tag = cs.e_tag;
  }
  if (p->n_tag != nt) return false;
  const double t1 = now_s();
  arslam::HostProblem h = arslam::host_problem(p, nullptr);
  const double t2 = now_s();
  // the same free tags and camera (the same reduced rows)
  if ((lay.cam_row >= 0) != (h.slot_free[0] != 0)) return false;
  for (int t = 0; t < nt; ++t)
    if ((lay.tag_row[t] >= 0) != (h.slot_free[3 + 6L * h.nc + 6L * t] != 0)) return false;
  // every capture's tiles pairwise in the loaded factor's tiles (lay.pattern
  // is the filled pattern: llt_plan_build fills it in place; a new coupling in
  // a fill tile is gathered into it -- k_schur clears every tile of the factor
  // each step and the updates read-modify-write their targets)
  const int T = lay.T;
  std::vector<int> ts;
  // (only the captures of the appended residual blocks: the others' tile
  // pairs were in the pattern already)
  std::vector<char> touched(h.nc, 0);
  int first_touched = h.nc;
  for (long b = nb; b < p->n_obs; ++b) {
    touched[p->obs_cap[b]] = 1;
    first_touched = std::min(first_touched, p->obs_cap[b]);
  }
  for (int c = 0; c < h.nc; ++c) {
    if (!touched[c]) continue;
    ts.clear();
    if (lay.cam_row >= 0) {
      ts.push_back(lay.cam_row / 64);
      ts.push_back((lay.cam_row + 2) / 64);
    }
    for (int a = h.cap_blk_start[c]; a < h.cap_blk_start[c + 1]; ++a) {
      const int r0 = lay.tag_row[h.blk_tag[a]];
      if (r0 < 0) continue;
      ts.push_back(r0 / 64);
      ts.push_back((r0 + 5) / 64);
    }
    for (size_t a = 0; a < ts.size(); ++a)
      for (size_t b = 0; b < ts.size(); ++b)
        if (ts[a] >= ts[b] && plan.h_tile_id[(size_t)ts[a] * T + ts[b]] < 0) return false;
  }
  // the co-visibility graph the order was computed for, outgrown by a tenth: reload with a fresh order
  for (int c = 0; c < h.nc; ++c)
    if (touched[c]) covis_add(h, lay, c);
  if (covis_nt && 10 * covis_edges > 11 * prev_order_edges) return false;
  if (4L * h.nc > 5L * prev_order_nc) return false;   // (a quarter more captures: a fresh order)
  // only new captures got residual blocks: their contributions extend the gather plan
  const int extend_from = first_touched >= nc ? nc : -1;
  // the tag slots move with the capture count
  for (int &sl : lay.row_slot)
    if (sl >= 3) sl += 6 * (h.nc - nc);
  nc = h.nc;
  nc_user = p->n_cap;
  nb = h.nb;
  n = h.n;
  nb_global = h.nb_global;
  slot_free = h.slot_free;
  x0 = h.x0;
  const double t3 = now_s();
  upload_problem(h, lay, extend_from);
  soa = *p;
  pk_appended_only = true;
  setup_kind = ARSLAM_SETUP_APPEND;
  setup_s = now_s() - t0;
  static const bool prof = std::getenv("ARSLAM_SETUP_PROFILE") != nullptr;   // debug: setup phases
  if (prof)
    std::fprintf(stderr, "arslam append: nc %d side %.3f host %.3f check %.3f upload %.3f ms\n", nc,
                 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), 1e3 * (now_s() - t3));
  return true;
}

// ARSLAM_ELIM_MIXED on a grown pointer-keyed problem (the reference's
// solveIncremental, ar_slam_util.cpp:629-742: new captures, each with
// residual blocks of known tags).  A fresh load would recompute Ceres' set
// (ComputeStableSchurOrdering) and rebuild the layout, plan and gather plan;
// here the set only grows: every new capture whose tags are all on the
// reduced side joins it as an eliminated group, appended after the loaded
// groups (so the loaded groups, the f-blocks and the gather plan's summation
// order are kept, and the plan is extended as for captures), and tags never
// leave the reduced side -- a new capture that sees an eliminated tag, a new
// tag or a residual on an old capture reloads.  The set is then the loaded
// problem's Ceres set plus the new captures: an independent set (a new
// capture is adjacent only to its tags, all reduced), not necessarily the
// one Ceres would pick on the grown graph; the step is the same exact solve.
bool arslam_lm::try_extend_mixed(const arslam_soa_problem *p) {
  if (!loaded || multi() || elim_used != ARSLAM_ELIM_MIXED || !has_f || opt.elimination != ARSLAM_ELIM_MIXED)
    return false;
  const double t0 = now_s();
  const long nb_old = (long)mx.obs_cap.size();
  const int ng_old = (int)mx.kind.size(), nf = (int)mx.f_src.size();
  if (p->n_tag != mx.src_n_tag || p->n_cap < mx.src_n_cap || p->n_obs <= nb_old) return false;
  // the f-block of each original tag (-1: eliminated or not a parameter)
  std::vector<int> tag_f(p->n_tag, -1);
  for (int f = 0; f < nf; ++f)
    if (!mx.f_is_cap[f]) tag_f[mx.f_src[f]] = f;
  // the new residuals: on new captures only, every tag on the reduced side
  for (long b = nb_old; b < p->n_obs; ++b)
    if (p->obs_cap[b] < mx.src_n_cap || tag_f[p->obs_tag[b]] < 0) return false;
  arslam::MixedProblem m = mx;
  const int nc_new = p->n_cap - mx.src_n_cap;
  std::vector<int> cap_g(nc_new, -1);
  for (long b = nb_old; b < p->n_obs; ++b) {
    const int c = p->obs_cap[b], q = c - mx.src_n_cap;
    if (cap_g[q] < 0) {
      cap_g[q] = (int)m.kind.size();
      m.kind.push_back(arslam::kMixCap);
      m.group_src.push_back(c);
      m.cap_const.push_back(p->cap_const ? p->cap_const[c] : 0);
    }
    m.obs_cap.push_back(cap_g[q]);
    m.obs_tag.push_back(tag_f[p->obs_tag[b]]);
  }
  for (int q = 0; q < nc_new; ++q)
    if (cap_g[q] < 0) return false;   // (a capture without residual blocks: not a block of Ceres' problem)
  const int ng = (int)m.kind.size();
  m.src_n_cap = p->n_cap;
  m.cap.resize(6L * ng);
  m.soa = *p;
  m.soa.n_cap = ng;
  m.soa.n_tag = nf;
  m.soa.cap = m.cap.data();
  m.soa.tag = m.tag.data();
  m.soa.obs_cap = m.obs_cap.data();
  m.soa.obs_tag = m.obs_tag.data();
  m.soa.cap_const = m.cap_const.data();
  m.soa.tag_const = m.tag_const.data();
  std::vector<double> xv(3 + 6L * ng + 6L * nf);
  arslam::mixed_values(m, *p, xv.data());
  std::memcpy(m.cap.data(), xv.data() + 3, 6L * ng * sizeof(double));
  if (nf) std::memcpy(m.tag.data(), xv.data() + 3 + 6L * ng, 6L * nf * sizeof(double));
  const double t1 = now_s();
  arslam::HostProblem h = arslam::host_problem(&m.soa, nullptr);
  arslam::mixed_patch(h, m, *p);
  const double t2 = now_s();
  // the same free f-blocks and camera (the same reduced rows)
  if ((lay.cam_row >= 0) != (h.slot_free[0] != 0)) return false;
  for (int f = 0; f < nf; ++f)
    if ((lay.tag_row[f] >= 0) != (h.slot_free[3 + 6L * h.nc + 6L * f] != 0)) return false;
  // every new group's tiles pairwise in the loaded factor's tiles
  const int T = lay.T;
  std::vector<int> ts;
  for (int g = ng_old; g < ng; ++g) {
    ts.clear();
    if (lay.cam_row >= 0) {
      ts.push_back(lay.cam_row / 64);
      ts.push_back((lay.cam_row + 2) / 64);
    }
    for (int a = h.cap_blk_start[g]; a < h.cap_blk_start[g + 1]; ++a) {
      const int r0 = lay.tag_row[h.blk_tag[a]];
      if (r0 < 0) continue;
      ts.push_back(r0 / 64);
      ts.push_back((r0 + 5) / 64);
    }
    for (size_t a = 0; a < ts.size(); ++a)
      for (size_t b = 0; b < ts.size(); ++b)
        if (ts[a] >= ts[b] && plan.h_tile_id[(size_t)ts[a] * T + ts[b]] < 0) return false;
  }
  for (int g = ng_old; g < ng; ++g) covis_add(h, lay, g);
  if (covis_nt && 10 * covis_edges > 11 * prev_order_edges) return false;
  if (4L * h.nc > 5L * prev_order_nc) return false;   // (a quarter more groups: a fresh order)
  // the f-block slots move with the group count
  for (int &sl : lay.row_slot)
    if (sl >= 3) sl += 6 * (h.nc - nc);
  mx = std::move(m);
  mx.soa.cap = mx.cap.data();   // (the moved vectors keep their buffers; re-pointed for clarity)
  mx.soa.tag = mx.tag.data();
  mx.soa.obs_cap = mx.obs_cap.data();
  mx.soa.obs_tag = mx.obs_tag.data();
  mx.soa.cap_const = mx.cap_const.data();
  mx.soa.tag_const = mx.tag_const.data();
  ceres_e_cap += nc_new;
  nc = h.nc;
  nc_full = h.nc;
  nc_user = p->n_cap;
  nb = h.nb;
  n = h.n;
  nb_global = h.nb_global;
  slot_free = h.slot_free;
  x0 = h.x0;
  const double t3 = now_s();
  upload_problem(h, lay, ng_old);
  soa = *p;
  pk_appended_only = true;
  setup_kind = ARSLAM_SETUP_APPEND;
  setup_s = now_s() - t0;
  static const bool prof = std::getenv("ARSLAM_SETUP_PROFILE") != nullptr;   // debug: setup phases
  if (prof)
    std::fprintf(stderr, "arslam append (mixed): groups %d host %.3f check %.3f upload %.3f ms\n", ng,
                 1e3 * (t2 - t1), 1e3 * (t3 - t2), 1e3 * (now_s() - t3));
  return true;
}

// Same structure as the loaded problem, new parameter values (the pointer-keyed
// path when no block, residual or constant changed since the last load).
void arslam_lm::reload_values(const arslam_soa_problem *p_in) {
  const double t0 = now_s();
  if (elim_used == ARSLAM_ELIM_MIXED) {   // the regrouped slots from p_in's blocks
    fail_if(!loaded || p_in->n_obs != (int)mx.obs_cap.size() || p_in->n_cap != mx.src_n_cap ||
                p_in->n_tag != mx.src_n_tag, ARSLAM_E_STATE,
            "reload_values: structure differs from the loaded problem");
    arslam::mixed_values(mx, *p_in, x0.data());
    HIP_CHECK(hipMemcpyAsync(u_x0, x0.data(), n * sizeof(double), hipMemcpyHostToDevice, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    soa = *p_in;
    setup_kind = ARSLAM_SETUP_VALUES;
    setup_s = now_s() - t0;
    return;
  }
  const arslam_soa_problem swapped = arslam::swap_roles(*p_in);
  const arslam_soa_problem *p = elim_used == ARSLAM_ELIM_TAGS ? &swapped : p_in;
  fail_if(!loaded || p->n_cap != nc_full || p->n_tag != nt || (!multi() && p->n_obs != nb), ARSLAM_E_STATE,
          "reload_values: structure differs from the loaded problem");
  std::memcpy(x0.data(), p->camera, 3 * sizeof(double));
  if (multi()) {
    for (int c = 0; c < nc; ++c) std::memcpy(x0.data() + 3 + 6L * c, p->cap + 6L * own_caps[c], 6 * sizeof(double));
  } else if (nc) {
    std::memcpy(x0.data() + 3, p->cap, 6L * nc * sizeof(double));
  }
  if (nt) std::memcpy(x0.data() + 3 + 6L * nc, p->tag, 6L * nt * sizeof(double));
  HIP_CHECK(hipMemcpyAsync(u_x0, x0.data(), n * sizeof(double), hipMemcpyHostToDevice, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  soa = *p;
  setup_kind = ARSLAM_SETUP_VALUES;
  setup_s = now_s() - t0;
}

// Evaluate residuals/Jacobian at x: cost, gradient (unscaled), column norms
// and the norms the minimizer reads.  Ceres EvaluateGradientAndJacobian.
void arslam_lm::linearize_launch() {
  h_lin.alloc(32);
  // one rank: the reductions also store their results straight into the
  // page-locked h_lin (no copy launch); several: h_lin is copied after the exchanges
  const bool direct = !multi();
  timers[PH_LIN].start(stream);
  arslam::launch_linearize(P, x, d_g.p, d_colnorm.p, d_obs_tg.p, d_parts.p, stream);
  // (several ranks: this rank's partial cost and fixed cost also saved, the
  // step's reductions reuse d_red, for the scalar exchange; the LM diagonal
  // from the partial sums is final for the capture slots and this rank's own
  // subtree tags -- all their observations are this rank's -- the rest
  // follows the exchange, lin_norms)
  arslam::launch_lin_reduce(P, d_obs_tg.p, d_g.p, d_colnorm.p, d_parts.p, d_red.p, stream,
                            direct ? h_lin.p : nullptr, multi() ? d_red.p + kLinSave : nullptr);
  if (multi()) lin_xpending = true;
  const arslam::LmDiagArgs ld{n, d_scale.p, d_colnorm.p, opt.min_lm_diagonal, opt.max_lm_diagonal, d_diag.p};
  lin_seq = direct ? next_seq(h_lin.p + 16 + arslam::kHostSeq) : 0.0;
  arslam::launch_slot_norms(P, d_red.p, d_g.p, d_colnorm.p, x, d_norms_p, stream, direct ? h_lin.p + 16 : nullptr,
                            diag_in_lin ? &ld : nullptr, lin_seq);
  timers[PH_LIN].stop(stream);
}

// (several ranks) the norms and the LM diagonal again, from the exchanged sums
void arslam_lm::lin_norms() {
  const arslam::LmDiagArgs ld{n, d_scale.p, d_colnorm.p, opt.min_lm_diagonal, opt.max_lm_diagonal, d_diag.p};
  arslam::launch_slot_norms(P, d_red.p, d_g.p, d_colnorm.p, x, d_norms_p, stream, nullptr, diag_in_lin ? &ld : nullptr);
  lin_xpending = false;
  norms_pending = true;   // capture slots and the held f-side slots: combined with the next scalars
}

// (several ranks) a pending linearization's sums when no step carries them:
// every tag slot's gradient and column norm and the camera's f partials, one
// packed all-reduce (the tags' observations span the ranks)
void arslam_lm::complete_pending_lin() {
  if (!lin_xpending) return;
  const long t0 = 3 + 6L * nc;
  arslam::PackSegs sg;
  sg.add(d_g.p + t0, n - t0);
  sg.add(d_colnorm.p + t0, n - t0);
  sg.add(d_red.p + arslam::P_GF, 2);   // g_f, col_f
  d_lx.alloc(sg.total());
  arslam::launch_pack(sg, d_lx.p, false, stream);
  allreduce(d_lx.p, sg.total(), ARSLAM_OP_SUM);
  arslam::launch_pack(sg, d_lx.p, true, stream);
  lin_norms();
}

// Several ranks: the scalars of fl (indices into d_red) and, if a
// linearization's norms are pending, its capture-slot norms, all-gathered in
// one SUM all-reduce and combined in rank order (k_ag_put / k_ag_reduce: the
// same bits on every rank); the norms then go to h_lin like the rest of it.
void arslam_lm::exchange_scalars(arslam::AgFields fl, arslam::HostOut *ho) {
  const bool with_norms = norms_pending;
  if (with_norms) {
    // the norms over the slots each rank holds (captures; its f-side slots)
    const int nb0 = (int)(d_norms_p - d_red.p);
    for (int q = 0; q < 6; ++q) fl.add(nb0 + q, q % 3 == 0);   // max |g|, sum g^2, sum x^2 (captures, then f-side)
    fl.add(kLinSave, false);       // the linearization's cost
    fl.add(kLinSave + 1, false);   // ... and fixed cost
  }
  if (fl.n == 0 && !ho) return;   // (with ho the combining launch still stores the host words)
  d_ag.alloc((size_t)nranks * arslam::kAgFields);
  arslam::launch_ag_put(d_red.p, fl, d_ag.p, nranks, rank, stream);
  allreduce(d_ag.p, (size_t)nranks * arslam::kAgFields, ARSLAM_OP_SUM);
  if (with_norms && ho) {   // (the combining launch stores them with the step's words)
    h_lin.alloc(32);
    ho->add(d_norms_p, h_lin.p + 16, 6);
    ho->add(d_red.p + kLinSave, h_lin.p, 2);
  }
  arslam::launch_ag_reduce(d_ag.p, fl, d_red.p, nranks, stream, ho);
  if (with_norms) {
    if (!ho) {
      HIP_CHECK(hipMemcpyAsync(h_lin.p + 16, d_norms_p, 6 * sizeof(double), hipMemcpyDeviceToHost, stream));
      HIP_CHECK(hipMemcpyAsync(h_lin.p, d_red.p + kLinSave, 2 * sizeof(double), hipMemcpyDeviceToHost, stream));
    }
    norms_pending = false;
  }
}

// (after a stream sync that covers linearize_launch)
void arslam_lm::linearize_collect(double *x_cost, double *fixed_cost, double *gmax, double *gnorm,
                                  double *xnorm) {
  const double *red = h_lin.p, *norms = h_lin.p + 16;
  *x_cost = red[arslam::P_COST];
  *fixed_cost = red[arslam::P_FIXED];
  *gmax = std::max(norms[0], norms[3]);
  *gnorm = std::sqrt(norms[1] + norms[4]);
  *xnorm = std::sqrt(norms[2] + norms[5]);
  timers[PH_LIN].collect();
}

// Evaluate residuals/Jacobian at x: cost, gradient (unscaled), column norms
// and the norms the minimizer reads.  Ceres EvaluateGradientAndJacobian.
void arslam_lm::linearize(double *x_cost, double *fixed_cost, double *gmax, double *gnorm,
                          double *xnorm) {
  linearize_launch();
  complete_pending_lin();
  exchange_norms();
  lin_sync();
  linearize_collect(x_cost, fixed_cost, gmax, gnorm, xnorm);
}

void arslam_lm::write_back(const double *d_src) {
  h_x.alloc(n + 1);   // page-locked; [n]: the download's sequence word (one rank)
  static const bool dma = std::getenv("ARSLAM_WRITE_BACK_DMA") != nullptr;   // debug A/B: the copy engine
  if (!multi() && !dma) {
    // a kernel stores x into h_x and then the sequence word the host polls
    // (the copy engine's download and an event behind it took ~70 us per
    // Solve on the incremental flow)
    const double seq = next_seq(h_x.p + n);
    arslam::launch_copy_out(d_src, n, h_x.p, d_seq_done.p, h_x.p + n, seq, stream);
    flag_sync(h_x.p + n, seq);
  } else {
    HIP_CHECK(hipMemcpyAsync(h_x.p, d_src, n * sizeof(double), hipMemcpyDeviceToHost, stream));
  }
  if (multi()) {
    // the camera and each tag from the rank holding it (the others hold stale
    // values of other ranks' subtree tags, and of the camera when its rows are
    // not in the replicated top -- a split with one active rank and no top):
    // one all-reduce of the held values, zeros elsewhere
    const long t0 = 3 + 6L * nc;
    d_lx.alloc(3 + n - t0);
    arslam::launch_own_copy(P, 0, 3, d_src, d_lx.p, stream);
    arslam::launch_own_copy(P, t0, n - t0, d_src + t0, d_lx.p + 3, stream);
    allreduce(d_lx.p, 3 + n - t0, ARSLAM_OP_SUM);
    HIP_CHECK(hipMemcpyAsync(h_x.p, d_lx.p, 3 * sizeof(double), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipMemcpyAsync(h_x.p + t0, d_lx.p + 3, (n - t0) * sizeof(double), hipMemcpyDeviceToHost, stream));
  }
  if (multi() || dma) spin_sync();
  const double *h = h_x.p;
  std::memcpy(soa.camera, h, 3 * sizeof(double));
  if (elim_used == ARSLAM_ELIM_MIXED) {   // groups (not the direct ones: copies) and f-blocks to their blocks
    for (int g = 0; g < nc; ++g)
      if (mx.kind[g] != arslam::kMixDirect)
        std::memcpy((mx.kind[g] == arslam::kMixTag ? soa.tag : soa.cap) + 6L * mx.group_src[g], h + 3 + 6L * g,
                    6 * sizeof(double));
    for (int f = 0; f < nt; ++f)
      std::memcpy((mx.f_is_cap[f] ? soa.cap : soa.tag) + 6L * mx.f_src[f], h + 3 + 6L * nc + 6L * f,
                  6 * sizeof(double));
  } else if (multi()) {   // this rank's captures into the whole problem's array
    for (int c = 0; c < nc; ++c) std::memcpy(soa.cap + 6L * own_caps[c], h + 3 + 6L * c, 6 * sizeof(double));
  } else if (nc) {
    std::memcpy(soa.cap, h + 3, 6L * nc * sizeof(double));
  }
  if (nt && elim_used != ARSLAM_ELIM_MIXED) std::memcpy(soa.tag, h + 3 + 6L * nc, 6L * nt * sizeof(double));
  if (pk_stage) scatter_to_blocks();
}

// Pointer-keyed path: the staging arrays (which soa aliases, role-swapped or
// not) -> the caller's parameter blocks, as Ceres writes the user's blocks.
void arslam_lm::scatter_to_blocks() {
  const arslam_soa_problem &p = *pk_stage;
  std::memcpy(camera_ptr, p.camera, 3 * sizeof(double));
  for (size_t c = 0; c < cap_ptrs.size(); ++c) std::memcpy(cap_ptrs[c], p.cap + 6 * c, 6 * sizeof(double));
  for (size_t t = 0; t < tag_ptrs.size(); ++t) std::memcpy(tag_ptrs[t], p.tag + 6 * t, 6 * sizeof(double));
}

void arslam_lm::restore_patched_wait() {
  if (dbg_patched_wait < 0) return;
  const int w = dbg_patched_wait;
  dbg_patched_wait = -1;
  plan.h_dag_waits[w].y -= 1 << 28;
  HIP_CHECK(hipMemcpyAsync(plan.dag_waits + w, &plan.h_dag_waits[w], sizeof(int2), hipMemcpyHostToDevice, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
}

// Several ranks: every rank takes the same branch on the callbacks' answers
// (MAX over the ranks of continue 0 < terminate successfully 1 < abort 2).
int arslam_lm::agree_callback(int r) {
  if (!multi()) return r;
  const double v = r == ARSLAM_SOLVER_ABORT ? 2.0 : r == ARSLAM_SOLVER_TERMINATE_SUCCESSFULLY ? 1.0 : 0.0;
  d_cb.alloc(1);
  HIP_CHECK(hipMemcpyAsync(d_cb.p, &v, sizeof(double), hipMemcpyHostToDevice, stream));
  allreduce(d_cb.p, 1, ARSLAM_OP_MAX);
  double m = 0.0;
  HIP_CHECK(hipMemcpyAsync(&m, d_cb.p, sizeof(double), hipMemcpyDeviceToHost, stream));
  HIP_CHECK(hipStreamSynchronize(stream));
  return m >= 2.0 ? ARSLAM_SOLVER_ABORT : m >= 1.0 ? ARSLAM_SOLVER_TERMINATE_SUCCESSFULLY : ARSLAM_SOLVER_CONTINUE;
}

namespace {

void print_header() {
  std::printf("iter      cost      cost_change  |gradient|   |step|    tr_ratio  tr_radius  ls_iter  iter_time  total_time\n");
}

void print_row(const arslam_lm_iteration &it) {
  std::printf("% 4d % 8e   % 3.2e   % 3.2e  % 3.2e  % 3.2e % 3.2e     % 4d   % 3.2e   % 3.2e\n",
              it.iteration, it.cost, it.cost_change, it.gradient_max_norm, it.step_norm,
              it.relative_decrease, it.trust_region_radius, 0, it.iteration_time, it.cumulative_time);
  std::fflush(stdout);
}

}  // namespace

void arslam_lm::solve(arslam_lm_summary *s) {
  fail_if(!loaded, ARSLAM_E_STATE, "no problem loaded");
  const arslam_lm_options &o = opt;
  const double t_start = now_s();
  std::memset(s, 0, sizeof(*s));
  for (auto &t : timers) {
    t.acc_ms = 0.0;
    t.on = o.phase_timing != 0;
  }
  dom_ms = dom_flops = 0.0;
  dom_launches = 0;
  comm_bytes = 0.0;
  comm_calls = 0;
  norms_pending = lin_xpending = false;
  s->n_obs = nb;
  s->n_reduced = has_f ? (int)nR : 0;
  s->setup_time_s = setup_s;
  for (int i = 0; i < 5; ++i) s->setup_phase_s[i] = setup_phase[i];
  s->setup_kind = setup_kind;
  x = d_xa.p;
  xc = d_xb.p;
  xbest = x;   // (iteration 0's finalize makes it so)
  HIP_CHECK(hipMemcpyAsync(x, u_x0, n * sizeof(double), hipMemcpyDeviceToDevice, stream));
  const bool root = rank == 0;
  if (o.minimizer_progress_to_stdout && root) print_header();
  // the patched dependency of arslam_lm_debug_break_dependency lasts one solve
  struct RestoreWait {
    arslam_lm *h;
    ~RestoreWait() {
      try { h->restore_patched_wait(); } catch (...) {}
    }
  } restore_wait{this};
  any_iter_cb = iter_cb != nullptr;
  if (multi()) {   // a callback on any rank: every rank joins the per-iteration agreement
    const double mine = iter_cb ? 1.0 : 0.0;
    d_cb.alloc(1);
    HIP_CHECK(hipMemcpyAsync(d_cb.p, &mine, sizeof(double), hipMemcpyHostToDevice, stream));
    allreduce(d_cb.p, 1, ARSLAM_OP_MAX);
    double m = 0.0;
    HIP_CHECK(hipMemcpyAsync(&m, d_cb.p, sizeof(double), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    any_iter_cb = m > 0.0;
    comm_bytes = 0.0;   // (the per-step exchange count starts here)
    comm_calls = 0;
  }

  // ---- iteration 0 ----
  double x_cost, fixed_cost, gmax, gnorm, x_norm;
  linearize(&x_cost, &fixed_cost, &gmax, &gnorm, &x_norm);
  s->fixed_cost = fixed_cost;
  s->initial_cost = x_cost + fixed_cost;
  s->final_cost = s->initial_cost;
  if (!std::isfinite(x_cost)) {
    s->termination = ARSLAM_FAILURE;
    s->rule = ARSLAM_RULE_EVAL_FAILED;
    s->total_time_s = now_s() - t_start;
    return;
  }
  {
    // the scale, and from it the first step's LM diagonal (k_lm_diag's work)
    const arslam::LmDiagArgs ld{n, d_scale.p, d_colnorm.p, o.min_lm_diagonal, o.max_lm_diagonal, d_diag.p};
    arslam::launch_scale(P, d_colnorm.p, o.jacobi_scaling, d_scale.p, stream, &ld);
  }
  diag_in_lin = true;
  struct DiagInLin {   // (off again when the solve ends, however it ends)
    arslam_lm *h;
    ~DiagInLin() { h->diag_in_lin = false; }
  } diag_in_lin_guard{this};

  double radius = o.initial_trust_region_radius, decrease_factor = 2.0;
  bool reuse_diag = false;
  int n_invalid = 0;
  double minimum_cost = x_cost;
  arslam_lm_iteration it{};
  it.iteration = 0;
  it.cost = x_cost + fixed_cost;
  it.gradient_max_norm = gmax;
  it.gradient_norm = gnorm;
  it.step_is_valid = 1;
  it.step_is_successful = 1;
  double t_iter = t_start;

  // A successful step's re-linearization is only enqueued (lin_pending): the
  // next step's kernels follow it in the stream, and its results are read at
  // that step's one host sync, where the finalization below runs first.  If
  // it then stops the minimizer, the speculative step is dropped uncounted.
  bool lin_pending = false;
  double prev_gmax = 0.0, prev_gnorm = 0.0;
  auto finalize = [&]() -> bool {   // true: the minimizer stops
    if (lin_pending) {
      double fc;
      linearize_collect(&x_cost, &fc, &gmax, &gnorm, &x_norm);
      it.cost = x_cost + fixed_cost;
      it.gradient_max_norm = gmax;
      it.gradient_norm = gnorm;
      lin_pending = false;
    }
    // ---- FinalizeIterationAndCheckIfMinimizerCanContinue ----
    if (it.step_is_successful) {
      if (it.iteration > 0) s->num_successful_steps++;
      if (x_cost < minimum_cost || it.iteration == 0) {
        minimum_cost = x_cost;
        xbest = x;   // (by pointer: no copy; the step in flight writes xc)
        if (o.update_state_every_iteration) write_back(xbest);
      }
    } else {
      s->num_unsuccessful_steps++;
    }
    it.trust_region_radius = radius;
    const double tn = now_s();
    it.iteration_time = tn - t_iter;
    it.cumulative_time = tn - t_start;
    t_iter = tn;
    if (s->n_iters <= ARSLAM_LM_MAX_ITERS) s->iters[s->n_iters++] = it;
    if (o.minimizer_progress_to_stdout && root) print_row(it);
    if (iter_cb || any_iter_cb) {   // Ceres RunCallbacks: after the record, before the stop rules
      const int r = agree_callback(iter_cb ? iter_cb(iter_cb_ctx, &it) : ARSLAM_SOLVER_CONTINUE);
      if (r == ARSLAM_SOLVER_ABORT) {
        s->termination = ARSLAM_USER_FAILURE; s->rule = ARSLAM_RULE_USER_CALLBACK; return true;
      }
      if (r == ARSLAM_SOLVER_TERMINATE_SUCCESSFULLY) {
        s->termination = ARSLAM_USER_SUCCESS; s->rule = ARSLAM_RULE_USER_CALLBACK; return true;
      }
    }
    if (it.iteration >= o.max_num_iterations) {
      s->termination = ARSLAM_NO_CONVERGENCE; s->rule = ARSLAM_RULE_MAX_ITERS; return true;
    }
    if (it.step_is_successful && it.gradient_max_norm <= o.gradient_tolerance) {
      s->termination = ARSLAM_CONVERGENCE; s->rule = ARSLAM_RULE_GRADIENT; return true;
    }
    if (radius <= o.min_trust_region_radius) {
      s->termination = ARSLAM_CONVERGENCE; s->rule = ARSLAM_RULE_MIN_RADIUS; return true;
    }
    prev_gmax = it.gradient_max_norm;
    prev_gnorm = it.gradient_norm;
    const int next_iter = it.iteration + 1;
    it = arslam_lm_iteration{};
    it.iteration = next_iter;
    return false;
  };

  for (;;) {
    // the stop rules that do not read the pending linearization: decided now
    // (after reading it), so no step is computed past them
    const bool stop_rule = it.iteration >= o.max_num_iterations || radius <= o.min_trust_region_radius;
    if (lin_pending && stop_rule) {
      complete_pending_lin();
      exchange_norms();
      lin_sync();
    }
    const bool deferred = lin_pending && !stop_rule;
    if (!deferred && finalize()) break;

    // ---- ComputeTrustRegionStep: LM diagonal, DENSE_SCHUR solve ----
    s->num_linear_solves++;
    const bool exec_dag = has_f && opt.factor_executor == 1;
    // the LM diagonal is current: k_scale formed it for the first step and
    // every accepted step's linearization re-forms it (k_slot_norms); a
    // rejected or invalid step keeps it
    arslam::ExecReset er{};
    const bool reset_in_schur = exec_dag && has_f && nc > 0;
    if (reset_in_schur) {
      // flag + executor counters + the backward solve's y sentinels: in k_schur's launch
      er = arslam::exec_reset_args(plan, d_flag.p, d_yF.p, nR);
    } else if (exec_dag) {
      const arslam::LmDiagArgs ld{0, d_scale.p, d_colnorm.p, o.min_lm_diagonal, o.max_lm_diagonal, d_diag.p, d_yF.p, nR};
      arslam::launch_exec_reset(plan, d_flag.p, stream, &ld);
    } else {
      if (!reuse_diag)
        arslam::launch_lm_diag(P, d_scale.p, d_colnorm.p, o.min_lm_diagonal, o.max_lm_diagonal, d_diag.p, stream);
      HIP_CHECK(hipMemsetAsync(d_flag.p, 0, sizeof(int), stream));
    }
    reuse_diag = true;
    // several ranks: a pending linearization's sums ride with the top tiles
    // (below), unless this step has no such exchange
    static const bool dag_trace_env = std::getenv("ARSLAM_DAG_TRACE") != nullptr;
    if (lin_xpending && !(has_f && opt.factor_executor == 1 && !dag_trace_env)) complete_pending_lin();
    if (has_f) {
      timers[PH_SCHUR].start(stream);
      // one rank: the gather writes the final S (D_f^2 and the padding rows
      // included).  Several: this rank's captures' share; the D_f^2 of the
      // rank's own subtree rows now, of the top rows after their exchange
      // (below).  k_schur's extra blocks clear S's tiles first.
      // (one rank on the persistent executor: the fill tiles the gather does
      // not write are left as they are -- their first update stores)
      const bool fill_first_store = !multi() && opt.factor_executor == 1;
      arslam::launch_schur(P, x, d_scale.p, d_diag.p, radius, Sp, stream, !multi(),
                           fill_first_store ? n_clear : plan.n_tiles, reset_in_schur ? &er : nullptr);
      const bool force_indefinite = dbg_indefinite_mask >> std::min(s->num_linear_solves - 1, 63) & 1ull;
      const long hook_row = P.cam_row >= 0 ? P.cam_row : nR - 1;   // (a top row with several ranks)
      if (multi()) arslam::launch_prep_reduced(P, d_diag.p, radius, Sp, stream, 0);
      else if (force_indefinite) arslam::debug_set_reduced_diag(P, Sp, hook_row, -1.0, stream);   // test hook
      timers[PH_SCHUR].stop(stream);
      timers[PH_CHOL].start(stream);
      timing_begin();
      if (opt.factor_executor == 1) {
        const bool rec = opt.kernel_timing && upd_timing.used < upd_timing.cap;
        if (rec) HIP_CHECK(hipEventRecord(upd_timing.ev[2 * upd_timing.used], stream));
        static const char *trace_path = std::getenv("ARSLAM_DAG_TRACE");   // debug: dump one task timeline
        static const int trace_skip = std::getenv("ARSLAM_DAG_TRACE_SKIP") ? std::atoi(std::getenv("ARSLAM_DAG_TRACE_SKIP")) : 0;
        if (trace_path && !dag_traced && dag_trace_seen++ >= trace_skip) {
          DevBuf<unsigned long long> tr;
          tr.alloc(8 * plan.n_dag_tasks);
          HIP_CHECK(hipMemsetAsync(tr.p, 0, tr.n * 8, stream));
          arslam::launch_dense_llt_dag(plan, Sp, d_flag.p, stream, dag_workgroups, nullptr, tr.p, false, -1,
                                       fill_first_store ? n_clear : LONG_MAX);
          std::vector<unsigned long long> h(8 * plan.n_dag_tasks);
          HIP_CHECK(hipMemcpyAsync(h.data(), tr.p, h.size() * 8, hipMemcpyDeviceToHost, stream));
          HIP_CHECK(hipStreamSynchronize(stream));
          if (FILE *f = std::fopen(trace_path, "wb")) {
            const long n = plan.n_dag_tasks;
            std::fwrite(&n, 8, 1, f);
            std::fwrite(plan.h_dag_tasks.data(), sizeof(int4), n, f);
            std::fwrite(h.data(), 8, h.size(), f);
            const long nw = (long)plan.h_dag_waits.size();   // the dependency lists, for dag_critical.py
            std::fwrite(&nw, 8, 1, f);
            std::fwrite(plan.h_dag_wait_off.data(), sizeof(int), n + 1, f);
            std::fwrite(plan.h_dag_waits.data(), sizeof(int2), nw, f);
            std::fwrite(plan.h_dag_sub.data(), sizeof(int2), n, f);   // fused TRSM tiles
            std::fclose(f);
          }
          dag_traced = true;
        } else if (multi()) {
          // phase 0: this rank's subtree columns, and their updates of the top
          // tiles (its share of the top's Schur complement); then the top tiles
          // are summed over the ranks -- the step's one bulk exchange -- and
          // every rank factors the top columns (phase 1) on identical inputs
          timers[PH_FAC0].start(stream);
          arslam::launch_dense_llt_dag(plan, Sp, d_flag.p, stream, dag_workgroups, nullptr, nullptr, false, 0);
          timers[PH_FAC0].stop(stream);
          // (+ a pending linearization's top-tag sums and camera partials, in
          // front of the top tiles: the step's collectives stay two)
          const long tail = lin_xpending ? top_tail_len() : 0;
          if (tail) arslam::launch_top_tail(u_top_slots, n_top_slots, d_g.p, d_colnorm.p, d_red.p, Sp - tail, false, stream);
          allreduce(Sp - tail, (size_t)tail + (size_t)plan.n_top_tiles * 4096, ARSLAM_OP_SUM);
          if (tail) {
            arslam::launch_top_tail(u_top_slots, n_top_slots, d_g.p, d_colnorm.p, d_red.p, Sp - tail, true, stream);
            lin_norms();   // the LM diagonal of the top rows, then their D^2
          }
          arslam::launch_prep_reduced(P, d_diag.p, radius, Sp, stream, 1);
          if (force_indefinite) arslam::debug_set_reduced_diag(P, Sp, hook_row, -1.0, stream);   // test hook
          timers[PH_FAC1].start(stream);
          arslam::launch_dense_llt_dag(plan, Sp, d_flag.p, stream, dag_workgroups, nullptr, nullptr, false, 1);
          timers[PH_FAC1].stop(stream);
        } else {
          arslam::launch_dense_llt_dag(plan, Sp, d_flag.p, stream, dag_workgroups, nullptr, nullptr, false, -1,
                                       fill_first_store ? n_clear : LONG_MAX);
        }
        if (rec) {
          HIP_CHECK(hipEventRecord(upd_timing.ev[2 * upd_timing.used + 1], stream));
          upd_timing.used++;
          upd_timing.flops += plan.total_factor_flops;
        }
        static const char *hash_path = std::getenv("ARSLAM_FACTOR_HASH");   // debug: per-tile factor hashes
        if (hash_path) {
          std::vector<unsigned long long> h((size_t)plan.n_tiles * 4096), ld((size_t)plan.T * 4096);
          HIP_CHECK(hipMemcpyAsync(h.data(), Sp, h.size() * 8, hipMemcpyDeviceToHost, stream));
          HIP_CHECK(hipMemcpyAsync(ld.data(), plan.ldiag, ld.size() * 8, hipMemcpyDeviceToHost, stream));
          HIP_CHECK(hipStreamSynchronize(stream));
          if (FILE *f = std::fopen(hash_path, "ab")) {
            const long nt = plan.n_tiles, T = plan.T;
            std::fwrite(&nt, 8, 1, f);
            std::fwrite(&T, 8, 1, f);
            std::vector<long> tmap(plan.h_tile_id.begin(), plan.h_tile_id.end());
            std::fwrite(tmap.data(), 8, tmap.size(), f);
            for (const auto *v : {&h, &ld})
              for (size_t t = 0; t < v->size() / 4096; ++t) {
                unsigned long long x = 1469598103934665603ull;
                for (int e = 0; e < 4096; ++e) x = (x ^ (*v)[t * 4096 + e]) * 1099511628211ull;
                std::fwrite(&x, 8, 1, f);
              }
            std::fclose(f);
          }
        }
      } else {
        arslam::launch_dense_llt(plan, Sp, d_flag.p, stream, opt.kernel_timing ? &upd_timing : nullptr);
      }
      timers[PH_CHOL].stop(stream);
      timers[PH_SOLVE].start(stream);
      if (opt.factor_executor == 1)
        arslam::launch_dense_back_solve_dag(plan, Sp, nR, d_yF.p, d_flag.p, stream, dag_workgroups, false);
      else
        arslam::launch_dense_back_solve(plan, Sp, nR, d_z.p, d_yF.p, d_flag.p, stream);
      if (multi()) {
        // y of the top columns (identical on every rank) and of this rank's
        // own subtrees; no exchange: a rank's captures see only those tags
        // (a capture's tags lie on one root path of the elimination tree), so
        // each rank updates the tags it holds and keeps the others' stale,
        // and the sums over f-side slots count each slot on its holder
        // (DevProblem::f_own); the final tags are gathered in write_back
        arslam::launch_mask_y(P, d_yF.p, rank, stream, true);
      }
      timers[PH_SOLVE].stop(stream);
    }
    timers[PH_BACK].start(stream);
    // (k_update_f writes every f-side slot of xc, k_backsub every capture
    // slot, then evaluates the candidate's cost per capture: k_cost fused)
    arslam::launch_update_f(P, x, d_scale.p, d_yF.p, xc, d_fparts.p, stream);
    arslam::launch_backsub(P, x, d_scale.p, d_diag.p, radius, d_yF.p, xc, d_parts.p, stream, has_f, true);
    timers[PH_BACK].stop(stream);
    timers[PH_COST].start(stream);
    h_step.alloc(16);
    // (one rank: the scalars are also stored straight into the page-locked h_step)
    double step_seq = !multi() ? next_seq(h_step.p + arslam::kHostSeq) : 0.0;
    arslam::launch_reduce_parts(d_parts.p, nc, d_fparts.p, n_fparts, d_red.p, stream, d_flag.p,
                                !multi() ? h_step.p : nullptr, d_seq_done.p, step_seq);
    if (multi()) {
      // candidate cost, fixed, model change, capture step^2 by sum; the
      // non-finite flags, the f-side non-finite step, indefinite and executor
      // fault by max (every rank takes the same branch); with a pending
      // linearization's norms: one collective
      arslam::AgFields fl;
      for (int f : {(int)arslam::P_COST, (int)arslam::P_FIXED, (int)arslam::P_MODEL, (int)arslam::P_STEP2,
                    (int)arslam::NPART})   // (NPART: the f-side step^2, of the slots this rank holds)
        fl.add(f, false);
      for (int f : {(int)arslam::P_YBAD, (int)arslam::P_CBAD, arslam::NPART + 1, arslam::NPART + 2, arslam::NPART + 3})
        fl.add(f, true);
      // the step's words (and a pending linearization's norms) stored to the
      // host by the combining launch, then its sequence number
      arslam::HostOut ho;
      ho.add(d_red.p, h_step.p, arslam::NPART + 5);
      step_seq = next_seq(h_step.p + arslam::kHostSeq);
      ho.seq_word = h_step.p + arslam::kHostSeq;
      ho.seq = step_seq;
      exchange_scalars(fl, &ho);
    }
    timers[PH_COST].stop(stream);
    flag_sync(h_step.p + arslam::kHostSeq, step_seq);
    const double *red = h_step.p;
    // A stuck dependency wait of a persistent executor is a device fault, not
    // an indefinite system: fail loudly instead of shrinking the radius.
    if (red[arslam::NPART + 3] != 0.0)
      throw Error(ARSLAM_E_DEVICE, executor_fault_message((int)red[arslam::NPART + 4], rank, it.iteration, plan, stream));
    for (int ph = PH_SCHUR; ph < PH_N; ++ph) timers[ph].collect();
    timing_collect();
    if (deferred && finalize()) {
      s->num_linear_solves--;   // the speculative step is not part of the trace
      break;
    }

    const bool lin_fail = red[arslam::NPART + 2] != 0.0;   // LLT failure: Ceres' invalid step
    const bool ybad = red[arslam::P_YBAD] != 0.0 || red[arslam::NPART + 1] != 0.0;
    const double model_cost_change = red[arslam::P_MODEL];
    const bool valid = !lin_fail && !ybad && model_cost_change > 0.0;
    if (!valid) {
      // Ceres 2.0 HandleInvalidStep: ++num_consecutive_invalid_steps_ >= max -> FAILURE
      // (the 5th consecutive invalid step at the default 5, not recorded)
      if (++n_invalid >= o.max_num_consecutive_invalid_steps) {
        s->termination = ARSLAM_FAILURE; s->rule = ARSLAM_RULE_INVALID_STEPS; break;
      }
      radius = radius / decrease_factor;   // StepIsInvalid
      decrease_factor *= 2.0;
      reuse_diag = true;
      it.cost = x_cost + fixed_cost;
      it.gradient_max_norm = prev_gmax;
      it.gradient_norm = prev_gnorm;
      it.step_is_valid = 0;
      it.step_is_successful = 0;
      continue;
    }
    n_invalid = 0;
    it.step_is_valid = 1;
    double candidate_cost = red[arslam::P_COST];
    if (!std::isfinite(candidate_cost) || red[arslam::P_CBAD] != 0.0) candidate_cost = DBL_MAX;
    it.step_norm = std::sqrt(red[arslam::P_STEP2] + red[arslam::NPART]);
    // ---- ParameterToleranceReached ----
    if (it.step_norm <= o.parameter_tolerance * (x_norm + o.parameter_tolerance)) {
      s->termination = ARSLAM_CONVERGENCE; s->rule = ARSLAM_RULE_PARAMETER; break;
    }
    // ---- FunctionToleranceReached ----
    it.cost_change = x_cost - candidate_cost;
    if (std::fabs(it.cost_change) <= o.function_tolerance * x_cost) {
      s->termination = ARSLAM_CONVERGENCE; s->rule = ARSLAM_RULE_FUNCTION; break;
    }
    // ---- IsStepSuccessful ----
    it.relative_decrease = candidate_cost >= DBL_MAX ? -DBL_MAX
                                                     : (x_cost - candidate_cost) / model_cost_change;
    if (it.relative_decrease > o.min_relative_decrease) {
      // the candidate becomes x; the next candidate goes to a buffer that is
      // neither x nor the best point (the old x, unless it is the best: its
      // successor's cost is read only at the next sync, after the next step
      // is enqueued)
      double *old = x;
      x = xc;
      xc = old != xbest ? old : (d_xa.p != x && d_xa.p != xbest) ? d_xa.p : (d_xb.p != x && d_xb.p != xbest) ? d_xb.p : d_xbest.p;
      linearize_launch();   // read at the next step's sync (finalize)
      lin_pending = true;
      it.step_is_successful = 1;
      const double q = 2.0 * it.relative_decrease - 1.0;
      radius = radius / std::max(1.0 / 3.0, 1.0 - q * q * q);
      radius = std::min(o.max_trust_region_radius, radius);
      decrease_factor = 2.0;
      reuse_diag = false;
    } else {
      it.step_is_successful = 0;
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      reuse_diag = true;
      it.cost = candidate_cost + fixed_cost;
      it.gradient_max_norm = prev_gmax;
      it.gradient_norm = prev_gnorm;
    }
  }
  s->final_cost = minimum_cost + fixed_cost;
  s->minimizer_time_s = now_s() - t_start;
  write_back(xbest);
  s->total_time_s = now_s() - t_start;
  static const bool prof = std::getenv("ARSLAM_SETUP_PROFILE") != nullptr;   // debug: setup phases
  if (prof) std::fprintf(stderr, "arslam write_back %.3f ms\n", 1e3 * (s->total_time_s - s->minimizer_time_s));
  const long nb_all = nb_global;
  s->n_obs = (int)nb_all;
  s->final_rms_px = nb_all ? std::sqrt(2.0 * s->final_cost / (4.0 * nb_all)) : 0.0;
  s->t_linearize_ms = timers[PH_LIN].acc_ms;
  s->t_schur_ms = timers[PH_SCHUR].acc_ms;
  s->t_cholesky_ms = timers[PH_CHOL].acc_ms;
  s->t_solve_ms = timers[PH_SOLVE].acc_ms;
  s->t_backsub_ms = timers[PH_BACK].acc_ms;
  s->t_cost_ms = timers[PH_COST].acc_ms;
  s->t_factor_own_ms = timers[PH_FAC0].acc_ms;
  s->t_factor_top_ms = timers[PH_FAC1].acc_ms;
  s->t_dominant_ms = dom_ms;
  s->dominant_flops = dom_flops;
  s->n_dominant_launches = dom_launches;
  s->n_factor_tiles = plan.n_tiles;
  s->n_levels = plan.nlev;
  s->n_update_tiles = plan.total_upd_tiles;
  s->factor_update_flops = plan.total_upd_flops;
  s->factor_scalar_flops = scalar_flops;
  s->comm_bytes = comm_bytes;
  s->comm_calls = comm_calls;
  s->elimination_used = elim_used;
  s->ceres_e_captures = ceres_e_cap;
  s->ceres_e_tags = ceres_e_tag;
  s->n_ranks = nranks;
  s->n_owned_captures = multi() ? nc : nc_user;   // (one rank: every capture, whichever side is eliminated)
  s->n_top_tiles = multi() ? plan.n_top_tiles : 0;
  s->split_top_work = split_top_work;
  s->split_max_rank_work = split_max_rank_work;
  s->split_total_work = split_total_work;
  s->n_active_ranks = multi() ? split_active : 1;
  s->order_reused = last_order_reused ? 1 : 0;
}

// ===========================================================================
// C-ABI
// ===========================================================================

namespace {

template <class F>
int guarded(F &&f);
}  // namespace
namespace arslam {
void set_last_error(const std::string &msg) { g_last_error = msg; }
}  // namespace arslam
namespace {
template <class F>
int guarded(F &&f) {
  try {
    f();
    return ARSLAM_OK;
  } catch (const Error &e) {
    g_last_error = e.what();
    return e.code;
  } catch (const std::bad_alloc &) {
    g_last_error = "host out of memory";
    return ARSLAM_E_OUT_OF_MEMORY;
  } catch (const std::exception &e) {
    g_last_error = e.what();
    return ARSLAM_E_HIP;
  } catch (...) {
    g_last_error = "unknown error";
    return ARSLAM_E_HIP;
  }
}

}  // namespace

extern "C" {

int arslam_lm_options_init(arslam_lm_options *o) {
  if (!o) return ARSLAM_E_INVALID_ARG;
  std::memset(o, 0, sizeof(*o));
  o->max_num_iterations = 50;              // ar_slam_util.cpp:1004
  o->function_tolerance = 1e-6;            // Ceres 2.0 defaults below
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_relative_decrease = 1e-3;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
  o->elimination = ARSLAM_ELIM_AUTO;       // DENSE_SCHUR, ar_slam_util.cpp:1011
  o->minimizer_progress_to_stdout = 0;
  o->update_state_every_iteration = 0;
  o->device = -1;
  o->cholesky_skip_zero_tiles = 1;
  o->reduced_ordering = 2;
  o->kernel_timing = 0;
  o->factor_executor = 1;
  o->phase_timing = 0;
  return ARSLAM_OK;
}

int arslam_lm_create(arslam_lm **out, const arslam_lm_options *opt) {
  if (!out) return ARSLAM_E_INVALID_ARG;
  *out = nullptr;
  return guarded([&] {
    auto *h = new arslam_lm();
    if (opt) h->opt = *opt; else arslam_lm_options_init(&h->opt);
    if (h->opt.elimination < ARSLAM_ELIM_AUTO || h->opt.elimination > ARSLAM_ELIM_MIXED) {
      delete h;
      throw Error(ARSLAM_E_INVALID_ARG, "elimination must be ARSLAM_ELIM_AUTO, _CAPTURES, _TAGS or _MIXED");
    }
    *out = h;
  });
}

void arslam_lm_destroy(arslam_lm *h) { delete h; }

int arslam_lm_set_options(arslam_lm *h, const arslam_lm_options *opt) {
  if (!h || !opt) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    fail_if(opt->elimination < ARSLAM_ELIM_AUTO || opt->elimination > ARSLAM_ELIM_MIXED, ARSLAM_E_INVALID_ARG,
            "elimination must be ARSLAM_ELIM_AUTO, _CAPTURES, _TAGS or _MIXED");
    fail_if(opt->factor_executor != 0 && opt->factor_executor != 1, ARSLAM_E_INVALID_ARG,
            "factor_executor must be 0 or 1");
    fail_if(opt->max_num_iterations < 0 || opt->max_num_iterations > ARSLAM_LM_MAX_ITERS,
            ARSLAM_E_INVALID_ARG, "max_num_iterations out of range");
    // the stream and every device buffer live on the device of the first load
    fail_if(h->stream && opt->device >= 0 && opt->device != h->device,
            ARSLAM_E_INVALID_ARG, "a handle's device is fixed once it has loaded a problem: create a new handle");
    if (opt->device != h->opt.device || opt->reduced_ordering != h->opt.reduced_ordering ||
        opt->cholesky_skip_zero_tiles != h->opt.cholesky_skip_zero_tiles || opt->elimination != h->opt.elimination)
      h->loaded = false, h->pk_dirty = true;
    h->opt = *opt;
  });
}

int arslam_lm_get_options(const arslam_lm *h, arslam_lm_options *opt) {
  if (!h || !opt) return ARSLAM_E_INVALID_ARG;
  *opt = h->opt;
  return ARSLAM_OK;
}

int arslam_lm_add_residual_block(arslam_lm *h, const double corners[8], double *camera,
                                 double *capture, double *tag) {
  if (!h || !corners || !camera || !capture || !tag) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    fail_if(h->camera_ptr && h->camera_ptr != camera, ARSLAM_E_UNSUPPORTED,
            "one shared camera block per problem (ArSlamSolver::camera_)");
    fail_if(capture == camera || tag == camera || capture == tag, ARSLAM_E_INVALID_ARG,
            "parameter blocks must be distinct");
    fail_if(h->tag_of.count(capture) || h->cap_of.count(tag), ARSLAM_E_INVALID_ARG,
            "a block cannot be both a capture and a tag");
    h->camera_ptr = camera;
    auto ci = h->cap_of.find(capture);
    int c;
    if (ci == h->cap_of.end()) {
      c = (int)h->cap_ptrs.size();
      h->cap_of.emplace(capture, c);
      h->cap_ptrs.push_back(capture);
    } else {
      c = ci->second;
    }
    auto ti = h->tag_of.find(tag);
    int t;
    if (ti == h->tag_of.end()) {
      t = (int)h->tag_ptrs.size();
      h->tag_of.emplace(tag, t);
      h->tag_ptrs.push_back(tag);
    } else {
      t = ti->second;
    }
    if (ti == h->tag_of.end()) h->pk_appended_only = false;   // a new tag: new reduced rows
    h->pk_dirty = true;
    h->pk_obs_cap.push_back(c);
    h->pk_obs_tag.push_back(t);
    h->pk_corners.insert(h->pk_corners.end(), corners, corners + 8);
  });
}

int arslam_lm_set_parameter_block_constant(arslam_lm *h, double *block) {
  if (!h || !block) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    fail_if(block != h->camera_ptr && !h->cap_of.count(block) && !h->tag_of.count(block),
            ARSLAM_E_INVALID_ARG, "parameter block is not part of the problem");
    if (h->constant.insert(block).second) h->pk_dirty = true, h->pk_appended_only = false;
  });
}

int arslam_lm_set_parameter_block_variable(arslam_lm *h, double *block) {
  if (!h || !block) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    if (h->constant.erase(block)) h->pk_dirty = true, h->pk_appended_only = false;
  });
}

int arslam_lm_num_residual_blocks(const arslam_lm *h) {
  return h ? (int)h->pk_obs_cap.size() : 0;
}

int arslam_lm_solve(arslam_lm *h, arslam_lm_summary *summary) {
  if (!h || !summary) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    std::memset(summary, 0, sizeof(*summary));
    if (h->pk_obs_cap.empty()) {   // empty problem: nothing to do (Ceres returns immediately)
      summary->termination = ARSLAM_CONVERGENCE;
      return;
    }
    const double t_stage = now_s();
    const int nc = (int)h->cap_ptrs.size(), nt = (int)h->tag_ptrs.size();
    std::vector<double> cam(h->camera_ptr, h->camera_ptr + 3), cap(6L * nc), tag(6L * nt);
    std::vector<unsigned char> cc(nc), tc(nt);
    for (int c = 0; c < nc; ++c) {
      std::memcpy(&cap[6L * c], h->cap_ptrs[c], 6 * sizeof(double));
      cc[c] = h->constant.count(h->cap_ptrs[c]) ? 1 : 0;
    }
    for (int t = 0; t < nt; ++t) {
      std::memcpy(&tag[6L * t], h->tag_ptrs[t], 6 * sizeof(double));
      tc[t] = h->constant.count(h->tag_ptrs[t]) ? 1 : 0;
    }
    arslam_soa_problem p{};
    p.n_cap = nc; p.n_tag = nt; p.n_obs = (int)h->pk_obs_cap.size();
    p.camera = cam.data(); p.cap = cap.data(); p.tag = tag.data();
    p.obs_cap = h->pk_obs_cap.data(); p.obs_tag = h->pk_obs_tag.data();
    p.corners = h->pk_corners.data();
    p.camera_const = h->constant.count(h->camera_ptr) ? 1 : 0;
    p.cap_const = cc.data(); p.tag_const = tc.data();
    struct StageGuard {   // (the staging arrays go out of scope; the device problem stays)
      arslam_lm *h;
      ~StageGuard() { h->pk_stage = nullptr; h->soa = arslam_soa_problem{}; h->reuse_order = false; }
    } stage_guard{h};
    if (h->loaded && h->pk_loaded && !h->pk_dirty) {
      h->reload_values(&p);   // same problem, new values: no host rebuild, no re-upload of observations
    } else if (h->loaded && h->pk_loaded && h->pk_appended_only && (h->try_extend(&p) || h->try_extend_mixed(&p))) {
      h->pk_dirty = false;    // appended residual blocks within the loaded tile pattern: layout and plan kept
    } else {
      h->reuse_order = h->pk_loaded;   // a grown pointer-keyed problem (not the first load)
      h->load(&p);
      h->reuse_order = false;
      h->pk_loaded = true;
      h->pk_dirty = false;
    }
    static const bool prof = std::getenv("ARSLAM_SETUP_PROFILE") != nullptr;   // debug: setup phases
    if (prof) std::fprintf(stderr, "arslam stage+setup %.3f ms\n", 1e3 * (now_s() - t_stage));
    h->pk_stage = &p;
    // the final write_back also writes the caller's blocks (Ceres writes parameters back;
    // every iteration under update_state_every_iteration)
    h->solve(summary);
  });
}

int arslam_lm_reset(arslam_lm *h) {
  if (!h) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    h->camera_ptr = nullptr;
    h->cap_of.clear(); h->tag_of.clear();
    h->cap_ptrs.clear(); h->tag_ptrs.clear();
    h->pk_obs_cap.clear(); h->pk_obs_tag.clear(); h->pk_corners.clear();
    h->constant.clear();
    h->loaded = false;
    h->pk_dirty = true;
    h->pk_loaded = false;
    h->prev_tag_row.clear();
    h->prev_mx_tag_row.clear();
    h->prev_mx_cap_row.clear();
  });
}

int arslam_lm_load_soa(arslam_lm *h, const arslam_soa_problem *p) {
  if (!h || !p) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    h->pk_loaded = false;
    h->pk_dirty = true;
    h->reuse_order = false;   // a bulk load never reuses a pointer-keyed problem's order
    h->prev_tag_row.clear();
    h->load(p);
  });
}

int arslam_lm_solve_loaded(arslam_lm *h, arslam_lm_summary *summary) {
  if (!h || !summary) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    fail_if(h->pk_loaded, ARSLAM_E_STATE, "no problem loaded by arslam_lm_load_soa");
    h->solve(summary);
  });
}

int arslam_lm_solve_soa(arslam_soa_problem *p, const arslam_lm_options *opt,
                        arslam_lm_summary *summary) {
  if (!p || !summary) return ARSLAM_E_INVALID_ARG;
  arslam_lm *h = nullptr;
  int rc = arslam_lm_create(&h, opt);
  if (rc) return rc;
  rc = guarded([&] {
    h->load(p);
    h->solve(summary);
  });
  arslam_lm_destroy(h);
  return rc;
}

int arslam_comm_unique_id(unsigned char id[ARSLAM_COMM_ID_BYTES]) {
  if (!id) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    static_assert(sizeof(ncclUniqueId) <= ARSLAM_COMM_ID_BYTES, "id size");
    ncclUniqueId u;
    NCCL_CHECK(ncclGetUniqueId(&u));
    std::memset(id, 0, ARSLAM_COMM_ID_BYTES);
    std::memcpy(id, &u, sizeof(u));
  });
}

int arslam_lm_set_comm_callback(arslam_lm *h, int rank, int nranks, arslam_allreduce_fn fn, void *ctx) {
  if (!h || nranks < 1 || rank < 0 || rank >= nranks || ((nranks > 1 || h->force_multi) && !fn))
    return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    if (h->comm) { (void)ncclCommDestroy(h->comm); h->comm = nullptr; }
    h->rank = rank;
    h->nranks = nranks;
    h->comm_cb = h->multi() ? fn : nullptr;
    h->comm_cb_ctx = ctx;
    h->loaded = false;
    h->pk_dirty = true;
  });
}

int arslam_lm_set_comm(arslam_lm *h, int rank, int nranks, const unsigned char id[ARSLAM_COMM_ID_BYTES]) {
  if (!h || !id || nranks < 1 || rank < 0 || rank >= nranks) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    h->ensure_stream();
    if (h->comm) { (void)ncclCommDestroy(h->comm); h->comm = nullptr; }
    h->comm_cb = nullptr;
    h->rank = rank;
    h->nranks = nranks;
    h->loaded = false;
    h->pk_dirty = true;
    if (h->multi()) {   // (one rank only under arslam_debug_force_multirank)
      ncclUniqueId u;
      std::memcpy(&u, id, sizeof(u));
      NCCL_CHECK(ncclCommInitRank(&h->comm, nranks, u, rank));
    }
  });
}

int arslam_lm_owned_captures(const arslam_lm *h, int *out, int cap, int *n) {
  if (!h || !n || (cap > 0 && !out)) return ARSLAM_E_INVALID_ARG;
  if (!h->loaded) return ARSLAM_E_STATE;
  const int k = h->multi() ? (int)h->own_caps.size() : h->nc_user;   // (one rank: every capture)
  for (int i = 0; i < k && i < cap; ++i) out[i] = h->multi() ? h->own_caps[i] : i;
  *n = k;
  return ARSLAM_OK;
}

int arslam_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int arslam_lm_set_iteration_callback(arslam_lm *h, arslam_iteration_callback fn, void *ctx) {
  if (!h) return ARSLAM_E_INVALID_ARG;
  h->iter_cb = fn;
  h->iter_cb_ctx = ctx;
  return ARSLAM_OK;
}

int arslam_lm_debug_force_indefinite(arslam_lm *h, unsigned long long step_mask) {
  if (!h) return ARSLAM_E_INVALID_ARG;
  h->dbg_indefinite_mask = step_mask;
  return ARSLAM_OK;
}

int arslam_lm_debug_force_multirank(arslam_lm *h, int on) {
  if (!h || (on != 0 && on != 1)) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    if (h->comm) { (void)ncclCommDestroy(h->comm); h->comm = nullptr; }
    h->comm_cb = nullptr;
    h->rank = 0;
    h->nranks = 1;
    h->force_multi = on != 0;
    h->loaded = false;
    h->pk_dirty = true;
  });
}

int arslam_lm_debug_break_dependency(arslam_lm *h, long ticket, long *broken) {
  if (!h || ticket < 0) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    fail_if(!h->loaded || !h->has_f || h->opt.factor_executor != 1, ARSLAM_E_STATE,
            "break_dependency needs a loaded problem on the persistent executor");
    arslam::LltPlan &pl = h->plan;
    long t = ticket;
    while (t < pl.n_dag_tasks && pl.h_dag_wait_off[t] == pl.h_dag_wait_off[t + 1]) ++t;
    fail_if(t >= pl.n_dag_tasks, ARSLAM_E_INVALID_ARG, "no task at or after this ticket waits on anything");
    const int w = pl.h_dag_wait_off[t];
    h->restore_patched_wait();
    pl.h_dag_waits[w].y += 1 << 28;   // a count no task ever reaches (for the next solve only)
    h->dbg_patched_wait = w;
    HIP_CHECK(hipMemcpyAsync(pl.dag_waits + w, &pl.h_dag_waits[w], sizeof(int2), hipMemcpyHostToDevice,
                             h->stream));
    HIP_CHECK(hipStreamSynchronize(h->stream));
    if (broken) *broken = t;
  });
}

int arslam_lm_debug_tag_pair_tile(arslam_lm *h, const double *tag_a, const double *tag_b, int *status) {
  if (!h || !tag_a || !tag_b || !status) return ARSLAM_E_INVALID_ARG;
  return guarded([&] {
    fail_if(!h->loaded || h->multi() || h->elim_used != ARSLAM_ELIM_CAPTURES || !h->has_f, ARSLAM_E_STATE,
            "tag_pair_tile needs a pointer-keyed problem loaded with capture elimination on one rank");
    const auto ia = h->tag_of.find(const_cast<double *>(tag_a)), ib = h->tag_of.find(const_cast<double *>(tag_b));
    *status = -1;
    if (ia == h->tag_of.end() || ib == h->tag_of.end()) return;
    const int ra = h->lay.tag_row[ia->second], rb = h->lay.tag_row[ib->second];
    if (ra < 0 || rb < 0) return;
    const int T = h->lay.T;
    int st = 2;
    for (int x : {ra, ra + 5})
      for (int y : {rb, rb + 5}) {
        int ti = x / 64, tj = y / 64;
        if (ti < tj) std::swap(ti, tj);
        // (the tiles assembled at the load are numbered first, the fill after them)
        const int id = h->plan.h_tile_id[(size_t)ti * T + tj];
        st = std::min(st, id < 0 ? 0 : (id < h->plan.n_assembled ? 2 : 1));
      }
    *status = st;
  });
}

const char *arslam_lm_last_error(void) { return g_last_error.c_str(); }

#ifndef ARSLAM_BUILD_ID
#define ARSLAM_BUILD_ID "unknown"
#endif
// the build's commit and source digest (ar_slam_amd/build.py build_id): every
// A/B line and bench line names the library it measured
const char *arslam_lm_version(void) { return "arslam_lm 0.2 (gfx950, fp64) build " ARSLAM_BUILD_ID; }

}  // extern "C"
