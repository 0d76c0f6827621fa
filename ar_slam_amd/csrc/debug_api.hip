// debug_api.hip -- component entry points (include/arslam_lm_debug.h) that run
// one device stage in isolation so the parity tests can pin it to the oracle.
#include <chrono>
#include "lm_internal.h"
#include "arslam_lm.h"
#include "arslam_lm_debug.h"

#include <climits>
#include <cstdlib>
#include <cstdio>
#include <unistd.h>
#include <cstring>
#include <string>
#include <vector>

namespace arslam {
void debug_read_schur_stamps(unsigned long long *out);
void debug_residual_jacobian(int n, const double *cam, const double *cap, const double *tag,
                             const double *corners, double *r, double *J, hipStream_t s);
void debug_angle_axis(int n, const double *w, const double *p, double *out, int *branch, hipStream_t s);
}

namespace {
int hip_fail(hipError_t e) { return e == hipSuccess ? ARSLAM_OK : ARSLAM_E_HIP; }
}

#define DBG_CHECK(x)                 \
  do {                               \
    hipError_t _e = (x);             \
    if (_e != hipSuccess) return hip_fail(_e); \
  } while (0)

extern "C" int arslam_debug_residual_jacobian(int n, const double *cam, const double *cap,
                                              const double *tag, const double *corners, double *r,
                                              double *J) {
  if (n < 0 || (n && (!cam || !cap || !tag || !corners || !r || !J))) return ARSLAM_E_INVALID_ARG;
  if (n == 0) return ARSLAM_OK;
  double *d_in = nullptr, *d_r = nullptr, *d_J = nullptr;
  const size_t in_n = (size_t)n * 23;
  DBG_CHECK(hipMalloc(&d_in, in_n * sizeof(double)));
  DBG_CHECK(hipMalloc(&d_r, (size_t)n * 8 * sizeof(double)));
  DBG_CHECK(hipMalloc(&d_J, (size_t)n * 120 * sizeof(double)));
  std::vector<double> h(in_n);
  std::memcpy(h.data(), cam, (size_t)n * 3 * sizeof(double));
  std::memcpy(h.data() + 3L * n, cap, (size_t)n * 6 * sizeof(double));
  std::memcpy(h.data() + 9L * n, tag, (size_t)n * 6 * sizeof(double));
  std::memcpy(h.data() + 15L * n, corners, (size_t)n * 8 * sizeof(double));
  DBG_CHECK(hipMemcpy(d_in, h.data(), in_n * sizeof(double), hipMemcpyHostToDevice));
  arslam::debug_residual_jacobian(n, d_in, d_in + 3L * n, d_in + 9L * n, d_in + 15L * n, d_r, d_J, 0);
  DBG_CHECK(hipGetLastError());
  DBG_CHECK(hipDeviceSynchronize());
  DBG_CHECK(hipMemcpy(r, d_r, (size_t)n * 8 * sizeof(double), hipMemcpyDeviceToHost));
  DBG_CHECK(hipMemcpy(J, d_J, (size_t)n * 120 * sizeof(double), hipMemcpyDeviceToHost));
  (void)hipFree(d_in);
  (void)hipFree(d_r);
  (void)hipFree(d_J);
  return ARSLAM_OK;
}

extern "C" int arslam_debug_angle_axis_rotate(int n, const double *w, const double *p, double *out,
                                              int *branch) {
  if (n < 0 || (n && (!w || !p || !out || !branch))) return ARSLAM_E_INVALID_ARG;
  if (n == 0) return ARSLAM_OK;
  double *d = nullptr;
  int *d_b = nullptr;
  DBG_CHECK(hipMalloc(&d, (size_t)n * 9 * sizeof(double)));
  DBG_CHECK(hipMalloc(&d_b, (size_t)n * sizeof(int)));
  DBG_CHECK(hipMemcpy(d, w, (size_t)n * 3 * sizeof(double), hipMemcpyHostToDevice));
  DBG_CHECK(hipMemcpy(d + 3L * n, p, (size_t)n * 3 * sizeof(double), hipMemcpyHostToDevice));
  arslam::debug_angle_axis(n, d, d + 3L * n, d + 6L * n, d_b, 0);
  DBG_CHECK(hipGetLastError());
  DBG_CHECK(hipDeviceSynchronize());
  DBG_CHECK(hipMemcpy(out, d + 6L * n, (size_t)n * 3 * sizeof(double), hipMemcpyDeviceToHost));
  DBG_CHECK(hipMemcpy(branch, d_b, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
  (void)hipFree(d);
  (void)hipFree(d_b);
  return ARSLAM_OK;
}

extern "C" int arslam_debug_dense_llt_ex(long n, double *A, const double *b, double *y, int *info,
                                         int executor);
extern "C" int arslam_debug_dense_llt(long n, double *A, const double *b, double *y, int *info) {
  return arslam_debug_dense_llt_ex(n, A, b, y, info, 0);
}

extern "C" int arslam_debug_dense_llt_ex(long n, double *A, const double *b, double *y, int *info,
                                         int executor) {
  if (n <= 0 || !A || !b || !y || !info) return ARSLAM_E_INVALID_ARG;
  const long N = (n + 1 + arslam::kTile - 1) / arslam::kTile * arslam::kTile;
  const int T = (int)(N / arslam::kTile);
  // dense lower matrix with the rhs as row n and identity padding, then compact tiles
  std::vector<double> h((size_t)N * N, 0.0);
  for (long i = 0; i < n; ++i)
    for (long j = 0; j <= i; ++j) h[i * N + j] = A[i * n + j];
  for (long j = 0; j < n; ++j) h[n * N + j] = b[j];
  h[n * N + n] = 1e300;
  for (long i = n + 1; i < N; ++i) h[i * N + i] = 1.0;
  std::vector<uint8_t> pattern((size_t)T * T, 0);
  for (int i = 0; i < T; ++i)
    for (int j = 0; j <= i; ++j) pattern[(size_t)i * T + j] = 1;
  arslam::LltPlan plan;
  try {
    arslam::llt_plan_build(plan, T, N, pattern, 0);
  } catch (...) {
    return ARSLAM_E_HIP;
  }
  std::vector<double> tiles((size_t)plan.n_tiles * 4096, 0.0);
  for (int ti = 0; ti < T; ++ti)
    for (int tj = 0; tj <= ti; ++tj) {
      double *t = tiles.data() + (size_t)plan.h_tile_id[(size_t)ti * T + tj] * 4096;
      for (int r = 0; r < 64; ++r)
        for (int c = 0; c < 64; ++c) t[r * 64 + c] = h[(ti * 64 + r) * N + tj * 64 + c];
    }
  double *d_S = nullptr, *d_z = nullptr, *d_y = nullptr;
  int *d_flag = nullptr;
  DBG_CHECK(hipMalloc(&d_S, tiles.size() * sizeof(double)));
  DBG_CHECK(hipMalloc(&d_z, N * sizeof(double)));
  DBG_CHECK(hipMalloc(&d_y, N * sizeof(double)));
  DBG_CHECK(hipMalloc(&d_flag, sizeof(int)));
  DBG_CHECK(hipMemcpy(d_S, tiles.data(), tiles.size() * sizeof(double), hipMemcpyHostToDevice));
  DBG_CHECK(hipMemset(d_flag, 0, sizeof(int)));
  const char *eg = std::getenv("ARSLAM_DAG_GRID");
  int grid = eg ? std::max(1, std::atoi(eg)) : 512;
  {   // at most the resident workgroups (the claim cap is half the grid)
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
      grid = std::min(grid, arslam::kDagWorkgroupsPerCu * cus);
  }
  if (executor == 1 && std::getenv("ARSLAM_DAG_PROGRESS")) {
    // debug: host-visible progress words, polled while the kernel runs
    int *prog = nullptr;
    DBG_CHECK(hipHostMalloc(&prog, 4 * sizeof(int) * grid, hipHostMallocCoherent));
    std::memset(prog, 0xff, 4 * sizeof(int) * grid);
    hipStream_t st;
    DBG_CHECK(hipStreamCreate(&st));
    DBG_CHECK(hipMemcpy(d_S, tiles.data(), tiles.size() * sizeof(double), hipMemcpyHostToDevice));
    arslam::launch_dense_llt_dag(plan, d_S, d_flag, st, grid, prog);
    for (int it = 0; it < 30; ++it) {
      usleep(100000);
      if (hipStreamQuery(st) == hipSuccess) break;
      std::fprintf(stderr, "t=%d00ms:", it + 1);
      for (int g = 0; g < grid && g < 16; ++g)
        std::fprintf(stderr, " [wg%d t%d ph%d ty%d]", g, ((volatile int *)prog)[4 * g], ((volatile int *)prog)[4 * g + 1],
                     ((volatile int *)prog)[4 * g + 2]);
      std::fprintf(stderr, "\n");
    }
    if (hipStreamQuery(st) != hipSuccess) {
      std::fprintf(stderr, "DAG kernel did not finish\n");
      std::fflush(stderr);
      std::_Exit(3);
    }
  }
  if (executor == 1) arslam::launch_dense_llt_dag(plan, d_S, d_flag, 0, grid);
  else arslam::launch_dense_llt(plan, d_S, d_flag, 0);
  if (executor == 1) arslam::launch_dense_back_solve_dag(plan, d_S, n, d_y, d_flag, 0, grid);
  else arslam::launch_dense_back_solve(plan, d_S, n, d_z, d_y, d_flag, 0);
  arslam::launch_scatter_diag(plan, d_S, 0);
  DBG_CHECK(hipGetLastError());
  DBG_CHECK(hipDeviceSynchronize());
  DBG_CHECK(hipMemcpy(tiles.data(), d_S, tiles.size() * sizeof(double), hipMemcpyDeviceToHost));
  DBG_CHECK(hipMemcpy(y, d_y, n * sizeof(double), hipMemcpyDeviceToHost));
  DBG_CHECK(hipMemcpy(info, d_flag, sizeof(int), hipMemcpyDeviceToHost));
  for (long i = 0; i < n; ++i)
    for (long j = 0; j < n; ++j) {
      const double *t = tiles.data() + (size_t)plan.h_tile_id[(size_t)(i / 64) * T + (j <= i ? j / 64 : 0)] * 4096;
      A[i * n + j] = j <= i ? t[(i % 64) * 64 + (j % 64)] : 0.0;
    }
  arslam::llt_plan_free(plan);
  (void)hipFree(d_S);
  (void)hipFree(d_z);
  (void)hipFree(d_y);
  (void)hipFree(d_flag);
  return ARSLAM_OK;
}

namespace {
// The protocol simulation over grids and policies (arslam::dag_simulate):
// 1 if deadlock-free in every run, else -(grid * 16 + policy) of the first
// deadlock.  Grids: small ones, the executor's 448 (1.75 per CU on 256 CUs)
// and 512, and the small-graph rule of launch_dense_llt_dag.
int simulate_all(const arslam::LltPlan &plan) {
  const long n = plan.n_dag_tasks;
  const int small = (int)std::min<long>(448, std::max<long>(std::min<long>(64, n), n / 4));
  for (int wk : {1, 2, 7, 64, small, 448, 512})
    for (int pol = 0; pol < arslam::kDagSimPolicies; ++pol)
      for (unsigned seed = 1; seed <= (pol == 0 || pol == 3 ? 3u : 1u); ++seed)
        if (!arslam::dag_simulate(plan, wk, seed, pol)) return -(wk * 16 + pol);
  // a 448-workgroup grid of which only k ever become resident (a GPU shared
  // with another process, or several ranks' launches on one GPU)
  for (int k : {1, 2, 7, 64})
    for (int pol = 0; pol < arslam::kDagSimPolicies; ++pol)
      if (!arslam::dag_simulate(plan, 448, 1u, pol, k)) return -(100000 * k + 448 * 16 + pol);
  return 1;
}
}  // namespace

extern "C" int arslam_debug_reduced_plan(const arslam_soa_problem *p, int ordering, int skip_zero_tiles,
                                         arslam_plan_info *info, int *tag_row) {
  if (!p || !info || ordering < 0 || ordering > 2) return ARSLAM_E_INVALID_ARG;
  try {
    std::memset(info, 0, sizeof(*info));
    static const bool prof = std::getenv("ARSLAM_SETUP_PROFILE") != nullptr;   // debug: setup phases
    auto clk = []() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t0 = prof ? clk() : 0.0;
    const arslam::HostProblem h = arslam::host_problem(p, nullptr);
    const double t1 = prof ? clk() : 0.0;
    arslam::ReducedLayout L = arslam::reduced_layout(h, ordering, skip_zero_tiles != 0, nullptr, nullptr);
    const double t2 = prof ? clk() : 0.0;
    info->n_reduced = L.nR;
    info->n_padded = L.N;
    info->pad_rows = L.pad_rows;
    info->tiles_per_side = L.T;
    info->n_parts = L.n_parts;
    info->camera_row = L.cam_row;
    if (tag_row)
      for (int t = 0; t < h.nt; ++t) tag_row[t] = L.tag_row[t];
    if (L.nR > 0) {
      arslam::LltPlan plan;
      arslam::llt_plan_symbolic(plan, L.T, L.N, L.pattern);
      if (prof) std::fprintf(stderr, "arslam plan: host_problem %.3f layout %.3f plan %.3f ms\n", t1 - t0, t2 - t1, clk() - t2);
      info->n_levels = plan.nlev;
      info->n_assembled_tiles = plan.n_assembled;
      info->n_factor_tiles = plan.n_tiles;
      info->n_update_tiles = plan.total_upd_tiles;
      info->n_update_items = (long)plan.h_items.size();
      info->n_split_targets = (long)plan.h_split.size();
      info->update_flops = plan.total_upd_flops;
      info->factor_flops = plan.total_factor_flops;
      info->scalar_flops = L.scalar_flops;
      info->n_dag_tasks = plan.n_dag_tasks;
      info->fill_first_ok = plan.fill_first_ok ? 1 : 0;
      info->dag_valid = arslam::dag_check(plan) ? 1 : 0;
      if (const char *dump = std::getenv("ARSLAM_DAG_DUMP")) {   // debug: the task graph, for offline analysis
        if (FILE *f = std::fopen(dump, "wb")) {
          const long n = plan.n_dag_tasks, nw = (long)plan.h_dag_waits.size(), T = plan.T;
          std::fwrite(&n, 8, 1, f);
          std::fwrite(&nw, 8, 1, f);
          std::fwrite(&T, 8, 1, f);
          const long ni = (long)plan.h_items.size(), ntg = (long)plan.h_targets.size();
          std::fwrite(&ni, 8, 1, f);
          std::fwrite(&ntg, 8, 1, f);
          std::fwrite(plan.h_dag_tasks.data(), sizeof(int4), n, f);
          std::fwrite(plan.h_dag_wait_off.data(), sizeof(int), n + 1, f);
          std::fwrite(plan.h_dag_waits.data(), sizeof(int2), nw, f);
          std::fwrite(plan.h_dag_sub.data(), sizeof(int2), n, f);
          std::fwrite(plan.h_tile_id.data(), sizeof(int), (size_t)T * T, f);
          std::fwrite(plan.h_items.data(), sizeof(int4), plan.h_items.size(), f);
          std::fwrite(plan.h_targets.data(), sizeof(int2), plan.h_targets.size(), f);
          std::fwrite(plan.h_dag_cont.data(), sizeof(int), n, f);
          std::fwrite(plan.h_dag_maxdep.data(), sizeof(int), n, f);
          std::fclose(f);
        }
      }
      if (info->dag_valid) info->dag_valid = simulate_all(plan);
    }
    return ARSLAM_OK;
  } catch (const arslam::ApiError &e) {
    return e.code;
  } catch (...) {
    return ARSLAM_E_INVALID_ARG;
  }
}

extern "C" int arslam_debug_reduced_plan_side(const arslam_soa_problem *p, int elimination, arslam_plan_info *info) {
  if (!p || !info || elimination < ARSLAM_ELIM_CAPTURES || elimination > ARSLAM_ELIM_MIXED) return ARSLAM_E_INVALID_ARG;
  try {
    std::memset(info, 0, sizeof(*info));
    // the device problem of that side, as arslam_lm's load builds it (one rank)
    std::vector<uint8_t> e_cap, e_tag;
    arslam::MixedProblem mx;
    const arslam_soa_problem swapped = arslam::swap_roles(*p);
    const arslam_soa_problem *q = p;
    int side = elimination;
    if (side == ARSLAM_ELIM_MIXED) {
      const arslam::SchurSide cs = arslam::ceres_schur_side(p, &e_cap, &e_tag);
      if (cs.e_cam || cs.e_tag == 0) side = ARSLAM_ELIM_CAPTURES;
      else if (cs.e_cap == 0) side = ARSLAM_ELIM_TAGS;
      else mx = arslam::mixed_problem(*p, e_cap, e_tag), q = &mx.soa;
    }
    if (side == ARSLAM_ELIM_TAGS) q = &swapped;
    arslam::HostProblem h = arslam::host_problem(q, nullptr);
    if (side == ARSLAM_ELIM_MIXED) arslam::mixed_patch(h, mx, *p);
    arslam::ReducedLayout L = arslam::reduced_layout(h, 2, true, nullptr, nullptr);
    info->n_reduced = L.nR;
    info->n_padded = L.N;
    info->pad_rows = L.pad_rows;
    info->tiles_per_side = L.T;
    info->n_parts = L.n_parts;
    info->camera_row = L.cam_row;
    info->scalar_flops = L.scalar_flops;
    if (L.nR > 0) {
      arslam::LltPlan plan;
      arslam::llt_plan_symbolic(plan, L.T, L.N, L.pattern);
      info->n_levels = plan.nlev;
      info->n_assembled_tiles = plan.n_assembled;
      info->n_factor_tiles = plan.n_tiles;
      info->n_update_tiles = plan.total_upd_tiles;
      info->n_update_items = (long)plan.h_items.size();
      info->update_flops = plan.total_upd_flops;
      info->factor_flops = plan.total_factor_flops;
      info->n_dag_tasks = plan.n_dag_tasks;
      info->dag_valid = arslam::dag_check(plan) ? 1 : 0;
    }
    return side;
  } catch (const arslam::ApiError &e) {
    return e.code;
  } catch (...) {
    return ARSLAM_E_INVALID_ARG;
  }
}

namespace {
arslam::LltPlan one_rank_plan(const arslam_soa_problem *p) {
  const arslam::HostProblem h = arslam::host_problem(p, nullptr);
  arslam::ReducedLayout L = arslam::reduced_layout(h, 2, true, nullptr, nullptr);
  if (L.nR <= 0) throw arslam::ApiError(ARSLAM_E_INVALID_ARG, "no reduced system");
  arslam::LltPlan plan;
  arslam::llt_plan_symbolic(plan, L.T, L.N, L.pattern);
  return plan;
}
}  // namespace

extern "C" int arslam_debug_dag_simulate(const arslam_soa_problem *p, int n_workers, unsigned seed, int policy,
                                         int *ok) {
  if (!p || !ok || n_workers < 1 || policy < 0) return ARSLAM_E_INVALID_ARG;
  try {
    *ok = arslam::dag_simulate(one_rank_plan(p), n_workers, seed, policy) ? 1 : 0;
    return ARSLAM_OK;
  } catch (const arslam::ApiError &e) {
    return e.code;
  } catch (...) {
    return ARSLAM_E_INVALID_ARG;
  }
}

extern "C" int arslam_debug_dag_simulate_started(const arslam_soa_problem *p, int n_workers, int n_started,
                                                 unsigned seed, int policy, int *ok) {
  if (!p || !ok || n_workers < 1 || n_started < 0 || policy < 0) return ARSLAM_E_INVALID_ARG;
  try {
    *ok = arslam::dag_simulate(one_rank_plan(p), n_workers, seed, policy, n_started) ? 1 : 0;
    return ARSLAM_OK;
  } catch (const arslam::ApiError &e) {
    return e.code;
  } catch (...) {
    return ARSLAM_E_INVALID_ARG;
  }
}

extern "C" int arslam_debug_dag_workgroup_limit(int k) {
  arslam::set_dag_workgroup_limit(k);
  return ARSLAM_OK;
}

extern "C" int arslam_debug_dag_fault_detail(const arslam_soa_problem *p, const int rec[9], char *buf, int len) {
  if (!p || !rec || !buf || len <= 0) return ARSLAM_E_INVALID_ARG;
  try {
    const std::string s = arslam::dag_fault_detail(one_rank_plan(p), rec);
    std::snprintf(buf, (size_t)len, "%s", s.c_str());
    return ARSLAM_OK;
  } catch (const arslam::ApiError &e) {
    return e.code;
  } catch (...) {
    return ARSLAM_E_INVALID_ARG;
  }
}

extern "C" int arslam_debug_rank_split(const arslam_soa_problem *p, int nranks, int rank, arslam_split_info *info,
                                       int *cap_owner) {
  if (!p || !info || nranks < 1 || rank < 0 || rank >= nranks) return ARSLAM_E_INVALID_ARG;
  try {
    std::memset(info, 0, sizeof(*info));
    const arslam::HostProblem h = arslam::host_problem(p, nullptr);
    arslam::ReducedLayout L = arslam::reduced_layout(h, 2, true, nullptr, nullptr);
    const arslam::RankSplit split = arslam::rank_split(h, L, nranks);
    info->tiles_per_side = L.T;
    info->top_work = split.top_work;
    info->max_rank_work = split.max_rank_work;
    info->total_work = split.total_work;
    info->n_active = split.n_active;
    for (int c = 0; c < h.nc; ++c) {
      if (cap_owner) cap_owner[c] = split.cap_owner[c];
      info->n_owned_captures += split.cap_owner[c] == rank;
    }
    if (L.nR > 0) {
      const std::vector<int> cls = split.col_class(rank);
      for (int k = 0; k < L.T; ++k) {
        info->n_top_cols += cls[k] == 1;
        info->n_own_cols += cls[k] == 0;
      }
      arslam::LltPlan plan;
      arslam::llt_plan_symbolic(plan, L.T, L.N, L.pattern, nranks > 1 ? &cls : nullptr);
      info->n_top_tiles = plan.n_top_tiles;
      info->n_tiles = plan.n_tiles;
      info->n_dag_tasks = plan.n_dag_tasks;
      info->phase_split = plan.phase_split;
      info->dag_valid = arslam::dag_check(plan) ? 1 : 0;
      if (info->dag_valid) info->dag_valid = simulate_all(plan);
    }
    return ARSLAM_OK;
  } catch (const arslam::ApiError &e) {
    return e.code;
  } catch (...) {
    return ARSLAM_E_INVALID_ARG;
  }
}

extern "C" int arslam_debug_ceres_e_blocks(const arslam_soa_problem *p, int out[4]) {
  if (!p || !out) return ARSLAM_E_INVALID_ARG;
  try {
    const arslam::SchurSide cs = arslam::ceres_schur_side(p);
    out[0] = cs.e_cap;
    out[1] = cs.e_tag;
    out[2] = cs.e_cam;
    out[3] = cs.max_tag_obs;
    return ARSLAM_OK;
  } catch (const arslam::ApiError &e) {
    return e.code;
  } catch (...) {
    return ARSLAM_E_INVALID_ARG;
  }
}

extern "C" int arslam_debug_mixed_groups(const arslam_soa_problem *p, int out[4], unsigned char *e_cap,
                                         unsigned char *e_tag) {
  if (!p || !out) return ARSLAM_E_INVALID_ARG;
  try {
    std::vector<uint8_t> ec, et;
    (void)arslam::ceres_schur_side(p, &ec, &et);
    if (e_cap) std::copy(ec.begin(), ec.end(), e_cap);
    if (e_tag) std::copy(et.begin(), et.end(), e_tag);
    const arslam::MixedProblem m = arslam::mixed_problem(*p, ec, et);
    arslam::HostProblem h = arslam::host_problem(&m.soa, nullptr);
    arslam::mixed_patch(h, m, *p);
    out[0] = h.nc;
    out[1] = h.nt;
    out[2] = m.n_direct;
    out[3] = h.maxblk;
    return ARSLAM_OK;
  } catch (const arslam::ApiError &e) {
    return e.code;
  } catch (...) {
    return ARSLAM_E_INVALID_ARG;
  }
}

// diagnostic build only (-DARSLAM_SCHUR_STAMPS): accumulated per-phase cycles of k_schur
extern "C" int arslam_debug_schur_stamps(unsigned long long out[16]) {
  if (!out) return ARSLAM_E_INVALID_ARG;
  arslam::debug_read_schur_stamps(out);
  return ARSLAM_OK;
}

extern "C" int arslam_debug_gather_extend(const arslam_soa_problem *p, int c0, int *identical, int *n_dest) {
  if (!p || !identical || !n_dest || c0 < 0 || c0 > p->n_cap) return ARSLAM_E_INVALID_ARG;
  try {
    // the first c0 captures' residual blocks, in p's order
    std::vector<int> oc, ot;
    std::vector<double> cr;
    for (int b = 0; b < p->n_obs; ++b)
      if (p->obs_cap[b] < c0) {
        oc.push_back(p->obs_cap[b]);
        ot.push_back(p->obs_tag[b]);
        cr.insert(cr.end(), p->corners + 8L * b, p->corners + 8L * b + 8);
      }
    arslam_soa_problem q = *p;
    q.n_cap = c0;
    q.n_obs = (int)oc.size();
    q.obs_cap = oc.data();
    q.obs_tag = ot.data();
    q.corners = cr.data();
    const arslam::HostProblem hs = arslam::host_problem(&q, nullptr);
    const arslam::ReducedLayout L = arslam::reduced_layout(hs, 2, true, nullptr, nullptr);
    arslam::SchurGather G = arslam::schur_gather_plan(hs, L);
    const arslam::HostProblem hf = arslam::host_problem(p, nullptr);
    arslam::schur_gather_extend(G, hf, L, c0);
    const arslam::SchurGather F = arslam::schur_gather_plan(hf, L);
    bool same = G.cap_off == F.cap_off && G.dest_row == F.dest_row && G.dest_start == F.dest_start &&
                G.items == F.items && G.splits == F.splits && G.n_pslots == F.n_pslots &&
                G.max_contrib == F.max_contrib && G.contrib.size() == F.contrib.size();
    for (size_t i = 0; same && i < G.contrib.size(); ++i)
      same = !std::memcmp(&G.contrib[i], &F.contrib[i], sizeof(arslam::SchurContrib));
    *identical = same ? 1 : 0;
    *n_dest = (int)F.dest_start.size() - 1;
    return ARSLAM_OK;
  } catch (const arslam::ApiError &e) {
    return e.code;
  } catch (...) {
    return ARSLAM_E_INVALID_ARG;
  }
}

// ---------------------------------------------------------------------------
// Box fingerprint (arslam_debug_box_fingerprint): the memory round trips the
// persistent executor's hand-offs are made of, measured in-process for a few
// milliseconds, so a bench line can be placed on the kind of box it ran on
// (the same library ran cfg3's factorization at ~597 us on some MI355X boxes
// and ~663 us on others).  One lane per measurement, bounded loops.
namespace {
__device__ __forceinline__ unsigned long long fp_rt() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;   // 100 MHz
}

// mode 0: never-matching CAS (the executor's counter poll), 1: agent-scope
// atomic load (sc1, the tile loads), over a random pointer cycle
__global__ void k_fp_chase(long *next, int n, int mode, unsigned long long *out, long *sink) {
  if (threadIdx.x != 0) return;
  long p = 0;
  for (int i = 0; i < 32; ++i) p = __hip_atomic_load(next + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t0 = fp_rt();
  for (int i = 0; i < n; ++i) {
    if (mode == 0) {
      long v = LONG_MIN;
      __hip_atomic_compare_exchange_strong(next + p, &v, LONG_MIN, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      p = v;
    } else {
      p = __hip_atomic_load(next + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  out[mode] = fp_rt() - t0;
  sink[0] = p;
}

// a write-through (agent-scope) vector store and its acknowledgement
// (s_waitcnt vmcnt(0)), one after another: the release of a published tile
__global__ void k_fp_store_ack(long *buf, int n, unsigned long long *out) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = fp_rt();
  for (int i = 0; i < n; ++i) {
    __hip_atomic_store(buf + 16L * (i & 1023), (long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  out[2] = fp_rt() - t0;
}

// ping-pong of two workgroups through agent-scope release / acquire flags
// (a hand-off and its answer); every wait bounded
__global__ void k_fp_pingpong(int *flags, int n, unsigned long long *out, int *xcc) {
  if (threadIdx.x != 0) return;
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (blockIdx.x < 2) xcc[blockIdx.x] = (int)(x & 7);
  if (blockIdx.x >= 2) return;
  int *a = flags, *b = flags + 64;
  const bool first = blockIdx.x == 0;
  const unsigned long long t0 = fp_rt();
  long spins = 0;
  for (int i = 1; i <= n && spins < (1L << 24); ++i) {
    if (first) {
      __hip_atomic_store(a, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      while (__hip_atomic_load(b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < i && ++spins < (1L << 24)) {}
    } else {
      while (__hip_atomic_load(a, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < i && ++spins < (1L << 24)) {}
      __hip_atomic_store(b, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (first) out[3] = spins >= (1L << 24) ? ~0ull : fp_rt() - t0;
}
}  // namespace

extern "C" int arslam_debug_box_fingerprint(int device, double out[6]) {
  if (!out) return ARSLAM_E_INVALID_ARG;
  int cur = 0;
  DBG_CHECK(hipGetDevice(&cur));
  if (device >= 0 && device != cur) DBG_CHECK(hipSetDevice(device));
  const int nel = 1 << 15, n = 2000;   // 256 KB pointer cycle over cache-line-spaced slots
  std::vector<long> h(nel, 0);
  std::vector<int> perm(nel / 16);
  for (int i = 0; i < (int)perm.size(); ++i) perm[i] = i;
  unsigned s = 12345;
  for (int i = (int)perm.size() - 1; i > 0; --i) {
    s = s * 1103515245u + 12345u;
    std::swap(perm[i], perm[s % (i + 1)]);
  }
  for (int i = 0; i < (int)perm.size(); ++i) h[16 * perm[i]] = 16L * perm[(i + 1) % perm.size()];
  long *d = nullptr, *sink = nullptr, *st = nullptr;
  unsigned long long *t = nullptr;
  int *flags = nullptr, *xcc = nullptr;
  hipStream_t stream = nullptr;
  auto cleanup = [&]() {
    if (stream) (void)hipStreamDestroy(stream);
    for (void *p : {(void *)d, (void *)sink, (void *)st, (void *)t, (void *)flags, (void *)xcc})
      if (p) (void)hipFree(p);
    if (device >= 0 && device != cur) (void)hipSetDevice(cur);
  };
  hipError_t e = hipSuccess;
  auto ok = [&](hipError_t r) { if (e == hipSuccess) e = r; return e == hipSuccess; };
  if (ok(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking)) && ok(hipMalloc(&d, nel * sizeof(long))) &&
      ok(hipMalloc(&sink, 64)) && ok(hipMalloc(&st, 1024 * 16 * sizeof(long))) && ok(hipMalloc(&t, 64)) &&
      ok(hipMalloc(&flags, 1024)) && ok(hipMalloc(&xcc, 64)) &&
      ok(hipMemcpyAsync(d, h.data(), nel * sizeof(long), hipMemcpyHostToDevice, stream)) &&
      ok(hipMemsetAsync(flags, 0, 1024, stream)) && ok(hipMemsetAsync(t, 0, 64, stream))) {
    hipLaunchKernelGGL(k_fp_chase, dim3(1), dim3(64), 0, stream, d, n, 0, t, sink);
    hipLaunchKernelGGL(k_fp_chase, dim3(1), dim3(64), 0, stream, d, n, 1, t, sink);
    hipLaunchKernelGGL(k_fp_store_ack, dim3(1), dim3(64), 0, stream, st, n, t);
    hipLaunchKernelGGL(k_fp_pingpong, dim3(8), dim3(64), 0, stream, flags, n, t, xcc);
    unsigned long long ht[4] = {0, 0, 0, 0};
    int hx[2] = {-1, -1};
    if (ok(hipGetLastError()) && ok(hipMemcpyAsync(ht, t, sizeof(ht), hipMemcpyDeviceToHost, stream)) &&
        ok(hipMemcpyAsync(hx, xcc, sizeof(hx), hipMemcpyDeviceToHost, stream)) && ok(hipStreamSynchronize(stream))) {
      for (int q = 0; q < 4; ++q) out[q] = ht[q] == ~0ull ? -1.0 : ht[q] * 10.0 / n;   // ns (100 MHz clock)
      out[4] = hx[0];
      out[5] = hx[1];
    }
  }
  cleanup();
  return hip_fail(e);
}
