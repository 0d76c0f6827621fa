// llt_plan.cpp -- host-side symbolic analysis of the reduced (tag + camera)
// system, built once per problem structure and replayed by every LM step:
//
//  1. ordering of the tags: natural, reverse Cuthill-McKee (band), or nested
//     dissection (recursive BFS-level vertex separators, each part aligned to
//     a 64-row tile so the tile elimination tree mirrors the dissection tree);
//  2. tile pattern of the reduced matrix (co-visible tags + the camera border
//     + the right-hand-side row) and its symbolic Cholesky fill;
//  3. a level schedule of the tile elimination tree: tile columns of equal
//     height are independent and are factored in one launch, their updates
//     applied in one launch; the backward solve walks the levels in reverse.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include "lm_internal.h"

#include <algorithm>
#include <deque>
#include <stdexcept>
#include <string>

namespace arslam {

namespace {

void check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <class T>
T *upload(const std::vector<T> &h, hipStream_t s) {
  if (h.empty()) return nullptr;
  T *d = nullptr;
  check(hipMalloc(&d, h.size() * sizeof(T)), "hipMalloc(plan)");
  check(hipMemcpyAsync(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s), "plan upload");
  return d;
}

}  // namespace

constexpr int kSplitMin = 6;   // k-lists longer than this are split

void llt_plan_symbolic(LltPlan &plan, int T, long lda, std::vector<uint8_t> &P) {
  llt_plan_free(plan);
  plan.T = T;
  plan.lda = lda;
  // compact tile numbering: assembled tiles (the input pattern + diagonal) first
  plan.h_tile_id.assign((size_t)T * T, -1);
  long nid = 0;
  for (int i = 0; i < T; ++i)
    for (int j = 0; j <= i; ++j)
      if (P[(long)i * T + j] || i == j) plan.h_tile_id[(long)i * T + j] = (int)nid++;
  plan.n_assembled = nid;
  // symbolic factorization at tile level
  std::vector<int> rows;
  for (int k = 0; k < T; ++k) {
    P[(long)k * T + k] = 1;
    rows.clear();
    for (int i = k + 1; i < T; ++i)
      if (P[(long)i * T + k]) rows.push_back(i);
    for (size_t a = 0; a < rows.size(); ++a)
      for (size_t b = 0; b <= a; ++b) P[(long)rows[a] * T + rows[b]] = 1;
  }
  // tile elimination tree and heights
  std::vector<int> parent(T, -1), height(T, 0);
  for (int k = 0; k < T; ++k)
    for (int i = k + 1; i < T; ++i)
      if (P[(long)i * T + k]) { parent[k] = i; break; }
  for (int k = 0; k < T; ++k)
    if (parent[k] >= 0) height[parent[k]] = std::max(height[parent[k]], height[k] + 1);
  int nlev = 0;
  for (int k = 0; k < T; ++k) nlev = std::max(nlev, height[k] + 1);
  std::vector<std::vector<int>> levcols(nlev);
  for (int k = 0; k < T; ++k) levcols[height[k]].push_back(k);
  plan.nlev = nlev;

  std::vector<int2> &panel = plan.h_panel, &targets = plan.h_targets, &gather = plan.h_gather,
                    &split = plan.h_split;
  std::vector<int> &kstart = plan.h_kstart, &ks = plan.h_ks, &bcols = plan.h_bcols, &gbeg = plan.h_gbeg;
  std::vector<int4> &items = plan.h_items;
  kstart.assign(1, 0);
  gbeg.assign(1, 0);
  plan.h_item_off.assign(1, 0);
  plan.h_panel_off.assign(1, 0);
  plan.h_upd_off.assign(1, 0);
  plan.h_bs_off.assign(1, 0);
  plan.h_bsg_off.assign(1, 0);
  plan.h_upd_flops.clear();
  plan.total_upd_flops = 0.0;
  plan.total_upd_tiles = 0;
  const double t3 = 64.0 * 64.0 * 64.0;
  std::vector<int> tgt_id((size_t)T * T, -1);
  for (int l = 0; l < nlev; ++l) {
    // panel tasks
    for (int k : levcols[l]) {
      panel.push_back(make_int2(k, k));
      for (int i = k + 1; i < T; ++i)
        if (P[(long)i * T + k]) panel.push_back(make_int2(i, k));
    }
    plan.h_panel_off.push_back((int)panel.size());
    // update targets of this level: (i,j), j <= i, both in some column k of the level
    std::vector<int2> lt;
    std::vector<std::vector<int>> lks;
    double fl = 0.0;
    for (int k : levcols[l]) {
      rows.clear();
      for (int i = k + 1; i < T; ++i)
        if (P[(long)i * T + k]) rows.push_back(i);
      for (size_t a = 0; a < rows.size(); ++a)
        for (size_t b = 0; b <= a; ++b) {
          const long key = (long)rows[a] * T + rows[b];
          int id = tgt_id[key];
          if (id < 0) {
            id = (int)lt.size();
            tgt_id[key] = id;
            lt.push_back(make_int2(rows[a], rows[b]));
            lks.emplace_back();
          }
          lks[id].push_back(k);
          fl += (a == b) ? 64.0 * 65.0 * 64.0 : 2.0 * t3;
          plan.total_upd_tiles++;
        }
    }
    std::vector<int4> litems;
    for (size_t t = 0; t < lt.size(); ++t) {
      tgt_id[(long)lt[t].x * T + lt[t].y] = -1;
      const int tg = (int)targets.size(), q0 = (int)ks.size();
      targets.push_back(lt[t]);
      ks.insert(ks.end(), lks[t].begin(), lks[t].end());
      kstart.push_back((int)ks.size());
      // split a long k-list into ~sqrt(m) chunks: chunk GEMMs run in parallel,
      // the last arriver reads ~sqrt(m) partial tiles
      const int m = (int)lks[t].size();
      if (m > kSplitMin) {
        int nch = std::min(255, (int)std::ceil(std::sqrt((double)m)));
        const int ch = (m + nch - 1) / nch;
        nch = (m + ch - 1) / ch;
        const int sid = (int)split.size();
        split.push_back(make_int2(nch, (int)plan.n_part));
        plan.n_part += nch;
        for (int c = 0; c < nch; ++c)
          litems.push_back(make_int4(tg, q0 + c * ch, std::min(q0 + (c + 1) * ch, q0 + m), sid * 256 + c));
      } else {
        litems.push_back(make_int4(tg, q0, q0 + m, -1));
      }
    }
    // longest items first (they bound the launch)
    std::stable_sort(litems.begin(), litems.end(),
                     [](const int4 &a, const int4 &b) { return a.z - a.y > b.z - b.y; });
    items.insert(items.end(), litems.begin(), litems.end());
    plan.h_item_off.push_back((int)items.size());
    plan.h_upd_off.push_back((int)targets.size());
    plan.h_upd_flops.push_back(fl);
    if (std::getenv("ARSLAM_PLAN_STATS")) {
      size_t mx = 0, tot = 0;
      for (size_t t = 0; t < lt.size(); ++t) { mx = std::max(mx, lks[t].size()); tot += lks[t].size(); }
      std::fprintf(stderr, "level %d: panel %d targets %zu ks %zu max_ks %zu\n", l,
                   plan.h_panel_off[l + 1] - plan.h_panel_off[l], lt.size(), tot, mx);
    }
    plan.total_upd_flops += fl;
  }
  // backward solve: levels from the root down; each column gathers from its
  // tile rows below the diagonal (ancestors, solved in earlier launches)
  for (int l = nlev - 1; l >= 0; --l) {
    for (int k : levcols[l]) {
      bcols.push_back(k);
      for (int i = k + 1; i < T; ++i)
        if (P[(long)i * T + k]) gather.push_back(make_int2(i, k));
      gbeg.push_back((int)gather.size());   // column's gathers: [gbeg[b], gbeg[b+1])
    }
    plan.h_bs_off.push_back((int)bcols.size());
    plan.h_bsg_off.push_back((int)gather.size());
  }
  for (int i = 0; i < T; ++i)   // fill tiles numbered after the assembled ones
    for (int j = 0; j <= i; ++j)
      if (P[(long)i * T + j] && plan.h_tile_id[(long)i * T + j] < 0) plan.h_tile_id[(long)i * T + j] = (int)nid++;
  plan.n_tiles = nid;
}

void llt_plan_upload(LltPlan &plan, hipStream_t s) {
  const int T = plan.T;
  plan.panel = upload(plan.h_panel, s);
  plan.upd_targets = upload(plan.h_targets, s);
  plan.upd_kstart = upload(plan.h_kstart, s);
  plan.upd_ks = upload(plan.h_ks, s);
  plan.upd_items = upload(plan.h_items, s);
  plan.upd_split = upload(plan.h_split, s);
  plan.n_split = (long)plan.h_split.size();
  check(hipMalloc(&plan.upd_cnt, std::max<size_t>(plan.h_split.size(), 1) * sizeof(int)), "hipMalloc(upd_cnt)");
  check(hipMalloc(&plan.upd_part, std::max<long>(plan.n_part, 1) * 4096 * sizeof(double)), "hipMalloc(upd_part)");
  plan.bs_cols = upload(plan.h_bcols, s);
  plan.bs_gather = upload(plan.h_gather, s);
  plan.bs_gbeg = upload(plan.h_gbeg, s);
  check(hipMalloc(&plan.bs_part, std::max<size_t>(plan.h_gather.size(), 1) * 64 * sizeof(double)), "hipMalloc(bs_part)");
  plan.tile_id = upload(plan.h_tile_id, s);
  check(hipMalloc(&plan.ldiag, 2 * (size_t)T * 64 * 64 * sizeof(double)), "hipMalloc(ldiag)");
  check(hipStreamSynchronize(s), "plan sync");
}

void llt_plan_build(LltPlan &plan, int T, long lda, std::vector<uint8_t> &P, hipStream_t s) {
  llt_plan_symbolic(plan, T, lda, P);
  llt_plan_upload(plan, s);
}

void llt_plan_free(LltPlan &plan) {
  for (void *p : {(void *)plan.panel, (void *)plan.upd_targets, (void *)plan.upd_kstart,
                  (void *)plan.upd_ks, (void *)plan.upd_items, (void *)plan.upd_split,
                  (void *)plan.upd_cnt, (void *)plan.upd_part, (void *)plan.bs_cols, (void *)plan.bs_gather,
                  (void *)plan.bs_gbeg, (void *)plan.bs_part, (void *)plan.tile_id, (void *)plan.ldiag})
    if (p) (void)hipFree(p);
  plan = LltPlan{};
}

}  // namespace arslam
