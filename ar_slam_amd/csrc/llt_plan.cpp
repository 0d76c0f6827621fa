// llt_plan.cpp -- host-side symbolic analysis for the reduced-system Cholesky:
// reverse Cuthill-McKee ordering of the tag co-visibility graph and the
// tile-level symbolic factorization (fill) that decides which tiles of the
// factor exist.  Built once per problem structure; the LM steps replay it.
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

// BFS levels from `start` within unvisited nodes; returns the last level's min-degree node
int bfs_far(int start, const std::vector<std::vector<int>> &adj, const std::vector<char> &done,
            int *depth) {
  std::vector<int> lev(adj.size(), -1);
  std::deque<int> q{start};
  lev[start] = 0;
  int last = start;
  while (!q.empty()) {
    const int u = q.front();
    q.pop_front();
    if (lev[u] > lev[last] || (lev[u] == lev[last] && adj[u].size() < adj[last].size())) last = u;
    for (int v : adj[u])
      if (!done[v] && lev[v] < 0) { lev[v] = lev[u] + 1; q.push_back(v); }
  }
  *depth = lev[last];
  return last;
}

}  // namespace

std::vector<int> rcm_order(int n, const std::vector<std::vector<int>> &adj) {
  std::vector<int> order;
  order.reserve(n);
  std::vector<char> done(n, 0);
  for (;;) {
    int start = -1;
    for (int v = 0; v < n; ++v)
      if (!done[v] && (start < 0 || adj[v].size() < adj[start].size())) start = v;
    if (start < 0) break;
    // pseudo-peripheral start node (George-Liu): walk to the far end until depth stops growing
    int depth = 0, far = bfs_far(start, adj, done, &depth);
    for (int it = 0; it < 8; ++it) {
      int d2 = 0;
      const int f2 = bfs_far(far, adj, done, &d2);
      if (d2 <= depth) break;
      depth = d2;
      start = far;
      far = f2;
    }
    start = far;
    std::deque<int> q{start};
    done[start] = 1;
    while (!q.empty()) {
      const int u = q.front();
      q.pop_front();
      order.push_back(u);
      std::vector<int> nb;
      for (int v : adj[u])
        if (!done[v]) { done[v] = 1; nb.push_back(v); }
      std::stable_sort(nb.begin(), nb.end(),
                       [&](int a, int b) { return adj[a].size() < adj[b].size(); });
      for (int v : nb) q.push_back(v);
    }
  }
  std::reverse(order.begin(), order.end());
  return order;
}

void llt_plan_build(LltPlan &plan, int T, long lda, std::vector<uint8_t> &P, hipStream_t s) {
  llt_plan_free(plan);
  plan.T = T;
  plan.lda = lda;
  // symbolic factorization at tile level: column k's rows fill every pair
  std::vector<int> rows;
  for (int k = 0; k < T; ++k) {
    P[(long)k * T + k] = 1;
    rows.clear();
    for (int i = k + 1; i < T; ++i)
      if (P[(long)i * T + k]) rows.push_back(i);
    for (size_t a = 0; a < rows.size(); ++a)
      for (size_t b = 0; b <= a; ++b) P[(long)rows[a] * T + rows[b]] = 1;
  }
  std::vector<int> trsm_rows, bs_cols;
  std::vector<int2> pairs, tiles;
  plan.h_trsm_off.assign(1, 0);
  plan.h_upd_off.assign(1, 0);
  plan.h_bs_off.assign(1, 0);
  plan.h_upd_flops.clear();
  const double t3 = 64.0 * 64.0 * 64.0;
  for (int k = 0; k < T; ++k) {
    rows.clear();
    for (int i = k + 1; i < T; ++i)
      if (P[(long)i * T + k]) rows.push_back(i);
    double fl = 0.0;
    for (size_t a = 0; a < rows.size(); ++a) {
      trsm_rows.push_back(rows[a]);
      for (size_t b = 0; b <= a; ++b) {
        pairs.push_back(make_int2(rows[a], rows[b]));
        // useful flops: off-diagonal tile 2*64^3, diagonal tile lower incl. diagonal 64*65*64
        fl += (a == b) ? 64.0 * 65.0 * 64.0 : 2.0 * t3;
      }
    }
    plan.h_trsm_off.push_back((int)trsm_rows.size());
    plan.h_upd_off.push_back((long)pairs.size());
    plan.h_upd_flops.push_back(fl);
    plan.total_upd_flops += fl;
    for (int j = 0; j < k; ++j)
      if (P[(long)k * T + j]) bs_cols.push_back(j);
    plan.h_bs_off.push_back((int)bs_cols.size());
    for (int j = 0; j <= k; ++j)
      if (P[(long)k * T + j]) tiles.push_back(make_int2(k, j));
  }
  plan.total_upd_tiles = (long)pairs.size();
  plan.n_tiles = (long)tiles.size();
  plan.trsm_rows = upload(trsm_rows, s);
  plan.upd_pairs = upload(pairs, s);
  plan.bs_cols = upload(bs_cols, s);
  plan.tiles = upload(tiles, s);
  check(hipStreamSynchronize(s), "plan sync");
}

void llt_plan_free(LltPlan &plan) {
  if (plan.trsm_rows) (void)hipFree(plan.trsm_rows);
  if (plan.upd_pairs) (void)hipFree(plan.upd_pairs);
  if (plan.bs_cols) (void)hipFree(plan.bs_cols);
  if (plan.tiles) (void)hipFree(plan.tiles);
  plan = LltPlan{};
}

}  // namespace arslam
