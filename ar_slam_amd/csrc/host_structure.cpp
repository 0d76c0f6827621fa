// host_structure.cpp -- host-only problem structure and reduced-system
// layout (see host_structure.h).  Restates the parameter-block bookkeeping of
// ceres::Problem as ar_slam builds it (AddResidualBlock, ar_slam_util.cpp:
// 720-727, 829-836, 956-963; SetParameterBlockConstant, :965, :972) and the
// DENSE_SCHUR split (captures eliminated, tags + camera reduced).
#include "host_structure.h"
#include "host_threads.h"

#include <algorithm>
#include <climits>
#include <chrono>
#include <iterator>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <deque>

namespace arslam {

namespace {

long round_up(long v, long m) { return (v + m - 1) / m * m; }

// BFS over `mark == tag` nodes from start; fills level of each visited node
// (-1 unvisited) and returns the visit order.
std::vector<int> bfs(int start, const std::vector<std::vector<int>> &adj, const std::vector<int> &mark,
                     int tag, std::vector<int> &lev) {
  std::vector<int> order{start};
  lev[start] = 0;
  for (size_t h = 0; h < order.size(); ++h) {
    const int u = order[h];
    for (int v : adj[u])
      if (mark[v] == tag && lev[v] < 0) {
        lev[v] = lev[u] + 1;
        order.push_back(v);
      }
  }
  return order;
}

// pseudo-peripheral node of the component of `start` (George-Liu)
int peripheral(int start, const std::vector<std::vector<int>> &adj, const std::vector<int> &mark,
               int tag, std::vector<int> &lev) {
  int best = start, depth = -1;
  for (int it = 0; it < 6; ++it) {
    const std::vector<int> ord = bfs(best, adj, mark, tag, lev);
    const int d = lev[ord.back()];
    int far = ord.back();
    for (int u : ord)   // among the last level, the one of least degree
      if (lev[u] == d && adj[u].size() < adj[far].size()) far = u;
    for (int u : ord) lev[u] = -1;
    if (d <= depth) break;
    depth = d;
    best = far;
  }
  return best;
}

double nd_beta() {
  // (debug sweeps; clamped to [0, 4]: a finite, non-negative weight)
  static const double b = std::getenv("ARSLAM_ND_BETA")
                              ? std::min(4.0, std::max(0.0, std::atof(std::getenv("ARSLAM_ND_BETA")) + 0.0))
                              : 0.3;
  return b;
}

// The geometric cuts' quantile window [q, 1 - q] and the smaller side's
// least share of the component (debug sweeps; clamped to [0.05, 0.45] and
// [0, 0.45]).
double nd_env(const char *name, double dflt, double lo, double hi) {
  const char *e = std::getenv(name);
  return e ? std::min(hi, std::max(lo, std::atof(e) + 0.0)) : dflt;
}
double nd_qlo() {
  static const double q = nd_env("ARSLAM_ND_QLO", 0.3, 0.05, 0.45);
  return q;
}
double nd_min_side() {
  static const double f = nd_env("ARSLAM_ND_MIN_SIDE", 0.2, 0.0, 0.45);
  return f;
}

// Elimination-tree height, in tile columns, of a dissection step: the
// separator's tiles plus the larger child's height, which grows about as
// sqrt(size) on these planar co-visibility graphs (cfg3: ~1 tile column per
// sqrt(tag) at the root); balance only breaks ties.
double height_score(long ssz, long na, long nb) {
  return std::ceil(6.0 * ssz / kTileRows) + nd_beta() * std::sqrt((double)std::max(na, nb)) +
         1e-6 * std::labs(na - nb);
}

// The two sides of a separator are dissected concurrently (host_fork2) and
// the directions of a geometric cut searched concurrently: the per-node arrays
// (mark, lev) are shared, but a branch only writes its own nodes and reads
// those and its separator's (the sides are not adjacent), and the parts come
// back in the serial order (side A's, side B's, then the separator).
struct Dissector {
  const std::vector<std::vector<int>> &adj;
  const std::vector<double> &xyz;   // optional 3-D embedding (tag positions), 3 per node
  int leaf;
  bool fast = false;
  std::vector<int> mark, lev;
  std::atomic<int> next_tag{1};

  Dissector(const std::vector<std::vector<int>> &a, const std::vector<double> &coords, int leaf_size)
      : adj(a), xyz(coords), leaf(leaf_size), mark(a.size(), 0), lev(a.size(), -1) {}

  // nodes: all with mark == tag; their parts appended to `parts` in elimination order
  void run(std::vector<int> nodes, int tag, std::vector<std::vector<int>> &parts) {
    if (nodes.empty()) return;
    // split into connected components
    std::vector<std::vector<int>> comps;
    for (int u : nodes) {
      if (lev[u] >= 0) continue;
      std::vector<int> c = bfs(u, adj, mark, tag, lev);
      comps.push_back(std::move(c));
    }
    for (int u : nodes) lev[u] = -1;
    for (auto &c : comps) dissect(c, tag, parts);
  }

  // BFS-level separator: the level that balances the two sides
  bool level_separator(std::vector<int> &comp, int tag, std::vector<int> &A, std::vector<int> &B,
                       std::vector<int> &S) {
    const int s = peripheral(comp[0], adj, mark, tag, lev);
    std::vector<int> ord = bfs(s, adj, mark, tag, lev);
    const int depth = lev[ord.back()];
    if (depth < 2) {
      for (int u : ord) lev[u] = -1;
      return false;
    }
    std::vector<int> cnt(depth + 1, 0);
    for (int u : ord) cnt[lev[u]]++;
    int sep = 1, acc = cnt[0];
    const int half = (int)ord.size() / 2;
    while (sep < depth - 1 && acc + cnt[sep] / 2 < half) acc += cnt[sep++];
    for (int u : ord) {
      if (lev[u] < sep) A.push_back(u);
      else if (lev[u] > sep) B.push_back(u);
      else S.push_back(u);
    }
    for (int u : ord) lev[u] = -1;
    return true;
  }

  // Minimum vertex cover of the cut's bipartite graph (side-1 boundary nodes
  // x side-2 boundary nodes, the cut edges), by augmenting paths and König's
  // construction: the smallest vertex separator that removes every cut edge
  // while keeping the remaining nodes on their sides.  On the co-visibility
  // graph (edges span up to ~3 tag spacings) it is often well below either
  // one-sided boundary.  cover[u] = 1 for the chosen nodes of comp.
  // (loc: scratch of adj.size() entries for the local numbering)
  int konig_cover(const std::vector<int> &comp, const std::vector<int> &side, int tag,
                  std::vector<char> &cover, std::vector<int> &loc) {
    std::vector<int> left, right;
    for (int u : comp) {
      bool bd = false;
      for (int v : adj[u])
        if (mark[v] == tag && side[v] != side[u]) { bd = true; break; }
      if (bd) (side[u] == 1 ? left : right).push_back(u);
    }
    std::vector<int> idx(0);
    // local numbering: left 0..nl-1, right nl..
    const int nl = (int)left.size(), nr = (int)right.size();
    for (int i = 0; i < nl; ++i) loc[left[i]] = i;
    for (int i = 0; i < nr; ++i) loc[right[i]] = nl + i;
    std::vector<std::vector<int>> g(nl);
    for (int i = 0; i < nl; ++i)
      for (int v : adj[left[i]])
        if (mark[v] == tag && side[v] == 2) g[i].push_back(loc[v] - nl);
    std::vector<int> mate_l(nl, -1), mate_r(nr, -1), seen(nr, -1);
    // Kuhn's augmenting paths (iterative DFS), greedy initial matching
    for (int i = 0; i < nl; ++i)
      for (int r : g[i])
        if (mate_r[r] < 0) { mate_l[i] = r; mate_r[r] = i; break; }
    std::vector<std::pair<int, int>> st;
    std::vector<int> par_r(nr, -1);
    for (int i0 = 0; i0 < nl; ++i0) {
      if (mate_l[i0] >= 0) continue;
      st.assign(1, {i0, 0});
      int found = -1;
      while (!st.empty() && found < 0) {
        auto &[i, k] = st.back();
        if (k >= (int)g[i].size()) { st.pop_back(); continue; }
        const int r = g[i][k++];
        if (seen[r] == i0) continue;
        seen[r] = i0;
        par_r[r] = i;
        if (mate_r[r] < 0) found = r;
        else st.push_back({mate_r[r], 0});
      }
      for (int r = found; r >= 0;) {   // flip the path
        const int i = par_r[r], nxt = mate_l[i];
        mate_l[i] = r;
        mate_r[r] = i;
        r = nxt;
      }
    }
    // König: Z = reachable from unmatched left nodes by alternating paths
    std::vector<char> zl(nl, 0), zr(nr, 0);
    std::vector<int> q;
    for (int i = 0; i < nl; ++i)
      if (mate_l[i] < 0) { zl[i] = 1; q.push_back(i); }
    for (size_t h = 0; h < q.size(); ++h)
      for (int r : g[q[h]])
        if (!zr[r] && mate_l[q[h]] != r) {
          zr[r] = 1;
          const int i = mate_r[r];
          if (i >= 0 && !zl[i]) { zl[i] = 1; q.push_back(i); }
        }
    int n = 0;
    for (int i = 0; i < nl; ++i) if (!zl[i]) { cover[left[i]] = 1; ++n; }
    for (int r = 0; r < nr; ++r) if (zr[r]) { cover[right[r]] = 1; ++n; }
    (void)idx;
    return n;
  }

  // Geometric separator: cut the component by a plane normal to one of its
  // principal axes at a quantile of the projections; the separator is the
  // minimum vertex cover of the cut edges (konig_cover).  The best
  // (smallest, then most balanced) of several cuts is kept.
  bool geometric_separator(std::vector<int> &comp, int tag, std::vector<int> &A, std::vector<int> &B,
                           std::vector<int> &S) {
    const int m = (int)comp.size();
    double c[3] = {0, 0, 0}, C[9] = {0};
    for (int u : comp)
      for (int a = 0; a < 3; ++a) c[a] += xyz[3L * u + a] / m;
    for (int u : comp)
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) C[3 * a + b] += (xyz[3L * u + a] - c[a]) * (xyz[3L * u + b] - c[b]);
    // two leading principal axes by power iteration with deflation
    double axes[2][3];
    double D[9];
    std::copy(C, C + 9, D);
    for (int k = 0; k < 2; ++k) {
      double v[3] = {1.0, 0.7, 0.3};
      double lam = 0.0;
      for (int it = 0; it < 100; ++it) {
        double w[3];
        for (int a = 0; a < 3; ++a) w[a] = D[3 * a] * v[0] + D[3 * a + 1] * v[1] + D[3 * a + 2] * v[2];
        const double nw = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        if (nw == 0.0) break;
        for (int a = 0; a < 3; ++a) v[a] = w[a] / nw;
        lam = nw;
      }
      for (int a = 0; a < 3; ++a) axes[k][a] = v[a];
      for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) D[3 * a + b] -= lam * v[a] * v[b];
    }
    // (fast, components of up to 512 tags: half the directions and every
    // other quantile, a quarter of the König covers -- the order was most of
    // an incremental reload; a slightly larger fill, e.g. cfg2 213 tiles
    // against 205)
    const bool big = !fast || m > 512;
    const int n_dir = big ? 6 : 3, n_q = 20, q_step = big ? 1 : 2;
    // each direction's best cut (its own scratch; large components search the
    // directions concurrently), then the first best over the directions in
    // order: the serial search's choice
    std::vector<double> dir_score(n_dir, -1.0);
    std::vector<std::vector<int>> dir_side(n_dir);
    auto search = [&](int k) {
      std::vector<int> side(adj.size(), 0), loc(adj.size(), -1);
      std::vector<char> cover(adj.size(), 0);
      std::vector<std::pair<double, int>> pr(m);
      double &best_score = dir_score[k];
      std::vector<int> &best_side = dir_side[k];
      // cut directions in the plane of the two principal axes
      const double ang = M_PI * k / n_dir, ca = std::cos(ang), sa = std::sin(ang);
      double dir[3];
      for (int a = 0; a < 3; ++a) dir[a] = ca * axes[0][a] + sa * axes[1][a];
      for (int i = 0; i < m; ++i) {
        const int u = comp[i];
        pr[i] = {dir[0] * xyz[3L * u] + dir[1] * xyz[3L * u + 1] + dir[2] * xyz[3L * u + 2], u};
      }
      std::sort(pr.begin(), pr.end());
      const int q0 = (int)std::lround(nd_qlo() * n_q);
      for (int qi = q0; qi <= n_q - q0; qi += q_step) {   // cut at quantiles 0.30 .. 0.70
        const int cut = m * qi / n_q;
        if (cut < 1 || cut >= m) continue;
        for (int i = 0; i < m; ++i) side[pr[i].second] = i < cut ? 1 : 2;
        for (int u : comp) cover[u] = 0;
        const int ssz = konig_cover(comp, side, tag, cover, loc);
        int na = 0, nbb = 0;
        for (int u : comp)
          if (!cover[u]) (side[u] == 1 ? na : nbb)++;
        if (std::min(na, nbb) < (int)(nd_min_side() * m)) continue;
        // elimination-tree height in tile columns: the separator's tiles plus
        // the larger child's height, which grows about as sqrt(size) on these
        // planar graphs (cfg3's tree: ~1 tile column per sqrt(tag))
        const double score = height_score(ssz, na, nbb);
        if (best_score < 0 || score < best_score) {
          best_score = score;
          best_side.assign(m, 0);
          for (int i = 0; i < m; ++i) best_side[i] = cover[comp[i]] ? 0 : side[comp[i]];
        }
      }
    };
    if (m >= 256) host_parallel_for(n_dir, search);
    else for (int k = 0; k < n_dir; ++k) search(k);
    double best_score = -1;
    int best_k = -1;
    for (int k = 0; k < n_dir; ++k)
      if (dir_score[k] >= 0 && (best_score < 0 || dir_score[k] < best_score)) {
        best_score = dir_score[k];
        best_k = k;
      }
    if (best_score < 0) return false;
    const std::vector<int> &best_side = dir_side[best_k];
    for (int i = 0; i < m; ++i) (best_side[i] == 1 ? A : best_side[i] == 2 ? B : S).push_back(comp[i]);
    return true;
  }

  void dissect(std::vector<int> &comp, int tag, std::vector<std::vector<int>> &parts) {
    if ((int)comp.size() <= leaf) {
      leaf_part(comp, tag, parts);
      return;
    }
    std::vector<int> A, B, S;
    bool ok = false;
    if (!xyz.empty()) {
      ok = geometric_separator(comp, tag, A, B, S);
      std::vector<int> A2, B2, S2;
      if (level_separator(comp, tag, A2, B2, S2) &&
          (!ok || height_score((long)S2.size(), (long)A2.size(), (long)B2.size()) <
                      height_score((long)S.size(), (long)A.size(), (long)B.size()))) {
        A.swap(A2); B.swap(B2); S.swap(S2);
        ok = true;
      }
    } else {
      ok = level_separator(comp, tag, A, B, S);
    }
    if (!ok) {
      leaf_part(comp, tag, parts);
      return;
    }
    absorb(A, B, S, tag);
    static const bool dbg = std::getenv("ARSLAM_ND_DEBUG") != nullptr;   // debug: the dissection tree
    if (dbg) std::fprintf(stderr, "nd: comp %zu -> A %zu B %zu S %zu\n", comp.size(), A.size(), B.size(), S.size());
    const int ta = ++next_tag, tb = ++next_tag, ts = ++next_tag;
    for (int u : A) mark[u] = ta;
    for (int u : B) mark[u] = tb;
    for (int u : S) mark[u] = ts;
    std::vector<std::vector<int>> pb;
    host_fork2(std::min(A.size(), B.size()) >= 128, [&] { run(A, ta, parts); }, [&] { run(B, tb, pb); });
    for (auto &q : pb) parts.push_back(std::move(q));
    parts.push_back(S);
  }

  // Grow the separator into the larger side (nodes adjacent to it first) until
  // its 6 rows per tag fill whole 64-row tiles: rows that would otherwise be
  // alignment padding become separator rows, and the children shrink.  Any
  // superset of a separator taken from one side still separates.
  void absorb(std::vector<int> &A, std::vector<int> &B, std::vector<int> &S, int tag) {
    const long rows = 6L * (long)S.size();
    int extra = (int)((round_up(rows, kTileRows) - rows) / 6);
    std::vector<int> &X = A.size() >= B.size() ? A : B;
    if (extra <= 0 || (int)X.size() <= extra) return;
    const int tx = ++next_tag;
    for (int u : X) mark[u] = tx;
    std::vector<char> take(adj.size(), 0);
    std::vector<int> frontier;
    for (int u : S)
      for (int v : adj[u])
        if (mark[v] == tx && !take[v] && extra > 0) { take[v] = 1; frontier.push_back(v); --extra; }
    for (size_t h = 0; h < frontier.size() && extra > 0; ++h)
      for (int v : adj[frontier[h]])
        if (mark[v] == tx && !take[v] && extra > 0) { take[v] = 1; frontier.push_back(v); --extra; }
    std::vector<int> keep;
    for (int u : X) (take[u] ? S : keep).push_back(u);
    for (int u : X) mark[u] = tag;
    X.swap(keep);
  }

  void leaf_part(std::vector<int> &comp, int tag, std::vector<std::vector<int>> &parts) {
    // within a leaf keep BFS order (locality)
    std::vector<int> ord = bfs(comp[0], adj, mark, tag, lev);
    for (int u : ord) lev[u] = -1;
    parts.push_back(ord);
  }
};

}  // namespace

std::vector<int> rcm_order(int n, const std::vector<std::vector<int>> &adj) {
  std::vector<int> order;
  order.reserve(n);
  std::vector<int> mark(n, 0), lev(n, -1);
  std::vector<char> done(n, 0);
  for (;;) {
    int start = -1;
    for (int v = 0; v < n; ++v)
      if (!done[v] && (start < 0 || adj[v].size() < adj[start].size())) start = v;
    if (start < 0) break;
    start = peripheral(start, adj, mark, 0, lev);
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

std::vector<std::vector<int>> nd_parts(int n, const std::vector<std::vector<int>> &adj, int leaf,
                                       const std::vector<double> &xyz, bool fast) {
  Dissector d(adj, xyz, leaf);
  d.fast = fast;
  std::vector<int> all(n);
  for (int i = 0; i < n; ++i) all[i] = i;
  std::vector<std::vector<int>> parts;
  d.run(all, 0, parts);
  return parts;
}


double scalar_cholesky_flops(const std::vector<std::vector<int>> &adj, const std::vector<int> &tag_row,
                             bool camera) {
  // tags in elimination order; symbolic factorization on the tag graph: the
  // higher-ordered neighbour set of a tag (its fill included) is merged into
  // its elimination-tree parent, the lowest of them
  std::vector<int> order;
  for (int t = 0; t < (int)tag_row.size(); ++t)
    if (tag_row[t] >= 0) order.push_back(t);
  std::sort(order.begin(), order.end(), [&](int a, int b) { return tag_row[a] < tag_row[b]; });
  std::vector<int> pos(tag_row.size(), -1);
  for (int i = 0; i < (int)order.size(); ++i) pos[order[i]] = i;
  const int n = (int)order.size();
  std::vector<std::vector<int>> up(n);   // higher-ordered neighbours (positions), sorted
  for (int i = 0; i < n; ++i) {
    for (int v : adj[order[i]])
      if (v < (int)pos.size() && pos[v] > i) up[i].push_back(pos[v]);
    std::sort(up[i].begin(), up[i].end());
    up[i].erase(std::unique(up[i].begin(), up[i].end()), up[i].end());
  }
  const double ncam = camera ? 3.0 : 0.0;
  double flops = 0.0;
  auto col = [&](double c) { flops += c * (c + 1.0) + c + 1.0; };
  std::vector<int> merged;
  for (int i = 0; i < n; ++i) {
    const double f = (double)up[i].size();
    for (int k = 0; k < 6; ++k) col((5 - k) + 6.0 * f + ncam);
    if (!up[i].empty()) {
      const int parent = up[i][0];
      merged.clear();
      std::set_union(up[parent].begin(), up[parent].end(), up[i].begin() + 1, up[i].end(),
                     std::back_inserter(merged));
      up[parent].swap(merged);
    }
    std::vector<int>().swap(up[i]);
  }
  for (int k = 0; k < (int)ncam; ++k) col(ncam - 1 - k);
  return flops;
}

// Ceres 2.0 (reorder_program.cc ComputeStableSchurOrdering, graph_algorithms.h
// StableIndependentSetOrdering): vertices are the
// non-constant parameter blocks in program order -- the order in which
// AddResidualBlock(cost, nullptr, camera, capture, tag) first saw them,
// ar_slam_util.cpp:723-727 -- with an edge between every two non-constant
// blocks of one residual.  The vertices are stable-sorted by ascending degree
// and taken greedily: a vertex none of whose neighbours is taken joins the
// independent set (the e-blocks).
SchurSide ceres_schur_side(const arslam_soa_problem *p, std::vector<uint8_t> *e_cap, std::vector<uint8_t> *e_tag) {
  SchurSide out;
  if (e_cap) e_cap->assign(p ? std::max(p->n_cap, 0) : 0, 0);
  if (e_tag) e_tag->assign(p ? std::max(p->n_tag, 0) : 0, 0);
  api_check(p != nullptr, ARSLAM_E_INVALID_ARG, "null problem");
  api_check(p->n_cap >= 0 && p->n_tag >= 0 && p->n_obs >= 0, ARSLAM_E_INVALID_ARG, "negative sizes");
  api_check(!p->n_obs || (p->obs_cap && p->obs_tag), ARSLAM_E_INVALID_ARG, "null observation arrays");
  const int nc = p->n_cap, nt = p->n_tag, nb = p->n_obs;
  for (int b = 0; b < nb; ++b) {
    api_check(p->obs_cap[b] >= 0 && p->obs_cap[b] < nc, ARSLAM_E_INVALID_ARG, "obs_cap out of range");
    api_check(p->obs_tag[b] >= 0 && p->obs_tag[b] < nt, ARSLAM_E_INVALID_ARG, "obs_tag out of range");
  }
  if (nb == 0) return out;
  auto cap_free = [&](int c) { return !(p->cap_const && p->cap_const[c]); };
  auto tag_free = [&](int t) { return !(p->tag_const && p->tag_const[t]); };
  const bool cam_free = !p->camera_const;
  // distinct (capture, tag) pairs of free blocks in both directions, in
  // O(observations): bucketed by capture (a counting sort), duplicates dropped
  // with a last-seen capture per tag (the adjacency lists are sets: their
  // order does not change the independent set)
  std::vector<int> tag_nobs(nt, 0);
  for (int b = 0; b < nb; ++b) out.max_tag_obs = std::max(out.max_tag_obs, ++tag_nobs[p->obs_tag[b]]);
  std::vector<int> by_cap_start(nc + 1, 0), by_cap(nb);
  for (int b = 0; b < nb; ++b) by_cap_start[p->obs_cap[b] + 1]++;
  for (int c = 0; c < nc; ++c) by_cap_start[c + 1] += by_cap_start[c];
  {
    std::vector<int> fill(by_cap_start.begin(), by_cap_start.end() - 1);
    for (int b = 0; b < nb; ++b) by_cap[fill[p->obs_cap[b]]++] = b;
  }
  {   // the most distinct tags of one capture and captures of one tag, constant blocks included
      // (the local system an e-block's k_schur wave holds: kMaxSchurBlocks)
    std::vector<int> last(nt, -1), ncap(nt, 0);
    for (int c = 0; c < nc; ++c) {
      int d = 0;
      for (int q = by_cap_start[c]; q < by_cap_start[c + 1]; ++q) {
        const int t = p->obs_tag[by_cap[q]];
        if (last[t] == c) continue;
        last[t] = c;
        ++d;
        out.max_tag_blk = std::max(out.max_tag_blk, ++ncap[t]);
      }
      out.max_cap_blk = std::max(out.max_cap_blk, d);
    }
  }
  std::vector<int> cap_adj_start(nc + 1, 0), cap_adj, tag_adj_start(nt + 1, 0), mark(nt, -1);
  cap_adj.reserve(nb);
  for (int c = 0; c < nc; ++c) {
    if (cap_free(c))
      for (int q = by_cap_start[c]; q < by_cap_start[c + 1]; ++q) {
        const int t = p->obs_tag[by_cap[q]];
        if (!tag_free(t) || mark[t] == c) continue;
        mark[t] = c;
        cap_adj.push_back(t);
        tag_adj_start[t + 1]++;
      }
    cap_adj_start[c + 1] = (int)cap_adj.size();
  }
  for (int t = 0; t < nt; ++t) tag_adj_start[t + 1] += tag_adj_start[t];
  std::vector<int> tag_adj(tag_adj_start[nt]);
  {
    std::vector<int> ft(tag_adj_start.begin(), tag_adj_start.end() - 1);
    for (int c = 0; c < nc; ++c)
      for (int q = cap_adj_start[c]; q < cap_adj_start[c + 1]; ++q) tag_adj[ft[cap_adj[q]]++] = c;
  }
  // vertex ids: 0 camera, 1 + c capture, 1 + nc + t tag; program order
  const int nv = 1 + nc + nt;
  std::vector<int> order;
  order.reserve(nv);
  std::vector<char> seen(nv, 0);
  auto visit = [&](int v, bool free_) {
    if (free_ && !seen[v]) { seen[v] = 1; order.push_back(v); }
  };
  for (int b = 0; b < nb; ++b) {
    visit(0, cam_free);
    visit(1 + p->obs_cap[b], cap_free(p->obs_cap[b]));
    visit(1 + nc + p->obs_tag[b], tag_free(p->obs_tag[b]));
  }
  const int cam_deg = (int)order.size() - (cam_free ? 1 : 0);
  auto degree = [&](int v) {
    if (v == 0) return cam_deg;
    if (v <= nc) return cap_adj_start[v] - cap_adj_start[v - 1] + (cam_free ? 1 : 0);
    const int t = v - 1 - nc;
    return tag_adj_start[t + 1] - tag_adj_start[t] + (cam_free ? 1 : 0);
  };
  std::vector<int> deg(nv, 0);
  int max_deg = 0;
  for (int v : order) max_deg = std::max(max_deg, deg[v] = degree(v));
  {   // stable sort by ascending degree: a counting sort
    std::vector<int> cnt(max_deg + 2, 0), sorted(order.size());
    for (int v : order) cnt[deg[v] + 1]++;
    for (int d = 0; d <= max_deg; ++d) cnt[d + 1] += cnt[d];
    for (int v : order) sorted[cnt[deg[v]]++] = v;
    order.swap(sorted);
  }
  enum : char { kWhite = 0, kGrey = 1, kBlack = 2 };
  std::vector<char> color(nv, kWhite);
  for (int v : order) {
    if (color[v] != kWhite) continue;
    color[v] = kBlack;
    if (v == 0) {
      ++out.e_cam;
      for (int u : order) if (u != 0 && color[u] == kWhite) color[u] = kGrey;   // every block shares a residual with it
      continue;
    }
    if (cam_free && color[0] == kWhite) color[0] = kGrey;
    if (v <= nc) {
      ++out.e_cap;
      if (e_cap) (*e_cap)[v - 1] = 1;
      for (int q = cap_adj_start[v - 1]; q < cap_adj_start[v]; ++q) {
        const int u = 1 + nc + cap_adj[q];
        if (color[u] == kWhite) color[u] = kGrey;
      }
    } else {
      ++out.e_tag;
      const int t = v - 1 - nc;
      if (e_tag) (*e_tag)[t] = 1;
      for (int q = tag_adj_start[t]; q < tag_adj_start[t + 1]; ++q) {
        const int u = 1 + tag_adj[q];
        if (color[u] == kWhite) color[u] = kGrey;
      }
    }
  }
  return out;
}

arslam_soa_problem swap_roles(const arslam_soa_problem &p) {
  arslam_soa_problem s = p;
  s.n_cap = p.n_tag; s.n_tag = p.n_cap;
  s.cap = p.tag; s.tag = p.cap;
  s.obs_cap = p.obs_tag; s.obs_tag = p.obs_cap;
  s.cap_const = p.tag_const; s.tag_const = p.cap_const;
  return s;
}

MixedProblem mixed_problem(const arslam_soa_problem &p, const std::vector<uint8_t> &e_cap,
                           const std::vector<uint8_t> &e_tag) {
  MixedProblem m;
  const int nc = p.n_cap, nt = p.n_tag, nb = p.n_obs;
  m.src_n_cap = nc;
  m.src_n_tag = nt;
  std::vector<int> cap_f(nc, -1), tag_f(nt, -1), cap_g(nc, -1), tag_g(nt, -1), cap_d(nc, -1);
  for (int t = 0; t < nt; ++t)
    if (!e_tag[t]) { tag_f[t] = (int)m.f_src.size(); m.f_src.push_back(t); m.f_is_cap.push_back(0); }
  for (int c = 0; c < nc; ++c)
    if (!e_cap[c]) { cap_f[c] = (int)m.f_src.size(); m.f_src.push_back(c); m.f_is_cap.push_back(1); }
  for (int c = 0; c < nc; ++c)
    if (e_cap[c]) { cap_g[c] = (int)m.kind.size(); m.kind.push_back(kMixCap); m.group_src.push_back(c); }
  for (int t = 0; t < nt; ++t)
    if (e_tag[t]) { tag_g[t] = (int)m.kind.size(); m.kind.push_back(kMixTag); m.group_src.push_back(t); }
  for (int b = 0; b < nb; ++b) {
    const int c = p.obs_cap[b], t = p.obs_tag[b];
    api_check(!(e_cap[c] && e_tag[t]), ARSLAM_E_INVALID_ARG, "mixed e-set: a residual joins two e-blocks");
    if (!e_cap[c] && !e_tag[t] && cap_d[c] < 0) {
      cap_d[c] = (int)m.kind.size();
      m.kind.push_back(kMixDirect);
      m.group_src.push_back(c);
    }
  }
  const int ng = (int)m.kind.size(), nf = (int)m.f_src.size();
  m.f_alias.assign(nf, -1);
  for (int c = 0; c < nc; ++c)
    if (cap_d[c] >= 0) { m.f_alias[cap_f[c]] = cap_d[c]; ++m.n_direct; }
  m.obs_cap.resize(nb);
  m.obs_tag.resize(nb);
  for (int b = 0; b < nb; ++b) {
    const int c = p.obs_cap[b], t = p.obs_tag[b];
    if (e_cap[c]) { m.obs_cap[b] = cap_g[c]; m.obs_tag[b] = tag_f[t]; }
    else if (e_tag[t]) { m.obs_cap[b] = tag_g[t]; m.obs_tag[b] = cap_f[c]; }
    else { m.obs_cap[b] = cap_d[c]; m.obs_tag[b] = tag_f[t]; }
  }
  m.cap.resize(6L * ng);
  m.tag.resize(6L * nf);
  m.cap_const.resize(ng);
  m.tag_const.resize(nf);
  for (int g = 0; g < ng; ++g) {
    const bool is_tag = m.kind[g] == kMixTag;
    const unsigned char *cst = is_tag ? p.tag_const : p.cap_const;
    m.cap_const[g] = cst ? cst[m.group_src[g]] : 0;
  }
  for (int f = 0; f < nf; ++f) {
    const unsigned char *cst = m.f_is_cap[f] ? p.cap_const : p.tag_const;
    m.tag_const[f] = cst ? cst[m.f_src[f]] : 0;
  }
  m.soa = p;
  m.soa.n_cap = ng;
  m.soa.n_tag = nf;
  m.soa.cap = m.cap.data();
  m.soa.tag = m.tag.data();
  m.soa.obs_cap = m.obs_cap.data();
  m.soa.obs_tag = m.obs_tag.data();
  m.soa.cap_const = m.cap_const.data();
  m.soa.tag_const = m.tag_const.data();
  std::vector<double> x(3 + 6L * ng + 6L * nf);
  mixed_values(m, p, x.data());
  if (ng) std::memcpy(m.cap.data(), x.data() + 3, 6L * ng * sizeof(double));
  if (nf) std::memcpy(m.tag.data(), x.data() + 3 + 6L * ng, 6L * nf * sizeof(double));
  return m;
}

void mixed_values(const MixedProblem &m, const arslam_soa_problem &p, double *x) {
  const long ng = (long)m.kind.size(), nf = (long)m.f_src.size();
  std::memcpy(x, p.camera, 3 * sizeof(double));
  for (long g = 0; g < ng; ++g) {
    const double *src = m.kind[g] == kMixTag ? p.tag : p.cap;
    std::memcpy(x + 3 + 6 * g, src + 6L * m.group_src[g], 6 * sizeof(double));
  }
  for (long f = 0; f < nf; ++f) {
    const double *src = m.f_is_cap[f] ? p.cap : p.tag;
    std::memcpy(x + 3 + 6 * ng + 6 * f, src + 6L * m.f_src[f], 6 * sizeof(double));
  }
}

void mixed_patch(HostProblem &h, const MixedProblem &m, const arslam_soa_problem &p) {
  const int ng = h.nc, nf = h.nt;
  // the direct groups' own f-block, last in their block lists
  std::vector<int> own(ng, -1);
  for (int f = 0; f < nf; ++f)
    if (m.f_alias[f] >= 0) own[m.f_alias[f]] = f;
  std::vector<int> start(ng + 1, 0), blk;
  blk.reserve(h.blk_tag.size() + m.n_direct);
  h.maxblk = 0;
  for (int g = 0; g < ng; ++g) {
    start[g] = (int)blk.size();
    blk.insert(blk.end(), h.blk_tag.begin() + h.cap_blk_start[g], h.blk_tag.begin() + h.cap_blk_start[g + 1]);
    if (own[g] >= 0) blk.push_back(own[g]);
    h.maxblk = std::max(h.maxblk, (int)blk.size() - start[g]);
  }
  start[ng] = (int)blk.size();
  h.cap_blk_start.swap(start);
  h.blk_tag.swap(blk);
  api_check(h.maxblk <= kMaxSchurBlocks, ARSLAM_E_UNSUPPORTED,
            "an eliminated block (or a direct group) couples more than 256 distinct blocks");
  // an f-block is free iff its original block is (a capture on the reduced side
  // may be used only by residuals of its own direct group)
  std::vector<char> used_c(p.n_cap, 0), used_t(p.n_tag, 0);
  for (int b = 0; b < p.n_obs; ++b) { used_c[p.obs_cap[b]] = 1; used_t[p.obs_tag[b]] = 1; }
  for (int f = 0; f < nf; ++f) {
    const int o = m.f_src[f];
    const bool fr = (m.f_is_cap[f] ? used_c[o] : used_t[o]) && !m.tag_const[f];
    for (int j = 0; j < 6; ++j) h.slot_free[3 + 6L * ng + 6L * f + j] = fr;
  }
  // the f-blocks' places for the ordering: a tag's translation; a capture's
  // the mean translation of the tags it sees (its own translation is minus the
  // camera centre, a mirror image of the tags' frame)
  std::vector<double> cap_xyz(3L * p.n_cap, 0.0);
  std::vector<int> cap_n(p.n_cap, 0);
  for (int b = 0; b < p.n_obs; ++b) {
    const int c = p.obs_cap[b];
    for (int a = 0; a < 3; ++a) cap_xyz[3L * c + a] += p.tag[6L * p.obs_tag[b] + a];
    cap_n[c]++;
  }
  h.nd_xyz.assign(3L * nf, 0.0);
  for (int f = 0; f < nf; ++f) {
    const int o = m.f_src[f];
    for (int a = 0; a < 3; ++a)
      h.nd_xyz[3L * f + a] = m.f_is_cap[f] ? (cap_n[o] ? cap_xyz[3L * o + a] / cap_n[o] : 0.0) : p.tag[6L * o + a];
  }
}

HostProblem host_problem(const arslam_soa_problem *p, const ReduceSumF64 &tag_deg_sum) {
  api_check(p != nullptr, ARSLAM_E_INVALID_ARG, "null problem");
  api_check(p->n_cap >= 0 && p->n_tag >= 0 && p->n_obs >= 0, ARSLAM_E_INVALID_ARG, "negative sizes");
  api_check(p->camera && (!p->n_cap || p->cap) && (!p->n_tag || p->tag), ARSLAM_E_INVALID_ARG,
            "null parameter arrays");
  api_check(!p->n_obs || (p->obs_cap && p->obs_tag && p->corners), ARSLAM_E_INVALID_ARG,
            "null observation arrays");
  HostProblem h;
  const int nc = h.nc = p->n_cap, nt = h.nt = p->n_tag, nb = h.nb = p->n_obs;
  const long n = h.n = 3 + 6L * nc + 6L * nt;
  // capture-major observation order (stable)
  h.cap_start.assign(nc + 1, 0);
  for (int b = 0; b < nb; ++b) {
    api_check(p->obs_cap[b] >= 0 && p->obs_cap[b] < nc, ARSLAM_E_INVALID_ARG, "obs_cap out of range");
    api_check(p->obs_tag[b] >= 0 && p->obs_tag[b] < nt, ARSLAM_E_INVALID_ARG, "obs_tag out of range");
    h.cap_start[p->obs_cap[b] + 1]++;
  }
  for (int c = 0; c < nc; ++c) {
    h.maxk = std::max(h.maxk, h.cap_start[c + 1]);
    h.cap_start[c + 1] += h.cap_start[c];
  }
  std::vector<int> order(nb);
  {
    std::vector<int> fill(h.cap_start.begin(), h.cap_start.end() - 1);
    for (int b = 0; b < nb; ++b) order[fill[p->obs_cap[b]]++] = b;
  }
  h.obs_tag.resize(nb);
  h.obs_lblk.resize(nb);
  h.cap_blk_start.assign(nc + 1, 0);
  h.corners.resize(8L * nb);
  h.blk_tag.reserve(nb);
  for (int c = 0; c < nc; ++c) {
    h.cap_blk_start[c] = (int)h.blk_tag.size();
    for (int q = h.cap_start[c]; q < h.cap_start[c + 1]; ++q) {
      const int b = order[q];
      const int t = p->obs_tag[b];
      h.obs_tag[q] = t;
      std::memcpy(&h.corners[8L * q], p->corners + 8L * b, 8 * sizeof(double));
      int u = -1;
      for (int i = h.cap_blk_start[c]; i < (int)h.blk_tag.size(); ++i)
        if (h.blk_tag[i] == t) { u = i - h.cap_blk_start[c]; break; }
      if (u < 0) { u = (int)h.blk_tag.size() - h.cap_blk_start[c]; h.blk_tag.push_back(t); }
      h.obs_lblk[q] = u + 1;
    }
    h.maxblk = std::max(h.maxblk, (int)h.blk_tag.size() - h.cap_blk_start[c]);
  }
  h.cap_blk_start[nc] = (int)h.blk_tag.size();
  api_check(h.maxblk <= kMaxSchurBlocks, ARSLAM_E_UNSUPPORTED,
            "an eliminated block (capture, or tag under tag elimination) couples more than 256 distinct blocks");
  // tag CSR over the capture-major order
  h.tag_start.assign(nt + 1, 0);
  h.tag_obs.resize(nb);
  h.obs_tpos.resize(nb);
  for (int q = 0; q < nb; ++q) h.tag_start[h.obs_tag[q] + 1]++;
  for (int t = 0; t < nt; ++t) h.tag_start[t + 1] += h.tag_start[t];
  {
    std::vector<int> fill(h.tag_start.begin(), h.tag_start.end() - 1);
    for (int q = 0; q < nb; ++q) {
      h.obs_tpos[q] = fill[h.obs_tag[q]]++;
      h.tag_obs[h.obs_tpos[q]] = q;
    }
  }
  // free slots (global tag use over ranks)
  std::vector<double> tag_deg(nt + 1, 0.0);
  for (int q = 0; q < nb; ++q) tag_deg[h.obs_tag[q]] += 1.0;
  tag_deg[nt] = nb;
  if (tag_deg_sum) tag_deg_sum(tag_deg);
  h.nb_global = (long)tag_deg[nt];
  h.slot_free.assign(n, 0);
  const bool cam_free = !p->camera_const && tag_deg[nt] > 0;
  for (int j = 0; j < 3; ++j) h.slot_free[j] = cam_free;
  for (int c = 0; c < nc; ++c) {
    const bool f = h.cap_start[c + 1] > h.cap_start[c] && !(p->cap_const && p->cap_const[c]);
    for (int j = 0; j < 6; ++j) h.slot_free[3 + 6L * c + j] = f;
  }
  for (int t = 0; t < nt; ++t) {
    const bool f = tag_deg[t] > 0 && !(p->tag_const && p->tag_const[t]);
    for (int j = 0; j < 6; ++j) h.slot_free[3 + 6L * nc + 6L * t + j] = f;
  }
  h.obs_active.resize(nb);
  for (int q = 0; q < nb; ++q) {
    const int c = p->obs_cap[order[q]];
    h.obs_active[q] = h.slot_free[0] || h.slot_free[3 + 6L * c] || h.slot_free[3 + 6L * nc + 6L * h.obs_tag[q]];
  }
  h.x0.resize(n);
  std::memcpy(h.x0.data(), p->camera, 3 * sizeof(double));
  if (nc) std::memcpy(h.x0.data() + 3, p->cap, 6L * nc * sizeof(double));
  if (nt) std::memcpy(h.x0.data() + 3 + 6L * nc, p->tag, 6L * nt * sizeof(double));
  return h;
}

ReducedLayout reduced_layout(const HostProblem &h, int ordering, bool sparse, const ReduceMaxU8 &adj_max,
                             const ReduceMaxU8 &pattern_max,
                             const std::vector<int> *reuse_tag_row, long reuse_edges, bool fast_order,
                             bool reuse_by_identity) {
  static const bool prof = std::getenv("ARSLAM_SETUP_PROFILE") != nullptr;   // debug: layout phases
  auto clk = []() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double tl[5] = {prof ? clk() : 0.0, 0, 0, 0, 0};
  // Rows exist only for free tags and a free camera (constant / unused blocks
  // are not parameters).  Tags are ordered natural, RCM or by nested
  // dissection; with ND every part starts on a tile boundary so the tile
  // elimination tree follows the dissection tree.
  const int nc = h.nc, nt = h.nt;
  ReducedLayout L;
  L.tag_row.assign(std::max(nt, 1), -1);
  std::vector<char> tfree(nt, 0);
  for (int t = 0; t < nt; ++t) tfree[t] = h.slot_free[3 + 6L * nc + 6L * t];
  std::vector<std::vector<int>> adj(nt);
  if (nt > 1) {   // (also for the natural order: the scalar flop count reads it)
    if (adj_max) {   // co-visibility is global over ranks
      api_check(nt <= 16384, ARSLAM_E_UNSUPPORTED, "multi-GPU reduced ordering limited to 16384 tags");
      std::vector<uint8_t> bm((size_t)nt * nt, 0);
      for (int c = 0; c < nc; ++c)
        for (int a = h.cap_blk_start[c]; a < h.cap_blk_start[c + 1]; ++a)
          for (int b = h.cap_blk_start[c]; b < h.cap_blk_start[c + 1]; ++b)
            if (a != b) bm[(size_t)h.blk_tag[a] * nt + h.blk_tag[b]] = 1;
      adj_max(bm);
      for (int a = 0; a < nt; ++a)
        for (int b = 0; b < nt; ++b)
          if (bm[(size_t)a * nt + b] && tfree[a] && tfree[b]) adj[a].push_back(b);
    } else {
      // per tag, the distinct tags of the captures whose blocks list it (a
      // stamp array dedupes them before the sort: the pairs repeat in every
      // capture that sees both; a mixed set's direct group lists its own
      // pose, which no residual of the group has as its tag)
      std::vector<int> tcap_start(nt + 1, 0), tcap(h.blk_tag.size());
      for (int t : h.blk_tag) tcap_start[t + 1]++;
      for (int t = 0; t < nt; ++t) tcap_start[t + 1] += tcap_start[t];
      {
        std::vector<int> fill(tcap_start.begin(), tcap_start.end() - 1);
        for (int c = 0; c < nc; ++c)
          for (int bb = h.cap_blk_start[c]; bb < h.cap_blk_start[c + 1]; ++bb) tcap[fill[h.blk_tag[bb]]++] = c;
      }
      std::vector<int> stamp(nt, -1);
      for (int a = 0; a < nt; ++a) {
        if (!tfree[a]) continue;
        std::vector<int> &v = adj[a];
        for (int q = tcap_start[a]; q < tcap_start[a + 1]; ++q) {
          const int c = tcap[q];
          for (int bb = h.cap_blk_start[c]; bb < h.cap_blk_start[c + 1]; ++bb) {
            const int b = h.blk_tag[bb];
            if (b != a && tfree[b] && stamp[b] != a) {
              stamp[b] = a;
              v.push_back(b);
            }
          }
        }
        std::sort(v.begin(), v.end());
      }
    }
  }
  for (auto &v : adj) L.n_edges += (long)v.size();
  if (prof) tl[1] = clk();
  // (tags past the earlier order's -- new parameter blocks are appended --
  // are placed after its rows, at the end of its last part: below)
  // (by identity: an entry per tag, -1 for a tag without an earlier row)
  const int n_old = reuse_tag_row ? std::min((int)reuse_tag_row->size(), nt) : 0;
  bool reuse = reuse_tag_row && (int)reuse_tag_row->size() <= std::max(nt, 1) && 10 * L.n_edges <= 11 * reuse_edges;
  if (reuse_by_identity) reuse = reuse && (int)reuse_tag_row->size() == nt;
  for (int t = 0; reuse && !reuse_by_identity && t < n_old; ++t) reuse = ((*reuse_tag_row)[t] >= 0) == (tfree[t] != 0);
  L.order_edges = reuse ? reuse_edges : L.n_edges;
  L.order_reused = reuse;
  std::vector<std::vector<int>> parts;
  if (reuse) {
    // (the earlier order; rows below)
  } else if (ordering == 2 && nt > 1) {
    // tag positions (initial values) embed the co-visibility graph for geometric separators
    std::vector<double> xyz(3L * nt);
    for (int t = 0; t < nt; ++t)
      for (int a = 0; a < 3; ++a)
        xyz[3L * t + a] = h.nd_xyz.empty() ? h.x0[3 + 6L * nc + 6L * t + a] : h.nd_xyz[3L * t + a];
    // leaves of up to 32 tags (192 rows = 3 whole tiles): a smaller dissection
    // would not shorten the elimination tree, only add padding and parts
    // (debug sweeps; clamped to [1, 4096])
    static const int leaf =
        std::getenv("ARSLAM_ND_LEAF") ? std::min(4096, std::max(1, std::atoi(std::getenv("ARSLAM_ND_LEAF")))) : 32;
    parts = nd_parts(nt, adj, leaf, xyz, fast_order);
  } else {
    std::vector<int> order;
    if (ordering == 1 && nt > 1) order = rcm_order(nt, adj);
    else for (int t = 0; t < nt; ++t) order.push_back(t);
    parts.push_back(order);
  }
  long row = 0, real = 0;
  if (reuse) {
    // (by identity: a tag whose earlier row is no longer a parameter leaves
    // those rows as padding, identity rows like the alignment padding)
    for (int t = 0; t < n_old; ++t) L.tag_row[t] = tfree[t] ? (*reuse_tag_row)[t] : -1;
    for (int t = 0; t < n_old; ++t)
      if (L.tag_row[t] >= 0) {
        row = std::max(row, (long)L.tag_row[t] + 6);
        real += 6;
      }
    // the tags new since the order was made, at the end of its last part (the
    // root separator): a valid order whatever they couple to, since every
    // part's elimination path ends there; the caller recomputes the order
    // once the tile elimination tree grows taller than a fresh one
    for (int t = 0; t < nt; ++t)
      if (tfree[t] && (t >= n_old || L.tag_row[t] < 0)) {
        L.tag_row[t] = (int)row;
        row += 6;
        real += 6;
      }
  }
  for (auto &part : parts) {
    bool any = false;
    for (int t : part) any = any || tfree[t];
    if (!any) continue;
    L.n_parts++;
    if (ordering == 2) row = round_up(row, kTileRows);
    for (int t : part) {
      if (!tfree[t]) continue;
      L.tag_row[t] = (int)row;
      row += 6;
      real += 6;
    }
  }
  L.pad_rows = row - real;
  L.row_slot.assign(row, -1);
  for (int t = 0; t < nt; ++t)
    if (L.tag_row[t] >= 0)
      for (int j = 0; j < 6; ++j) L.row_slot[L.tag_row[t] + j] = (int)(3 + 6L * nc + 6L * t + j);
  if (h.slot_free[0]) {
    L.cam_row = (int)row;
    for (int j = 0; j < 3; ++j) L.row_slot.push_back(j);
    row += 3;
  }
  L.nR = row;
  if (prof) tl[2] = clk();
  L.scalar_flops = scalar_cholesky_flops(adj, L.tag_row, L.cam_row >= 0);
  if (prof) tl[3] = clk();
  if (L.nR == 0) return L;
  L.N = round_up(L.nR + 1, kTileRows);
  const int T = L.T = (int)(L.N / kTileRows);
  L.pattern.assign((size_t)T * T, 0);
  if (!sparse) {
    for (int i = 0; i < T; ++i)
      for (int j = 0; j <= i; ++j) L.pattern[(size_t)i * T + j] = 1;
    return L;
  }
  std::vector<int> ts;
  for (int c = 0; c < nc; ++c) {
    ts.clear();
    if (L.cam_row >= 0) {
      ts.push_back(L.cam_row / kTileRows);
      ts.push_back((L.cam_row + 2) / kTileRows);
    }
    for (int a = h.cap_blk_start[c]; a < h.cap_blk_start[c + 1]; ++a) {
      const int r0 = L.tag_row[h.blk_tag[a]];
      if (r0 < 0) continue;
      ts.push_back(r0 / kTileRows);
      ts.push_back((r0 + 5) / kTileRows);
    }
    std::sort(ts.begin(), ts.end());
    ts.erase(std::unique(ts.begin(), ts.end()), ts.end());
    for (size_t a = 0; a < ts.size(); ++a)
      for (size_t b = 0; b <= a; ++b) L.pattern[(size_t)ts[a] * T + ts[b]] = 1;
  }
  const int rhs = (int)(L.nR / kTileRows);
  for (int j = 0; j <= rhs; ++j) L.pattern[(size_t)rhs * T + j] = 1;
  if (pattern_max) pattern_max(L.pattern);
  if (prof)
    std::fprintf(stderr, "arslam layout: adj %.3f order %.3f flops %.3f pattern %.3f ms\n", tl[1] - tl[0],
                 tl[2] - tl[1], tl[3] - tl[2], clk() - tl[3]);
  return L;
}

namespace {

struct GatherItem {
  long key;   // rX << 32 | rY
  int c;
  int px, py, nblk;
};

// capture c's lower blocks of the reduced system (and its rhs row) as gather items
void capture_gather_items(const HostProblem &h, const ReducedLayout &L, int c, std::vector<GatherItem> &items,
                          std::vector<std::pair<int, int>> &blk) {
  const int nblk = h.cap_blk_start[c + 1] - h.cap_blk_start[c];
  const long m = 1 + 6L * nblk;
  if (h.cap_start[c + 1] == h.cap_start[c]) return;   // no residuals: k_schur stores nothing
  blk.clear();
  if (L.cam_row >= 0) blk.emplace_back(L.cam_row, 0);
  for (int u = 0; u < nblk; ++u) {
    const int tr = L.tag_row[h.blk_tag[h.cap_blk_start[c] + u]];
    if (tr >= 0) blk.emplace_back(tr, 1 + 6 * u);
  }
  if (blk.empty()) return;
  blk.emplace_back((int)L.nR, (int)m);   // rhs row
  for (size_t a = 0; a < blk.size(); ++a)
    for (size_t b = 0; b < blk.size(); ++b) {
      const int rx = blk[a].first, ry = blk[b].first;
      if (rx < ry || ry == L.nR) continue;   // lower blocks; the rhs only as a row
      items.push_back({((long)rx << 32) | ry, c, blk[a].second, blk[b].second, nblk});
    }
}

SchurContrib gather_contrib(const SchurGather &G, const GatherItem &t) {
  const int m = 1 + 6 * t.nblk, U = schur_blk(t.px, m), V = schur_blk(t.py, m);
  if (U >= V) return {G.cap_off[t.c] + schur_block_off(U, V, t.nblk), 0, schur_blk_size(V, t.nblk)};
  return {G.cap_off[t.c] + schur_block_off(V, U, t.nblk), 1, schur_blk_size(U, t.nblk)};
}

// the gather launch's work items: a destination per item, or its contributions
// in chunks of kSchurChunk summed through partial slots (k_schur_combine).  An
// item's wave sums its contributions in G = 64 / (the block's elements) lane
// groups, so a destination stays one item up to 16 contributions per group (64
// at least): a 1-element block (camera, rhs) up to 1,024 -- problems of up to
// 1,024 captures need no combine launch.  Longer ones keep 64-contribution
// pieces (a 1,024-contribution item's wave outlasts the rest of the gather)
int gather_single_max(const SchurGather &G, int d, long nR, int cam_row) {
  const int rX = G.dest_row[2L * d], rY = G.dest_row[2L * d + 1];
  const int e = ((rX == nR || rX == cam_row) ? 1 : 6) * (rY == cam_row ? 1 : 6);
  return std::max(kSchurChunk, 16 * (64 / e));
}

void gather_partition(SchurGather &G, long nR, int cam_row) {
  G.items.clear();
  G.splits.clear();
  G.n_pslots = 0;
  G.max_contrib = 0;
  const int nd = (int)G.dest_start.size() - 1;
  for (int d = 0; d < nd; ++d) {
    const int k0 = G.dest_start[d], k1 = G.dest_start[d + 1];
    G.max_contrib = std::max(G.max_contrib, k1 - k0);
    const int chunk = kSchurChunk;
    if (k1 - k0 <= gather_single_max(G, d, nR, cam_row)) {
      G.items.insert(G.items.end(), {d, k0, k1, -1});
      continue;
    }
    const int pieces = (k1 - k0 + chunk - 1) / chunk;
    G.splits.insert(G.splits.end(), {d, G.n_pslots, pieces, 0});
    for (int q = 0; q < pieces; ++q)
      G.items.insert(G.items.end(), {d, k0 + q * chunk, std::min(k1, k0 + (q + 1) * chunk), G.n_pslots + q});
    G.n_pslots += pieces;
  }
}

}  // namespace

SchurGather schur_gather_plan(const HostProblem &h, const ReducedLayout &L) {
  SchurGather G;
  G.cap_off.assign(h.nc + 1, 0);
  std::vector<GatherItem> items;
  std::vector<std::pair<int, int>> blk;   // (global first row, local first column) of the capture's blocks
  for (int c = 0; c < h.nc; ++c) {
    const int nblk = h.cap_blk_start[c + 1] - h.cap_blk_start[c];
    G.cap_off[c + 1] = G.cap_off[c] + schur_slab_size(nblk);
    capture_gather_items(h, L, c, items, blk);
  }
  // stable sort by (rX, rY): two stable counting passes (rY, then rX; rows
  // are < nR + 1), so each destination's contributions stay in capture
  // order -- the gather's fixed summation order.  (A comparison sort of the
  // ~45 items per capture was half of the per-Solve setup of an incremental
  // flow.)
  {
    const long nrow = L.nR + 2;
    std::vector<int> cnt(nrow + 1);
    std::vector<GatherItem> tmp(items.size());
    for (int pass = 0; pass < 2; ++pass) {
      auto row = [&](const GatherItem &t) { return pass == 0 ? (long)(t.key & 0xffffffffL) : (long)(t.key >> 32); };
      std::fill(cnt.begin(), cnt.end(), 0);
      for (const GatherItem &t : items) cnt[row(t) + 1]++;
      for (long r = 0; r < nrow; ++r) cnt[r + 1] += cnt[r];
      for (const GatherItem &t : items) tmp[cnt[row(t)]++] = t;
      items.swap(tmp);
    }
  }
  G.contrib.reserve(items.size());
  for (size_t i = 0; i < items.size(); ++i) {
    if (i == 0 || items[i].key != items[i - 1].key) {
      G.dest_row.push_back((int)(items[i].key >> 32));
      G.dest_row.push_back((int)(items[i].key & 0xffffffffL));
      G.dest_start.push_back((int)G.contrib.size());
    }
    G.contrib.push_back(gather_contrib(G, items[i]));
  }
  G.dest_start.push_back((int)G.contrib.size());
  gather_partition(G, L.nR, L.cam_row);
  return G;
}

// The plan of a problem grown by the captures [c0, nc) whose captures below c0
// are unchanged (the same layout L): each destination keeps its contributions
// and gains the new captures' after them -- capture order, the summation order
// of a fresh plan -- and a block no capture had touched becomes a destination
// in (rX, rY) order.  Equal to schur_gather_plan of the grown problem.
void schur_gather_extend(SchurGather &G, const HostProblem &h, const ReducedLayout &L, int c0) {
  const int nc0 = (int)G.cap_off.size() - 1;
  if (c0 != nc0) throw std::logic_error("schur_gather_extend: not an append of captures");
  G.cap_off.resize(h.nc + 1);
  std::vector<GatherItem> items;
  std::vector<std::pair<int, int>> blk;
  for (int c = c0; c < h.nc; ++c) {
    const int nblk = h.cap_blk_start[c + 1] - h.cap_blk_start[c];
    G.cap_off[c + 1] = G.cap_off[c] + schur_slab_size(nblk);
    capture_gather_items(h, L, c, items, blk);
  }
  std::stable_sort(items.begin(), items.end(), [](const GatherItem &a, const GatherItem &b) { return a.key < b.key; });
  const int nd = (int)G.dest_start.size() - 1;
  std::vector<int> dest_row, dest_start;
  std::vector<SchurContrib> contrib;
  dest_row.reserve(G.dest_row.size() + 2 * items.size());
  dest_start.reserve(G.dest_start.size() + items.size());
  contrib.reserve(G.contrib.size() + items.size());
  const long kEnd = LONG_MAX;
  size_t i = 0;
  int d = 0;
  while (d < nd || i < items.size()) {
    const long ko = d < nd ? ((long)G.dest_row[2 * d] << 32) | G.dest_row[2 * d + 1] : kEnd;
    const long kn = i < items.size() ? items[i].key : kEnd;
    const long k = std::min(ko, kn);
    dest_row.push_back((int)(k >> 32));
    dest_row.push_back((int)(k & 0xffffffffL));
    dest_start.push_back((int)contrib.size());
    if (ko == k) {
      contrib.insert(contrib.end(), G.contrib.begin() + G.dest_start[d], G.contrib.begin() + G.dest_start[d + 1]);
      ++d;
    }
    for (; i < items.size() && items[i].key == k; ++i) contrib.push_back(gather_contrib(G, items[i]));
  }
  dest_start.push_back((int)contrib.size());
  G.dest_row.swap(dest_row);
  G.dest_start.swap(dest_start);
  G.contrib.swap(contrib);
  gather_partition(G, L.nR, L.cam_row);
}

}  // namespace arslam
