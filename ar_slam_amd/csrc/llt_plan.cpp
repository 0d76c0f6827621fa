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
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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


}  // namespace

constexpr int kSplitMin = 6;   // k-lists longer than this are split

// Task graph of the tile factorization for the persistent executor.  Tasks:
// POTRF(k) (also forms L_kk^{-1}), TRSM(i,k) (L_ik = A_ik L_kk^{-T}) and the
// plan's update items.  An item's product waits for the TRSMs of its
// columns; its application to the target waits until the target's earlier
// levels were applied (so every tile sums its updates in level order, as the
// level-synchronous path does).  Tickets follow an as-soon-as-possible time
// estimate, a topological order in which every awaited task -- including any
// chunk of an earlier level of the same target, which may be the one that
// applies it -- has a smaller ticket; so the ticketed persistent kernel
// cannot deadlock.
// Ticket order of the task graph by list scheduling: a simulation of
// kSimWorkersDefault workgroups that, whenever one is free, start the ready task
// with the longest remaining path to the end of the factorization (its
// bottom level).  Tickets follow the simulated start order, so the order is
// topological (a task starts after all of its producers finished) and tasks
// on the elimination tree's critical chain are drawn as soon as their inputs
// can be ready instead of behind a wave of updates that can wait.  Costs are
// calibrated on MI355X task traces (tools/dag_critical.py), in microseconds.
// Simulated with fewer workgroups than the executor's 512: the real tasks run
// slower than their calibrated costs while ~300 updates contend for the
// memory system, so a 512-wide simulation hands out tickets ahead of
// readiness, workgroups block on them, and chain tasks are drawn late.  A
// narrower simulation orders the chain earlier (cfg3 k_factor_dag 735 -> 716
// us at 192-256; 160 is worse, 810 us; tools/env_bench.sh).
constexpr int kSimWorkersDefault = 224;
int sim_workers() {   // (ARSLAM_SIM_WORKERS: debug sweeps)
  static const int w = std::getenv("ARSLAM_SIM_WORKERS") ? std::min(4096, std::max(1, std::atoi(std::getenv("ARSLAM_SIM_WORKERS"))))
                                                         : kSimWorkersDefault;
  return w;
}
// A POTRF node may also carry the TRSM of the column's first off-diagonal
// tile (sub = its compact tile id): 'late' waits are those of that TRSM,
// polled after L_kk is published.
struct DagNode {
  int phase = 0;   // multi-rank plans: 0 this rank's subtree columns, 1 the replicated top
  int type;
  int idx;
  int4 task;
  std::vector<int2> waits;
  int sub = -1;
  std::vector<int2> late;
};

static std::vector<int> dag_list_schedule(const std::vector<DagNode> &nodes, long nt, const LltPlan &plan,
                                          std::vector<double> *finish_out = nullptr,
                                          std::vector<double> *blevel_out = nullptr) {
  const int n = (int)nodes.size();
  std::vector<int> ready_prod(nt, -1);
  std::vector<std::vector<std::pair<int, int>>> by_tile(nt);   // (seq, node) of update items
  for (int v = 0; v < n; ++v) {
    const int4 t = nodes[v].task;
    if (t.x == 0 || t.x == 1) ready_prod[t.w] = v;
    else if (t.x == 2) by_tile[t.w].push_back({t.z, v});
    if (nodes[v].sub >= 0) ready_prod[nodes[v].sub] = v;
  }
  auto seq_nodes = [&](int tile, int seq, std::vector<int> &out) {
    for (const auto &sv : by_tile[tile])
      if (sv.first == seq) out.push_back(sv.second);
  };
  std::vector<std::vector<int>> succ(n);
  std::vector<int> ndep(n, 0);
  std::vector<double> cost(n);
  std::vector<int> pr;
  // task costs (us): POTRF base, per folded column, fused TRSM; TRSM; update
  // base, per column; INV.  The update items are weighted well above their
  // uncontended run time (4 + 4 per column): under the ~300 concurrent updates
  // of the wide levels they run ~2-3x slower and hold the memory system the
  // chain needs, and a schedule that budgets for that draws the chain tasks
  // ahead of them (cfg3 k_factor_dag 720 -> ~688 us with 16 + 16 per column;
  // flat from 12 + 12 to 20 + 12, worse at 24 + 24; round-2 sweeps).
  double cc[7] = {16.0, 4.0, 5.0, 6.0, 16.0, 16.0, 5.0};
  if (const char *e = std::getenv("ARSLAM_SIM_COST"))   // debug: list-schedule cost sweeps (tools/sim_sweep.sh)
    std::sscanf(e, "%lf,%lf,%lf,%lf,%lf,%lf,%lf", &cc[0], &cc[1], &cc[2], &cc[3], &cc[4], &cc[5], &cc[6]);
  for (int v = 0; v < n; ++v) {
    const DagNode &nd = nodes[v];
    pr.clear();
    std::vector<int2> all(nd.waits);
    all.insert(all.end(), nd.late.begin(), nd.late.end());
    for (const int2 &w : all) {
      if (w.x < nt) {
        if (ready_prod[w.x] >= 0) pr.push_back(ready_prod[w.x]);
      } else if (w.y > 0) {
        seq_nodes(w.x - (int)nt, w.y - 1, pr);   // the level before the awaited count (earlier levels chain)
      }
    }
    if (nd.task.x == 2 && nd.task.z > 0) seq_nodes(nd.task.w, nd.task.z - 1, pr);   // in-order application
    std::sort(pr.begin(), pr.end());
    pr.erase(std::unique(pr.begin(), pr.end()), pr.end());
    for (int u : pr) {
      if (u == v) continue;
      succ[u].push_back(v);
      ndep[v]++;
    }
    if (nd.task.x == 0) {
      const int nk = nd.task.z >= 0 ? plan.h_items[nd.task.z].z - plan.h_items[nd.task.z].y : 0;
      cost[v] = cc[0] + cc[1] * nk + (nd.sub >= 0 ? cc[2] : 0.0);
    } else if (nd.task.x == 1) {
      cost[v] = cc[3];
    } else if (nd.task.x == 3) {
      cost[v] = cc[6];
    } else {
      const int4 it = plan.h_items[nd.task.y];
      cost[v] = cc[4] + cc[5] * (it.z - it.y);
    }
  }
  // bottom levels (nodes are created producers-first: a reverse sweep is a valid order)
  std::vector<int> topo;
  topo.reserve(n);
  {
    std::vector<int> d = ndep;
    std::vector<int> st;
    for (int v = 0; v < n; ++v)
      if (!d[v]) st.push_back(v);
    while (!st.empty()) {
      const int u = st.back();
      st.pop_back();
      topo.push_back(u);
      for (int v : succ[u])
        if (--d[v] == 0) st.push_back(v);
    }
    if ((int)topo.size() != n) throw std::runtime_error("dag_list_schedule: task graph has a cycle");
  }
  std::vector<double> blevel(n, 0.0);
  for (int q = n - 1; q >= 0; --q) {
    const int u = topo[q];
    double m = 0.0;
    for (int v : succ[u]) m = std::max(m, blevel[v]);
    blevel[u] = cost[u] + m;
  }
  // simulation
  auto cmp = [&](int a, int b) {   // max-heap on bottom level, then creation order
    if (blevel[a] != blevel[b]) return blevel[a] < blevel[b];
    return a > b;
  };
  std::vector<int> heap;
  std::vector<int> d = ndep;
  for (int v = 0; v < n; ++v)
    if (!d[v]) heap.push_back(v);
  std::make_heap(heap.begin(), heap.end(), cmp);
  typedef std::pair<double, int> Ev;   // (finish time, node)
  std::vector<Ev> events;
  auto ev_cmp = [](const Ev &a, const Ev &b) { return a.first > b.first || (a.first == b.first && a.second > b.second); };
  std::vector<int> order;
  order.reserve(n);
  int busy = 0;
  double now = 0.0;
  std::vector<double> through(blevel_out ? n : 0);
  const int n_workers = sim_workers();
  while ((int)order.size() < n || !events.empty()) {
    while (busy < n_workers && !heap.empty()) {
      std::pop_heap(heap.begin(), heap.end(), cmp);
      const int v = heap.back();
      heap.pop_back();
      order.push_back(v);
      events.push_back({now + cost[v], v});
      if (finish_out) (*finish_out)[v] = now + cost[v];
      if (blevel_out) through[v] = now + blevel[v];   // longest path through v, as scheduled
      std::push_heap(events.begin(), events.end(), ev_cmp);
      ++busy;
    }
    if (events.empty()) break;
    std::pop_heap(events.begin(), events.end(), ev_cmp);
    const Ev e = events.back();
    events.pop_back();
    now = e.first;
    --busy;
    for (int v : succ[e.second])
      if (--d[v] == 0) {
        heap.push_back(v);
        std::push_heap(heap.begin(), heap.end(), cmp);
      }
  }
  if ((int)order.size() != n) throw std::runtime_error("dag_list_schedule: not every task was scheduled");
  if (blevel_out) *blevel_out = through;
  return order;
}

void dag_build(LltPlan &plan) {
  const int T = plan.T;
  const long nt = plan.n_tiles;
  auto tid = [&](int i, int j) { return plan.h_tile_id[(long)i * T + j]; };
  const int nlev = plan.nlev;
  // the phase of a level (multi-rank plans: phase 0 = this rank's subtree
  // columns, phase 1 = the replicated top separators, llt_plan_symbolic)
  const int lev_per_phase = plan.n_phases > 1 ? nlev / plan.n_phases : nlev;
  auto phase_of_level = [&](int l) { return l / lev_per_phase; };
  // applications per target tile and per-(target, level) sequence number,
  // over both phases in order (a top tile's phase-1 items follow its phase-0 ones)
  std::vector<int> n_apply(nt, 0);
  std::vector<int> item_seq(plan.h_items.size(), 0);
  for (int l = 0; l < nlev; ++l) {
    const int t0 = plan.h_upd_off[l], t1 = plan.h_upd_off[l + 1];
    std::vector<int> seq_of_target(t1 - t0, 0);
    for (int t = t0; t < t1; ++t) {
      const int2 tg = plan.h_targets[t];
      seq_of_target[t - t0] = n_apply[tid(tg.x, tg.y)]++;
    }
    for (int it = plan.h_item_off[l]; it < plan.h_item_off[l + 1]; ++it)
      item_seq[it] = seq_of_target[plan.h_items[it].x - t0];
  }
  typedef DagNode Node;
  std::vector<Node> nodes;
  for (int l = 0; l < nlev; ++l) {
    // factor tasks of the level's columns
    for (int p = plan.h_panel_off[l]; p < plan.h_panel_off[l + 1]; ++p) {
      const int2 pk = plan.h_panel[p];
      const int i = pk.x, k = pk.y;
      Node n;
      n.phase = phase_of_level(l);
      if (i == k) {
        n.type = 0;
        n.task = make_int4(0, k, -1, tid(k, k));
        if (n_apply[tid(k, k)]) n.waits.push_back(make_int2((int)nt + tid(k, k), n_apply[tid(k, k)]));
      } else {
        n.type = 1;
        n.task = make_int4(1, i, k, tid(i, k));
        n.waits.push_back(make_int2(tid(k, k), 1));
        if (n_apply[tid(i, k)]) n.waits.push_back(make_int2((int)nt + tid(i, k), n_apply[tid(i, k)]));
      }
      n.idx = p;
      nodes.push_back(std::move(n));
    }
    // update items of the level
    for (int it = plan.h_item_off[l]; it < plan.h_item_off[l + 1]; ++it) {
      const int4 item = plan.h_items[it];
      const int2 tg = plan.h_targets[item.x];
      const int tt = tid(tg.x, tg.y);
      Node n;
      n.phase = phase_of_level(l);
      n.type = 2;
      n.idx = it;
      n.task = make_int4(2, it, item_seq[it], tt);
      for (int q = item.y; q < item.z; ++q) {
        const int k = plan.h_ks[q];
        n.waits.push_back(make_int2(tid(tg.x, k), 1));
        if (tg.y != tg.x) n.waits.push_back(make_int2(tid(tg.y, k), 1));
      }
      nodes.push_back(std::move(n));
    }
  }
  // Fold the last update of each diagonal tile into its POTRF task when that
  // update is one unsplit item of the same phase: the POTRF then computes
  // A_kk - sum L_kj L_kj^T itself, taking a task and a hand-off off the
  // critical chain.  (A multi-rank top tile's phase-0 items are this rank's
  // share of a sum that is all-reduced between the phases: never folded into
  // a phase-1 POTRF.)
  {
    std::vector<int> last_item(nt, -1), last_count(nt, 0);
    for (size_t m = 0; m < nodes.size(); ++m) {
      if (nodes[m].type != 2) continue;
      const int tt = nodes[m].task.w, seq = nodes[m].task.z;
      if (seq + 1 != n_apply[tt]) continue;   // not the final level of this tile
      last_item[tt] = (int)m;
      last_count[tt]++;
    }
    std::vector<char> drop(nodes.size(), 0);
    for (auto &n : nodes) {
      if (n.type != 0) continue;
      const int tt = n.task.w;
      const int m = last_item[tt];
      if (m < 0 || last_count[tt] != 1 || plan.h_items[nodes[m].task.y].w >= 0 || nodes[m].phase != n.phase)
        continue;
      n.task.z = nodes[m].task.y;   // item folded into the POTRF
      std::vector<int2> w;
      for (const int2 &x : n.waits)
        if (x.x != (int)nt + tt) w.push_back(x);
      if (n_apply[tt] > 1) w.push_back(make_int2((int)nt + tt, n_apply[tt] - 1));
      w.insert(w.end(), nodes[m].waits.begin(), nodes[m].waits.end());
      n.waits = std::move(w);
      drop[m] = 1;
    }
    std::vector<Node> kept;
    for (size_t m = 0; m < nodes.size(); ++m)
      if (!drop[m]) kept.push_back(std::move(nodes[m]));
    nodes.swap(kept);
  }
  // Fuse the TRSM of each column's first off-diagonal tile (the elimination
  // tree parent's row) into the column's POTRF task: on a chain of
  // separator columns, POTRF(k) -> TRSM(parent, k) -> POTRF(parent) is the
  // critical path, and the fused task solves the tile against the L_kk it
  // still holds in LDS (no draw, no hand-off, no reload of L_kk).  The
  // TRSM's own waits become the task's late waits.  (Same column: same phase.)
  {
    std::vector<int> trsm_node(nt, -1);
    for (size_t m = 0; m < nodes.size(); ++m)
      if (nodes[m].type == 1) trsm_node[nodes[m].task.w] = (int)m;
    std::vector<char> drop(nodes.size(), 0);
    for (auto &n : nodes) {
      if (n.type != 0) continue;
      const int k = n.task.y;
      int par = -1;
      for (int i = k + 1; i < T && par < 0; ++i)
        if (tid(i, k) >= 0) par = i;
      if (par < 0) continue;
      const int m = trsm_node[tid(par, k)];
      if (m < 0) continue;
      n.sub = tid(par, k);
      for (const int2 &x : nodes[m].waits)
        if (x.x != tid(k, k)) n.late.push_back(x);
      drop[m] = 1;
    }
    std::vector<Node> kept;
    for (size_t m = 0; m < nodes.size(); ++m)
      if (!drop[m]) kept.push_back(std::move(nodes[m]));
    nodes.swap(kept);
  }
  // L_kk^{-1} of every column (for the backward solve) as its own task, off
  // the chain: the POTRF task can go straight on to its parent
  for (int k = 0; k < T; ++k) {
    if (tid(k, k) < 0) continue;
    Node n;
    n.type = 3;
    n.idx = k;
    n.phase = plan.h_col_class.empty() ? 0 : (plan.h_col_class[k] == 1 ? 1 : 0);
    n.task = make_int4(3, k, 0, tid(k, k));
    n.waits.push_back(make_int2(tid(k, k), 1));
    nodes.push_back(std::move(n));
  }
  // tickets: each phase list-scheduled on its own (phase 1 runs in a later
  // launch, after the multi-rank exchange), phase 0 first
  std::vector<int> order;
  for (int ph = 0; ph < std::max(plan.n_phases, 1); ++ph) {
    std::vector<int> idx;
    for (int v = 0; v < (int)nodes.size(); ++v)
      if (nodes[v].phase == ph) idx.push_back(v);
    std::vector<Node> sub;
    sub.reserve(idx.size());
    for (int v : idx) sub.push_back(nodes[v]);
    for (int o : dag_list_schedule(sub, nt, plan)) order.push_back(idx[o]);
    if (ph == 0) plan.phase_split = (long)order.size();
  }
  plan.h_dag_tasks.clear();
  plan.h_dag_waits.clear();
  plan.h_dag_sub.clear();
  plan.h_dag_phase.clear();
  plan.h_dag_wait_off.assign(1, 0);
  for (int o : order) {
    plan.h_dag_tasks.push_back(nodes[o].task);
    plan.h_dag_phase.push_back(nodes[o].phase);
    plan.h_dag_waits.insert(plan.h_dag_waits.end(), nodes[o].waits.begin(), nodes[o].waits.end());
    plan.h_dag_sub.push_back(make_int2(nodes[o].sub, (int)plan.h_dag_waits.size()));
    plan.h_dag_waits.insert(plan.h_dag_waits.end(), nodes[o].late.begin(), nodes[o].late.end());
    plan.h_dag_wait_off.push_back((int)plan.h_dag_waits.size());
  }
  plan.n_dag_tasks = (long)plan.h_dag_tasks.size();
  // Continuations: a finished task may claim one designated successor and run
  // it at once on the same workgroup instead of leaving it to be drawn.  The
  // 512 workgroups hold drawn tasks that wait (the factorization keeps ~30 %
  // of them busy), so in the contended first half of the factorization a
  // ready chain task used to be drawn 10-25 us after its last producer ended.
  // POTRF(k) with fused TRSM (par, k) -> POTRF(par) (the solved tile stays
  // in LDS; the fold reuses it for column k's term).
  // maxdep[c] = the largest ticket among c's early producers other than its
  // claimers (>= 0 marks a target): a claim needs those drawn.  Late waits (a
  // POTRF's fused TRSM) are not counted, so a claimed target may wait on
  // undrawn tickets; the kernel bounds claimed targets in flight to half the
  // grid, so workgroups stay free to draw (k_factor_dag, dag_simulate).
  {
    const long n = plan.n_dag_tasks;
    plan.h_dag_cont.assign(n, -1);
    plan.h_dag_maxdep.assign(n, -1);
    std::vector<int> potrf_of(T, -1), ready_tk(nt, -1);
    std::vector<std::vector<std::pair<int, int>>> apply_tk(nt);   // (seq, ticket) of update items
    for (long t = 0; t < n; ++t) {
      const int4 tk = plan.h_dag_tasks[t];
      if (tk.x == 0) potrf_of[tk.y] = (int)t;
      if (tk.x == 0 || tk.x == 1) ready_tk[tk.w] = (int)t;
      if (plan.h_dag_sub[t].x >= 0) ready_tk[plan.h_dag_sub[t].x] = (int)t;
      if (tk.x == 2) apply_tk[tk.w].push_back({tk.z, (int)t});
    }
    // early producers of every task (the in-order application's predecessor
    // level included for update items)
    std::vector<std::vector<int>> prod(n);
    for (long t = 0; t < n; ++t) {
      const int4 tk = plan.h_dag_tasks[t];
      const int early_end = plan.h_dag_sub[t].x >= 0 ? plan.h_dag_sub[t].y : plan.h_dag_wait_off[t + 1];
      std::vector<int> &pr = prod[t];
      for (int q = plan.h_dag_wait_off[t]; q < early_end; ++q) {
        const int2 w = plan.h_dag_waits[q];
        if (w.x < nt) {
          if (ready_tk[w.x] >= 0) pr.push_back(ready_tk[w.x]);
        } else {
          for (const auto &sv : apply_tk[w.x - nt])
            if (sv.first < w.y) pr.push_back(sv.second);
        }
      }
      if (tk.x == 2 && tk.z > 0)
        for (const auto &sv : apply_tk[tk.w])
          if (sv.first == tk.z - 1) pr.push_back(sv.second);
      std::sort(pr.begin(), pr.end());
      pr.erase(std::unique(pr.begin(), pr.end()), pr.end());
    }
    for (long t = 0; t < n; ++t) {
      const int4 tk = plan.h_dag_tasks[t];
      const int sb = plan.h_dag_sub[t].x;
      if (tk.x != 0 || sb < 0) continue;
      int par = -1;
      for (int i = tk.y + 1; i < T && par < 0; ++i)
        if (tid(i, tk.y) == sb) par = i;
      if (par < 0 || potrf_of[par] < 0 || potrf_of[par] <= t) continue;
      if (plan.h_dag_phase[potrf_of[par]] != plan.h_dag_phase[t]) continue;   // never across the exchange
      plan.h_dag_cont[t] = potrf_of[par];
    }
    plan.h_dag_cont_akk.assign(n, -1);
    for (long t = 0; t < n; ++t) {
      const int c = plan.h_dag_cont[t];
      if (c < 0 || plan.h_dag_tasks[c].z < 0) continue;
      const int4 it = plan.h_items[plan.h_dag_tasks[c].z];
      if (it.z - it.y == 1 && plan.h_ks[it.y] == plan.h_dag_tasks[t].y)
        plan.h_dag_cont_akk[t] = tid(plan.h_dag_tasks[c].y, plan.h_dag_tasks[c].y);
    }
    // (generic successor claims -- every task claiming the successor it is the
    // last producer of -- and ready claims of near-critical successors were
    // measured slower in round 2 and removed: the claimed successors were
    // often not the ones the chain waited for, and the extra polling cost more
    // workgroup time than the late draws it saved)
    std::vector<std::vector<int>> claimers(n);
    for (long t = 0; t < n; ++t)
      if (plan.h_dag_cont[t] >= 0) claimers[plan.h_dag_cont[t]].push_back((int)t);
    for (long c = 0; c < n; ++c) {
      if (claimers[c].empty()) continue;
      int md = 0;
      for (int u : prod[c])
        if (std::find(claimers[c].begin(), claimers[c].end(), u) == claimers[c].end()) md = std::max(md, u);
      plan.h_dag_maxdep[c] = md;
    }
    plan.h_dag_rec.assign((size_t)n * kDagRecInts, -1);
    for (long t = 0; t < n; ++t) {
      int *r = plan.h_dag_rec.data() + t * kDagRecInts;
      const int4 tk = plan.h_dag_tasks[t];
      r[kRecType] = tk.x, r[kRecY] = tk.y, r[kRecZ] = tk.z, r[kRecW] = tk.w;
      r[kRecSub] = plan.h_dag_sub[t].x, r[kRecLate] = plan.h_dag_sub[t].y;
      r[kRecWait0] = plan.h_dag_wait_off[t], r[kRecWait1] = plan.h_dag_wait_off[t + 1];
      const int c = plan.h_dag_cont[t];
      r[kRecCont] = c, r[kRecContAkk] = plan.h_dag_cont_akk[t], r[kRecMaxdep] = plan.h_dag_maxdep[t];
      if (c >= 0)
        r[kRecContMaxdep] = plan.h_dag_maxdep[c], r[kRecContWait0] = plan.h_dag_wait_off[c],
        r[kRecContLate] = plan.h_dag_sub[c].y;
      if (tk.x == 0 && tk.z >= 0) {
        const int4 it = plan.h_items[tk.z];
        r[kRecQ0] = it.y, r[kRecQ1] = it.z, r[kRecFoldK0] = plan.h_ks[it.y], r[kRecFoldTile0] = tid(tk.y, plan.h_ks[it.y]);
      } else if (tk.x == 2) {
        const int4 it = plan.h_items[tk.y];
        const int2 tg = plan.h_targets[it.x];
        r[kRecQ0] = it.y, r[kRecQ1] = it.z, r[kRecSid] = it.w, r[kRecTi] = tg.x, r[kRecTj] = tg.y;
        if (it.w >= 0) r[kRecSplitN] = plan.h_split[it.w >> 8].x, r[kRecSplitP] = plan.h_split[it.w >> 8].y;
        r[kRecTile0I] = tid(tg.x, plan.h_ks[it.y]), r[kRecTile0J] = tid(tg.y, plan.h_ks[it.y]);
      }
    }
    plan.h_dag_ks_tiles.assign(std::max<size_t>(plan.h_ks.size(), 1), make_int2(-1, -1));
    for (const int4 &it : plan.h_items) {
      const int2 tg = plan.h_targets[it.x];
      for (int q = it.y; q < it.z; ++q)
        plan.h_dag_ks_tiles[q] = make_int2(tid(tg.x, plan.h_ks[q]), tid(tg.y, plan.h_ks[q]));
    }
  }
  // Fill tiles are not cleared on one rank: the first update of each stores
  // 0 - acc instead of reading the tile (k_factor_dag, first_store).  That is
  // only sound if every fill tile's first application (sequence 0) is an
  // unfolded update item of the DAG: a tile with no update, or whose only
  // update was folded into its POTRF, would be read uncleared.  Checked here,
  // not assumed; the solver clears every tile when it fails.
  {
    plan.fill_first_ok = plan.n_phases == 1;
    std::vector<char> first(nt, 0);
    for (const int4 &tk : plan.h_dag_tasks)
      if (tk.x == 2 && tk.z == 0) first[tk.w] = 1;
    for (long t = plan.n_assembled; t < nt && plan.fill_first_ok; ++t) plan.fill_first_ok = first[t] != 0;
  }
  long n_potrf = 0, n_trsm = 0;
  for (size_t t = 0; t < plan.h_dag_tasks.size(); ++t) {
    n_potrf += plan.h_dag_tasks[t].x == 0;
    n_trsm += plan.h_dag_tasks[t].x == 1 || plan.h_dag_sub[t].x >= 0;
  }
  const double t3 = 64.0 * 64.0 * 64.0;
  plan.total_factor_flops = plan.total_upd_flops + n_potrf * (t3 / 3.0 + t3 / 3.0) + n_trsm * 2.0 * t3;
}

// Symbolic Cholesky fill of a lower tile pattern (in place, diagonal set) and
// the tile elimination tree (parent[k]: the first row below the diagonal).
void tile_fill(int T, std::vector<uint8_t> &P, std::vector<int> &parent) {
  std::vector<int> rows;
  for (int k = 0; k < T; ++k) {
    P[(long)k * T + k] = 1;
    rows.clear();
    for (int i = k + 1; i < T; ++i)
      if (P[(long)i * T + k]) rows.push_back(i);
    for (size_t a = 0; a < rows.size(); ++a)
      for (size_t b = 0; b <= a; ++b) P[(long)rows[a] * T + rows[b]] = 1;
  }
  parent.assign(T, -1);
  for (int k = 0; k < T; ++k)
    for (int i = k + 1; i < T; ++i)
      if (P[(long)i * T + k]) { parent[k] = i; break; }
}

void llt_plan_symbolic(LltPlan &plan, int T, long lda, std::vector<uint8_t> &P, const std::vector<int> *col_class) {
  llt_plan_reset(plan);
  plan.T = T;
  plan.lda = lda;
  const bool multi = col_class != nullptr;
  std::vector<int> cls = multi ? *col_class : std::vector<int>(T, 0);
  plan.h_col_class.assign(cls.begin(), cls.end());
  plan.n_phases = multi ? 2 : 1;
  const std::vector<uint8_t> assembled = P;
  std::vector<int> parent;
  tile_fill(T, P, parent);
  // compact tile numbering.  One rank: the assembled tiles (the input pattern
  // + diagonal) first, then the fill.  Several ranks: the top columns' tiles
  // first (the prefix all-reduced between the two phases), then this rank's
  // own subtree columns'; another rank's tiles are not stored here.
  plan.h_tile_id.assign((size_t)T * T, -1);
  long nid = 0;
  if (multi) {
    for (int want : {1, 0})
      for (int i = 0; i < T; ++i)
        for (int j = 0; j <= i; ++j)
          if (P[(long)i * T + j] && cls[j] == want) plan.h_tile_id[(long)i * T + j] = (int)nid++;
    plan.n_top_tiles = 0;
    for (int i = 0; i < T; ++i)
      for (int j = 0; j <= i; ++j)
        if (P[(long)i * T + j] && cls[j] == 1) plan.n_top_tiles++;
    plan.n_assembled = plan.n_top_tiles;
  } else {
    for (int i = 0; i < T; ++i)
      for (int j = 0; j <= i; ++j)
        if (assembled[(long)i * T + j] || i == j) plan.h_tile_id[(long)i * T + j] = (int)nid++;
    plan.n_assembled = nid;
    for (int i = 0; i < T; ++i)   // fill tiles numbered after the assembled ones
      for (int j = 0; j <= i; ++j)
        if (P[(long)i * T + j] && plan.h_tile_id[(long)i * T + j] < 0) plan.h_tile_id[(long)i * T + j] = (int)nid++;
  }
  plan.n_tiles = nid;
  // tile elimination tree heights
  std::vector<int> height(T, 0);
  for (int k = 0; k < T; ++k)
    if (parent[k] >= 0) height[parent[k]] = std::max(height[parent[k]], height[k] + 1);
  int nlev = 0;
  for (int k = 0; k < T; ++k) nlev = std::max(nlev, height[k] + 1);
  std::vector<std::vector<int>> levcols(nlev);
  for (int k = 0; k < T; ++k) levcols[height[k]].push_back(k);
  // levels of each phase (phase 0: class-0 columns, phase 1: class-1), one
  // set of level lists per phase
  plan.nlev = nlev * plan.n_phases;

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
  std::vector<int> rows;
  for (int lp = 0; lp < plan.nlev; ++lp) {
    const int l = lp % nlev, phase = lp / nlev;
    std::vector<int> cols;
    for (int k : levcols[l])
      if (cls[k] == phase) cols.push_back(k);
    // panel tasks
    for (int k : cols) {
      panel.push_back(make_int2(k, k));
      for (int i = k + 1; i < T; ++i)
        if (P[(long)i * T + k]) panel.push_back(make_int2(i, k));
    }
    plan.h_panel_off.push_back((int)panel.size());
    // update targets of this level: (i,j), j <= i, both in some column k of the level
    std::vector<int2> lt;
    std::vector<std::vector<int>> lks;
    double fl = 0.0;
    for (int k : cols) {
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
    plan.total_upd_flops += fl;
  }
  // backward solve: levels from the root down; each column gathers from its
  // tile rows below the diagonal (ancestors, solved in earlier launches).
  // Several ranks: the top columns and this rank's own (their ancestors are
  // own or top columns).
  for (int l = nlev - 1; l >= 0; --l) {
    for (int k : levcols[l]) {
      if (cls[k] == 2) continue;
      bcols.push_back(k);
      for (int i = k + 1; i < T; ++i)
        if (P[(long)i * T + k]) gather.push_back(make_int2(i, k));
      gbeg.push_back((int)gather.size());   // column's gathers: [gbeg[b], gbeg[b+1])
    }
    plan.h_bs_off.push_back((int)bcols.size());
    plan.h_bsg_off.push_back((int)gather.size());
  }
  dag_build(plan);
}

RankSplit rank_split(const HostProblem &h, const ReducedLayout &L, int nranks) {
  RankSplit out;
  const int T = L.T, nc = h.nc;
  out.cap_owner.assign(nc, 0);
  out.col_owner.assign(T, -1);
  std::vector<long> rank_obs(nranks, 0);
  auto least_loaded = [&]() {
    int r = 0;
    for (int q = 1; q < nranks; ++q)
      if (rank_obs[q] < rank_obs[r]) r = q;
    return r;
  };
  if (L.nR == 0 || T == 0 || nranks <= 1) {
    for (int c = 0; c < nc; ++c) {
      const int r = nranks <= 1 ? 0 : least_loaded();
      out.cap_owner[c] = r;
      rank_obs[r] += h.cap_start[c + 1] - h.cap_start[c];
    }
    if (nranks <= 1) out.col_owner.assign(T, 0);
    return out;
  }
  std::vector<uint8_t> P = L.pattern;
  std::vector<int> parent;
  tile_fill(T, P, parent);
  std::vector<std::vector<int>> ch(T);
  for (int k = 0; k < T; ++k)
    if (parent[k] >= 0) ch[parent[k]].push_back(k);
  // work of a column: its tile tasks (POTRF, TRSMs, update pairs); of a subtree: the sum
  std::vector<double> w(T), W(T);
  for (int k = 0; k < T; ++k) {
    double c = 0;
    for (int i = k + 1; i < T; ++i) c += P[(long)i * T + k];
    w[k] = W[k] = (c + 1.0) * (c + 2.0) / 2.0;
  }
  for (int k = 0; k < T; ++k)
    if (parent[k] >= 0) W[parent[k]] += W[k];
  for (int k = 0; k < T; ++k) out.total_work += w[k];
  // the observations of the captures each column would own (the lowest
  // column of their tags), summed over subtrees, and the tiles of each column
  std::vector<double> cob(T, 0.0), tiles(T, 0.0);
  double top_only_obs = 0.0;
  for (int c = 0; c < nc; ++c) {
    int low = T;
    for (int a = h.cap_blk_start[c]; a < h.cap_blk_start[c + 1]; ++a) {
      const int r0 = L.tag_row[h.blk_tag[a]];
      if (r0 >= 0) low = std::min(low, r0 / kTileRows);
    }
    const double ob = h.cap_start[c + 1] - h.cap_start[c];
    if (low < T) cob[low] += ob; else top_only_obs += ob;
  }
  std::vector<double> COB = cob;
  for (int k = 0; k < T; ++k)
    if (parent[k] >= 0) COB[parent[k]] += COB[k];
  for (int k = 0; k < T; ++k)
    for (int i = k; i < T; ++i) tiles[k] += P[(long)i * T + k] || i == k;
  // Grow the replicated top from the root (the heaviest subtree root of the
  // frontier into the top, descending a separator chain one column at a
  // time) and deal the frontier's subtrees to A <= nranks active ranks; keep
  // the (top, A) of the least modelled step time.  The factorization is
  // bound by its critical chain (every leaf-to-root path crosses the top),
  // about the same for every split, so the model is
  // what the split changes: the per-capture work of the busiest rank (its
  // observations, ~3 ns each on cfg3: linearize, Schur, back-substitution)
  // and the exchange of the top tiles (2 (N-1)/N x 32 KB per tile at
  // ~100 GB/s).  A deeper split adds top tiles faster than it removes
  // per-capture work, so ranks may stay idle in phase 0 (they then own only
  // captures that see top tags alone).  Tile-task work breaks ties.
  const double kObsUs = 0.003, kTileUs = 32768.0 / 100e3 * 2.0 * (nranks - 1) / nranks;
  int active_forced = 0;
  if (const char *e = std::getenv("ARSLAM_SPLIT_ACTIVE"))   // debug: fix A (clamped to [0, nranks]; 0 = the model's)
    active_forced = std::min(nranks, std::max(0, std::atoi(e)));
  std::vector<char> top(T, 0);
  std::vector<int> frontier;
  for (int k = 0; k < T; ++k)
    if (parent[k] < 0) frontier.push_back(k);
  double best = -1.0, topw = 0.0, top_tiles = 0.0;
  std::vector<char> best_top;
  std::vector<int> best_front, best_asg;
  for (int iter = 0; iter <= T; ++iter) {
    std::vector<int> ord = frontier;
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return COB[a] != COB[b] ? COB[a] > COB[b] : a > b; });
    for (int A = 1; A <= std::min<int>(nranks, (int)ord.size()); ++A) {
      if (active_forced > 0 && A != std::min<int>(active_forced, (int)ord.size())) continue;
      // subtrees largest-first onto the least loaded of the A active ranks
      // (observations), then the top-only captures onto the least loaded rank
      std::vector<double> bins(nranks, 0.0), wbin(nranks, 0.0);
      std::vector<int> asg(ord.size());
      for (size_t q = 0; q < ord.size(); ++q) {
        int r = 0;
        for (int x = 1; x < A; ++x)
          if (bins[x] < bins[r]) r = x;
        asg[q] = r;
        bins[r] += COB[ord[q]];
        wbin[r] += W[ord[q]];
      }
      std::vector<double> ob = bins;
      *std::min_element(ob.begin(), ob.end()) += top_only_obs;
      const double mo = *std::max_element(ob.begin(), ob.end());
      const double mw = *std::max_element(wbin.begin(), wbin.end());
      const double est = kObsUs * mo + kTileUs * top_tiles + 1e-9 * (topw + mw);
      if (best < 0 || est < best * (1.0 - 1e-12)) {
        best = est;
        best_top = top;
        best_front = ord;
        best_asg = asg;
        out.top_work = topw;
        out.max_rank_work = mw;
        out.n_active = A;
      }
    }
    int v = -1;
    for (int f : frontier)
      if (v < 0 || W[f] > W[v] || (W[f] == W[v] && f > v)) v = f;
    if (v < 0 || ch[v].empty()) break;
    top[v] = 1;
    topw += w[v];
    top_tiles += tiles[v];
    frontier.erase(std::find(frontier.begin(), frontier.end(), v));
    frontier.insert(frontier.end(), ch[v].begin(), ch[v].end());
  }
  std::vector<int> root_rank(T, -1);
  for (size_t q = 0; q < best_front.size(); ++q) root_rank[best_front[q]] = best_asg[q];
  for (int k = T - 1; k >= 0; --k) {
    if (best_top[k]) out.col_owner[k] = -1, out.n_top_cols++;
    else if (root_rank[k] >= 0) out.col_owner[k] = root_rank[k];
    else out.col_owner[k] = parent[k] >= 0 ? out.col_owner[parent[k]] : 0;
  }
  // captures: the owner of the lowest tile column among their tags' rows
  std::vector<int> top_only;
  for (int c = 0; c < nc; ++c) {
    int low = T;
    for (int a = h.cap_blk_start[c]; a < h.cap_blk_start[c + 1]; ++a) {
      const int r0 = L.tag_row[h.blk_tag[a]];
      if (r0 >= 0) low = std::min(low, r0 / kTileRows);
    }
    if (low < T && out.col_owner[low] >= 0) {
      out.cap_owner[c] = out.col_owner[low];
      rank_obs[out.col_owner[low]] += h.cap_start[c + 1] - h.cap_start[c];
    } else {
      top_only.push_back(c);
    }
  }
  for (int c : top_only) {
    const int r = least_loaded();
    out.cap_owner[c] = r;
    rank_obs[r] += h.cap_start[c + 1] - h.cap_start[c];
  }
  return out;
}

bool dag_check(const LltPlan &plan) {
  const long nt = plan.n_tiles;
  std::vector<int> cnt(2 * nt + 1, 0), arrived(plan.h_split.size(), 0);
  for (long t = 0; t < plan.n_dag_tasks; ++t) {
    for (int w = plan.h_dag_wait_off[t]; w < plan.h_dag_wait_off[t + 1]; ++w)
      if (cnt[plan.h_dag_waits[w].x] < plan.h_dag_waits[w].y) return false;
    const int4 task = plan.h_dag_tasks[t];
    if (task.x == 3) continue;
    if (task.x == 0 || task.x == 1) {
      cnt[task.w] = 1;
      if (plan.h_dag_sub[t].x >= 0) cnt[plan.h_dag_sub[t].x] = 1;
      continue;
    }
    const int sid = plan.h_items[task.y].w;
    if (sid >= 0 && ++arrived[sid >> 8] < plan.h_split[sid >> 8].x) continue;   // not the last chunk
    if (cnt[nt + task.w] != task.z) return false;   // level order of the applications
    cnt[nt + task.w]++;
  }
  return true;
}

// Interleavings of n_workers concurrent workgroups running the persistent
// executor's protocol (k_factor_dag) step by step.  Returns false on a
// deadlock: a reachable state in which no workgroup can move.
//   draw      the next ticket, or the continuation target the workgroup claimed;
//   early     the task's early waits met (a POTRF's own; every wait of the
//             other types).  A drawn continuation target then runs only if no
//             predecessor claimed it; a POTRF publishes L_kk (ready[kk]);
//   late      a POTRF with a fused TRSM: the TRSM's waits, then the solved
//             tile (ready[sub]) is published;
//   apply     an update item: split arrival, then the level-ordered application.
// A finished POTRF claims its continuation target when every early producer
// of the target other than its claimers has been drawn (maxdep) and fewer than
// n_workers / 2 claimed targets are in flight, and runs it next.
// Policies (which movable workgroup moves next):
//   0  random (seed);
//   1  draws first, then the workgroup holding the youngest ticket (every free
//      workgroup takes a task as early as it can, the oldest task waits
//      longest: the most workgroups held by blocked tasks);
//   2  draws first, then the oldest ticket;
//   3  draws first, then random.
// policy | kDagSimNoCap (tests only) drops the in-flight cap on claimed
// targets, which the protocol needs: the simulation must then find deadlocks.
// n_started >= 0: only that many workgroups ever start (the rest of the grid is
// never resident), each starting when the schedule picks it; the cap is half
// the workgroups started so far (k_factor_dag), or half the grid under
// policy | kDagSimGridCap (round 5's protocol, which these schedules break).
bool dag_simulate(const LltPlan &plan, int n_workers, unsigned seed, int policy, int n_started) {
  const bool no_cap = (policy & kDagSimNoCap) != 0, grid_cap = (policy & kDagSimGridCap) != 0;
  policy &= kDagSimNoCap - 1;
  const long nt = plan.n_tiles, n = plan.n_dag_tasks;
  std::vector<int> cnt(2 * nt + 1, 0), arrived(plan.h_split.size(), 0);
  const bool has_cont = !plan.h_dag_cont.empty();
  auto maxdep = [&](long t) { return has_cont ? plan.h_dag_maxdep[t] : -1; };
  std::vector<char> claimed(n, 0);
  enum { DRAW = 0, EARLY = 1, APPLY = 2, LATE = 3 };
  struct W { long t = -1; int phase = DRAW; long next = -1; bool cont = false; bool up = true; };
  const int n_res = n_started < 0 ? n_workers : std::min(n_started, n_workers);
  std::vector<W> ws(n_res);
  int started = n_res;
  if (n_started >= 0) {
    started = 0;
    for (W &w : ws) w.up = false;
  }
  long ticket = 0, finished = 0;
  int inflight = 0;   // claimed continuations running: at most started / 2 (as k_factor_dag)
  unsigned rng = seed ? seed : 1u;
  auto rnd = [&]() { rng = rng * 1664525u + 1013904223u; return rng >> 8; };
  auto met = [&](int q0, int q1) {
    for (int q = q0; q < q1; ++q)
      if (cnt[plan.h_dag_waits[q].x] < plan.h_dag_waits[q].y) return false;
    return true;
  };
  auto early_end = [&](long t) { return plan.h_dag_sub[t].x >= 0 ? plan.h_dag_sub[t].y : plan.h_dag_wait_off[t + 1]; };
  auto movable = [&](const W &w) {
    if (!w.up) return true;   // (start)
    switch (w.phase) {
      case DRAW: return w.next >= 0 || ticket < n;
      case EARLY: return met(plan.h_dag_wait_off[w.t], early_end(w.t));
      case LATE: return met(plan.h_dag_sub[w.t].y, plan.h_dag_wait_off[w.t + 1]);
      default: return cnt[nt + plan.h_dag_tasks[w.t].w] >= plan.h_dag_tasks[w.t].z;
    }
  };
  auto done = [&](W &w) {
    ++finished;
    const int c = has_cont ? plan.h_dag_cont[w.t] : -1;
    w.next = -1;
    const int cap = grid_cap ? n_workers / 2 : started / 2;
    if (c >= 0 && ticket > maxdep(c) && !claimed[c] && (no_cap || inflight < cap)) {
      claimed[c] = 1;
      w.next = c;
      ++inflight;
    }
    if (w.cont) --inflight;
    w.phase = DRAW;
  };
  auto move = [&](W &w) {
    if (!w.up) {
      w.up = true;
      ++started;
      return;
    }
    if (w.phase == DRAW) {
      if (w.next >= 0) {
        w.t = w.next;
        w.next = -1;
        w.cont = true;
      } else {
        w.t = ticket++;
        w.cont = false;
      }
      w.phase = EARLY;
      return;
    }
    const int4 task = plan.h_dag_tasks[w.t];
    if (w.phase == EARLY) {
      if (!w.cont && maxdep(w.t) >= 0) {
        if (claimed[w.t]) {   // a predecessor runs it
          w.phase = DRAW;
          return;
        }
        claimed[w.t] = 1;
      }
      if (task.x == 3) return done(w);
      if (task.x != 2) {
        cnt[task.w] = 1;   // L_kk (POTRF) or the solved tile (TRSM)
        if (task.x == 0 && plan.h_dag_sub[w.t].x >= 0) {
          w.phase = LATE;
          return;
        }
        return done(w);
      }
      const int sid = plan.h_items[task.y].w;
      if (sid >= 0 && ++arrived[sid >> 8] < plan.h_split[sid >> 8].x) return done(w);
      w.phase = APPLY;
      return;
    }
    if (w.phase == LATE) {
      cnt[plan.h_dag_sub[w.t].x] = 1;
      return done(w);
    }
    cnt[nt + task.w]++;
    done(w);
  };
  std::vector<int> cand;
  while (finished < n) {
    cand.clear();
    bool draw = false;
    for (int m = 0; m < n_res; ++m)
      if (movable(ws[m])) {
        if (policy != 0 && ws[m].phase == DRAW && !draw) {   // draws first: keep only draws
          draw = true;
          cand.clear();
        }
        if (!draw || ws[m].phase == DRAW) cand.push_back(m);
      }
    if (cand.empty()) return false;
    int pick = cand[0];
    if (policy == 0 || policy == 3 || draw) {
      pick = cand[rnd() % (unsigned)cand.size()];
    } else {
      for (int m : cand) {
        const bool younger = ws[m].t > ws[pick].t;
        if (policy == 1 ? younger : ws[m].t < ws[pick].t) pick = m;
      }
    }
    move(ws[pick]);
  }
  return true;
}

std::string dag_fault_detail(const LltPlan &plan, const int *rec) {
  const long nt = plan.n_tiles, n = plan.n_dag_tasks;
  const int t = rec[kFaultTicket], ctr = rec[kFaultCounter];
  auto task_name = [&](long u) {
    if (u < 0 || u >= n) return std::string("?");
    const int4 k = plan.h_dag_tasks[u];
    char b[96];
    if (k.x == 0) std::snprintf(b, sizeof(b), "POTRF %d%s", k.y, plan.h_dag_sub[u].x >= 0 ? "+TRSM" : "");
    else if (k.x == 1) std::snprintf(b, sizeof(b), "TRSM (%d,%d)", k.y, k.z);
    else if (k.x == 2) std::snprintf(b, sizeof(b), "update item %d (level %d of tile %d)", k.y, k.z, k.w);
    else std::snprintf(b, sizeof(b), "INV %d", k.y);
    return std::string(b);
  };
  std::string s = "ticket " + std::to_string(t) + " (" + task_name(t) + ")";
  if (ctr < 0 || ctr >= 2 * nt) return s;
  // the tickets that advance the awaited counter
  std::vector<long> prod;
  for (long u = 0; u < n; ++u) {
    const int4 k = plan.h_dag_tasks[u];
    if (ctr < nt ? ((k.x == 0 || k.x == 1) && k.w == ctr) || plan.h_dag_sub[u].x == ctr
                 : k.x == 2 && k.w == ctr - nt && k.z < rec[kFaultNeed])
      prod.push_back(u);
  }
  s += ": " + std::string(ctr < nt ? "ready[" : "applied[") + std::to_string(ctr < nt ? ctr : ctr - nt) + "] = " +
       std::to_string(rec[kFaultSeen]) + " < " + std::to_string(rec[kFaultNeed]) + ", advanced by";
  for (size_t q = 0; q < prod.size() && q < 6; ++q) {
    s += (q ? ", " : " ") + std::string("ticket ") + std::to_string(prod[q]) + " (" + task_name(prod[q]) + ")";
    if (!plan.h_dag_maxdep.empty() && plan.h_dag_maxdep[prod[q]] >= 0) s += " [continuation target]";
  }
  if (prod.size() > 6) s += ", ...";
  s += "; tickets drawn " + std::to_string(rec[kFaultDrawn]) + ", claimed continuations in flight " +
       std::to_string(rec[kFaultInflight]) + ", workgroup " + std::to_string(rec[kFaultBlock]);
  if (rec[kFaultFirstStuck] > 0) {   // where the stuck chain starts (the earliest waits give up first)
    const long first = (long)INT_MAX - rec[kFaultFirstStuck];
    s += "; smallest ticket timed out: " + std::to_string(first) + " (" + task_name(first) + ")";
  }
  return s;
}

void llt_plan_upload(LltPlan &plan, hipStream_t s) {
  const int T = plan.T;
  plan.n_split = (long)plan.h_split.size();
  // lay the arrays out in one arena (256-byte aligned), stage the host ones in
  // one buffer, and copy them with one transfer
  struct Piece { void **dst; const void *src; size_t bytes; };
  std::vector<Piece> pieces;
  auto add = [&](void **dst, const void *src, size_t bytes) { pieces.push_back({dst, src, bytes}); };
  auto addv = [&](auto **dst, const auto &v) { add(reinterpret_cast<void **>(dst), v.data(), v.size() * sizeof(v[0])); };
  addv(&plan.panel, plan.h_panel);
  addv(&plan.upd_targets, plan.h_targets);
  addv(&plan.upd_kstart, plan.h_kstart);
  addv(&plan.upd_ks, plan.h_ks);
  addv(&plan.upd_items, plan.h_items);
  addv(&plan.upd_split, plan.h_split);
  add(reinterpret_cast<void **>(&plan.upd_cnt), nullptr, std::max<size_t>(plan.h_split.size(), 1) * sizeof(int));
  add(reinterpret_cast<void **>(&plan.upd_part), nullptr, std::max<long>(plan.n_part, 1) * 4096 * sizeof(double));
  addv(&plan.bs_cols, plan.h_bcols);
  addv(&plan.bs_gather, plan.h_gather);
  addv(&plan.bs_gbeg, plan.h_gbeg);
  add(reinterpret_cast<void **>(&plan.bs_part), nullptr, std::max<size_t>(plan.h_gather.size(), 1) * 64 * sizeof(double));
  add(reinterpret_cast<void **>(&plan.bs_counters), nullptr, ((size_t)T + 1) * sizeof(int));
  addv(&plan.tile_id, plan.h_tile_id);
  std::vector<signed char> cls(plan.h_col_class.begin(), plan.h_col_class.end());
  if (cls.empty()) cls.assign(T, 0);
  addv(&plan.tile_class, cls);
  // L_kk, L_kk^{-1}, and the 16x16 block inverses (4 x 16 x 18) of each column
  add(reinterpret_cast<void **>(&plan.ldiag), nullptr, ((size_t)2 * T * 64 * 64 + (size_t)T * 1152) * sizeof(double));
  addv(&plan.dag_waits, plan.h_dag_waits);
  addv(&plan.dag_rec, plan.h_dag_rec);
  addv(&plan.dag_ks_tiles, plan.h_dag_ks_tiles);
  add(reinterpret_cast<void **>(&plan.dag_claimed), nullptr, std::max<long>(plan.n_dag_tasks, 1) * sizeof(int));
  add(reinterpret_cast<void **>(&plan.dag_counters), nullptr, (2 * (size_t)plan.n_tiles + kDagCounterExtra) * sizeof(int));
  size_t total = 0, staged = 0;
  std::vector<size_t> off(pieces.size());
  for (size_t i = 0; i < pieces.size(); ++i) {   // host arrays first: one contiguous copy
    if (!pieces[i].src || !pieces[i].bytes) continue;
    off[i] = total;
    total += (pieces[i].bytes + 255) & ~size_t(255);
  }
  staged = total;
  for (size_t i = 0; i < pieces.size(); ++i) {
    if (pieces[i].src && pieces[i].bytes) continue;
    off[i] = total;
    total += (pieces[i].bytes + 255) & ~size_t(255);
  }
  if (total > plan.arena_bytes) {
    if (plan.arena) (void)hipFree(plan.arena);
    plan.arena = nullptr;
    plan.arena_bytes = 0;
    const size_t want = total + total / 2;   // (grows by half again: a growing problem reallocates rarely)
    check(hipMalloc(&plan.arena, want), "hipMalloc(plan arena)");
    plan.arena_bytes = want;
  }
  std::vector<char> host(staged);
  for (size_t i = 0; i < pieces.size(); ++i) {
    *pieces[i].dst = pieces[i].bytes ? plan.arena + off[i] : nullptr;
    if (pieces[i].src && pieces[i].bytes) std::memcpy(host.data() + off[i], pieces[i].src, pieces[i].bytes);
  }
  if (staged) check(hipMemcpyAsync(plan.arena, host.data(), staged, hipMemcpyHostToDevice, s), "plan upload");
  check(hipStreamSynchronize(s), "plan sync");   // (the staging buffer goes out of scope)
}

void llt_plan_build(LltPlan &plan, int T, long lda, std::vector<uint8_t> &P, hipStream_t s,
                    const std::vector<int> *col_class) {
  llt_plan_symbolic(plan, T, lda, P, col_class);
  llt_plan_upload(plan, s);
}

void llt_plan_reset(LltPlan &plan) {
  char *arena = plan.arena;
  const size_t bytes = plan.arena_bytes;
  plan = LltPlan{};
  plan.arena = arena;
  plan.arena_bytes = bytes;
}

void llt_plan_free(LltPlan &plan) {
  if (plan.arena) (void)hipFree(plan.arena);
  plan = LltPlan{};
}

}  // namespace arslam
