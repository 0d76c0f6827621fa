"""Ceres 2.0's automatic DENSE_SCHUR e-block choice, restated in plain Python.

TEST INFRASTRUCTURE ONLY (the checker for arslam_debug_ceres_e_blocks and the
ARSLAM_ELIM_AUTO rule); nothing in ar_slam_amd/ imports it.

ArSlamSolver::optimize sets linear_solver_type = DENSE_SCHUR and no
linear_solver_ordering (ar_slam_util.cpp:1003-1012).  Ceres then puts every
parameter block in one group, and ReorderProgramForSchurTypeLinearSolver
(Ceres 2.0 internal/ceres/reorder_program.cc) calls ComputeStableSchurOrdering:
  * CreateHessianGraph: a vertex per non-constant parameter block, an edge
    between every two non-constant blocks of one residual block;
  * the vertices in program order (the order AddResidualBlock first saw the
    blocks: camera, capture, tag per residual, ar_slam_util.cpp:723-727);
  * StableIndependentSetOrdering (graph_algorithms.h): stable sort by
    ascending degree, then greedily take every vertex none of whose
    neighbours has been taken -- the taken vertices are the e-blocks.
Ceres itself is not in this image; this follows the published
algorithm, so the e-block choice is parity-unpinned against Ceres.
"""


def ceres_e_blocks(obs_cap, obs_tag, n_cap, n_tag, camera_const=False, cap_const=None, tag_const=None,
                   members=False):
    """Returns {captures, tags, camera, max_tag_obs} of Ceres' independent set (members: also
    e_cap / e_tag, a 0/1 flag per capture and per tag, and e_cam)."""
    cap_free = [not (cap_const is not None and cap_const[c]) for c in range(n_cap)]
    tag_free = [not (tag_const is not None and tag_const[t]) for t in range(n_tag)]
    cam_free = not camera_const
    # vertex keys: ("f",), ("c", c), ("t", t)
    order, seen = [], set()
    adj = {}

    def vertex(v, free):
        if free and v not in seen:
            seen.add(v)
            order.append(v)
            adj[v] = set()

    tag_nobs = [0] * n_tag
    for c, t in zip(obs_cap, obs_tag):
        c, t = int(c), int(t)
        tag_nobs[t] += 1
        blocks = [(("f",), cam_free), (("c", c), cap_free[c]), (("t", t), tag_free[t])]
        for v, free in blocks:
            vertex(v, free)
        live = [v for v, free in blocks if free]
        for i in range(len(live)):
            for j in range(i + 1, len(live)):
                adj[live[i]].add(live[j])
                adj[live[j]].add(live[i])
    queue = sorted(order, key=lambda v: len(adj[v]))   # Python's sort is stable
    color = {v: 0 for v in order}                      # 0 white, 1 grey, 2 black
    taken = []
    for v in queue:
        if color[v] != 0:
            continue
        color[v] = 2
        taken.append(v)
        for u in adj[v]:
            if color[u] == 0:
                color[u] = 1
    if members:
        e_cap, e_tag = [0] * n_cap, [0] * n_tag
        for v in taken:
            if v[0] == "c":
                e_cap[v[1]] = 1
            elif v[0] == "t":
                e_tag[v[1]] = 1
        return dict(e_cap=e_cap, e_tag=e_tag, e_cam=int(("f",) in taken))
    return dict(captures=sum(1 for v in taken if v[0] == "c"),
                tags=sum(1 for v in taken if v[0] == "t"),
                camera=sum(1 for v in taken if v[0] == "f"),
                max_tag_obs=max(tag_nobs) if tag_nobs else 0)
