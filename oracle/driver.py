"""CPU restatement of ArSlamSolver's drivers over the oracle (TEST INFRASTRUCTURE ONLY).

Restates, with the oracle's ceres::Solve restatement (or_solve) as the
optimizer:
  * solve()            BFS from the capture with most tags  ar_slam_util.cpp:744-866
  * addConnectedCaptures                                    :868-886
  * solveIncremental() / solveCapture()                      :629-742
  * the initialisers initCapturePose / initArPose            :98-128
The problem grows exactly as ceres::Problem does in the reference: every
optimize() solves all residual blocks added so far, parameter blocks in
first-use order.  Unsolved captures live in the reference's own container,
std::unordered_set<CaptureHandle> with hash = index (ar_slam_util.hpp:140-145,
492; oracle/stl_uset.cpp), so solveIncremental visits them in libstdc++'s
bucket order and seeds with its begin() (ar_slam_util.cpp:643, 657-676), as
the C++ mirror does.  Used only by tests/ to check ar_slam_amd/host against it.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import oracle as O

_STL = None


def _stl():
    global _STL
    if _STL is None:
        O.build()
        L = C.CDLL(os.path.join(O.HERE, "liboracle_stl.so"))
        L.or_uset_new.restype = C.c_void_p
        L.or_uset_free.argtypes = [C.c_void_p]
        L.or_uset_insert.argtypes = [C.c_void_p, C.c_uint]
        L.or_uset_erase.argtypes = [C.c_void_p, C.c_uint]
        L.or_uset_size.argtypes = [C.c_void_p]
        L.or_uset_list.argtypes = [C.c_void_p, C.POINTER(C.c_uint)]
        _STL = L
    return _STL


class UnorderedHandleSet:
    """std::unordered_set<CaptureHandle> (ar_slam_util.hpp:492), through oracle/stl_uset.cpp."""

    def __init__(self):
        self._L = _stl()
        self._h = self._L.or_uset_new()

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.or_uset_free(self._h)

    def insert(self, idx):
        self._L.or_uset_insert(self._h, idx)

    def erase(self, idx):
        return self._L.or_uset_erase(self._h, idx)

    def __len__(self):
        return self._L.or_uset_size(self._h)

    def items(self):
        """The elements in iteration order, begin() first."""
        out = (C.c_uint * max(len(self), 1))()
        n = self._L.or_uset_list(self._h, out)
        return [int(out[i]) for i in range(n)]


class OracleSlam:
    def __init__(self, camera=(3000.0, 0.0, 0.0), **opts):
        self.camera = np.array(camera, np.float64)
        self.captures = []    # dict(uid, blocks, init_block, pose)
        self.arucos = []      # dict(id, blocks, initialized, pose)
        self.blocks = []      # dict(rect, cap, ar, added)
        self.aruco_map = {}
        self.unsolved = UnorderedHandleSet()
        self.opts = opts
        self.order = []       # added blocks, in AddResidualBlock order
        self.solve_order = []  # the capture of each optimize() call
        self.n_solves = 0

    def add_detections(self, uid, ids, corners):
        c = len(self.captures)
        self.captures.append(dict(uid=uid, blocks=[], init_block=None, pose=np.zeros(6)))
        for i, ar_id in enumerate(ids):
            if ar_id not in self.aruco_map:
                self.aruco_map[ar_id] = len(self.arucos)
                self.arucos.append(dict(id=ar_id, blocks=[], initialized=False, pose=np.zeros(6)))
            a = self.aruco_map[ar_id]
            b = len(self.blocks)
            self.blocks.append(dict(rect=np.asarray(corners[i], np.float64), cap=c, ar=a, added=False))
            self.captures[c]["blocks"].append(b)
            self.arucos[a]["blocks"].append(b)
        self.unsolved.insert(c)
        return c

    # ---- problem ----
    def _add_blocks(self, c):
        cap = self.captures[c]
        for b in cap["blocks"]:
            blk = self.blocks[b]
            ar = self.arucos[blk["ar"]]
            if not ar["initialized"]:
                ar["initialized"] = True
                ar["pose"] = O.init_ar_pose(blk["rect"], self.camera, cap["pose"])
            assert not blk["added"], "block for capture was somehow already added?"
            blk["added"] = True
            self.order.append(b)
        self.solve_order.append(c)

    def _optimize(self):
        caps, tags = [], []
        cpos, tpos = {}, {}
        obs_cap, obs_tag, corners = [], [], []
        for b in self.order:
            blk = self.blocks[b]
            if blk["cap"] not in cpos:
                cpos[blk["cap"]] = len(caps)
                caps.append(blk["cap"])
            if blk["ar"] not in tpos:
                tpos[blk["ar"]] = len(tags)
                tags.append(blk["ar"])
            obs_cap.append(cpos[blk["cap"]])
            obs_tag.append(tpos[blk["ar"]])
            corners.append(blk["rect"])
        cap = np.array([self.captures[c]["pose"] for c in caps])
        tag = np.array([self.arucos[a]["pose"] for a in tags])
        cam, cap, tag, s = O.solve(self.camera.copy(), cap, tag, np.array(obs_cap, np.int32),
                                   np.array(obs_tag, np.int32), np.array(corners), **self.opts)
        self.camera = cam
        for i, c in enumerate(caps):
            self.captures[c]["pose"] = cap[i].copy()
        for i, a in enumerate(tags):
            self.arucos[a]["pose"] = tag[i].copy()
        self.n_solves += 1
        self.last_summary = s

    def _init_capture(self, c, b):
        blk = self.blocks[b]
        self.captures[c]["pose"] = O.init_capture_pose(blk["rect"], self.camera, self.arucos[blk["ar"]]["pose"])

    # ---- drivers ----
    def solve(self):
        best = 0
        for i in range(1, len(self.captures)):
            if len(self.captures[i]["blocks"]) > len(self.captures[best]["blocks"]):
                best = i
        self.captures[best]["init_block"] = -1
        open_ = [best]
        while open_:
            c = open_.pop(0)
            if c != best:
                self._init_capture(c, self.captures[c]["init_block"])
            self._add_blocks(c)
            self._optimize()
            for bb in self.captures[c]["blocks"]:
                for b in self.arucos[self.blocks[bb]["ar"]]["blocks"]:
                    cc = self.blocks[b]["cap"]
                    if self.captures[cc]["init_block"] is None:
                        self.captures[cc]["init_block"] = b
                        open_.append(cc)

    def solve_incremental(self):   # ar_slam_util.cpp:629-678
        if len(self.unsolved) and len(self.unsolved) == len(self.captures):
            c = self.unsolved.items()[0]      # *unsolved_captures_.begin()
            self.unsolved.erase(c)
            self._add_blocks(c)
            self._optimize()
        repeat = True
        while repeat:
            repeat = False
            # the set's iteration order; nothing is inserted during the loop, so
            # an erase only removes the element (the rest keep their order)
            order = self.unsolved.items()
            i = 0
            while i < len(order):
                c = order[i]
                hit = None
                for b in self.captures[c]["blocks"]:
                    if self.arucos[self.blocks[b]["ar"]]["initialized"]:
                        hit = b
                        break
                if hit is not None:
                    repeat = True
                    self.unsolved.erase(c)     # itr = unsolved_captures_.erase(itr)
                    order.pop(i)
                    self._init_capture(c, hit)
                    self._add_blocks(c)
                    self._optimize()
                    if i >= len(order):        # itr == end()
                        break
                i += 1   # ++itr: after an erase this skips the next element, as the reference's loop does
