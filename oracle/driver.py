"""CPU restatement of ArSlamSolver's drivers over the oracle (TEST INFRASTRUCTURE ONLY).

Restates, with the oracle's ceres::Solve restatement (or_solve) as the
optimizer:
  * solve()            BFS from the capture with most tags  ar_slam_util.cpp:744-866
  * addConnectedCaptures                                    :868-886
  * solveIncremental() / solveCapture()                      :629-742
  * the initialisers initCapturePose / initArPose            :98-128
The problem grows exactly as ceres::Problem does in the reference: every
optimize() solves all residual blocks added so far, parameter blocks in
first-use order.  Unsolved captures are visited in ascending index (the
reference's unordered_set order is the standard library's), as the C++
mirror does.  Used only by tests/ to check ar_slam_amd/host against it.
"""
from __future__ import annotations

import numpy as np

from . import oracle as O


class OracleSlam:
    def __init__(self, camera=(3000.0, 0.0, 0.0), **opts):
        self.camera = np.array(camera, np.float64)
        self.captures = []    # dict(uid, blocks, init_block, pose)
        self.arucos = []      # dict(id, blocks, initialized, pose)
        self.blocks = []      # dict(rect, cap, ar, added)
        self.aruco_map = {}
        self.unsolved = []
        self.opts = opts
        self.order = []       # added blocks, in AddResidualBlock order
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
        self.unsolved.append(c)
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

    def solve_incremental(self):
        self.unsolved.sort()
        if self.unsolved and len(self.unsolved) == len(self.captures):
            c = self.unsolved.pop(0)
            self._add_blocks(c)
            self._optimize()
        repeat = True
        while repeat:
            repeat = False
            i = 0
            while i < len(self.unsolved):
                c = self.unsolved[i]
                hit = None
                for b in self.captures[c]["blocks"]:
                    if self.arucos[self.blocks[b]["ar"]]["initialized"]:
                        hit = b
                        break
                if hit is not None:
                    repeat = True
                    self.unsolved.pop(i)
                    self._init_capture(c, hit)
                    self._add_blocks(c)
                    self._optimize()
                    if i >= len(self.unsolved):
                        break
                i += 1   # after an erase this skips the next element, as the reference's loop does
