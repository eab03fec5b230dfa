"""Batched monocular front end over a device-resident frame sequence: the headline path.

One step = ORBextractor::operator() on B frames (ORBextractor.cc:1513-1629) plus
TrackWithMotionModel's SearchByProjection(CurrentFrame, LastFrame, th, bMono)
(Tracking.cc:966-994, ORBmatcher.cc:1620-1789) of every frame against its predecessor,
and optionally (local_map=True) TrackLocalMap's SearchLocalPoints (Tracking.cc:1280-1336:
IsInFrustum + SearchByProjection(F, vpLocalMapPoints, th), ORBmatcher.cc:61-173) of every
frame against the MapPoints of its `local_window` predecessors, all in HBM:

* the batch is split into `lanes` contiguous chunks, each extracted by its own
  ORBextractor on its own HIP stream, so one chunk's latency-bound kernels (octree,
  describe) overlap another's;
* one ORBmatcher matches all B-1 pairs on a third stream once every lane is done (a
  stream of its own, created before the lanes' streams), with TrackWithMotionModel's
  second search at 2*th of a pair left under 20 matches (Tracking.cc:988-994);
* pipelined (default): keypoint / descriptor / match buffers are double-buffered, so
  batch j is extracted while batch j-1 is matched; the next use of a buffer waits for
  the matching that last read it (events in both directions).  Not pipelined: the same
  launches with a single buffer set, each step waiting for the previous step's match.

bench.py times this object; tests/test_gpu_pipeline.py checks every frame and every
pair of its output against the CPU parity oracle.
"""
from __future__ import annotations

import sys

import numpy as np

from .extractor import ORBextractor
from .matcher import ORBmatcher


class SequencePipeline:
    def __init__(self, batch: int, width: int, height: int, lanes: int = 2, pipelined: bool = True,
                 match: bool = True, device: int = 0, params=(1000, 1.2, 8, 20, 7), fx: float = 500.0,
                 fy: float = 500.0, cx: float = 320.0, cy: float = 240.0, depth: float = 5.0, th: float = 15.0,
                 nnratio: float = 0.9, check_ori: bool = True, match_stream=None,
                 nbuf: int = 2, matcher_mode: int | None = None, match_after_stage: int = 0,
                 lane_offset_stage: int | None = None, match_cu_stride: int = 1,
                 match_priority: int = 0, on_matched=None, local_map: bool = False, local_window: int = 3,
                 local_th: float = 1.0, level0_in_place: bool = True, retry_below: int = 20,
                 first_in_phase: bool = True):
        import torch

        self.B, self.W, self.H = int(batch), int(width), int(height)
        self.S = max(1, min(int(lanes), self.B))
        self.match = bool(match)
        self.pipelined = bool(pipelined) and self.match
        self.dev = torch.device("cuda", device)
        self.fx, self.fy, self.cx, self.cy, self.depth, self.th = fx, fy, cx, cy, depth, th
        # TrackWithMotionModel searches a pair again at 2*th when it found fewer than 20
        # matches (Tracking.cc:988-994); 0: one search (the bare SearchByProjection)
        self.retry_below = int(retry_below)
        # The matcher's stream is created here, before the extraction lanes' streams
        # (orbx_stream_create; match_cu_stride k > 1 also confines it to CUs 0, k,
        # 2k, ...; match_priority: its HIP stream priority).  HIP hands out its hardware queues in stream-creation order, and
        # the three busy streams run concurrently only on queues of their own: created
        # after the lanes' streams, or taken from torch's stream pool, the same matcher
        # stream measured 193-197k frames/s against 214-217k (k = 1 and k = 4 alike;
        # profiles/r02_n_stream_order_ab.log)
        self._own_ms = None
        if match_stream is not None:
            self.ms = match_stream
        else:
            from .extractor import stream_create
            self._own_ms = stream_create(device, max(1, int(match_cu_stride)), int(match_priority))
            self.ms = torch.cuda.ExternalStream(self._own_ms, device=self.dev)
        self.exs = [ORBextractor(*params, device=device) for _ in range(self.S)]
        # the monocular front end never reads mvImagePyramid: level 0 stays in the batch's
        # frames (no copy into the pyramid; orbx_extractor_set_level0_in_place)
        for e in self.exs:
            e.set_level0_in_place(level0_in_place)
        self.matcher = ORBmatcher(nnratio, check_ori, device=device)
        # matcher_mode: orbx_matcher_set_footprint.  Default 5 (lean split: one 1024-thread
        # workgroup per problem sorts and scores with only the grid and the claims in LDS,
        # then a one-wave kernel replays with only the claims in LDS).  Beside the pipelined
        # extraction 4 (lean, replay in the scoring workgroup) measured 190-192k frames/s
        # against 185-190k for 0 (grid, descriptors and query state in LDS, ~118 KB per
        # workgroup), 176-181k for 1 (256 threads) and 167-169k for 2 (split launches);
        # 5 measured 197.4k vs 196.3k for 4 at C1 and 66.3k vs 63.9k at configs[4]
        # (profiles/r02_e_*, r02_k_*, r02_m_split_ab.log)
        self.matcher.set_footprint(5 if matcher_mode is None else matcher_mode)
        self.sf = self.exs[0].GetScaleFactors()
        self.cap = self.exs[0].max_keypoints(self.W, self.H)
        # TrackLocalMap stage: every keypoint of the batch makes a MapPoint (id b*cap + i,
        # at `depth` on its ray: Tracking::CreateNewKeyFrame's UnprojectStereo), which
        # TrackWithMotionModel projects (global ids) and frame b's local map lists -- the
        # MapPoints of frames b-1 .. b-local_window, every slot (empty slots are bad).
        # SearchLocalPoints uses ORBmatcher(0.8) (Tracking.cc:1320).
        self.local_map = bool(local_map) and self.match
        self.local_th = float(local_th)
        if self.local_map:
            self.lmatcher = ORBmatcher(0.8, False, device=device)
            self.lmatcher.set_footprint(5 if matcher_mode is None else matcher_mode)
            off, ids = [0], []
            for b in range(self.B):
                for f in range(max(0, b - int(local_window)), b):
                    ids.append(np.arange(f * self.cap, (f + 1) * self.cap, dtype=np.int32))
                off.append(off[-1] + (b - max(0, b - int(local_window))) * self.cap)
            self.local_off = np.array(off, np.int32)
            self.d_local_ids = torch.from_numpy(np.concatenate(ids) if ids else np.zeros(1, np.int32)).to(self.dev)
        self.bounds = [(self.B * c // self.S, self.B * (c + 1) // self.S) for c in range(self.S)]
        self.streams = [torch.cuda.ExternalStream(e.stream_handle(), device=self.dev) for e in self.exs]
        nbuf = max(2, int(nbuf)) if self.pipelined else 1
        B, cap = self.B, self.cap
        i32 = dict(dtype=torch.int32, device=self.dev)
        self.kps = [torch.empty((B, cap, 7), **i32) for _ in range(nbuf)]
        self.desc = [torch.empty((B, cap, 32), dtype=torch.uint8, device=self.dev) for _ in range(nbuf)]
        self.n = [torch.empty((B,), **i32) for _ in range(nbuf)]
        self.mp = [torch.empty((B, cap), **i32) for _ in range(nbuf)]
        self.nm = [torch.empty((B,), **i32) for _ in range(nbuf)]
        if self.local_map:
            from .matcher import mappoint_table
            self.tab = [mappoint_table(B, cap, self.dev) for _ in range(nbuf)]
            self.nm_local = [torch.empty((B,), **i32) for _ in range(nbuf)]
            self._lt = []  # (start, end) event pairs of the local stage while timing
        self.ev_ex = [[torch.cuda.Event() for _ in range(self.S)] for _ in range(nbuf)]  # [buffer][lane]
        self.ev_m = [torch.cuda.Event() for _ in range(nbuf)]
        self.used = [False] * nbuf
        self.T_of = [None] * nbuf  # the poses of the batch extracted into each buffer
        # match_after_stage k (pipelined only): the matching of batch j-1 also waits until
        # every lane's extraction of batch j has passed stage k (1 pyramid, 2 blur + FAST
        # strength, 3 FAST cells, 4 octree), so it runs beside the later stages
        self.stage_ev = [e.set_stage_event(match_after_stage) for e in self.exs] \
            if (self.pipelined and match_after_stage) else None
        # lane_offset_stage k: lane c starts each batch once lane c-1 has passed stage k of
        # it, so the lanes run out of phase (one lane's latency-bound stages beside the
        # other's issue-bound ones) instead of in step.  Default 2 (after the blur + FAST
        # strength stage): 193.6-197.4k frames/s against 192.8-194.3k in step, extraction
        # alone 216.5k against 210.8k (profiles/r02_l_lane_offset_ab.log).  None: 2, or 4
        # (after the octree) for pyramids deeper than 8 levels, whose longer matcher runs
        # best beside one lane's describe and the other's first stages (configs[4]
        # 99.8-101.0k -> 105.7-106.0k frames/s; configs[1] with 4: 214.5-215.4k against
        # 224.4-225.1k with 2; tools/g_r3zy.sh, tools/g_r3zz.sh)
        # (round 5: 3 for deep pyramids, with the LDS-DMA describe at every frame size --
        # offset 3 110.5-111.4k frames/s, 4 107.6-107.9k, 2 105.3-106.3k at configs[4], r05c)
        if lane_offset_stage is None:
            lane_offset_stage = 3 if int(params[2]) > 8 else 2
        self.lane_offset_stage = int(lane_offset_stage)
        self.first_in_phase = bool(first_in_phase)
        self.lane_ev = [e.set_stage_event(lane_offset_stage) for e in self.exs] \
            if (lane_offset_stage and not match_after_stage and self.S > 1) else None
        # on_matched(b): called right after a batch's matching is enqueued on self.ms and
        # before the event that releases its buffer b for reuse -- work the consumer
        # enqueues on self.ms there (e.g. copying the results out) finishes before the
        # buffer is overwritten
        self.on_matched = on_matched
        from . import _lib
        _lib.track(self)
        self._timing = False
        self._ext_timed = self._match_timed = False
        self.it = 0            # extractions issued
        self.pending = None    # buffer extracted but not yet matched (pipelined)
        self.last = None       # buffer holding the newest complete result

    def close(self):
        """Wait for this pipeline's work, then release its matchers, its extractors and the
        matcher stream it created (idempotent; results are unreadable afterwards)."""
        from .extractor import release_owned
        release_owned(self, streams=[getattr(self, "ms", None)], owners=[
            getattr(self, "matcher", None), getattr(self, "lmatcher", None), *getattr(self, "exs", [])],
            own_streams=["_own_ms"])

    def __del__(self, _finalizing=sys.is_finalizing):
        if not _finalizing():  # at interpreter exit the atexit hook has closed it already
            try:
                self.close()
            except Exception:
                pass

    # -- launches -----------------------------------------------------------------
    def _extract(self, frames, Tcw, b):
        self.T_of[b] = Tcw
        for c in range(self.S):
            b0, b1 = self.bounds[c]
            if self.used[b] and self.match:
                self.streams[c].wait_event(self.ev_m[b])  # the matching that last read buffer b is done
            # the lane offset (lane c waits for lane c-1's stage) -- except, with
            # first_in_phase, on a run's first batch (nothing pending to match): there the
            # lanes start together, and the offset forms on the second batch, where the
            # first batch's matching runs beside the waiting lane instead of nothing
            # (first_in_phase; r05as: +0.4 % at 20 steps, within noise; r06fp: +0.6 % over six
            # interleaved pairs at 20 steps, five of them faster -- on since round 6)
            if self.lane_ev and c > 0 and not (self.first_in_phase and self.match and self.pipelined
                                               and self.pending is None):
                from .extractor import stream_wait_event
                stream_wait_event(self.streams[c].cuda_stream, self.lane_ev[c - 1])
            self.exs[c].extract_batch_device(frames[b0:b1], self.kps[b][b0:b1], self.desc[b][b0:b1],
                                             self.n[b][b0:b1])
            self._lane_tail(b, c)
            self.ev_ex[b][c].record(self.streams[c])
        self.used[b] = True

    def _lane_tail(self, b, c):
        """Per-frame work a subclass enqueues on lane c's stream after its extraction of
        buffer b (before the event the matcher waits for)."""

    def _match(self, b, after_next=False):
        Tcw = self.T_of[b]
        for c in range(self.S):
            self.ms.wait_event(self.ev_ex[b][c])
        if after_next and self.stage_ev:
            from .extractor import stream_wait_event
            for ev in self.stage_ev:
                stream_wait_event(self.ms.cuda_stream, ev)
        if self.local_map:
            self._match_local(b, Tcw)
        else:
            self.matcher.match_sequence_device_ex(self.kps[b], self.desc[b], self.n[b], Tcw, self.mp[b], self.nm[b],
                                                  self.sf, self.fx, self.fy, self.cx, self.cy, self.W, self.H,
                                                  depth=self.depth, th=self.th, retry_below=self.retry_below,
                                                  stream=self.ms.cuda_stream)
        if self.on_matched is not None:
            self.on_matched(b)
        self.ev_m[b].record(self.ms)

    def _match_local(self, b, Tcw):
        """MapPoints of the batch, TrackWithMotionModel against them, then SearchLocalPoints."""
        import torch

        from .matcher import create_mappoints_device
        s = self.ms.cuda_stream
        tab = self.tab[b]
        create_mappoints_device(self.kps[b], self.n[b], Tcw, self.sf, self.fx, self.fy, self.cx, self.cy, tab,
                                const_depth=self.depth, stream=s)
        self.matcher.match_sequence_device_ex(self.kps[b], self.desc[b], self.n[b], Tcw, self.mp[b], self.nm[b],
                                              self.sf, self.fx, self.fy, self.cx, self.cy, self.W, self.H,
                                              th=self.th, d_mp_pos=tab["pos"], global_ids=True,
                                              retry_below=self.retry_below, stream=s)
        timed = self._timing
        if timed:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(self.ms)
        mps = dict(tab, desc=self.desc[b].view(-1, 32))
        self.lmatcher.search_local_points_device(mps, self.kps[b], self.desc[b], self.n[b], Tcw, self.local_off,
                                                 self.d_local_ids, self.mp[b], self.nm_local[b], self.sf, self.fx,
                                                 self.fy, self.cx, self.cy, self.W, self.H, th=self.local_th,
                                                 stream=s)
        if timed:
            ev[1].record(self.ms)
            self._lt.append(ev)

    def step(self, frames, Tcw):
        """Issue one step (asynchronous).  Pipelined: extracts this batch and matches the
        previous one (with the poses passed alongside that batch); call drain() after the
        last step.  `frames` and `Tcw` must stay untouched until the batch is matched."""
        nbuf = len(self.kps)
        b = self.it % nbuf
        self._extract(frames, Tcw, b)
        self.it += 1
        if not self.match:
            self.last = b
            return
        if self.pipelined:
            if self.pending is not None:
                self._match(self.pending, after_next=True)
                self.last = self.pending
            self.pending = b
        else:
            self._match(b)
            self.last = b

    def nbuf_ok(self) -> bool:
        """Two pipeline buffers (the layout an external double-buffered feeder pairs with)."""
        return len(self.kps) == 2

    def drain(self, Tcw=None):
        if self.pipelined and self.pending is not None:
            self._match(self.pending)
            self.last = self.pending
            self.pending = None

    def run(self, frames, Tcw, k: int):
        """k steps, pipeline fill and drain included (K extractions and K matchings)."""
        for _ in range(k):
            self.step(frames, Tcw)
        self.drain(Tcw)

    # -- results ------------------------------------------------------------------
    def results(self, b=None) -> dict:
        """Device tensors of the newest complete batch, or of buffer b (call after
        synchronising, or after ev_m[b] for a buffer whose matching was issued)."""
        b = self.last if b is None else b
        r = {"kps": self.kps[b], "desc": self.desc[b], "n": self.n[b], "mp": self.mp[b], "nm": self.nm[b]}
        if self.local_map:
            r["nm_local"] = self.nm_local[b]
        return r

    def host_results(self, b=None) -> dict:
        r = self.results(b)
        B, cap = self.B, self.cap
        from . import _lib as L
        out = {"kps": r["kps"].cpu().numpy().view(np.uint8).reshape(B, cap, 28).view(L.KEYPOINT_DTYPE).reshape(B, cap),
               "desc": r["desc"].cpu().numpy(), "n": r["n"].cpu().numpy(), "mp": r["mp"].cpu().numpy(),
               "nm": r["nm"].cpu().numpy()}
        if "nm_local" in r:
            out["nm_local"] = r["nm_local"].cpu().numpy()
        return out

    def status(self) -> np.ndarray:
        """Octree status words of every frame of the newest extraction (0 = complete)."""
        return np.concatenate([e.status(b1 - b0) for e, (b0, b1) in zip(self.exs, self.bounds)])

    def set_timing(self, enable: bool, stage: str | None = None):
        """HIP-event timing of the following steps: every stage of every lane and the
        matcher, or (stage given) only that stage's launches -- an extraction stage's two
        boundary events per lane, or the matcher's ("match")."""
        ext = enable and stage != "match"
        for e in self.exs:
            e.set_timing(ext, None if stage == "match" else stage)
        self._match_timed = bool(enable) and self.match and stage in (None, "match")
        if self.match:
            self.matcher.set_timing(self._match_timed)
        self._ext_timed = bool(ext)
        self._timing = bool(enable)
        if enable and self.local_map:
            self._lt = []

    def stage_times(self) -> dict:
        """HIP-event stage times (ms per launch) averaged over the lanes' extractors (each
        lane's launches time its own frames), plus the matcher's ("match"): the stages
        set_timing selected."""
        out = {}
        if self._ext_timed:
            per = [e.stage_times() for e in self.exs]
            out = {k: sum(p[k] for p in per) / len(per) for k in per[0]}
        if self._match_timed:
            out["match"] = self.matcher.last_ms()
        if self.local_map and self._lt:
            out["local_map"] = sum(a.elapsed_time(b) for a, b in self._lt) / len(self._lt)
        return out


def sequence_poses(off: np.ndarray, fx: float = 500.0, fy: float = 500.0, depth: float = 5.0) -> np.ndarray:
    """mTcw rows 0..2 of each view of synth.sequence: a pure translation that makes the
    canvas shift `off` pixels at depth `depth`."""
    T = np.zeros((len(off), 12), np.float32)
    for b in range(len(off)):
        T[b] = [1, 0, 0, -off[b, 0] * depth / fx, 0, 1, 0, -off[b, 1] * depth / fy, 0, 0, 1, 0]
    return T
