"""Batched RGB-D front end over a device-resident sequence: configs[4]'s step.

One step, for B RGB-D frames in HBM (gray image + registered 16-bit depth image each), the
hot path of Tracking::GrabImageRGBD (Tracking.cc:247-289) and of the tracking search that
follows it:
  1. ORBextractor::operator() on the gray images (Frame.cc:217), the batch split into
     lanes on their own extractor streams (pipeline.SequencePipeline);
  2. the RGB-D Frame constructor's steps after extraction (Frame.cc:227-230):
     UndistortKeyPoints and ComputeStereoFromRGBD with GrabImageRGBD's convertTo(CV_32F,
     mDepthMapFactor) (Tracking.cc:265-271) applied to the pixels read -- one kernel
     (orbx_compute_stereo_from_rgbd_device) -> mvKeysUn, mvuRight, mvDepth;
  3. Tracking::UpdateLastFrame (Tracking.cc:893-954): frame b-1's temporal MapPoints at
     UnprojectStereo for its nearest keypoints with depth, beside the map MapPoints it
     already tracks (set_tracked / tracked_from);
  4. TrackWithMotionModel's SearchByProjection(CurrentFrame, LastFrame, th = 15,
     bMono = false) (Tracking.cc:966-994, ORBmatcher.cc:1620-1789) of frame b against frame
     b-1, b >= 1, with the retry at 2*th of a pair left with fewer than 20 matches
     (Tracking.cc:988-994): the stereo octave ranges for motion along the optical axis
     beyond mb, the mvuRight gate, the rotation check, temporal claims not blocking, the
     undistorted image bounds (Frame::ComputeImageBounds) for the grid.
Steps 2-3 run per frame on each extraction lane's stream right after its frames, step 4
on the matcher stream beside the next batch's extraction.  No frame of the
sequence is a keyframe (UpdateLastFrame returns early for the last keyframe, Tracking.cc:
902; a caller with keyframes passes their LastFrames' MapPoints through set_tracked and
skips those frames' temporal points itself).  Optimizer::PoseOptimization, which consumes
the matches in the reference, is out of scope: every frame's pose is given.

bench.py --workload tum5k times this object; tests/test_gpu_rgbd.py checks every frame
and pair of its output against the CPU parity oracle.
"""
from __future__ import annotations

import numpy as np

from .frame import ComputeImageBounds, camera, rgbd_device
from .matcher import create_mappoints_device, last_frame_table, mappoint_table, update_last_frame_device
from .pipeline import SequencePipeline
from .stereo import th_depth as _th_depth

RETRY_BELOW = 20  # Tracking.cc:989: "if (nmatches < 20)" -> search again at 2*th


class RGBDSequencePipeline(SequencePipeline):
    def __init__(self, batch: int, width: int, height: int, fx: float, fy: float, cx: float, cy: float, dist,
                 bf: float, depth_map_factor: float = 5000.0, th_depth_factor: float = 40.0,
                 params=(5000, 1.2, 12, 20, 7), th: float = 15.0, retry_below: int = RETRY_BELOW, **kw):
        # lane 1 starts each batch after lane 0's octree (stage 4): the RGB-D step's matcher
        # (steps 2-4, far heavier than the monocular search) then runs beside one lane's
        # describe and the other's first stages -- 87.0-87.1k RGB-D frames/s against
        # 83.2-85.7k after the FAST cells (3, SequencePipeline's deep-pyramid default), 85.1-86.1k
        # after the blur (2), 82.1-83.3k after the pyramid (1) (profiles/r06_rgbd_lane_offset_ab.txt)
        kw.setdefault("lane_offset_stage", 4)
        # steps 2-3 (the RGB-D Frame, UpdateLastFrame) per frame, so on each extraction
        # lane's stream right after its frames (frame_on_lanes) or on the matcher stream
        # before the search
        self.frame_on_lanes = bool(kw.pop("frame_on_lanes", True))
        super().__init__(batch, width, height, params=params, fx=fx, fy=fy, cx=cx, cy=cy, th=th, **kw)
        import torch

        if not self.match:
            raise ValueError("the RGB-D pipeline is the tracking step: match=True")
        self.cam = camera(fx, fy, cx, cy, *dist)
        self.image_bounds = ComputeImageBounds(self.cam, width, height, device=self.dev.index or 0)
        self.bf = float(bf)
        self.mb = float(np.float32(bf) / np.float32(fx))  # mb = mbf / fx (Frame.cc:260)
        self.th_depth = _th_depth(bf, fx, th_depth_factor)  # mThDepth = mbf * ThDepth / fx
        # Tracking.cc:166-170: mDepthMapFactor = 1.0f / DepthMapFactor (1 when ~0)
        f = np.float32(depth_map_factor)
        self.depth_map_factor = 1.0 if abs(float(f)) < 1e-5 else float(np.float32(1.0) / f)
        self.retry_below = int(retry_below)
        nbuf = len(self.kps)
        B, cap = self.B, self.cap
        f32 = dict(dtype=torch.float32, device=self.dev)
        self.kpu = [torch.empty((B, cap, 7), dtype=torch.int32, device=self.dev) for _ in range(nbuf)]
        self.ur = [torch.empty((B, cap), **f32) for _ in range(nbuf)]
        self.dp = [torch.empty((B, cap), **f32) for _ in range(nbuf)]
        self.lf = [last_frame_table(B, cap, self.dev) for _ in range(nbuf)]
        self.D_of = [None] * nbuf
        self._next_depth = None
        self.obs_in = self.pos_in = None
        self._rt = []  # (start, end) events of steps 2-4 while timing

    # -- launches -----------------------------------------------------------------
    def step(self, frames, Tcw, depth=None):
        """Issue one step (asynchronous): B gray frames (B, H, W) u8, poses Tcw (B, 12) f32 and
        depth images (B, H, W) u16 (or f32) in HBM, all untouched until the batch is matched."""
        if depth is None:
            raise ValueError("an RGB-D step needs the depth images")
        self._next_depth = depth
        super().step(frames, Tcw)

    def run(self, frames, Tcw, k: int, depth=None):
        for _ in range(k):
            self.step(frames, Tcw, depth)
        self.drain(Tcw)

    def _extract(self, frames, Tcw, b):
        self.D_of[b] = self._next_depth
        super()._extract(frames, Tcw, b)

    def _frame_steps(self, b, b0, b1, stream):
        """Steps 2-3 for frames b0..b1-1 of buffer b on `stream`."""
        T = self.T_of[b][b0:b1]
        lf = {k: v[b0:b1] for k, v in self.lf[b].items()}
        rgbd_device(self.cam, self.kps[b][b0:b1], self.n[b][b0:b1], self.D_of[b][b0:b1], self.bf,
                    self.depth_map_factor, self.kpu[b][b0:b1], self.ur[b][b0:b1], self.dp[b][b0:b1], stream=stream)
        update_last_frame_device(self.kpu[b][b0:b1], self.n[b][b0:b1], self.dp[b][b0:b1], T, self.fx, self.fy,
                                 self.cx, self.cy, self.th_depth, lf,
                                 d_obs_in=None if self.obs_in is None else self.obs_in[b0:b1],
                                 d_pos_in=None if self.pos_in is None else self.pos_in[b0:b1], stream=stream)

    def _lane_tail(self, b, c):
        if self.frame_on_lanes:
            b0, b1 = self.bounds[c]
            self._frame_steps(b, b0, b1, self.streams[c].cuda_stream)

    def _match(self, b, after_next=False):
        import torch
        T = self.T_of[b]
        for c in range(self.S):
            self.ms.wait_event(self.ev_ex[b][c])
        if after_next and self.stage_ev:
            from .extractor import stream_wait_event
            for ev in self.stage_ev:
                stream_wait_event(self.ms.cuda_stream, ev)
        if self._timing:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record(self.ms)
        s = self.ms.cuda_stream
        lf = self.lf[b]
        if not self.frame_on_lanes:
            self._frame_steps(b, 0, self.B, s)
        self.matcher.match_sequence_device_ex(
            self.kpu[b], self.desc[b], self.n[b], T, self.mp[b], self.nm[b], self.sf, self.fx, self.fy, self.cx,
            self.cy, self.W, self.H, th=self.th, mono=False, bf=self.bf, b=self.mb, d_u_right=self.ur[b],
            d_mp_pos=lf["mp_pos"], d_has_mp=lf["has_mp"], d_mp_obs=lf["mp_obs"], global_ids=True,
            retry_below=self.retry_below, bounds=self.image_bounds, stream=s)
        if self._timing:
            ev[1].record(self.ms)
            self._rt.append(ev)
        if self.on_matched is not None:
            self.on_matched(b)
        self.ev_m[b].record(self.ms)

    # -- the MapPoints LastFrames already track -------------------------------------
    def set_tracked(self, obs_in, pos_in):
        """Every frame's map MapPoints as a LastFrame (before UpdateLastFrame): obs_in (B, cap)
        i32 Observations() (-1 = NULL), pos_in (B, cap, 3) f32 world positions; None: none."""
        self.obs_in, self.pos_in = obs_in, pos_in

    def tracked_from(self, mask, observations: int = 2, b=None):
        """(obs_in, pos_in) for set_tracked: every slot of `mask` ((B, cap) bool) whose
        keypoint has a depth in buffer b's newest results carries a map MapPoint with
        `observations` at its UnprojectStereo position (orbx_create_mappoints_device over
        mvKeysUn) -- made once at setup for a batch stepped repeatedly (call after
        synchronising)."""
        import torch
        b = self.last if b is None else b
        tab = mappoint_table(self.B, self.cap, self.dev)
        create_mappoints_device(self.kpu[b], self.n[b], self.T_of[b], self.sf, self.fx, self.fy, self.cx, self.cy,
                                tab, d_depth=self.dp[b], stream=self.ms.cuda_stream)
        self.ms.synchronize()
        m = torch.as_tensor(np.asarray(mask.cpu() if hasattr(mask, "cpu") else mask), device=self.dev).bool()
        obs = torch.where(m & (self.dp[b] > 0), torch.tensor(int(observations), dtype=torch.int32, device=self.dev),
                          torch.tensor(-1, dtype=torch.int32, device=self.dev)).contiguous()
        return obs, tab["pos"].view(self.B, self.cap, 3).contiguous()

    # -- results ------------------------------------------------------------------
    def set_timing(self, enable: bool, stage: str | None = None):
        super().set_timing(enable, stage)
        self._rt = []

    def stage_times(self) -> dict:
        """The extraction stages and "match" as SequencePipeline reports them, plus "rgbd_track":
        HIP-event ms of steps 2-4 (RGB-D Frame, UpdateLastFrame, the search and its retry)."""
        out = super().stage_times()
        if self._rt:
            out["rgbd_track"] = sum(a.elapsed_time(c) for a, c in self._rt) / len(self._rt)
        return out

    def results(self, b=None) -> dict:
        b = self.last if b is None else b
        r = super().results(b)
        r.update({"kpu": self.kpu[b], "ur": self.ur[b], "dp": self.dp[b], **self.lf[b]})
        return r

    def host_results(self, b=None) -> dict:
        from . import _lib as L
        b = self.last if b is None else b
        out = super().host_results(b)
        B, cap = self.B, self.cap
        out["kpu"] = self.kpu[b].cpu().numpy().view(np.uint8).reshape(B, cap, 28).view(L.KEYPOINT_DTYPE).reshape(B, cap)
        for name, t in (("ur", self.ur[b]), ("dp", self.dp[b]), ("mp_obs", self.lf[b]["mp_obs"]),
                        ("mp_pos", self.lf[b]["mp_pos"]), ("has_mp", self.lf[b]["has_mp"])):
            out[name] = t.cpu().numpy()
        return out
