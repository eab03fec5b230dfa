"""Batched stereo front end over a device-resident sequence: configs[2]'s step.

One step, for B rectified stereo frames in HBM (the Frame constructor's hot path and the
tracking search that follows it):
  1. ORBextractor::operator() on the left and the right images, by two extractors on two
     streams (mpORBextractorLeft / mpORBextractorRight, Frame.cc:127-131);
  2. Frame::ComputeStereoMatches of every frame (Frame.cc:673-885) -> mvuRight, mvDepth;
  3. Tracking::UpdateLastFrame (Tracking.cc:893-954): frame b-1's temporal MapPoints at
     UnprojectStereo for its nearest keypoints with depth, beside the MapPoints it already
     tracks (`obs_in` / `pos_in`, e.g. those of the map);
  4. Tracking::TrackWithMotionModel's SearchByProjection(CurrentFrame, LastFrame, th = 7,
     bMono = false) (Tracking.cc:966-994, ORBmatcher.cc:1620-1789) of frame b against
     frame b-1, b >= 1: the stereo octave ranges (bForward / bBackward for motion along the
     optical axis beyond mb), the mvuRight gate, the rotation check, the claims of the
     temporal points (Observations() == 0) not blocking later ones, and the second search
     at 2*th of a pair left under 20 matches.
No frame of the sequence is a keyframe: UpdateLastFrame returns early for the last keyframe
(Tracking.cc:902), which this pipeline does not model -- a caller with keyframes passes
their LastFrames' MapPoints as obs_in / pos_in and must not step those frames' temporal
points.
Step 2 runs on a matcher stream and steps 3-4 on a tracking stream, beside the next
steps' extraction: four extractor pairs in rotation, so a pair's pyramids and outputs stay
untouched until its matching is done; the right image's extraction starts after the left
one's blur stage (out of phase).

benchmarks/stereo_bench.py (bench.py --workload kitti) times this object; tests/test_gpu_stereo_track.py
checks every frame and pair of its output against the CPU parity oracle.
"""
from __future__ import annotations

import sys

import numpy as np

from .extractor import ORBextractor
from .matcher import ORBmatcher, last_frame_table, update_last_frame_device


def th_depth(bf: float, fx: float, th_depth_factor: float = 35.0) -> float:
    """Tracking's mThDepth = mbf * (float)fSettings["ThDepth"] / fx (Tracking.cc), in float."""
    return float(np.float32(bf) * np.float32(th_depth_factor) / np.float32(fx))


class StereoSequencePipeline:
    def __init__(self, batch: int, width: int, height: int, fx: float, fy: float, cx: float, cy: float, bf: float,
                 params=(2000, 1.2, 8, 20, 7), track: bool = True, th: float = 7.0, nnratio: float = 0.9,
                 check_ori: bool = True, th_depth_factor: float = 35.0, max_d: float | None = None,
                 matcher_mode: int | None = None, device: int = 0, level0_in_place: bool = True,
                 retry_below: int = 20, nsets: int = 4, lane_offset_stage: int = 2, track_stream: bool = True):
        import torch

        from .extractor import stream_create
        self.B, self.W, self.H = int(batch), int(width), int(height)
        self.fx, self.fy, self.cx, self.cy, self.bf = float(fx), float(fy), float(cx), float(cy), float(bf)
        self.b = float(np.float32(bf) / np.float32(fx))  # mb = mbf / fx (Frame.cc:61)
        self.max_d = float(fx) if max_d is None else float(max_d)  # maxD = mbf / minZ, minZ = mb
        self.th, self.track = float(th), bool(track)
        self.retry_below = int(retry_below)  # TrackWithMotionModel's 2*th search below 20 matches (Tracking.cc:988-994)
        self.th_depth = th_depth(bf, fx, th_depth_factor)
        self.dev = torch.device("cuda", device)
        # the matcher stream first: HIP assigns hardware queues in stream-creation order, and
        # a stream created after the extractors' can share one with an extraction stream
        # 
        self._own_ms = stream_create(device, 1, 0)
        self.ms = torch.cuda.ExternalStream(self._own_ms, device=self.dev)
        # UpdateLastFrame + the search on a stream of their own, so step k's tracking runs
        # beside step k+1's stereo matching (as the keyframe stream's triangulation does).
        # With two extractor pairs and no lane offset it measured 1-2 % slower (r05bd); with
        # the offset and four pairs it is the faster form (r05ca-cc, interleaved: three pairs
        # on one stream 57.0-58.0k stereo frames/s, on two 58.4-59.3k, four pairs on two
        # 59.8-60.7k, five 59.8-60.0k).  track_stream False: one stream
        self._own_ts = stream_create(device, 1, 0) if track_stream else None
        self.ts = torch.cuda.ExternalStream(self._own_ts, device=self.dev) if self._own_ts else self.ms
        # extractor pairs in rotation: a set is re-extracted only after the matching that last
        # read it (ev_m).  Four: with the right image's lane offset (below) the matching no
        # longer keeps up with two (r05bq-br, one matcher stream, interleaved: two sets
        # 54.7-54.9k stereo frames/s, three 57.2-58.2k, four 56.6-57.6k; before the offset
        # three measured 0.8 % slower, r05ap), and with the tracking on its own stream four
        # beat three (above)
        self.nsets = max(2, int(nsets))
        self.sets = [(ORBextractor(*params, device=device), ORBextractor(*params, device=device))
                     for _ in range(self.nsets)]
        # level 0 read from the caller's frames when their rows are 64-byte aligned
        # (extractor.device_frames): no copy into the pyramid, and ComputeStereoMatches'
        # octave-0 SAD windows read it there (orbx_extractor_set_level0_in_place)
        for pair in self.sets:
            for e in pair:
                e.set_level0_in_place(level0_in_place)
        # lane offset: the right image's extraction starts once the left one's has passed
        # stage 2 (blur + FAST strength), as the monocular pipeline's lanes, so the two run
        # out of phase instead of in step (r05bm, interleaved: 53.6-54.0k in step, 54.6-55.1k
        # after stage 2, 54.0-55.1k after stage 3, 53.1-53.9k after stage 1).
        # lane_offset_stage 0: in step
        lo = int(lane_offset_stage)
        self.lane_ev = [a.set_stage_event(lo) for a, _ in self.sets] if lo > 0 else None
        self.smatcher = ORBmatcher(0.6, True, device=device)  # ComputeStereoMatches' handle (stream, arena)
        self.tmatcher = ORBmatcher(nnratio, check_ori, device=device)  # TrackWithMotionModel: ORBmatcher(0.9, true)
        self.tmatcher.set_footprint(5 if matcher_mode is None else matcher_mode)
        self.sf = self.sets[0][0].GetScaleFactors()
        self.cap = self.sets[0][0].max_keypoints(self.W, self.H)
        B, cap = self.B, self.cap
        i32 = dict(dtype=torch.int32, device=self.dev)
        f32 = dict(dtype=torch.float32, device=self.dev)
        u8 = dict(dtype=torch.uint8, device=self.dev)
        self.buf = [{"kl": torch.empty((B, cap, 7), **i32), "dl": torch.empty((B, cap, 32), **u8),
                     "nl": torch.empty((B,), **i32), "kr": torch.empty((B, cap, 7), **i32),
                     "dr": torch.empty((B, cap, 32), **u8), "nr": torch.empty((B,), **i32),
                     "ur": torch.empty((B, cap), **f32), "dp": torch.empty((B, cap), **f32),
                     "mp": torch.empty((B, cap), **i32), "nm": torch.empty((B,), **i32),
                     **last_frame_table(B, cap, self.dev)} for _ in range(self.nsets)]
        self.streams = [(torch.cuda.ExternalStream(a.stream_handle(), device=self.dev),
                         torch.cuda.ExternalStream(c.stream_handle(), device=self.dev)) for a, c in self.sets]
        self.ev_l = [torch.cuda.Event() for _ in range(self.nsets)]
        self.ev_r = [torch.cuda.Event() for _ in range(self.nsets)]
        self.ev_m = [torch.cuda.Event() for _ in range(self.nsets)]
        self.ev_s = [torch.cuda.Event() for _ in range(self.nsets)]  # a set's stereo matching done
        self.used = [False] * self.nsets
        self.it = 0
        self.last = None
        self._timing = False
        self._st = []  # (stereo start, track start, end) events while timing
        from . import _lib
        _lib.track(self)

    def close(self):
        """Wait for this pipeline's work, then release its matchers, its extractor pairs and
        the streams it created (idempotent)."""
        from .extractor import release_owned
        release_owned(self, streams=[getattr(self, "ts", None), getattr(self, "ms", None)],
                      owners=[getattr(self, "smatcher", None), getattr(self, "tmatcher", None),
                              *(e for pair in getattr(self, "sets", []) for e in pair)],
                      own_streams=["_own_ts", "_own_ms"])

    def __del__(self, _finalizing=sys.is_finalizing):
        if not _finalizing():
            try:
                self.close()
            except Exception:
                pass

    def step(self, d_left, d_right, d_Tcw=None, obs_in=None, pos_in=None):
        """Issue one step (asynchronous): B stereo frames d_left / d_right (B, H, W) u8 with
        poses d_Tcw (B, 12) f32 (needed when tracking); obs_in (B, cap) i32 / pos_in
        (B, cap, 3) f32: the MapPoints each frame already tracks as a LastFrame (-1 = none)
        or None.  Inputs must stay untouched until the step's matching is done."""
        import torch

        k = self.it % self.nsets
        (exl, exr), (sl, sr), bk = self.sets[k], self.streams[k], self.buf[k]
        if self.used[k]:  # the matching that last read this set's pyramids is done
            sl.wait_event(self.ev_m[k])
            sr.wait_event(self.ev_m[k])
        exl.extract_batch_device(d_left, bk["kl"], bk["dl"], bk["nl"])
        if self.lane_ev:
            from .extractor import stream_wait_event
            stream_wait_event(sr.cuda_stream, self.lane_ev[k])
        exr.extract_batch_device(d_right, bk["kr"], bk["dr"], bk["nr"])
        self.ev_l[k].record(sl)
        self.ev_r[k].record(sr)
        self.ms.wait_event(self.ev_l[k])
        self.ms.wait_event(self.ev_r[k])
        if self._timing:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(self.ms)
        self.smatcher.ComputeStereoMatchesBatchDevice(exl, exr, bk["kl"], bk["dl"], bk["nl"], bk["kr"], bk["dr"],
                                                      bk["nr"], self.bf, self.max_d, bk["ur"], bk["dp"],
                                                      stream=self.ms)
        if self._timing:
            ev[1].record(self.ms)
        if self.ts is not self.ms:
            self.ev_s[k].record(self.ms)
            self.ts.wait_event(self.ev_s[k])
        if self.track:
            if d_Tcw is None:
                raise ValueError("tracking needs the frames' poses")
            self._last_T = d_Tcw
            s = self.ts.cuda_stream
            update_last_frame_device(bk["kl"], bk["nl"], bk["dp"], d_Tcw, self.fx, self.fy, self.cx, self.cy,
                                     self.th_depth, bk, d_obs_in=obs_in, d_pos_in=pos_in, stream=s)
            self.tmatcher.match_sequence_device_ex(
                bk["kl"], bk["dl"], bk["nl"], d_Tcw, bk["mp"], bk["nm"], self.sf, self.fx, self.fy, self.cx, self.cy,
                self.W, self.H, th=self.th, mono=False, bf=self.bf, b=self.b, d_u_right=bk["ur"],
                d_mp_pos=bk["mp_pos"], d_has_mp=bk["has_mp"], d_mp_obs=bk["mp_obs"], global_ids=True,
                retry_below=self.retry_below, stream=s)
        if self._timing:
            ev[2].record(self.ts)
            self._st.append(ev)
        self.ev_m[k].record(self.ts)  # after the stereo matching (waited for) and the tracking
        self.used[k] = True
        self.last = k
        self.it += 1

    def tracked_from(self, mask, observations: int = 2, k=None):
        """(obs_in, pos_in) for step(): every slot of `mask` ((B, cap) bool, host or device)
        whose keypoint has a depth in set k's newest results (default: the newest step's)
        carries a tracked MapPoint with `observations` at its UnprojectStereo position
        (orbx_create_mappoints_device) -- a LastFrame's map MapPoints, made once at setup for
        a batch that is stepped repeatedly (call after synchronising)."""
        import torch

        from .matcher import create_mappoints_device, mappoint_table
        k = self.last if k is None else k
        bk = self.buf[k]
        tab = mappoint_table(self.B, self.cap, self.dev)
        T = getattr(self, "_last_T", None)
        if T is None:
            raise ValueError("tracked_from needs a step with poses first")
        create_mappoints_device(bk["kl"], bk["nl"], T, self.sf, self.fx, self.fy, self.cx, self.cy, tab,
                                d_depth=bk["dp"], stream=self.ms.cuda_stream)
        self.ms.synchronize()
        m = torch.as_tensor(np.asarray(mask.cpu() if hasattr(mask, "cpu") else mask), device=self.dev).bool()
        obs = torch.where(m & (bk["dp"] > 0), torch.tensor(int(observations), dtype=torch.int32, device=self.dev),
                          torch.tensor(-1, dtype=torch.int32, device=self.dev)).contiguous()
        return obs, tab["pos"].view(self.B, self.cap, 3).contiguous()

    def set_timing(self, enable: bool):
        for ex in (e for st in self.sets for e in st):
            ex.set_timing(enable)
        self._timing = bool(enable)
        self._st = []

    def stage_times(self) -> dict:
        """HIP-event ms per launch: the extraction stages (averaged over every extractor's
        launches, left and right), "stereo" and "track" (UpdateLastFrame + the search)."""
        from ._lib import OrbxError
        per = []
        for e in (e for st in self.sets for e in st):
            try:
                per.append(e.stage_times())
            except OrbxError:  # a set not reached by the timed steps (fewer steps than sets)
                pass
        out = {s: sum(p[s] for p in per) / len(per) for s in per[0]}
        if self._st:
            out["stereo"] = sum(a.elapsed_time(b) for a, b, _ in self._st) / len(self._st)
            if self.track:
                out["track"] = sum(b.elapsed_time(c) for _, b, c in self._st) / len(self._st)
        return out

    def status_clean(self, k=None) -> bool:
        k = self.last if k is None else k
        return not any(ex.status().any() for ex in self.sets[k])

    def host_results(self, k=None) -> dict:
        """Host copies of set k's (default: the newest step's) outputs (call after synchronising)."""
        from . import _lib as L
        k = self.last if k is None else k
        bk = self.buf[k]
        B, cap = self.B, self.cap
        kp = lambda t: t.cpu().numpy().view(np.uint8).reshape(B, cap, 28).view(L.KEYPOINT_DTYPE).reshape(B, cap)  # noqa
        out = {"kl": kp(bk["kl"]), "kr": kp(bk["kr"])}
        for name in ("dl", "dr", "nl", "nr", "ur", "dp", "mp", "nm", "mp_obs", "mp_pos", "has_mp"):
            out[name] = bk[name].cpu().numpy()
        return out
