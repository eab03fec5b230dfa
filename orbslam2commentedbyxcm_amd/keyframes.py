"""Frame-sharded stereo keyframe stream with the cross-keyframe exchange (configs[3]).

One step on every rank = for its B stereo keyframes of a W*B-keyframe window:

1. the stereo Frame constructor's hot path (Frame.cc:99-178): mpORBextractorLeft and
   mpORBextractorRight on two streams (orbx_extract_batch_device), then
   ComputeStereoMatches (Frame.cc:673-885, orbx_compute_stereo_matches_batch_device);
2. KeyFrame::ComputeBoW (KeyFrame.cc:66-74): the DBoW2 FeatureVector at levelsup 4
   (orbx_vocabulary_transform_batch_device);
3. the MapPoints a stereo keyframe is born with (Tracking::CreateNewKeyFrame,
   Tracking.cc:1069-1121: every stereo point closer than mThDepth gets one);
4. the exchange: every rank's keyframe slab -- keypoints, descriptors, mvuRight,
   has-MapPoint flags, FeatureVector -- is all-gathered device to device
   (``all_gather_into_tensor`` on RCCL over xGMI; one contiguous slab per rank, no
   packing);
5. LocalMapping::CreateNewMapPoints' matching loop (LocalMapping.cc:235-305) for each
   local keyframe against its covisible neighbours, which live on the other ranks
   (keyframe g of the window is on rank g % W): the baseline test (cc:270-283), F12
   (ComputeF12, cc:606-625) and SearchForTriangulation (ORBmatcher.cc:850-1056) of every
   pair in one launch (orbx_search_for_triangulation_batch_device), ORBmatcher(0.6, false).

Step k+1's extraction overlaps step k's stereo / BoW / gather / triangulation: sets of
extractor pairs, slabs, gathered buffers and triangulation outputs rotate (four by
default, `nsets`), and a set is reused only after the triangulation that last read
it (its event) -- so the gather of a later step never overwrites neighbours that an
earlier step's triangulation is still reading.  `windows` > 1 gives each step its own keyframe window
(same poses, another texture), so a cross-step ordering fault changes bytes.  The neighbour plan (covisibility proxy: the nn
keyframes whose views overlap most, then the baseline skip) depends only on the poses and
is made once on the host, as LocalMapping does per keyframe.

benchmarks/euroc_bench.py (bench.py --workload euroc) times this object;
tests/test_gpu_keyframes.py checks its output against the CPU parity oracle (also through
a one-rank RCCL group with collective=True, the all_gather_into_tensor path), and
tests/test_distributed.py covers the layout, the plan and the gather at world size 2 on
gloo.
"""
from __future__ import annotations

import sys
from dataclasses import dataclass

import numpy as np

# EuRoC stereo settings (the public ORB-SLAM2 Examples/Stereo/EuRoC.yaml; the
# reference tree ships no settings files): rectified 752x480, 1200 features.
EUROC = dict(width=752, height=480, nfeatures=1200, scale=1.2, nlevels=8, ini_th=20, min_th=7,
             fx=435.2046959714599, fy=435.2046959714599, cx=367.4517211914062, cy=252.2008514404297,
             bf=47.90639384423901, th_depth=35.0)

KP_BYTES = 28  # orbx_keypoint / cv::KeyPoint


def _al(x: int) -> int:
    return (x + 255) & ~255


class SlabLayout:
    """Byte layout of one rank's keyframe slab: B keyframes, each field a [B][...] array
    in the batched calls' layouts, every field 256-B aligned.  The gathered buffer is W
    slabs back to back, so keyframe (rank q, local i) sits at q * nbytes + field offset
    + i * field stride."""

    FIELDS = (  # name, bytes per keyframe as a function of cap, numpy dtype, trailing shape
        ("kps", lambda c: c * KP_BYTES, np.int32, lambda c: (c, 7)),
        ("desc", lambda c: c * 32, np.uint8, lambda c: (c, 32)),
        ("n", lambda c: 4, np.int32, lambda c: ()),
        ("u_right", lambda c: c * 4, np.float32, lambda c: (c,)),
        ("has_mp", lambda c: c, np.uint8, lambda c: (c,)),
        ("fv_node", lambda c: c * 4, np.int32, lambda c: (c,)),
        ("fv_off", lambda c: (c + 1) * 4, np.int32, lambda c: (c + 1,)),
        ("fv_idx", lambda c: c * 4, np.int32, lambda c: (c,)),
        ("nfv", lambda c: 4, np.int32, lambda c: ()),
    )

    def __init__(self, batch: int, cap: int):
        self.B, self.cap = int(batch), int(cap)
        self.offset, self.stride = {}, {}
        o = 0
        for name, per, _, _ in self.FIELDS:
            self.offset[name] = o
            self.stride[name] = per(self.cap)
            o = _al(o + self.B * per(self.cap))
        self.nbytes = o

    def views(self, slab) -> dict:
        """Typed [B, ...] views (torch tensors) into a uint8 slab tensor."""
        import torch

        tdt = {np.int32: torch.int32, np.uint8: torch.uint8, np.float32: torch.float32}
        out = {}
        for name, per, dt, shp in self.FIELDS:
            o, nb = self.offset[name], self.B * per(self.cap)
            out[name] = slab[o:o + nb].view(tdt[dt]).view((self.B,) + shp(self.cap))
        return out

    def address(self, base: int, rank: int, local: int, name: str) -> int:
        return base + rank * self.nbytes + self.offset[name] + local * self.stride[name]

    def records(self, base: int, world: int, poses) -> list:
        """orbx_keyframe_device records of every keyframe of a gathered buffer at device
        address `base`, in record order rank * B + local; poses[rank * B + local] is
        that keyframe's host Tcw."""
        from .matcher import keyframe_device

        recs = []
        for q in range(world):
            for i in range(self.B):
                a = {name: self.address(base, q, i, name) for name, *_ in self.FIELDS}
                recs.append(keyframe_device(a["kps"], a["desc"], a["n"], a["has_mp"], a["fv_node"], a["fv_off"],
                                            a["fv_idx"], a["nfv"], poses[q * self.B + i], a["u_right"]))
        return recs


def window_index(rank: int, local: int, world: int) -> int:
    """Keyframe g of the step window lives on rank g % world as local g // world."""
    return local * world + rank


def record_index(g: int, world: int, batch: int) -> int:
    return (g % world) * batch + g // world


@dataclass
class NeighbourPlan:
    pairs: np.ndarray    # (P, 2) record indices (KF1 = a local keyframe, KF2 = a neighbour)
    F12: np.ndarray      # (P, 3, 3) float32
    kf1_window: np.ndarray  # (P,) window index of KF1
    kf2_window: np.ndarray  # (P,) window index of KF2
    skipped_baseline: int


def compute_f12(T1, T2, fx, fy, cx, cy) -> np.ndarray:
    from .distributed import compute_f12 as f
    return f(T1, T2, fx, fy, cx, cy)


def plan_neighbours(poses: np.ndarray, rank: int, world: int, batch: int, nn: int, mb: float,
                    cam: dict) -> NeighbourPlan:
    """For each keyframe of this rank: GetBestCovisibilityKeyFrames(nn) proxied by
    stream adjacency (the nn keyframes of the window nearest in stream order, the earlier
    one first on a tie: g-1, g+1, g-2, ...), the stereo baseline skip `baseline <
    pKF2->mb` (LocalMapping.cc:270-276), and F12 (LocalMapping.cc:606-625).  Per-rank
    work does not depend on the world size (bar the window ends).  poses: (W*B, 3|4, 4)
    Tcw by window index."""
    N = world * batch
    pairs, F, k1, k2 = [], [], [], []
    skipped = 0
    centres = [-(np.asarray(T, np.float32)[:3, :3].T @ np.asarray(T, np.float32)[:3, 3]) for T in poses]
    for i in range(batch):
        g = window_index(rank, i, world)
        order = sorted((abs(h - g), h) for h in range(N) if h != g)[:nn]
        for _, h in order:
            base = np.asarray(centres[h] - centres[g], np.float32)
            if float(np.sqrt(np.sum(base.astype(np.float64) ** 2))) < mb:
                skipped += 1
                continue
            pairs.append((record_index(g, world, batch), record_index(h, world, batch)))
            F.append(compute_f12(poses[g][:3], poses[h][:3], cam["fx"], cam["fy"], cam["cx"], cam["cy"]))
            k1.append(g)
            k2.append(h)
    return NeighbourPlan(np.array(pairs, np.int32).reshape(-1, 2), np.array(F, np.float32).reshape(-1, 3, 3),
                         np.array(k1, np.int64), np.array(k2, np.int64), skipped)


def stream_poses(off: np.ndarray, fx: float, fy: float, depth: float) -> np.ndarray:
    """Tcw (4x4) of each view of synth.StereoSequence: a translation that shifts the
    plane at `depth` by off pixels."""
    T = np.tile(np.eye(4, dtype=np.float32), (len(off), 1, 1))
    T[:, 0, 3] = -off[:, 0] * depth / fx
    T[:, 1, 3] = -off[:, 1] * depth / fy
    return T


def gather_slabs(slab, gathered, group=None, force: bool = False, async_op: bool = False):
    """Every rank's slab into `gathered` (world x slab bytes), rank order.  RCCL:
    one all_gather_into_tensor, device to device, enqueued behind the current stream's
    work (ProcessGroupNCCL's stream waits on it).  async_op False: the current stream
    waits on the collective before anything enqueued after it; True: nothing waits yet --
    the returned work handle's wait() makes the stream current at that point wait (the
    triangulation stream, so the matcher stream runs on past the exchange).  gloo (the
    CPU tests, and the several-ranks-on-one-GPU rehearsal): all_gather, staged through
    host memory for device tensors, synchronous.  World size 1 is a device copy unless
    `force`, which issues the collective anyway (the one-GPU hardware test of the RCCL
    path).  Returns the pending work handle or None."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    if world == 1 and not force:
        if gathered.data_ptr() != slab.data_ptr():
            gathered.copy_(slab)
        return None
    if slab.is_cuda and dist.get_backend(group) != "gloo":
        work = dist.all_gather_into_tensor(gathered, slab, group=group, async_op=async_op)
        return work if async_op else None
    src = slab.cpu() if slab.is_cuda else slab
    dst = gathered.new_empty(gathered.shape, device="cpu") if gathered.is_cuda else gathered
    dist.all_gather(list(dst.view(world, -1).unbind(0)), src, group=group)
    if dst is not gathered:
        gathered.copy_(dst)
    return None


class StereoKeyFramePipeline:
    """Device-resident configs[3] step for one rank (see the module docstring)."""

    def __init__(self, batch: int, rank: int = 0, world: int = 1, device: int = 0, nn: int = 10, seq_seed: int = 3,
                 vocab_text: bytes | None = None, settings: dict | None = None, group=None, windows: int = 1,
                 on_step_done=None, collective: bool = False, level0_in_place: bool = True, nsets: int = 4,
                 lane_offset_stage: int = 3, gather_async: bool = True):
        import torch

        from . import synth
        from .extractor import ORBextractor
        from .matcher import FrameView, ORBmatcher
        from .vocabulary import ORBVocabulary

        s = dict(EUROC if settings is None else settings)
        self.s, self.B, self.rank, self.world, self.group = s, int(batch), int(rank), int(world), group
        # collective: the slab exchange runs through the process group even at world size 1
        # (a one-rank RCCL all_gather_into_tensor into its own gathered buffers), so the
        # N-GPU data path -- collective, gathered buffers, keyframe tables into them -- is
        # the one under test on a single GPU; world > 1 always exchanges
        self.collective = self.world > 1 or bool(collective)
        # the exchange's work handle is waited for on the triangulation stream only
        # (gather_async False: the round-4 order, the matcher stream waits for it)
        self.gather_async = bool(gather_async)
        self.W, self.H = s["width"], s["height"]
        self.dev = torch.device("cuda", device)
        self.mb = s["bf"] / s["fx"]
        self.th_depth = s["bf"] * s["th_depth"] / s["fx"]  # Tracking.cc:106 mThDepth = mbf * ThDepth / fx
        disp = 13  # plane depth bf / 13 = 3.69 m: inside mThDepth (3.85 m), so every stereo point is "close"
        self.depth = s["bf"] / disp
        N = self.world * self.B
        # keyframes ~13 px apart on average (a stereo baseline at this depth), so about half
        # of the g +- 1 neighbours fail LocalMapping's baseline test and the rest pass
        # window w: the same walk (poses, neighbour plan) over its own texture
        self.seqs = [synth.StereoSequence(seq_seed, N, self.W, self.H, step=16, margin=256, disp=disp,
                                          canvas_seed=seq_seed + 1000 * w if w else None)
                     for w in range(max(1, int(windows)))]
        self.seq = self.seqs[0]
        self.poses = stream_poses(self.seq.off, s["fx"], s["fy"], self.depth)
        self.local = [window_index(self.rank, i, self.world) for i in range(self.B)]
        views = [sq.views(self.local) for sq in self.seqs]
        self.left_np, self.right_np = views[0]
        prm = (s["nfeatures"], s["scale"], s["nlevels"], s["ini_th"], s["min_th"])
        # the matcher stream first: HIP assigns hardware queues in stream-creation order, and
        # a stream created after the extractors' (or from torch's pool) can share one with
        # an extraction stream
        from .extractor import stream_create
        self._own_ms = stream_create(device, 1)
        self.ms = torch.cuda.ExternalStream(self._own_ms, device=self.dev)
        # SearchForTriangulation on a stream of its own: the triangulation of step j runs
        # beside the stereo matching and BoW of step j + 1 instead of after them
        self._own_ts = stream_create(device, 1)
        self.ts = torch.cuda.ExternalStream(self._own_ts, device=self.dev)
        # extractor pairs / slabs in rotation: a set is rewritten only after the triangulation
        # that last read it (ev_m), so with two sets step j+1's extraction waited for step
        # j-1's triangulation -- the GPU idled between the steps' extractions.  Four sets
        # give it slack (r05ao-az, interleaved: two 48.6-49.6k, three 49.0-50.2k, four
        # 54.4-55.2k, five 52.8-54.5k, six and eight 50-52k keyframes/s: beyond four the
        # eight extractor streams outnumber the hardware queues)
        self.nsets = max(2, int(nsets))
        self.sets = [(ORBextractor(*prm, device=device), ORBextractor(*prm, device=device))
                     for _ in range(self.nsets)]
        # level 0 read in place from the pitched input frames below (no copy into the
        # pyramids; the stereo matching reads it there)
        for pair in self.sets:
            for e in pair:
                e.set_level0_in_place(level0_in_place)
        # lane offset: the right image's extraction starts once the left one's has passed
        # stage 3 (FAST cells), so the two run out of phase instead of in step (r05bn,
        # interleaved: in step 49.5-50.2k keyframes/s, after stage 2 49.4-51.9k, after
        # stage 3 50.6-52.5k; r05bo: after stage 3 49.4-51.2k against 48.4-51.2k after
        # stage 4).  lane_offset_stage 0: in step
        lo = int(lane_offset_stage)
        self.lane_ev = [a.set_stage_event(lo) for a, _ in self.sets] if lo > 0 else None
        self.sf = self.sets[0][0].GetScaleFactors()
        self.cap = self.sets[0][0].max_keypoints(self.W, self.H)
        self.stereo = ORBmatcher(0.6, True, device=device)
        self.tri = ORBmatcher(0.6, False, device=device)  # LocalMapping.cc:243
        self.voc = ORBVocabulary(device)
        if vocab_text is None:
            vocab_text = synth.vocabulary_text(7, 10, 6, 0, 0)
        self.vocab_text = vocab_text
        if not self.voc.loadFromText(vocab_text):
            raise RuntimeError("vocabulary rejected")
        from . import _lib
        _lib.track(self)
        self.lay = SlabLayout(self.B, self.cap)
        u8 = dict(dtype=torch.uint8, device=self.dev)
        i32 = dict(dtype=torch.int32, device=self.dev)
        self.slabs = [torch.zeros(self.lay.nbytes, **u8) for _ in range(self.nsets)]
        self.sv = [self.lay.views(sl) for sl in self.slabs]
        self.right = [{"kps": torch.empty((self.B, self.cap, 7), **i32),
                       "desc": torch.empty((self.B, self.cap, 32), **u8),
                       "n": torch.empty((self.B,), **i32),
                       "depth": torch.empty((self.B, self.cap), dtype=torch.float32, device=self.dev)}
                      for _ in range(self.nsets)]
        self.bow = [{"bow_word": torch.empty((self.B, self.cap), **i32),
                     "bow_value": torch.empty((self.B, self.cap), dtype=torch.float64, device=self.dev),
                     "nbow": torch.empty((self.B,), **i32)} for _ in range(self.nsets)]
        # one gathered buffer per set: step j+1's all-gather (set k') must not overwrite the
        # neighbours step j's triangulation (set k) is reading on the other stream
        self.gathered = [torch.zeros(self.world * self.lay.nbytes, **u8) for _ in range(self.nsets)] \
            if self.collective else None
        self.plan = plan_neighbours(self.poses, self.rank, self.world, self.B, nn, self.mb, s)
        P = max(len(self.plan.pairs), 1)
        self.m12 = [torch.empty((P, self.cap), **i32) for _ in range(self.nsets)]
        self.tri_pairs = [torch.empty((P, self.cap, 2), **i32) for _ in range(self.nsets)]
        self.tri_n = [torch.empty((P,), **i32) for _ in range(self.nsets)]
        win_poses = [None] * (self.world * self.B)
        for g in range(self.world * self.B):
            win_poses[record_index(g, self.world, self.B)] = self.poses[g]
        self._rec_poses = win_poses
        from . import _lib as L
        self.cam = FrameView(keys=np.zeros(0, L.KEYPOINT_DTYPE), desc=np.zeros((0, 32), np.uint8), fx=s["fx"],
                             fy=s["fy"], cx=s["cx"], cy=s["cy"], bf=s["bf"], b=self.mb, max_x=float(self.W),
                             max_y=float(self.H), scale_factors=self.sf, level_sigma2=self.sf * self.sf)
        self.streams = [(torch.cuda.ExternalStream(a.stream_handle(), device=self.dev),
                         torch.cuda.ExternalStream(b.stream_handle(), device=self.dev)) for a, b in self.sets]
        self.ev_l = [torch.cuda.Event() for _ in range(self.nsets)]
        self.ev_r = [torch.cuda.Event() for _ in range(self.nsets)]
        self.ev_m = [torch.cuda.Event() for _ in range(self.nsets)]
        self.ev_s = [torch.cuda.Event() for _ in range(self.nsets)]  # stereo + BoW (+ all-gather) of a set done
        self.used = [False] * self.nsets
        self.window_of = [0] * self.nsets  # the window each set last held
        # on_step_done(k): called after a step's triangulation is enqueued on self.ts and
        # before the event that releases set k -- consumer work enqueued on self.ts there
        # (e.g. copying the results out) finishes before the set is reused
        self.on_step_done = on_step_done
        self.it = 0
        self.last = 0
        from .extractor import device_frames
        self.inputs = [(device_frames(lf, self.dev), device_frames(rg, self.dev)) for lf, rg in views]
        self.d_left, self.d_right = self.inputs[0]
        torch.cuda.synchronize(self.dev)
        # the keyframe tables are fixed per buffer: build the ctypes arrays once
        from .matcher import keyframe_table
        bufs = self.gathered if self.collective else self.slabs
        self._tabs = [keyframe_table(self.lay.records(b.data_ptr(), self.world, self._rec_poses)) for b in bufs]

    def close(self):
        """Wait for this pipeline's work, then release its matchers, vocabulary, extractor
        pairs and the streams it created (idempotent)."""
        from .extractor import release_owned
        release_owned(self, streams=[getattr(self, "ts", None), getattr(self, "ms", None)],
                      owners=[getattr(self, "stereo", None), getattr(self, "tri", None), getattr(self, "voc", None),
                              *(e for pair in getattr(self, "sets", []) for e in pair)],
                      own_streams=["_own_ts", "_own_ms"])

    def __del__(self, _finalizing=sys.is_finalizing):
        if not _finalizing():
            try:
                self.close()
            except Exception:
                pass

    def step(self):
        """Issue one step (asynchronous)."""
        import torch

        k = self.it % self.nsets
        (exl, exr), (sl, sr) = self.sets[k], self.streams[k]
        v, rt, bw = self.sv[k], self.right[k], self.bow[k]
        if self.used[k]:  # the work that last read this set's pyramids, slab and gathered buffer is done
            sl.wait_event(self.ev_m[k])
            sr.wait_event(self.ev_m[k])
        w = self.it % len(self.inputs)
        self.window_of[k] = w
        d_left, d_right = self.inputs[w]
        exl.extract_batch_device(d_left, v["kps"], v["desc"], v["n"])
        if self.lane_ev:
            from .extractor import stream_wait_event
            stream_wait_event(sr.cuda_stream, self.lane_ev[k])
        exr.extract_batch_device(d_right, rt["kps"], rt["desc"], rt["n"])
        self.ev_l[k].record(sl)
        self.ev_r[k].record(sr)
        ms = self.ms
        ms.wait_event(self.ev_l[k])
        ms.wait_event(self.ev_r[k])
        s = self.s
        self.stereo.ComputeStereoMatchesBatchDevice(exl, exr, v["kps"], v["desc"], v["n"], rt["kps"], rt["desc"],
                                                    rt["n"], s["bf"], s["fx"], v["u_right"], rt["depth"], stream=ms)
        out = {"bow_word": bw["bow_word"], "bow_value": bw["bow_value"], "nbow": bw["nbow"],
               "fv_node": v["fv_node"], "fv_off": v["fv_off"], "fv_idx": v["fv_idx"], "nfv": v["nfv"]}
        self.voc.transform_batch_device(v["desc"], v["n"], self.cap, 4, out, stream=ms.cuda_stream)
        work = None
        with torch.cuda.stream(ms):
            # Tracking::CreateNewKeyFrame: a MapPoint for every stereo point closer than mThDepth
            torch.logical_and(v["u_right"] >= 0, rt["depth"] < self.th_depth, out=v["has_mp"].view(torch.bool))
            if self.collective:
                # off the matcher stream's path (round 5): the collective waits for this set's
                # slab, the triangulation stream waits for the collective, and the matcher
                # stream goes on to the next step's stereo matching meanwhile.  Reuse stays
                # ordered: the next exchange into gathered[k] is issued behind the matcher
                # stream's wait for set k's extraction, which waits for ev_m[k] -- this
                # step's triangulation, the buffer's last reader
                work = gather_slabs(self.slabs[k], self.gathered[k], self.group, force=True,
                                    async_op=self.gather_async)
        self.ev_s[k].record(ms)
        ts = self.ts
        ts.wait_event(self.ev_s[k])
        if work is not None:
            with torch.cuda.stream(ts):
                work.wait()
        if len(self.plan.pairs):
            self.tri.SearchForTriangulationBatchDevice(self._tabs[k], self.cam, self.plan.pairs, self.plan.F12,
                                                       self.cap, self.m12[k], self.tri_pairs[k], self.tri_n[k],
                                                       stream=ts)
        if self.on_step_done is not None:
            self.on_step_done(k)
        self.ev_m[k].record(ts)  # after the stereo, BoW and gather (waited for) and the triangulation
        self.used[k] = True
        self.last = k
        self.it += 1

    def run(self, steps: int):
        for _ in range(steps):
            self.step()

    def set_timing(self, enable: bool):
        for ex in (e for st in self.sets for e in st):
            ex.set_timing(enable)
        self.stereo.set_timing(enable)
        self.tri.set_timing(enable)

    def stage_times(self) -> dict:
        """HIP-event ms per launch: extraction stages averaged over the extractors (L and R
        of every set) that ran a timed extraction, the stereo matching and the triangulation."""
        from ._lib import OrbxError
        per = []
        for e in (e for st in self.sets for e in st):
            try:
                per.append(e.stage_times())
            except OrbxError:  # a set not reached by the timed steps (fewer steps than sets)
                pass
        st = {k: sum(p[k] for p in per) / len(per) for k in per[0]}
        st["stereo"] = self.stereo.last_ms()
        if len(self.plan.pairs):
            st["triangulation"] = self.tri.last_ms()
        return st

    def results(self, k=None) -> dict:
        """Device tensors of set k (default: the newest step's): every field the step
        writes, the triangulation outputs and (collective) the gathered buffer."""
        k = self.last if k is None else k
        v, rt = self.sv[k], self.right[k]
        P = len(self.plan.pairs)
        r = {"kps": v["kps"], "dl": v["desc"], "nl": v["n"], "kr": rt["kps"], "dr": rt["desc"], "nr": rt["n"],
             "ur": v["u_right"], "depth": rt["depth"], "has_mp": v["has_mp"], "fv_node": v["fv_node"],
             "fv_off": v["fv_off"], "fv_idx": v["fv_idx"], "nfv": v["nfv"], "tri_n": self.tri_n[k][:P],
             "tri_pairs": self.tri_pairs[k][:P]}
        if self.collective:
            r["gathered"] = self.gathered[k]
        return r

    def to_host(self, r: dict) -> dict:
        """Host form of results() (or of clones of it)."""
        from . import _lib as L
        B, cap = self.B, self.cap

        def kp(t):
            return t.cpu().numpy().view(np.uint8).reshape(B, cap, KP_BYTES).view(L.KEYPOINT_DTYPE).reshape(B, cap)

        out = {name: t.cpu().numpy() for name, t in r.items() if name not in ("kps", "kr")}
        out["kl"], out["kr"] = kp(r["kps"]), kp(r["kr"])
        return out

    def host_results(self) -> dict:
        """Host copies of the newest step's outputs (call after synchronising)."""
        return self.to_host(self.results())

    def status(self) -> bool:
        """True if every extraction of the newest step completed its octree."""
        return not any(ex.status().any() for ex in self.sets[self.last])
