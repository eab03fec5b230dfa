"""Whole-batch parity checks of the batched device paths against the oracle.

TEST INFRASTRUCTURE ONLY (used by tests/, bench.py's parity leg and smoke()): every
frame of a batch is re-extracted by the C restatement and every matched pair re-run
through its SearchByProjection(Frame&, const Frame&, th, bMono) (ORBmatcher.cc:
1620-1789), in a thread pool (the oracle's ctypes calls release the GIL).
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import oracle as O


def _threads(threads):
    return threads or max(1, min(16, len(os.sched_getaffinity(0))))


def extract_all(frames: np.ndarray, params=(1000, 1.2, 8, 20, 7), threads: int = 0):
    """Oracle extraction of every frame -> list of (keypoints, descriptors)."""
    O.build()
    p = O.params(*params)

    def one(img):
        k, d, _ = O.extract(img, p)
        return k, d

    with ThreadPoolExecutor(_threads(threads)) as ex:
        return list(ex.map(one, frames))


def compare_extraction(ref, kps, desc, n) -> list[int]:
    """Frames whose device keypoints (all 28 bytes) / descriptors differ from `ref`."""
    bad = []
    for b, (kr, dr) in enumerate(ref):
        m = int(n[b])
        if m != len(kr):
            bad.append(b)
            continue
        kg = kps[b, :m].view(np.uint8).reshape(m, 28)
        if not (np.array_equal(kg, kr.view(np.uint8).reshape(m, 28)) and np.array_equal(desc[b, :m], dr)):
            bad.append(b)
    return bad


def sequence_matches(ref, T: np.ndarray, sf, fx=500.0, fy=500.0, cx=320.0, cy=240.0, W=640, H=480, depth=5.0,
                     th=15.0, check_ori=True, threads: int = 0, retry: bool = True):
    """Oracle TrackWithMotionModel matching of frame b against b-1 for every b >= 1, on
    the oracle's own extraction `ref`, with the MapPoints orbx_match_sequence_device
    defines (every last-frame keypoint i is MapPoint i at `depth` on its ray); retry: the
    second search at 2*th below 20 matches (SequencePipeline's default), else one search
    (orbx_match_sequence_device)."""
    from orbslam2commentedbyxcm_amd.matcher import FrameView, MapPoints
    F32 = np.float32

    def view(k, d, t):
        return FrameView(keys=k, desc=d, fx=fx, fy=fy, cx=cx, cy=cy, max_x=float(W), max_y=float(H),
                         scale_factors=sf, Tcw=np.vstack([t.reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32))

    def one(b):
        (lk, ld), (ck, cd) = ref[b - 1], ref[b]
        Tl = T[b - 1]
        xc0 = (lk["x"] - F32(cx)) / F32(fx) * F32(depth)
        xc1 = (lk["y"] - F32(cy)) / F32(fy) * F32(depth)
        xc2 = np.full(len(lk), F32(depth), np.float32)
        Xw = np.stack([Tl[c] * (xc0 - Tl[3]) + Tl[4 + c] * (xc1 - Tl[7]) + Tl[8 + c] * (xc2 - Tl[11])
                       for c in range(3)], 1).astype(np.float32)
        mps = MapPoints(desc=ld, observations=np.ones(len(lk), np.int32), pos=Xw)
        cur = np.full(len(ck), -1, np.int32)
        if retry:  # TrackWithMotionModel: again at 2*th below 20 matches (Tracking.cc:988-994)
            nr, _ = O.track_motion_model(view(ck, cd, T[b]), cur, view(lk, ld, Tl), np.arange(len(lk), dtype=np.int32),
                                         mps, th, True, check_ori)
        else:
            nr = O.sbp_frame(view(ck, cd, T[b]), cur, view(lk, ld, Tl), np.arange(len(lk), dtype=np.int32), mps, th,
                             True, check_ori)
        return nr, cur

    with ThreadPoolExecutor(_threads(threads)) as ex:
        return [None] + list(ex.map(one, range(1, len(ref))))


def check_sequence(frames: np.ndarray, T: np.ndarray, res: dict, sf, threads: int = 0,
                   params=(1000, 1.2, 8, 20, 7), **kw) -> dict:
    """Every frame's extraction and every pair's matches of a SequencePipeline result
    (host copies: kps, desc, n, mp, nm) against the oracle."""
    ref = extract_all(frames, params=params, threads=threads)
    bad_frames = compare_extraction(ref, res["kps"], res["desc"], res["n"])
    out = {"frames_checked": len(frames), "frames_mismatched": len(bad_frames), "first_bad_frames": bad_frames[:8]}
    if "mp" in res:
        mref = sequence_matches(ref, T, sf, threads=threads, **kw)
        bad_pairs = []
        for b in range(1, len(frames)):
            nr, cur = mref[b]
            m = int(res["n"][b])
            if int(res["nm"][b]) != nr or not np.array_equal(res["mp"][b, :m], cur):
                bad_pairs.append(b)
        ok0 = int(res["nm"][0]) == 0 and bool((res["mp"][0] == -1).all())
        out.update({"pairs_checked": len(frames) - 1, "pairs_mismatched": len(bad_pairs) + (0 if ok0 else 1),
                    "first_bad_pairs": bad_pairs[:8],
                    "mean_matches_per_pair_ref": float(np.mean([mref[b][0] for b in range(1, len(frames))]))
                    if len(frames) > 1 else 0.0})
    out["bit_exact"] = out["frames_mismatched"] == 0 and out.get("pairs_mismatched", 0) == 0
    return out


def sequence_local(ref, T: np.ndarray, sf, cap: int, local_window: int = 3, fx=500.0, fy=500.0, cx=320.0, cy=240.0,
                   W=640, H=480, depth=5.0, th=15.0, local_th=1.0, threads: int = 0):
    """Oracle of SequencePipeline(local_map=True) on the oracle's own extraction `ref`:
    every keypoint's MapPoint (ora_create_mappoints at `depth`, id f*cap + i), then per
    frame b >= 1 TrackWithMotionModel's SearchByProjection against frame b-1's MapPoints
    (ORBmatcher(0.9, true)) and Tracking::SearchLocalPoints against the MapPoints of frames
    b-1 .. b-local_window (ORBmatcher(0.8)).  -> per frame (nm, nm_local, frame_mp)."""
    from orbslam2commentedbyxcm_amd.matcher import FrameView, MapPoints
    B = len(ref)
    N = B * cap

    def view(k, d, t):
        return FrameView(keys=k, desc=d, fx=fx, fy=fy, cx=cx, cy=cy, max_x=float(W), max_y=float(H),
                         scale_factors=sf, Tcw=np.vstack([t.reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32))

    pos = np.zeros((N, 3), np.float32)
    nrm = np.zeros((N, 3), np.float32)
    mx = np.zeros(N, np.float32)
    mn = np.zeros(N, np.float32)
    desc = np.zeros((N, 32), np.uint8)
    bad = np.ones(N, np.uint8)
    for f, (k, d) in enumerate(ref):
        m = O.create_mappoints(view(k, d, T[f]), const_depth=depth)
        sl = slice(f * cap, f * cap + len(k))
        pos[sl], nrm[sl], mx[sl], mn[sl] = m["pos"], m["normal"], m["max_distance"], m["min_distance"]
        desc[sl] = d
        bad[sl] = 1 - m["valid"]
    obs = (1 - bad).astype(np.int32)
    mps = MapPoints(desc=desc, observations=obs, pos=pos, bad=bad, max_distance=mx, min_distance=mn, normal=nrm)

    def one(b):
        (lk, ld), (ck, cd) = ref[b - 1], ref[b]
        cur = np.full(len(ck), -1, np.int32)
        last_mp = np.where(bad[(b - 1) * cap:(b - 1) * cap + len(lk)] == 0,
                           np.arange((b - 1) * cap, (b - 1) * cap + len(lk)), -1).astype(np.int32)
        nm, _ = O.track_motion_model(view(ck, cd, T[b]), cur, view(lk, ld, T[b - 1]), last_mp, mps, th, True, True)
        ids = np.concatenate([np.arange(f * cap, (f + 1) * cap, dtype=np.int32)
                              for f in range(max(0, b - local_window), b)])
        nl = O.search_local_points(view(ck, cd, T[b]), cur, ids, mps, local_th, 0.8)
        return nm, nl, cur

    with ThreadPoolExecutor(_threads(threads)) as ex:
        return [None] + list(ex.map(one, range(1, B)))


def check_sequence_local(frames: np.ndarray, T: np.ndarray, res: dict, sf, cap: int, threads: int = 0,
                         params=(1000, 1.2, 8, 20, 7), **kw) -> dict:
    """A SequencePipeline(local_map=True) result (kps, desc, n, mp, nm, nm_local) against
    sequence_local: every frame's extraction and every frame's final mvpMapPoints."""
    ref = extract_all(frames, params=params, threads=threads)
    bad_frames = compare_extraction(ref, res["kps"], res["desc"], res["n"])
    out = {"frames_checked": len(frames), "frames_mismatched": len(bad_frames), "first_bad_frames": bad_frames[:8]}
    mref = sequence_local(ref, T, sf, cap, threads=threads, **kw)
    bad_pairs = []
    for b in range(1, len(frames)):
        nm, nl, cur = mref[b]
        m = int(res["n"][b])
        if int(res["nm"][b]) != nm or int(res["nm_local"][b]) != nl or not np.array_equal(res["mp"][b, :m], cur):
            bad_pairs.append(b)
    out.update({"pairs_checked": len(frames) - 1, "pairs_mismatched": len(bad_pairs), "first_bad_pairs": bad_pairs[:8],
                "mean_matches_per_pair_ref": float(np.mean([mref[b][0] for b in range(1, len(frames))])),
                "mean_local_matches_ref": float(np.mean([mref[b][1] for b in range(1, len(frames))]))})
    out["bit_exact"] = out["frames_mismatched"] == 0 and out["pairs_mismatched"] == 0
    return out
