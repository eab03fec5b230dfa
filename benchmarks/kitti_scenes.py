"""configs[2]'s synthetic KITTI stream and its oracle: rectified 1241x376 stereo pairs of a
textured plane along synth.kitti_walk (motion along the optical axis beyond the baseline
both ways, rolls, depths 12-28 m on both sides of mThDepth), KITTI 00-02's calibration.

Shared by benchmarks/stereo_bench.py (bench.py --workload kitti) and the GPU parity tests."""
from __future__ import annotations

import numpy as np

from orbslam2commentedbyxcm_amd import synth
from orbslam2commentedbyxcm_amd.matcher import FrameView, MapPoints

W, H, NF = 1241, 376, 2000
PARAMS = (NF, 1.2, 8, 20, 7)           # KITTI00-02.yaml: 2000 features, 1.2, 8 levels, FAST 20/7
FX = FY = 718.856                      # Camera.fx / fy
CX, CY = 607.1928, 185.2157            # Camera.cx / cy
BF = 386.1448                          # Camera.bf
TH_DEPTH_FACTOR = 35.0                 # ThDepth
Z0 = 15.0                              # the plane's distance from the reference camera
TRACKED_OBS = 2                        # Observations() of the MapPoints a LastFrame already tracks


def sequence(seed: int, n: int, workers: int = 1):
    """n stereo frames: (left (n, H, W) u8, right (n, H, W) u8, Tcw (n, 12) f32)."""
    rels = synth.kitti_walk(seed, n)
    left, right = synth.plane_stereo_views(seed, rels, BF / FX, W, H, FX, FY, CX, CY, Z0, workers=workers)
    T = np.stack([np.asarray(r, np.float32)[:3, :4].reshape(12) for r in rels]).astype(np.float32)
    return left, right, T


def tracked_mask(seed: int, B: int, cap: int, frac: float = 0.5) -> np.ndarray:
    """Which keypoint slots of each LastFrame already carry a tracked map MapPoint (where
    they also have a depth): a seeded fraction."""
    return np.random.default_rng(seed + 77).random((B, cap)) < frac


def oracle_frame(O, p, sf, left, right, Tcw):
    """Oracle stereo Frame: extraction of both images + ComputeStereoMatches (maxD = fx)."""
    kl, dl, _ = O.extract(left, p)
    kr, dr, _ = O.extract(right, p)
    T = np.vstack([np.asarray(Tcw, np.float32).reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32)
    v = FrameView(keys=kl, desc=dl, fx=FX, fy=FY, cx=CX, cy=CY, bf=BF, b=float(np.float32(BF) / np.float32(FX)),
                  max_x=float(W), max_y=float(H), scale_factors=sf, level_sigma2=sf * sf, Tcw=T)
    ur, dp = O.compute_stereo_matches(v, kr, dr, O.pyramid(left, p), O.pyramid(right, p), FX)
    v.u_right = ur
    v.depth = dp
    v.kr, v.dr = kr, dr
    return v


def oracle_track(O, last, cur, tracked, th_depth, th=7.0, check_ori=True):
    """UpdateLastFrame of `last` (its tracked slots carry MapPoints at UnprojectStereo with
    TRACKED_OBS observations) + TrackWithMotionModel's SearchByProjection(cur, last, th,
    bMono=false), again at 2*th below 20 matches.
    -> (cur_mp with ids = last keypoint index, nmatches, last's mp_obs, mp_pos)."""
    n = len(last.keys)
    obs_in = np.where(tracked[:n] & (last.depth > 0), TRACKED_OBS, -1).astype(np.int32)
    pos_in = O.create_mappoints(last, last.depth)["pos"]
    obs, pos, _ = O.update_last_frame(last, last.depth, th_depth, obs_in, pos_in)
    last_mp = np.where(obs >= 0, np.arange(n), -1).astype(np.int32)
    mps = MapPoints(desc=last.desc, observations=np.maximum(obs, 0), pos=pos)
    ref = np.full(len(cur.keys), -1, np.int32)
    nm, _ = O.track_motion_model(cur, ref, last, last_mp, mps, th, False, check_ori)  # retry at 2*th below 20
    return ref, nm, obs, pos
