"""configs[4]'s synthetic TUM RGB-D stream and its oracle: 640x480 gray + registered
16-bit depth frames of a textured plane along synth.tum_walk (hand-held motion, depths
1.6-3.9 m on both sides of mThDepth, motion along the optical axis beyond mb both ways),
rendered through TUM1's lens distortion, with Kinect-like depth holes; ORB settings of
configs[4] (5000 features, scale 1.2, 12 levels, FAST 20/7).

Shared by the RGB-D bench (bench.py --workload tum5k) and the GPU parity tests."""
from __future__ import annotations

import numpy as np

from orbslam2commentedbyxcm_amd import synth
from orbslam2commentedbyxcm_amd.matcher import FrameView, MapPoints

W, H = 640, 480
PARAMS = (5000, 1.2, 12, 20, 7)        # configs[4]: nFeatures=5000, 12 levels (TUM1.yaml: scale 1.2, FAST 20/7)
CAM = synth.TUM1
FX, FY, CX, CY = CAM["fx"], CAM["fy"], CAM["cx"], CAM["cy"]
DIST = CAM["dist"]                     # k1 k2 p1 p2 k3
K = [FX, FY, CX, CY]
BF = CAM["bf"]                         # Camera.bf
TH_DEPTH_FACTOR = CAM["th_depth"]      # ThDepth
DEPTH_MAP_FACTOR = CAM["depth_map_factor"]  # DepthMapFactor (the image stores metres x 5000)
# Tracking.cc:166-170: mDepthMapFactor = 1.0f / DepthMapFactor
M_DEPTH_MAP_FACTOR = float(np.float32(1.0) / np.float32(DEPTH_MAP_FACTOR))
Z0 = 2.2                               # the plane's distance from the reference camera
TH = 15.0                              # Tracking.cc:979-983: th = 15 unless STEREO
TRACKED_OBS = 2                        # Observations() of the MapPoints a LastFrame already tracks


def sequence(seed: int, n: int, workers: int = 1):
    """n RGB-D frames: (gray (n, H, W) u8, depth (n, H, W) u16, Tcw (n, 12) f32)."""
    rels = synth.tum_walk(seed, n, z0=Z0)
    gray, depth = synth.plane_rgbd_views(seed, rels, W, H, FX, FY, CX, CY, DIST, Z0,
                                         depth_map_factor=DEPTH_MAP_FACTOR, workers=workers)
    T = np.stack([np.asarray(r, np.float32)[:3, :4].reshape(12) for r in rels]).astype(np.float32)
    return gray, depth, T


def tracked_mask(seed: int, B: int, cap: int, frac: float = 0.5) -> np.ndarray:
    """Which keypoint slots of each LastFrame already carry a tracked map MapPoint (where
    they also have a depth): a seeded fraction."""
    return np.random.default_rng(seed + 77).random((B, cap)) < frac


def th_depth() -> float:
    return float(np.float32(BF) * np.float32(TH_DEPTH_FACTOR) / np.float32(FX))


def oracle_frame(O, p, sf, gray, depth, Tcw, bounds):
    """Oracle RGB-D Frame (Frame.cc:192-264): extraction, UndistortKeyPoints,
    ComputeStereoFromRGBD on the u16 image with mDepthMapFactor.  The view's keys are
    mvKeysUn (what the matchers read); .kd holds mvKeys."""
    kd, dl, _ = O.extract(gray, p)
    ku = O.undistort_keypoints(K, DIST, kd)
    ur, dp = O.compute_stereo_from_rgbd(kd, ku, depth, BF, M_DEPTH_MAP_FACTOR)
    T = np.vstack([np.asarray(Tcw, np.float32).reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32)
    v = FrameView(keys=ku, desc=dl, fx=FX, fy=FY, cx=CX, cy=CY, bf=BF, b=float(np.float32(BF) / np.float32(FX)),
                  min_x=float(bounds[0]), max_x=float(bounds[1]), min_y=float(bounds[2]), max_y=float(bounds[3]),
                  scale_factors=sf, level_sigma2=sf * sf, Tcw=T, u_right=ur)
    v.depth = dp
    v.kd = kd
    return v


def oracle_track(O, last, cur, tracked, th_depth_m, th=TH, check_ori=True):
    """UpdateLastFrame of `last` (its tracked slots carry MapPoints at UnprojectStereo with
    TRACKED_OBS observations) + TrackWithMotionModel's search (SearchByProjection(cur, last,
    th, bMono=false), again at 2*th below 20 matches).
    -> (cur_mp with ids = last keypoint index, nmatches, last's mp_obs, mp_pos, retried)."""
    n = len(last.keys)
    obs_in = np.where(tracked[:n] & (last.depth > 0), TRACKED_OBS, -1).astype(np.int32)
    pos_in = O.create_mappoints(last, last.depth)["pos"]
    obs, pos, _ = O.update_last_frame(last, last.depth, th_depth_m, obs_in, pos_in)
    last_mp = np.where(obs >= 0, np.arange(n), -1).astype(np.int32)
    mps = MapPoints(desc=last.desc, observations=np.maximum(obs, 0), pos=pos)
    ref = np.full(len(cur.keys), -1, np.int32)
    nm, retried = O.track_motion_model(cur, ref, last, last_mp, mps, th, False, check_ori)
    return ref, nm, obs, pos, retried
