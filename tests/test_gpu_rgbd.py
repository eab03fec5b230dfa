"""configs[4]'s RGB-D front end at its shape (640x480, 5000 features x 12 levels, TUM1
calibration with distortion, 16-bit depth at factor 5000 with holes) through
RGBDSequencePipeline -- extraction, UndistortKeyPoints + ComputeStereoFromRGBD
(Frame.cc:192-264, 586-628, 888-909; GrabImageRGBD's depth conversion, Tracking.cc:
265-271), Tracking::UpdateLastFrame's temporal MapPoints (Tracking.cc:893-954) and
TrackWithMotionModel's search (th 15, bMono false, the retry at 2*th below 20 matches,
Tracking.cc:966-994; ORBmatcher.cc:1620-1789) -- every frame, every LastFrame and every
pair against the oracle, including pairs forced under 20 matches."""
import numpy as np
import pytest

import tum_rgbd_scenes as S

pytestmark = pytest.mark.gpu

B = 16
SEED = 4000
SPARSE, SPARSE_NEXT = 2, 3     # frame 2 keeps depth in one small region; frame 3's pose is off by 3 degrees
EMPTY = 6                      # frame 6 has no depth at all: its LastFrame carries no MapPoint


def _perturb(t12, deg):
    from orbslam2commentedbyxcm_amd import synth
    Tm = np.vstack([np.asarray(t12, np.float64).reshape(3, 4), [0, 0, 0, 1]])
    R = np.eye(4)
    R[:3, :3] = synth.rotation("y", deg)
    return (R @ Tm)[:3, :4].reshape(12).astype(np.float32)


@pytest.fixture(scope="module")
def scene():
    gray, depth, T = S.sequence(SEED, B, workers=8)
    keep = np.zeros(depth.shape[1:], bool)
    keep[210:250, 300:350] = True
    depth[SPARSE][~keep] = 0
    depth[EMPTY][:] = 0
    T[SPARSE_NEXT] = _perturb(T[SPARSE_NEXT], 3.0)
    return gray, depth, T


@pytest.fixture(scope="module")
def bounds(oracle):
    return oracle.compute_image_bounds(S.K, S.DIST, S.W, S.H)


@pytest.fixture(scope="module")
def oracle_views(oracle, scene, bounds):
    from concurrent.futures import ThreadPoolExecutor
    gray, depth, T = scene
    p = oracle.params(*S.PARAMS)
    sf = np.array(p.scale[:p.nlevels], np.float32)
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(lambda b: S.oracle_frame(oracle, p, sf, gray[b], depth[b], T[b], bounds), range(B)))


def _run(pl, scene, tracked=None, steps=2):
    import torch

    from orbslam2commentedbyxcm_amd.extractor import device_frames
    gray, depth, T = scene
    dev = pl.dev
    d_gray = device_frames(gray, dev)
    d_depth = torch.from_numpy(depth).to(dev)
    d_T = torch.from_numpy(T).to(dev)
    pl.set_tracked(None, None)
    if tracked is not None:
        pl.run(d_gray, d_T, 1, d_depth)
        torch.cuda.synchronize(dev)
        pl.set_tracked(*pl.tracked_from(tracked))
    pl.run(d_gray, d_T, steps, d_depth)
    torch.cuda.synchronize(dev)
    return pl.host_results()


def _check_frames(h, views):
    for b, v in enumerate(views):
        n = h["n"][b]
        assert n == len(v.keys), b
        assert np.array_equal(h["kps"][b, :n].view(np.uint8), v.kd.view(np.uint8)), b
        assert np.array_equal(h["desc"][b, :n], v.desc), b
        assert np.array_equal(h["kpu"][b, :n].view(np.uint8), v.keys.view(np.uint8)), b
        assert np.array_equal(h["ur"][b, :n], v.u_right), b
        assert np.array_equal(h["dp"][b, :n], v.depth), b
        assert (h["ur"][b, n:] == -1).all() and (h["dp"][b, n:] == -1).all(), b


def _check_track(oracle, h, views, tracked, th_depth, cap, check_ori=True):
    assert (h["mp"][0] == -1).all() and h["nm"][0] == 0
    retried, forward, backward = [], 0, 0
    for b in range(1, B):
        last, cur = views[b - 1], views[b]
        ref, nr, obs, pos, rt = S.oracle_track(oracle, last, cur, tracked[b - 1], th_depth, check_ori=check_ori)
        n0 = len(last.keys)
        assert np.array_equal(h["mp_obs"][b - 1, :n0], obs), b
        assert np.array_equal(h["mp_pos"][b - 1, :n0][obs >= 0], pos[obs >= 0]), b
        assert np.array_equal(h["has_mp"][b - 1, :n0], (obs >= 0).astype(np.uint8)), b
        mp = h["mp"][b, :len(cur.keys)]
        got = np.where(mp >= 0, mp - (b - 1) * cap, -1)
        assert h["nm"][b] == nr, (b, h["nm"][b], nr, rt)
        assert np.array_equal(got, ref), (b, np.nonzero(got != ref)[0][:10])
        if rt:
            retried.append(b)
        Tl, Tc = last.Tcw, cur.Tcw
        tlc = Tl[:3, :3] @ (-(Tc[:3, :3].T @ Tc[:3, 3])) + Tl[:3, 3]
        forward += tlc[2] > last.b
        backward += -tlc[2] > last.b
    return retried, forward, backward


def test_rgbd_frame_single_call(oracle, orbx_built, scene, oracle_views):
    """orbx_compute_stereo_from_rgbd (the drop-in Frame constructor's steps): u16 with the
    camera (undistortion in the same pass), float32 images with factor 1 (read as is) and
    with a factor (converted), and mvKeysUn passed in (no camera)."""
    from orbslam2commentedbyxcm_amd.frame import ComputeStereoFromRGBD, camera
    gray, depth, T = scene
    cam = camera(*S.K, *S.DIST)
    for b in (0, 1, SPARSE, EMPTY):
        v = oracle_views[b]
        ku, ur, dp = ComputeStereoFromRGBD(v.kd, depth[b], S.BF, S.M_DEPTH_MAP_FACTOR, cam=cam)
        assert np.array_equal(ku.view(np.uint8), v.keys.view(np.uint8)), b
        assert np.array_equal(ur, v.u_right) and np.array_equal(dp, v.depth), b
    v = oracle_views[1]
    df = (depth[1].astype(np.float32) * np.float32(S.M_DEPTH_MAP_FACTOR)).astype(np.float32)
    df[::7, ::5] = np.nan  # NaN depths are no depth (d > 0 is false)
    for img, f in ((df, 1.0), (df * 2, 0.5), (depth[1].astype(np.float32), S.M_DEPTH_MAP_FACTOR)):
        _, ur, dp = ComputeStereoFromRGBD(v.kd, img, S.BF, f, keys_un=v.keys)
        ru, rd = oracle.compute_stereo_from_rgbd(v.kd, v.keys, img, S.BF, f)
        assert np.array_equal(ur, ru) and np.array_equal(dp, rd)
        assert (dp > 0).sum() > 1000
    _, ur, dp = ComputeStereoFromRGBD(v.kd[:0], depth[1], S.BF, S.M_DEPTH_MAP_FACTOR, cam=cam)
    assert len(ur) == 0 and len(dp) == 0


def test_rgbd_pipeline_configs4(oracle, orbx_built, scene, oracle_views):
    """B = 16 RGB-D frames at 5000 x 12, half the LastFrame keypoints with depth tracking
    map MapPoints: every frame's mvKeys / descriptors / mvKeysUn / mvuRight / mvDepth, every
    LastFrame's MapPoints and every pair's mvpMapPoints / nmatches, with two pairs under 20
    matches (a LastFrame with depth in one small region and a pose 3 degrees off: the retry
    at 2*th finds more; a LastFrame without depth: 0 both times)."""
    from orbslam2commentedbyxcm_amd.rgbd import RGBDSequencePipeline
    pl = RGBDSequencePipeline(B, S.W, S.H, S.FX, S.FY, S.CX, S.CY, S.DIST, S.BF, params=S.PARAMS)
    tracked = S.tracked_mask(SEED, B, pl.cap)
    h = _run(pl, scene, tracked)
    assert not pl.status().any()
    _check_frames(h, oracle_views)
    retried, fwd, bwd = _check_track(oracle, h, oracle_views, tracked, pl.th_depth, pl.cap)
    assert SPARSE_NEXT in retried and EMPTY + 1 in retried, retried
    assert h["nm"][EMPTY + 1] == 0 and 20 <= h["nm"][SPARSE_NEXT] < 100, h["nm"]
    assert fwd >= 2 and bwd >= 2, (fwd, bwd)
    assert (h["mp_obs"] == S.TRACKED_OBS).sum() > 5000 and (h["mp_obs"] == 0).sum() > 5000
    assert min(h["nm"][b] for b in range(1, B) if b not in retried) > 1000


@pytest.mark.parametrize("footprint", [5, 0])
def test_rgbd_pipeline_all_temporal(oracle, orbx_built, scene, oracle_views, footprint):
    """No tracked MapPoints (every visited point temporal, no claim blocks), one step, two
    launch shapes of the first search (the retry pass is always one launch of the one-wave form)."""
    from orbslam2commentedbyxcm_amd.rgbd import RGBDSequencePipeline
    pl = RGBDSequencePipeline(B, S.W, S.H, S.FX, S.FY, S.CX, S.CY, S.DIST, S.BF, params=S.PARAMS,
                              matcher_mode=footprint, pipelined=False)
    h = _run(pl, scene, None, steps=1)
    _check_frames(h, oracle_views)
    retried, _, _ = _check_track(oracle, h, oracle_views, np.zeros((B, pl.cap), bool), pl.th_depth, pl.cap)
    assert EMPTY + 1 in retried
