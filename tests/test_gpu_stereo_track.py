"""configs[2] with its SearchByProjection leg: the stereo front end at KITTI's shape
(1241x376, 2000 features) through StereoSequencePipeline -- extraction of L and R,
ComputeStereoMatches, Tracking::UpdateLastFrame's temporal MapPoints and the stereo
TrackWithMotionModel search (th 7, bMono false: bForward / bBackward, the mvuRight gate,
non-blocking claims of the temporal points, the rotation check) -- every frame and every
pair against the oracle (ORBextractor.cc, Frame.cc:673-885, Tracking.cc:893-994,
ORBmatcher.cc:1620-1789)."""
import numpy as np
import pytest

import kitti_scenes as K

pytestmark = pytest.mark.gpu

B = 16


@pytest.fixture(scope="module")
def scene():
    return K.sequence(11, B, workers=8)


@pytest.fixture(scope="module")
def oracle_views(oracle, scene):
    from concurrent.futures import ThreadPoolExecutor
    left, right, T = scene
    p = oracle.params(*K.PARAMS)
    sf = np.array(p.scale[:p.nlevels], np.float32)
    with ThreadPoolExecutor(8) as ex:
        return list(ex.map(lambda b: K.oracle_frame(oracle, p, sf, left[b], right[b], T[b]), range(B)))


def _check_frames(h, views):
    for b, v in enumerate(views):
        nl, nr = h["nl"][b], h["nr"][b]
        assert nl == len(v.keys) and nr == len(v.kr), b
        assert np.array_equal(h["kl"][b, :nl].view(np.uint8), v.keys.view(np.uint8)), b
        assert np.array_equal(h["dl"][b, :nl], v.desc), b
        assert np.array_equal(h["kr"][b, :nr].view(np.uint8), v.kr.view(np.uint8)), b
        assert np.array_equal(h["dr"][b, :nr], v.dr), b
        assert np.array_equal(h["ur"][b, :nl], v.u_right), b
        assert np.array_equal(h["dp"][b, :nl], v.depth), b


def _check_track(oracle, h, views, tracked, th_depth, cap, check_ori=True):
    assert (h["mp"][0] == -1).all() and h["nm"][0] == 0
    forward = backward = 0
    for b in range(1, B):
        last, cur = views[b - 1], views[b]
        ref, nr, obs, pos = K.oracle_track(oracle, last, cur, tracked[b - 1], th_depth, check_ori=check_ori)
        n0 = len(last.keys)
        # UpdateLastFrame's outputs for frame b-1 (used by pair b)
        assert np.array_equal(h["mp_obs"][b - 1, :n0], obs), b
        assert np.array_equal(h["mp_pos"][b - 1, :n0][obs >= 0], pos[obs >= 0]), b
        assert np.array_equal(h["has_mp"][b - 1, :n0], (obs >= 0).astype(np.uint8)), b
        mp = h["mp"][b, :len(cur.keys)]
        got = np.where(mp >= 0, mp - (b - 1) * cap, -1)
        assert h["nm"][b] == nr, (b, h["nm"][b], nr)
        assert np.array_equal(got, ref), (b, np.nonzero(got != ref)[0][:10])
        assert nr > 100, (b, nr)
        Tl, Tc = last.Tcw, cur.Tcw
        tlc = Tl[:3, :3] @ (-(Tc[:3, :3].T @ Tc[:3, 3])) + Tl[:3, 3]
        forward += tlc[2] > last.b
        backward += -tlc[2] > last.b
    return forward, backward


def _run(pl, scene, tracked=None, steps=2, pitched=True):
    """pitched: the frames in HBM with 1280-byte rows (extractor.device_frames), so the
    extractors read level 0 in place and ComputeStereoMatches reads it from the frames;
    packed 1241-byte rows take the copy into the pyramids."""
    import torch

    from orbslam2commentedbyxcm_amd.extractor import device_frames
    left, right, T = scene
    dev = pl.dev
    if pitched:
        d_left, d_right = device_frames(left, dev), device_frames(right, dev)
        assert d_left.stride(1) == 1280
    else:
        d_left, d_right = (torch.from_numpy(a).to(dev) for a in (left, right))
    d_T = torch.from_numpy(T).to(dev)
    obs_in = pos_in = None
    if tracked is not None:
        pl.step(d_left, d_right, d_T)
        torch.cuda.synchronize(dev)
        obs_in, pos_in = pl.tracked_from(tracked)
    for _ in range(steps):
        pl.step(d_left, d_right, d_T, obs_in, pos_in)
    torch.cuda.synchronize(dev)
    return pl.host_results()


@pytest.mark.parametrize("pitched", [True, False])
def test_stereo_track_kitti_tracked_and_temporal(oracle, orbx_built, scene, oracle_views, pitched):
    """Half the LastFrame keypoints with depth already track map MapPoints (blocking
    claims), the other visited ones get temporal points (non-blocking).  Frames with a
    64-byte-multiple row pitch (level 0 read in place) and packed."""
    from orbslam2commentedbyxcm_amd.stereo import StereoSequencePipeline
    pl = StereoSequencePipeline(B, K.W, K.H, K.FX, K.FY, K.CX, K.CY, K.BF, params=K.PARAMS)
    tracked = K.tracked_mask(11, B, pl.cap)
    h = _run(pl, scene, tracked, pitched=pitched)
    assert pl.status_clean()
    _check_frames(h, oracle_views)
    fwd, bwd = _check_track(oracle, h, oracle_views, tracked, pl.th_depth, pl.cap)
    assert fwd >= 2 and bwd >= 2, (fwd, bwd)
    assert (h["mp_obs"] == K.TRACKED_OBS).sum() > 1000 and (h["mp_obs"] == 0).sum() > 1000


@pytest.mark.parametrize("footprint", [5, 0, 2])
def test_stereo_track_kitti_all_temporal(oracle, orbx_built, scene, oracle_views, footprint):
    """No tracked MapPoints: every visited LastFrame point is temporal (Observations() 0), so
    no claim blocks and later queries overwrite earlier ones; the rotation check then removes
    a keypoint when any of its entries falls outside the three maxima.  All launch shapes
    of the sequence matcher."""
    from orbslam2commentedbyxcm_amd.stereo import StereoSequencePipeline
    pl = StereoSequencePipeline(B, K.W, K.H, K.FX, K.FY, K.CX, K.CY, K.BF, params=K.PARAMS, matcher_mode=footprint)
    h = _run(pl, scene, None, steps=1)
    _check_frames(h, oracle_views)
    none = np.zeros((B, pl.cap), bool)
    _check_track(oracle, h, oracle_views, none, pl.th_depth, pl.cap)


def test_stereo_track_kitti_near_threshold(oracle, orbx_built, scene, oracle_views):
    """mThDepth of 3.8 m (ThDepth 7): no keypoint lies within it, so UpdateLastFrame visits
    exactly the 101 nearest (Tracking.cc:951-952) -- the device's ranking path -- and the
    search runs without the rotation check."""
    from orbslam2commentedbyxcm_amd.stereo import StereoSequencePipeline
    pl = StereoSequencePipeline(B, K.W, K.H, K.FX, K.FY, K.CX, K.CY, K.BF, params=K.PARAMS, th_depth_factor=7.0,
                                check_ori=False)
    tracked = K.tracked_mask(12, B, pl.cap, frac=0.3)
    h = _run(pl, scene, tracked, steps=1)
    assert ((h["mp_obs"] == 0).sum(axis=1)[:B - 1] <= 101).all()
    _check_track(oracle, h, oracle_views, tracked, pl.th_depth, pl.cap, check_ori=False)
