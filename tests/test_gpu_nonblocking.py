"""SearchByProjection(Frame&, const Frame&, th, bMono) (ORBmatcher.cc:1620-1789) with
MapPoints whose Observations() is 0 -- Tracking::UpdateLastFrame's temporal points -- and
the rotation check on.  Such a claim does not block the keypoint (cc:1716-1718), so a later
query takes it again: the keypoint keeps the last MapPoint, both acceptances count in
nmatches and both enter rotHist (in different bins when the two queries' angles differ),
and ComputeThreeMaxima's removal NULLs the keypoint when *either* entry's bin is dropped
(cc:1772-1784).  Dense re-claims on a rolled view pair, through the single drop-in call
(one-wave replay) and the batched sequence matcher (256-thread block replay, and the other
launch shapes)."""
import numpy as np
import pytest

import match_scenes as S
from orbslam2commentedbyxcm_amd.matcher import FrameView, MapPoints, ORBmatcher

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("zero_frac", [0.5, 1.0])
@pytest.mark.parametrize("scene", ["roll20", "tilt"])
def test_single_call_nonblocking_rotation(oracle, orbx_built, zero_frac, scene):
    A, B = S.posed_views(oracle, 21, scene)
    mps = S.posed_mappoints(A, 21, obs_zero_frac=zero_frac)
    mps.bad = None
    last_mp = np.arange(len(A.keys), dtype=np.int32)
    for th in (15.0, 30.0):  # the wider window: more queries reach each keypoint
        m = ORBmatcher(0.9, True)
        cur_gpu = np.full(len(B.keys), -1, np.int32)
        n_gpu = m.SearchByProjectionFrame(B, cur_gpu, A, last_mp, mps, th, True)
        cur_ref = np.full(len(B.keys), -1, np.int32)
        n_ref = oracle.sbp_frame(B, cur_ref, A, last_mp, mps, th, True, True)
        assert n_gpu == n_ref, (th, n_gpu, n_ref)
        assert np.array_equal(cur_gpu, cur_ref), (th, np.nonzero(cur_gpu != cur_ref)[0][:10])
        assert n_ref > 100
        # re-claims happened: more acceptances than keypoints left holding a MapPoint
        # would be the case without the rotation removal; check that the scene is dense
        cur_all = np.full(len(B.keys), -1, np.int32)
        n_all = oracle.sbp_frame(B, cur_all, A, last_mp, mps, th, True, False)
        assert n_all > (cur_all >= 0).sum(), "no keypoint was claimed twice"


@pytest.mark.parametrize("footprint", [5, 0, 1, 2, 3])
@pytest.mark.parametrize("zero_frac", [0.5, 1.0])
def test_sequence_nonblocking_rotation(oracle, orbx_built, footprint, zero_frac):
    """The batched matcher with per-MapPoint Observations() (orbx_sequence.mp_obs, global ids)
    over a posed sequence, every launch shape, against the oracle pair by pair."""
    import torch

    from orbslam2commentedbyxcm_amd import ORBextractor
    B = 6
    imgs, rels, T = S.posed_sequence(23, B)
    dev = torch.device("cuda", 0)
    ex = ORBextractor(*S.C1)
    cap = ex.max_keypoints(640, 480)
    d_kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
    d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.empty((B,), dtype=torch.int32, device=dev)
    ex.extract_batch_device(torch.from_numpy(imgs).to(dev), d_kps, d_desc, d_n)
    torch.cuda.synchronize()
    n = d_n.cpu().numpy()
    kps = d_kps.cpu().numpy().view(np.uint8).reshape(B, cap, 28).view(oracle.KEYPOINT_DTYPE).reshape(B, cap)
    desc = d_desc.cpu().numpy()
    rng = np.random.default_rng(24)
    pos = np.zeros((B, cap, 3), np.float32)
    obs = np.full((B, cap), 1, np.int32)
    for k in range(B):
        kk = kps[k][: n[k]]
        X, _ = S.plane_points(rels[k], kk["x"], kk["y"])
        pos[k, : n[k]] = S.to_world(X).astype(np.float32)
        obs[k, : n[k]] = np.where(rng.random(n[k]) < zero_frac, 0, rng.integers(1, 4, n[k]))
    d_T, d_pos, d_obs = (torch.from_numpy(a).to(dev) for a in (T, pos, obs))
    d_mp = torch.empty((B, cap), dtype=torch.int32, device=dev)
    d_nm = torch.empty((B,), dtype=torch.int32, device=dev)
    sf = ex.GetScaleFactors()
    m = ORBmatcher(0.9, True)
    m.set_footprint(footprint)
    m.match_sequence_device_ex(d_kps, d_desc, d_n, d_T, d_mp, d_nm, sf, S.FX, S.FY, S.CX, S.CY, 640, 480, th=15.0,
                               d_mp_pos=d_pos, d_mp_obs=d_obs, global_ids=True, stream=ex.stream_handle())
    torch.cuda.synchronize()
    mp, nm = d_mp.cpu().numpy(), d_nm.cpu().numpy()
    for p in range(B - 1):
        lk, ck = kps[p][: n[p]], kps[p + 1][: n[p + 1]]
        Tl = np.vstack([T[p].reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32)
        Tc = np.vstack([T[p + 1].reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32)
        last = FrameView(keys=lk, desc=desc[p][: n[p]], fx=S.FX, fy=S.FY, cx=S.CX, cy=S.CY, scale_factors=sf, Tcw=Tl)
        cur = FrameView(keys=ck, desc=desc[p + 1][: n[p + 1]], fx=S.FX, fy=S.FY, cx=S.CX, cy=S.CY, scale_factors=sf,
                        Tcw=Tc)
        mps = MapPoints(desc=desc[p][: n[p]], observations=obs[p][: n[p]], pos=pos[p][: n[p]])
        ref = np.full(n[p + 1], -1, np.int32)
        nr = oracle.sbp_frame(cur, ref, last, np.arange(n[p], dtype=np.int32), mps, 15.0, True, True)
        got = mp[p + 1][: n[p + 1]]
        got = np.where(got >= 0, got - p * cap, -1)
        assert nm[p + 1] == nr, (p, nm[p + 1], nr)
        assert np.array_equal(got, ref), (p, np.nonzero(got != ref)[0][:10])
        assert nr > 150


def test_sequence_mp_obs_needs_global_ids(orbx_built):
    import torch

    from orbslam2commentedbyxcm_amd import _lib as L
    dev = torch.device("cuda", 0)
    z = torch.zeros((2, 16, 7), dtype=torch.int32, device=dev)
    d = torch.zeros((2, 16, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros((2,), dtype=torch.int32, device=dev)
    T = torch.zeros((2, 12), dtype=torch.float32, device=dev)
    o = torch.zeros((2, 16), dtype=torch.int32, device=dev)
    m = ORBmatcher(0.9, True)
    with pytest.raises(L.OrbxError):
        m.match_sequence_device_ex(z, d, n, T, o, n, np.ones(8, np.float32), 500, 500, 320, 240, 640, 480,
                                   d_mp_obs=o, global_ids=False)
