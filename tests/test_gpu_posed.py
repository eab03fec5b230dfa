"""GPU parity of the projection matchers under general camera motion.

The scenes (match_scenes.POSED) are views of one textured plane from cameras that roll
8-25 degrees about the optical axis, tilt a few degrees about the other two, and move
along the optical axis by more than the stereo baseline.  Every Tcw has a full rotation
(the world frame is not a camera frame), so R*X + t, the epipole, the forward / backward
octave ranges of SearchByProjection(Frame&, const Frame&) (ORBmatcher.cc:1650-1701,
including GetFeaturesInArea's disabled level filter for nLastOctave == 0, Frame.cc:515)
and the rotation histogram (ORBmatcher.cc:1750-1786, 1935-1977) all see non-trivial
input.  Each call is compared with the CPU oracle.
"""
import numpy as np
import pytest

import match_scenes as S
from orbslam2commentedbyxcm_amd.matcher import ORBmatcher, Track

pytestmark = pytest.mark.gpu

SCENES = list(S.POSED)


def _track(t):
    return Track(in_view=t.in_view, proj_x=t.proj_x, proj_y=t.proj_y, proj_xr=t.proj_xr,
                 scale_level=t.scale_level, view_cos=t.view_cos)


@pytest.mark.parametrize("scene", SCENES)
@pytest.mark.parametrize("stereo", [False, True])
def test_posed_search_by_projection_frame(oracle, orbx_built, scene, stereo):
    """a12 with bForward / bBackward (stereo) and the rotation check on a real roll."""
    A, B = S.posed_views(oracle, 1, scene, stereo=stereo)
    mps = S.posed_mappoints(A, 1)
    rng = np.random.default_rng(2)
    last_mp = np.arange(len(A.keys), dtype=np.int32)
    last_mp[rng.random(len(A.keys)) < 0.1] = -1
    outlier = (rng.random(len(A.keys)) < 0.05).astype(np.uint8)
    th = 7.0 if stereo else 15.0
    counts = {}
    for check_ori in (False, True):
        m = ORBmatcher(0.9, check_ori)
        cur_gpu = np.full(len(B.keys), -1, np.int32)
        n_gpu = m.SearchByProjectionFrame(B, cur_gpu, A, last_mp, mps, th, not stereo, last_outlier=outlier)
        cur_ref = np.full(len(B.keys), -1, np.int32)
        n_ref = oracle.sbp_frame(B, cur_ref, A, last_mp, mps, th, not stereo, check_ori, last_outlier=outlier)
        assert n_gpu == n_ref, (n_gpu, n_ref)
        assert np.array_equal(cur_gpu, cur_ref), np.nonzero(cur_gpu != cur_ref)[0][:10]
        counts[check_ori] = (n_ref, S.rotation_bins(A.keys, B.keys, cur_ref))
    n_all, bins_all = counts[False]
    n_ori, bins_ori = counts[True]
    assert n_all > 300
    assert (bins_all > 0).sum() >= 3          # a non-degenerate histogram before the filter
    assert n_ori < n_all                      # ComputeThreeMaxima removed some matches
    assert (bins_ori > 0).sum() <= 3
    # the dominant bin is the roll between the views, not bin 0
    rel = np.asarray(B.rel)[:3, :3] @ np.asarray(A.rel)[:3, :3].T
    roll = np.degrees(np.arctan2(rel[1, 0], rel[0, 0]))
    assert int(np.argmax(bins_all)) == int(np.round((-roll % 360) * 30 / 360)) % 30


def test_posed_forward_level_zero_queries(oracle, orbx_built):
    """bForward with nLastOctave == 0: GetFeaturesInArea(u, v, r, 0) checks no level at
    all (Frame.cc:515), so octave-0 queries may take any octave.  The same queries with
    the default octave window would match differently; both agree with the oracle."""
    A, B = S.posed_views(oracle, 3, "forward", stereo=True)
    mps = S.posed_mappoints(A, 3)
    last_mp = np.where(A.keys["octave"] == 0, np.arange(len(A.keys)), -1).astype(np.int32)
    assert (last_mp >= 0).sum() > 150
    m = ORBmatcher(0.9, False)
    cur_gpu = np.full(len(B.keys), -1, np.int32)
    n_gpu = m.SearchByProjectionFrame(B, cur_gpu, A, last_mp, mps, 7.0, False)
    cur_ref = np.full(len(B.keys), -1, np.int32)
    n_ref = oracle.sbp_frame(B, cur_ref, A, last_mp, mps, 7.0, False, False)
    assert n_gpu == n_ref and np.array_equal(cur_gpu, cur_ref)
    # matched at octaves above 1: only possible without a level filter
    assert (B.keys["octave"][cur_ref >= 0] > 1).sum() > 0


@pytest.mark.parametrize("scene", SCENES)
def test_posed_search_by_projection_local(oracle, orbx_built, scene):
    """a11 fed by IsInFrustum (Frame.cc:412-477) of the world MapPoints in the posed frame."""
    A, B = S.posed_views(oracle, 4, scene, stereo=scene in ("forward", "tilt"))
    mps = S.with_depth_info(S.posed_mappoints(A, 4), A, 4)
    t = oracle.is_in_frustum(B, mps)
    assert t.in_view.sum() > 0.5 * len(A.keys)
    assert len(np.unique(t.scale_level[t.in_view > 0])) >= 3
    rng = np.random.default_rng(5)
    queries = rng.permutation(len(A.keys)).astype(np.int32)
    f0 = np.full(len(B.keys), -1, np.int32)
    sel = rng.random(len(B.keys)) < 0.15
    f0[sel] = rng.integers(0, len(A.keys), sel.sum())
    for th, nnratio in ((1.0, 0.8), (5.0, 0.6)):
        m = ORBmatcher(nnratio, False)
        fg = f0.copy()
        ng = m.SearchByProjectionLocal(B, fg, queries, mps, _track(t), th)
        fr = f0.copy()
        nr = oracle.sbp_local(B, fr, queries, mps, _track(t), th, nnratio)
        assert ng == nr and nr > 100, (ng, nr)
        assert np.array_equal(fg, fr), np.nonzero(fg != fr)[0][:10]


@pytest.mark.parametrize("scene", SCENES)
def test_posed_search_by_projection_keyframe(oracle, orbx_built, scene):
    """a13 (relocalisation): PredictScale on the true camera distances, rotation check."""
    A, B = S.posed_views(oracle, 6, scene)
    mps = S.with_depth_info(S.posed_mappoints(A, 6), A, 6)
    rng = np.random.default_rng(6)
    kf_mp = np.arange(len(A.keys), dtype=np.int32)
    kf_mp[rng.random(len(A.keys)) < 0.1] = -1
    already = (rng.random(len(A.keys)) < 0.1).astype(np.uint8)
    for th, orb_dist, check_ori in ((10.0, 100, True), (3.0, 64, False)):
        m = ORBmatcher(0.9, check_ori)
        cur_gpu = np.full(len(B.keys), -1, np.int32)
        n_gpu = m.SearchByProjectionKeyFrame(B, cur_gpu, A, kf_mp, mps, th, orb_dist, already_found=already)
        cur_ref = np.full(len(B.keys), -1, np.int32)
        n_ref = oracle.sbp_keyframe(B, cur_ref, A, kf_mp, mps, th, orb_dist, check_ori, already_found=already)
        assert n_gpu == n_ref and n_ref > 100, (n_gpu, n_ref)
        assert np.array_equal(cur_gpu, cur_ref), np.nonzero(cur_gpu != cur_ref)[0][:10]


@pytest.mark.parametrize("scene,scale", [("roll20", 1.0), ("forward", 1.4), ("backward", 0.7), ("tilt", 1.0)])
def test_posed_search_by_projection_sim3(oracle, orbx_built, scene, scale):
    """a14 (loop closing) with a Sim3 whose rotation is a general one."""
    A, B = S.posed_views(oracle, 7, scene)
    mps = S.with_depth_info(S.posed_mappoints(A, 7), A, 7)
    rng = np.random.default_rng(8)
    n = len(A.keys)
    Scw = (np.float32(scale) * np.asarray(B.Tcw, np.float32)[:3, :4]).astype(np.float32)
    points = rng.permutation(n)[: int(0.9 * n)].astype(np.int32)
    matched0 = np.full(len(B.keys), -1, np.int32)
    m = ORBmatcher(0.75, False)
    got = matched0.copy()
    n_gpu = m.SearchByProjectionSim3(B, Scw, points, got, mps, 10)
    ref = matched0.copy()
    n_ref = oracle.sbp_sim3(B, Scw, points, ref, mps, 10)
    assert n_gpu == n_ref and n_ref > 50, (n_gpu, n_ref)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("scene", SCENES)
@pytest.mark.parametrize("stereo", [False, True])
def test_posed_search_for_triangulation(oracle, orbx_built, scene, stereo):
    """a15 with the epipole inside the image (motion along the optical axis) and a
    general F12 (ComputeF12, LocalMapping.cc:606-625)."""
    A, B = S.posed_views(oracle, 9, scene, stereo=stereo)
    rng = np.random.default_rng(9)
    has1 = (rng.random(len(A.keys)) < 0.2).astype(np.uint8)
    has2 = (rng.random(len(B.keys)) < 0.2).astype(np.uint8)
    fv1, fv2 = S.fv(A), S.fv(B)
    F12 = S.fundamental(A, B)
    for check_ori in (False, True):
        m = ORBmatcher(0.6, check_ori)
        pg = m.SearchForTriangulation(A, has1, fv1, B, has2, fv2, F12, False)
        pr = oracle.search_for_triangulation(A, has1, fv1, B, has2, fv2, F12, False, check_ori)
        assert np.array_equal(pg, pr), (len(pg), len(pr))
        assert len(pr) > 20


def test_posed_search_for_triangulation_batch_device(oracle, orbx_built):
    """The batched device SearchForTriangulation over keyframes from all four posed
    scenes (stereo and monocular), every ordered pair."""
    import torch

    from test_gpu_match import _upload_kfs
    from orbslam2commentedbyxcm_amd.matcher import FrameView

    # four keyframes of one plane: two stereo, two monocular (mvuRight < 0 throughout)
    views = S.posed_views(oracle, 10, "roll20", stereo=True,
                          extra=[S._rel([("z", -15.0), ("y", 2.0)], [0.0, 0.1, 0.6]),
                                 S._rel([("z", 9.0)], [0.0, 0.0, -0.7])])
    for V in views[2:]:
        V.u_right = None
    rng = np.random.default_rng(12)
    has = [(rng.random(len(V.keys)) < 0.2).astype(np.uint8) for V in views]
    fvs = [S.fv(V) for V in views]
    dev = torch.device("cuda", 0)
    cap = max(len(V.keys) for V in views) + 11
    keep, recs = _upload_kfs(views, has, fvs, cap, dev)
    pairs = [(i, j) for i in range(4) for j in range(4) if i != j]
    F12 = np.stack([S.fundamental(views[i], views[j]) for i, j in pairs])
    P = len(pairs)
    d_m12 = torch.empty((P, cap), dtype=torch.int32, device=dev)
    d_pairs = torch.empty((P, cap, 2), dtype=torch.int32, device=dev)
    d_np = torch.empty((P,), dtype=torch.int32, device=dev)
    cam = FrameView(keys=views[0].keys[:0], desc=views[0].desc[:0], scale_factors=views[0].scale_factors,
                    level_sigma2=views[0].level_sigma2)
    for check_ori in (False, True):
        m = ORBmatcher(0.6, check_ori)
        m.SearchForTriangulationBatchDevice(recs, cam, np.array(pairs), F12, cap, d_m12, d_pairs, d_np)
        torch.cuda.synchronize(dev)
        pg, npg = d_pairs.cpu().numpy(), d_np.cpu().numpy()
        total = 0
        for p, (i, j) in enumerate(pairs):
            pr = oracle.search_for_triangulation(views[i], has[i], fvs[i], views[j], has[j], fvs[j], F12[p],
                                                 False, check_ori)
            assert npg[p] == len(pr), (p, npg[p], len(pr))
            assert np.array_equal(pg[p, :npg[p]], pr), p
            total += len(pr)
        assert total > 200


@pytest.mark.parametrize("stereo,check_ori,footprint", [(False, True, 5), (True, True, 5), (True, False, 0),
                                                        (True, True, 2)])
def test_posed_match_sequence_device(oracle, orbx_built, stereo, check_ori, footprint):
    """Batched TrackWithMotionModel matching (orbx_match_sequence_device_ex) over a posed
    sequence: world MapPoint positions per last-frame keypoint, a has-MapPoint mask, and
    for stereo mvuRight plus the forward / backward octave ranges; every pair against the
    oracle's SearchByProjection(Frame&, const Frame&, th, bMono)."""
    import torch

    from orbslam2commentedbyxcm_amd import ORBextractor
    from orbslam2commentedbyxcm_amd.matcher import FrameView, MapPoints

    B = 8
    imgs, rels, T = S.posed_sequence(20, B)
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
    rng = np.random.default_rng(21)
    bf = 0.54 * S.FX if stereo else 0.0
    b = bf / S.FX
    pos = np.zeros((B, cap, 3), np.float32)
    ur = np.full((B, cap), -1.0, np.float32)
    has = np.zeros((B, cap), np.uint8)
    for k in range(B):
        kk = kps[k][: n[k]]
        X, z = S.plane_points(rels[k], kk["x"], kk["y"])
        pos[k, : n[k]] = S.to_world(X * (1.0 + rng.normal(0, 0.002, n[k]))[:, None]).astype(np.float32)
        u = (kk["x"] - bf / z + rng.normal(0, 0.5, n[k])).astype(np.float32)
        u[rng.random(n[k]) < 0.3] = -1.0
        ur[k, : n[k]] = u
        has[k, : n[k]] = rng.random(n[k]) < 0.9
    d_T = torch.from_numpy(T).to(dev)
    d_pos = torch.from_numpy(pos).to(dev)
    d_ur = torch.from_numpy(ur).to(dev) if stereo else None
    d_has = torch.from_numpy(has).to(dev)
    d_mp = torch.empty((B, cap), dtype=torch.int32, device=dev)
    d_nm = torch.empty((B,), dtype=torch.int32, device=dev)
    sf = ex.GetScaleFactors()
    m = ORBmatcher(0.9, check_ori)
    m.set_footprint(footprint)
    th = 7.0 if stereo else 15.0
    m.match_sequence_device_ex(d_kps, d_desc, d_n, d_T, d_mp, d_nm, sf, S.FX, S.FY, S.CX, S.CY, 640, 480, th=th,
                               mono=not stereo, bf=bf, b=b, d_u_right=d_ur, d_mp_pos=d_pos, d_has_mp=d_has,
                               stream=ex.stream_handle())
    torch.cuda.synchronize()
    mp, nm = d_mp.cpu().numpy(), d_nm.cpu().numpy()
    assert (mp[0] == -1).all() and nm[0] == 0
    forward = backward = 0
    occupied = []
    for p in range(B - 1):
        lk, ck = kps[p][: n[p]], kps[p + 1][: n[p + 1]]
        Tl = np.vstack([T[p].reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32)
        Tc = np.vstack([T[p + 1].reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32)
        last = FrameView(keys=lk, desc=desc[p][: n[p]], fx=S.FX, fy=S.FY, cx=S.CX, cy=S.CY, bf=bf, b=b,
                         scale_factors=sf, Tcw=Tl)
        cur = FrameView(keys=ck, desc=desc[p + 1][: n[p + 1]], fx=S.FX, fy=S.FY, cx=S.CX, cy=S.CY, bf=bf, b=b,
                        scale_factors=sf, Tcw=Tc, u_right=ur[p + 1][: n[p + 1]] if stereo else None)
        mps = MapPoints(desc=desc[p][: n[p]], observations=np.ones(n[p], np.int32), pos=pos[p][: n[p]])
        last_mp = np.where(has[p][: n[p]] > 0, np.arange(n[p]), -1).astype(np.int32)
        ref = np.full(n[p + 1], -1, np.int32)
        nr = oracle.sbp_frame(cur, ref, last, last_mp, mps, th, not stereo, check_ori)
        assert nm[p + 1] == nr, (p, nm[p + 1], nr)
        assert np.array_equal(mp[p + 1][: n[p + 1]], ref), (p, np.nonzero(mp[p + 1][: n[p + 1]] != ref)[0][:10])
        assert nr > 150, (p, nr)
        dz = (S.SEQ_Z[p + 1] - S.SEQ_Z[p])
        forward += dz > b and stereo
        backward += -dz > b and stereo
        occupied.append((S.rotation_bins(lk, ck, ref) > 0).sum())
    if stereo:
        assert forward >= 2 and backward >= 2
    assert max(occupied) >= 2


def _sequence_on_gpu(oracle, B, seed, prm=S.C1):
    import torch

    from orbslam2commentedbyxcm_amd import ORBextractor
    imgs, rels, T = S.posed_sequence(seed, B)
    dev = torch.device("cuda", 0)
    ex = ORBextractor(*prm)
    cap = ex.max_keypoints(640, 480)
    d_kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
    d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.empty((B,), dtype=torch.int32, device=dev)
    ex.extract_batch_device(torch.from_numpy(imgs).to(dev), d_kps, d_desc, d_n)
    torch.cuda.synchronize()
    n = d_n.cpu().numpy()
    kps = d_kps.cpu().numpy().view(np.uint8).reshape(B, cap, 28).view(oracle.KEYPOINT_DTYPE).reshape(B, cap)
    return dict(ex=ex, cap=cap, d_kps=d_kps, d_desc=d_desc, d_n=d_n, n=n, kps=kps, desc=d_desc.cpu().numpy(),
                rels=rels, T=T, dev=dev)


def _mappoint_table(seq, seed):
    """Every keypoint of the sequence as a MapPoint (id = frame * cap + index): world
    position on the plane, MapPoint::UpdateNormalAndDepth's normal and distances from the
    frame that made it, Observations() in 0..3, a few bad."""
    rng = np.random.default_rng(seed)
    B, cap = len(seq["n"]), seq["cap"]
    N = B * cap
    pos = np.zeros((N, 3), np.float32)
    desc = np.zeros((N, 32), np.uint8)
    nrm = np.zeros((N, 3), np.float32)
    mx = np.ones(N, np.float32)
    mn = np.ones(N, np.float32)
    sf = seq["ex"].GetScaleFactors()
    for f in range(B):
        k = seq["kps"][f][: seq["n"][f]]
        X, _ = S.plane_points(seq["rels"][f], k["x"], k["y"])
        P = S.to_world(X * (1.0 + rng.normal(0, 0.002, len(k)))[:, None]).astype(np.float32)
        T = np.vstack([seq["T"][f].reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32)
        Ow = -(T[:3, :3].T @ T[:3, 3])
        PO = P - Ow[None, :]
        dist = np.linalg.norm(PO.astype(np.float64), axis=1).astype(np.float32)
        sl = slice(f * cap, f * cap + len(k))
        pos[sl], desc[sl] = P, seq["desc"][f][: len(k)]
        nrm[sl] = (PO / dist[:, None]).astype(np.float32)
        mx[sl] = (dist * sf[k["octave"]]).astype(np.float32)
        mn[sl] = (mx[sl] / sf[-1]).astype(np.float32)
    obs = rng.integers(0, 4, N).astype(np.int32)
    bad = (rng.random(N) < 0.03).astype(np.uint8)
    return dict(pos=pos, desc=desc, normal=nrm, max_distance=mx, min_distance=mn, observations=obs, bad=bad)


@pytest.mark.parametrize("th,nnratio,footprint,stereo", [(1.0, 0.8, 5, False), (3.0, 0.8, 5, True),
                                                          (5.0, 0.6, 2, False), (1.0, 0.8, 0, True)])
def test_search_local_points_device(oracle, orbx_built, th, nnratio, footprint, stereo):
    """Tracking::SearchLocalPoints on the device (orbx_search_local_points_device): for each
    frame of a posed sequence, its local map = the MapPoints of its neighbours in the
    sequence, its mvpMapPoints pre-set as TrackWithMotionModel would have left them (some
    of them bad), IsInFrustum + SearchByProjection(F, vpLocalMapPoints, th) vs the oracle."""
    import torch

    from orbslam2commentedbyxcm_amd.matcher import FrameView, MapPoints

    B = 8
    seq = _sequence_on_gpu(oracle, B, 30)
    cap, n = seq["cap"], seq["n"]
    tab = _mappoint_table(seq, 31)
    rng = np.random.default_rng(32)
    # local maps: the MapPoints of frames b-2, b-1, b+1 (existing slots), shuffled per frame
    lists, off = [], [0]
    for b in range(B):
        ids = np.concatenate([np.arange(f * cap, f * cap + n[f]) for f in (b - 2, b - 1, b + 1) if 0 <= f < B])
        ids = rng.permutation(ids).astype(np.int32)
        lists.append(ids)
        off.append(off[-1] + len(ids))
    local_ids = np.concatenate(lists).astype(np.int32)
    # mvpMapPoints before the search: ~25 % of keypoints hold an id from the local map
    fmp0 = np.full((B, cap), -1, np.int32)
    for b in range(B):
        sel = np.nonzero(rng.random(n[b]) < 0.25)[0]
        fmp0[b, sel] = rng.choice(lists[b], len(sel), replace=False)
    ur = np.full((B, cap), -1.0, np.float32)
    bf = 0.54 * S.FX if stereo else 0.0
    if stereo:
        for b in range(B):
            k = seq["kps"][b][: n[b]]
            _, z = S.plane_points(seq["rels"][b], k["x"], k["y"])
            u = (k["x"] - bf / z + rng.normal(0, 0.5, n[b])).astype(np.float32)
            u[rng.random(n[b]) < 0.3] = -1.0
            ur[b, : n[b]] = u
    dev = seq["dev"]
    d_tab = {k: torch.from_numpy(v).to(dev) for k, v in tab.items()}
    d_fmp = torch.from_numpy(fmp0).to(dev)
    d_nm = torch.full((B,), -7, dtype=torch.int32, device=dev)
    sf = seq["ex"].GetScaleFactors()
    m = ORBmatcher(nnratio, False)
    m.set_footprint(footprint)
    m.search_local_points_device(d_tab, seq["d_kps"], seq["d_desc"], seq["d_n"],
                                 torch.from_numpy(seq["T"]).to(dev), np.array(off), torch.from_numpy(local_ids).to(dev),
                                 d_fmp, d_nm, sf, S.FX, S.FY, S.CX, S.CY, 640, 480, th=th, bf=bf,
                                 d_u_right=torch.from_numpy(ur).to(dev) if stereo else None)
    torch.cuda.synchronize()
    fmp, nm = d_fmp.cpu().numpy(), d_nm.cpu().numpy()
    mps = MapPoints(desc=tab["desc"], observations=tab["observations"], pos=tab["pos"], bad=tab["bad"],
                    max_distance=tab["max_distance"], min_distance=tab["min_distance"], normal=tab["normal"])
    total = 0
    for b in range(B):
        F = FrameView(keys=seq["kps"][b][: n[b]], desc=seq["desc"][b][: n[b]], fx=S.FX, fy=S.FY, cx=S.CX, cy=S.CY,
                      bf=bf, scale_factors=sf, Tcw=np.vstack([seq["T"][b].reshape(3, 4), [0, 0, 0, 1]]),
                      u_right=ur[b][: n[b]] if stereo else None)
        ref = fmp0[b][: n[b]].copy()
        nr = oracle.search_local_points(F, ref, lists[b], mps, th, nnratio)
        assert nm[b] == nr, (b, nm[b], nr)
        assert np.array_equal(fmp[b][: n[b]], ref), (b, np.nonzero(fmp[b][: n[b]] != ref)[0][:10])
        total += nr
    assert total > 100 * B


def test_create_mappoints_device(oracle, orbx_built):
    """Tracking::CreateNewKeyFrame's MapPoints on the device (UnprojectStereo +
    UpdateNormalAndDepth) == the oracle's, bit for bit, for per-keypoint depths (some not
    positive) on a posed sequence, and for the constant-depth form."""
    import torch

    from orbslam2commentedbyxcm_amd.matcher import FrameView, create_mappoints_device, mappoint_table

    B = 6
    seq = _sequence_on_gpu(oracle, B, 40)
    cap, n = seq["cap"], seq["n"]
    rng = np.random.default_rng(41)
    depth = np.zeros((B, cap), np.float32)
    for b in range(B):
        k = seq["kps"][b][: n[b]]
        _, z = S.plane_points(seq["rels"][b], k["x"], k["y"])
        d = z.astype(np.float32)
        d[rng.random(n[b]) < 0.2] = -1.0
        depth[b, : n[b]] = d
    sf = seq["ex"].GetScaleFactors()
    d_T = torch.from_numpy(seq["T"]).to(seq["dev"])
    for const in (None, 5.0):
        tab = mappoint_table(B, cap, seq["dev"])
        create_mappoints_device(seq["d_kps"], seq["d_n"], d_T, sf, S.FX, S.FY, S.CX, S.CY, tab,
                                d_depth=None if const else torch.from_numpy(depth).to(seq["dev"]),
                                const_depth=const or 0.0)
        torch.cuda.synchronize()
        got = {k: v.cpu().numpy() for k, v in tab.items()}
        for b in range(B):
            F = FrameView(keys=seq["kps"][b][: n[b]], desc=seq["desc"][b][: n[b]], fx=S.FX, fy=S.FY, cx=S.CX,
                          cy=S.CY, scale_factors=sf, Tcw=np.vstack([seq["T"][b].reshape(3, 4), [0, 0, 0, 1]]))
            r = oracle.create_mappoints(F, None if const else depth[b][: n[b]], const or 0.0)
            sl = slice(b * cap, b * cap + n[b])
            v = r["valid"] > 0
            assert np.array_equal(got["bad"][sl], 1 - r["valid"]) and got["bad"][b * cap + n[b]:(b + 1) * cap].all()
            assert np.array_equal(got["observations"][sl], r["valid"].astype(np.int32))
            for k in ("pos", "normal", "max_distance", "min_distance"):
                assert np.array_equal(got[k][sl][v].view(np.uint32), r[k][v].view(np.uint32)), (b, k)
