"""The oracle's Tracking::UpdateLastFrame (oracle/orbx_oracle_match.c ora_update_last_frame)
against a literal Python transcription of Tracking.cc:905-953 (vector of (depth, index)
pairs, std::sort, the visiting loop with its break), on seeded depth fields that put the
mThDepth break before, at and after the 100-point floor, with ties in depth."""
import numpy as np
import pytest

from orbslam2commentedbyxcm_amd.matcher import FrameView


def _transcription(depth, obs_in, th_depth):
    """Tracking.cc:905-953, the MapPoint bookkeeping only: which keypoints get a temporal point."""
    v = sorted((float(np.float32(z)), i) for i, z in enumerate(depth) if z > 0)
    obs = obs_in.copy()
    made = np.zeros(len(depth), bool)
    n_points = 0
    for z, i in v:
        if obs[i] < 0 or obs[i] < 1:  # !pMP || pMP->Observations() < 1
            obs[i] = 0
            made[i] = True
        n_points += 1
        if z > th_depth and n_points > 100:
            break
    return obs, made


def _frame(n, rng):
    keys = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                              ("octave", "<i4"), ("class_id", "<i4")])
    keys["x"] = rng.uniform(0, 1241, n)
    keys["y"] = rng.uniform(0, 376, n)
    sf = (1.2 ** np.arange(8)).astype(np.float32)
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = np.array([[0.9, -0.1, 0.42], [0.12, 0.99, 0.0], [-0.41, 0.05, 0.91]], np.float32)
    T[:3, 3] = [0.3, -0.2, 1.1]
    return FrameView(keys=keys, desc=np.zeros((n, 32), np.uint8), fx=718.856, fy=718.856, cx=607.1928, cy=185.2157,
                     bf=386.1448, b=0.537, scale_factors=sf, level_sigma2=sf * sf, Tcw=T)


@pytest.mark.parametrize("seed,n,th,frac_depth,frac_obs", [
    (0, 2000, 18.8, 0.5, 0.5),    # many within th_depth: the first point beyond it ends the walk
    (1, 2000, 3.0, 0.5, 0.3),     # none within: exactly the 101 nearest
    (2, 300, 12.0, 0.4, 0.0),     # fewer than 100 with depth at all
    (3, 1500, 14.0, 0.6, 0.9),    # mostly tracked already
    (4, 800, 10.0, 0.9, 0.2),     # ~100 within: the floor and the threshold meet
])
def test_update_last_frame_matches_transcription(oracle, seed, n, th, frac_depth, frac_obs):
    rng = np.random.default_rng(seed)
    F = _frame(n, rng)
    depth = np.where(rng.random(n) < frac_depth, rng.uniform(2.0, 40.0, n), -1).astype(np.float32)
    depth[rng.random(n) < 0.05] = np.float32(9.5)  # ties in depth: broken by index
    if seed == 4:
        depth = np.where(depth > 0, rng.uniform(9.0, 11.0, n), -1).astype(np.float32)
    obs_in = np.where(rng.random(n) < frac_obs, rng.integers(0, 4, n), -1).astype(np.int32)
    pos_in = rng.normal(0, 5, (n, 3)).astype(np.float32)
    obs, pos, created = oracle.update_last_frame(F, depth, th, obs_in, pos_in)
    want, made = _transcription(depth, obs_in, np.float32(th))
    assert np.array_equal(obs, want)
    assert created == made.sum() > 0
    # temporal points sit at UnprojectStereo (the CreateNewKeyFrame restatement's positions)
    ref = oracle.create_mappoints(F, depth)["pos"]
    assert np.array_equal(pos[made], ref[made])
    assert np.array_equal(pos[~made], pos_in[~made])
