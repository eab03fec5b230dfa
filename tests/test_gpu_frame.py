"""GPU parity of the Frame steps (f3): UndistortKeyPoints / ComputeImageBounds /
AssignFeaturesToGrid against the oracle, host-buffer and batched device forms."""
from __future__ import annotations

import numpy as np
import pytest

from orbslam2commentedbyxcm_amd import KEYPOINT_DTYPE
from orbslam2commentedbyxcm_amd import frame as FR

pytestmark = pytest.mark.gpu

CAMS = {  # Examples/*/*.yaml
    "tum1": ([517.306408, 516.469215, 318.643040, 255.313989], [0.262383, -0.953104, -0.005358, 0.002628, 1.163314]),
    "euroc": ([458.654, 457.296, 367.215, 248.375], [-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05, 0.0]),
    "kitti": ([718.856, 718.856, 607.1928, 185.2157], [0.0, 0.0, 0.0, 0.0, 0.0]),
}


def _keys(seed, n, W, H):
    rng = np.random.default_rng(seed)
    k = np.zeros(n, KEYPOINT_DTYPE)
    k["x"] = rng.uniform(-2, W + 2, n).astype(np.float32)
    k["y"] = rng.uniform(-2, H + 2, n).astype(np.float32)
    k["x"][:8] = [0, W, 0, W, 0.5, W - 0.5, W / 2, 31.25]
    k["y"][:8] = [0, 0, H, H, 0.5, H - 0.5, H / 2, 17.75]
    k["size"] = 31
    k["angle"] = rng.uniform(0, 360, n)
    k["octave"] = rng.integers(0, 8, n)
    k["response"] = rng.uniform(0, 100, n)
    k["class_id"] = -1
    return k


@pytest.mark.parametrize("name", list(CAMS))
def test_undistort_bounds_grid(oracle, orbx_built, name):
    K, D = CAMS[name]
    W, H = (1241, 376) if name == "kitti" else ((752, 480) if name == "euroc" else (640, 480))
    cam = FR.camera(*K, *D)
    keys = _keys(1, 3000, W, H)
    ku = FR.UndistortKeyPoints(cam, keys)
    kr = oracle.undistort_keypoints(K, D, keys)
    assert np.array_equal(ku.view(np.uint8), kr.view(np.uint8))
    b = FR.ComputeImageBounds(cam, W, H)
    br = oracle.compute_image_bounds(K, D, W, H)
    assert np.array_equal(b.view(np.uint32), br.view(np.uint32))
    s, i = FR.AssignFeaturesToGrid(ku, b)
    sr, ir = oracle.assign_features_to_grid(kr, br)
    assert np.array_equal(s, sr) and np.array_equal(i, ir)


@pytest.mark.parametrize("counts,cap", [([1000, 0, 1, 2000, 777], 2000), ([8192, 5000], 8192)])
def test_batched_device(oracle, orbx_built, counts, cap):
    import torch

    K, D = CAMS["tum1"]
    cam = FR.camera(*K, *D)
    B = len(counts)
    keys = np.zeros((B, cap), KEYPOINT_DTYPE)
    for b in range(B):
        keys[b] = _keys(10 + b, cap, 640, 480)
    d_keys = torch.from_numpy(keys.view(np.int32).reshape(B, cap, 7).copy()).cuda()
    d_n = torch.tensor(counts, dtype=torch.int32, device="cuda")
    d_un = torch.full_like(d_keys, -9)
    FR.undistort_device(cam, d_keys, d_n, cap, d_un)
    b4 = oracle.compute_image_bounds(K, D, 640, 480)
    d_cs = torch.full((B, 64 * 48 + 1), -5, dtype=torch.int32, device="cuda")
    d_ci = torch.full((B, cap), -5, dtype=torch.int32, device="cuda")
    FR.grid_device(d_un, d_n, cap, b4, d_cs, d_ci)
    torch.cuda.synchronize()
    un = d_un.cpu().numpy().reshape(B, cap * 7).view(KEYPOINT_DTYPE).reshape(B, cap)
    cs, ci = d_cs.cpu().numpy(), d_ci.cpu().numpy()
    for b, c in enumerate(counts):
        n = min(c, cap)
        kr = oracle.undistort_keypoints(K, D, keys[b, :n])
        assert np.array_equal(un[b, :n].view(np.uint8), kr.view(np.uint8))
        assert (d_un.cpu().numpy()[b, n:] == -9).all()
        sr, ir = oracle.assign_features_to_grid(kr, b4)
        assert np.array_equal(cs[b], sr) and np.array_equal(ci[b, :sr[-1]], ir)
