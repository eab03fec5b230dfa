"""GPU parity of §8(f) rank 4 against the C oracle: Fuse (both overloads, search part),
SearchBySim3 and MapPoint::ComputeDistinctiveDescriptors."""
from __future__ import annotations

import numpy as np
import pytest

import match_scenes as S
from orbslam2commentedbyxcm_amd.matcher import ComputeDistinctiveDescriptors, MapPoints, ORBmatcher

pytestmark = pytest.mark.gpu


def _mps_of(oracle_view, seed):
    """MapPoints back-projected from a view (world = camera shifted by the view's pose)."""
    m = S.mappoints_from(oracle_view, seed)
    m.pos = (m.pos - np.asarray(oracle_view.Tcw, np.float32)[:3, 3][None, :]).astype(np.float32)
    return S.with_depth_info(m, oracle_view, seed)


def _concat(a: MapPoints, b: MapPoints) -> MapPoints:
    cat = lambda x, y: np.concatenate([x, y])  # noqa: E731
    return MapPoints(desc=cat(a.desc, b.desc), observations=cat(a.observations, b.observations), pos=cat(a.pos, b.pos),
                     bad=cat(a.bad, b.bad), max_distance=cat(a.max_distance, b.max_distance),
                     min_distance=cat(a.min_distance, b.min_distance), normal=cat(a.normal, b.normal))


@pytest.mark.parametrize("seed,stereo,th", [(0, False, 3.0), (1, True, 3.0), (2, True, 1.5), (3, False, 6.0)])
def test_fuse(oracle, orbx_built, seed, stereo, th):
    A, B = S.two_views(oracle, seed, stereo=stereo)
    mps = _mps_of(A, seed)
    rng = np.random.default_rng(seed + 40)
    n = len(A.keys)
    points = rng.permutation(n).astype(np.int32)
    points[rng.random(n) < 0.05] = -1
    skip = (rng.random(n) < 0.1).astype(np.uint8)
    m = ORBmatcher(0.6, True)
    got = m.Fuse(B, points, skip, mps, th)
    ref = oracle.fuse(B, points, skip, mps, th)
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:10]
    assert (ref >= 0).sum() > 50


@pytest.mark.parametrize("seed,scale,th", [(4, 1.0, 4.0), (5, 1.3, 4.0), (6, 0.8, 8.0)])
def test_fuse_sim3(oracle, orbx_built, seed, scale, th):
    A, B = S.two_views(oracle, seed)
    mps = _mps_of(A, seed)
    rng = np.random.default_rng(seed + 41)
    n = len(A.keys)
    Scw = (np.float32(scale) * np.asarray(B.Tcw, np.float32)[:3, :4]).astype(np.float32)
    points = rng.permutation(n)[: int(0.8 * n)].astype(np.int32)
    skip = (rng.random(n) < 0.1).astype(np.uint8)
    m = ORBmatcher(0.75, False)
    got = m.FuseSim3(B, Scw, points, skip, mps, th)
    ref = oracle.fuse_sim3(B, Scw, points, skip, mps, th)
    assert np.array_equal(got, ref), np.nonzero(got != ref)[0][:10]
    assert (ref >= 0).sum() > 50


@pytest.mark.parametrize("seed,s12,th", [(7, 1.0, 7.5), (8, 1.05, 7.5), (9, 1.0, 3.0)])
def test_search_by_sim3(oracle, orbx_built, seed, s12, th):
    A, B = S.two_views(oracle, seed, dx=-6, dy=4)
    ma, mb = _mps_of(A, seed), _mps_of(B, seed + 1)
    mps = _concat(ma, mb)
    nA, nB = len(A.keys), len(B.keys)
    rng = np.random.default_rng(seed + 42)
    mp1 = np.arange(nA, dtype=np.int32)
    mp1[rng.random(nA) < 0.2] = -1
    mp2 = np.arange(nA, nA + nB, dtype=np.int32)
    mp2[rng.random(nB) < 0.2] = -1
    already1 = (rng.random(nA) < 0.05).astype(np.uint8)
    already2 = (rng.random(nB) < 0.05).astype(np.uint8)
    T1, T2 = np.asarray(A.Tcw, np.float32), np.asarray(B.Tcw, np.float32)
    R12 = (T1[:3, :3] @ T2[:3, :3].T).astype(np.float32)
    t12 = (T1[:3, 3] - R12 @ T2[:3, 3]).astype(np.float32)
    m12_0 = np.full(nA, -1, np.int32)
    m12_0[already1.astype(bool)] = 12345
    m = ORBmatcher(0.75, True)
    got = m12_0.copy()
    ng = m.SearchBySim3(A, mp1, B, mp2, got, mps, s12, R12, t12, th, already1, already2)
    ref = m12_0.copy()
    nr = oracle.search_by_sim3(A, mp1, already1, B, mp2, already2, mps, s12, R12, t12, th, ref)
    assert ng == nr and np.array_equal(got, ref), (ng, nr)
    assert nr > 50


@pytest.mark.parametrize("seed", [0, 1])
def test_compute_distinctive_descriptors(oracle, orbx_built, seed):
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, 12, 500)
    counts[:6] = [0, 1, 2, 63, 64, 130]  # empty, single, even / odd, more than a wave
    base = rng.integers(0, 256, (len(counts), 32), dtype=np.uint8)
    descs = []
    for k, c in enumerate(counts):
        bits = np.unpackbits(np.repeat(base[k:k + 1], c, 0), axis=1)
        bits ^= (rng.random(bits.shape) < rng.uniform(0.02, 0.3)).astype(np.uint8)
        descs.append(np.packbits(bits, axis=1))
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    desc = np.concatenate(descs) if off[-1] else np.zeros((0, 32), np.uint8)
    best, out = ComputeDistinctiveDescriptors(off, desc)
    ref = oracle.distinctive_descriptors(off, desc)
    assert np.array_equal(best, ref)
    for k in range(len(counts)):
        if ref[k] >= 0:
            assert np.array_equal(out[k], desc[off[k] + ref[k]])
