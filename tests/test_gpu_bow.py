"""GPU parity of the vocabulary-node and initialisation matchers (§8(f) rank 2):
SearchByBoW(KF, F), SearchByBoW(KF, KF) and SearchForInitialization, against the C
oracle (oracle/orbx_oracle_match.c), byte for byte.  FeatureVectors come from the
synthetic node map of match_scenes (small and large nodes, > 64 candidates) and, end
to end, from the GPU vocabulary transform."""
from __future__ import annotations

import numpy as np
import pytest

import match_scenes as S
from orbslam2commentedbyxcm_amd.matcher import ORBmatcher, feature_vector_csr

pytestmark = pytest.mark.gpu


def _mp_ids(n, seed, null_frac=0.2, base=0):
    rng = np.random.default_rng(seed)
    mp = np.arange(base, base + n, dtype=np.int32)
    mp[rng.random(n) < null_frac] = -1  # NULL or isBad()
    return mp


@pytest.mark.parametrize("seed,nnodes,check_ori,ratio", [(0, 40, True, 0.7), (1, 40, False, 0.7), (2, 5, True, 0.7),
                                                         (3, 300, True, 0.75), (4, 2, False, 0.9)])
def test_search_by_bow_frame(oracle, orbx_built, seed, nnodes, check_ori, ratio):
    A, B = S.two_views(oracle, seed, dx=5 + seed, dy=-3)
    fv1, fv2 = S.fv(A, nnodes=nnodes), S.fv(B, nnodes=nnodes)
    mp = _mp_ids(len(A.keys), seed + 50, base=1000)
    m = ORBmatcher(ratio, check_ori)
    ng, mg = m.SearchByBoWFrame(A, mp, fv1, B, fv2)
    nr, mr = oracle.search_by_bow_frame(A, mp, fv1, B, fv2, ratio, check_ori)
    assert ng == nr and np.array_equal(mg, mr), (ng, nr, np.nonzero(mg != mr)[0][:10])
    assert nr > 30


@pytest.mark.parametrize("seed,nnodes,check_ori,ratio", [(5, 40, True, 0.75), (6, 5, True, 0.75),
                                                         (7, 100, False, 0.6), (8, 1, True, 0.9)])
def test_search_by_bow_keyframes(oracle, orbx_built, seed, nnodes, check_ori, ratio):
    A, B = S.two_views(oracle, seed, dx=-4, dy=6)
    fv1, fv2 = S.fv(A, nnodes=nnodes), S.fv(B, nnodes=nnodes)
    mp1 = _mp_ids(len(A.keys), seed + 60, 0.15)
    mp2 = _mp_ids(len(B.keys), seed + 70, 0.3, base=5000)
    m = ORBmatcher(ratio, check_ori)
    ng, mg = m.SearchByBoWKeyFrames(A, mp1, fv1, B, mp2, fv2)
    nr, mr = oracle.search_by_bow_keyframes(A, mp1, fv1, B, mp2, fv2, ratio, check_ori)
    assert ng == nr and np.array_equal(mg, mr), (ng, nr, np.nonzero(mg != mr)[0][:10])
    assert nr > 30


def test_search_by_bow_empty_and_disjoint(oracle, orbx_built):
    A, B = S.two_views(oracle, 9)
    m = ORBmatcher(0.7, True)
    mp = _mp_ids(len(A.keys), 1)
    empty = (np.zeros(0, np.int32), np.zeros(1, np.int32), np.zeros(0, np.int32))
    n, out = m.SearchByBoWFrame(A, mp, empty, B, S.fv(B))
    assert n == 0 and (out == -1).all()
    # disjoint node sets: nothing shared
    n1 = S.vocab_nodes(A)
    n2 = S.vocab_nodes(B) + 1000
    n, out = m.SearchByBoWFrame(A, mp, feature_vector_csr(n1), B, feature_vector_csr(n2))
    assert n == 0 and (out == -1).all()


@pytest.mark.parametrize("seed,window,check_ori,passes", [(0, 100, True, 2), (1, 50, True, 1), (2, 100, False, 1),
                                                          (3, 200, True, 1), (4, 10, True, 3)])
def test_search_for_initialization(oracle, orbx_built, seed, window, check_ori, passes):
    """Tracking::MonocularInitialization: ORBmatcher(0.9, true), windowSize 100, called
    again on later frames with the updated vbPrevMatched."""
    A, B = S.two_views(oracle, seed, dx=9, dy=-6)
    m = ORBmatcher(0.9, check_ori)
    prev_g = np.ascontiguousarray(np.stack([A.keys["x"], A.keys["y"]], 1).astype(np.float32))
    prev_r = prev_g.copy()
    for _ in range(passes):
        ng, mg = m.SearchForInitialization(A, B, prev_g, window)
        nr, mr, prev_r = oracle.search_for_initialization(A, B, prev_r, window, 0.9, check_ori)
        assert ng == nr and np.array_equal(mg, mr), (ng, nr, np.nonzero(mg != mr)[0][:10])
        assert np.array_equal(prev_g.view(np.uint32), prev_r.view(np.uint32))
    assert nr > 20


def test_bow_end_to_end_with_vocabulary(oracle, orbx_built):
    """extract -> ORBVocabulary.transform (GPU) -> SearchByBoW (GPU) equals the oracle
    on the same FeatureVectors, and the FeatureVectors equal the oracle transform's."""
    from orbslam2commentedbyxcm_amd import synth
    from orbslam2commentedbyxcm_amd.vocabulary import ORBVocabulary

    A, B = S.two_views(oracle, 12, dx=6, dy=2)
    text = synth.vocabulary_text(3, 10, 5, 0, 0, centres=A.desc)
    V, OV = ORBVocabulary(0), oracle.Vocab(text)
    assert V.loadFromText(text)
    for levelsup in (4, 3):
        fvs = []
        for X in (A, B):
            _, _, fn, fo, fi = V.transform_arrays(X.desc, levelsup)
            _, _, en, eo, ei = OV.transform(X.desc, levelsup)
            assert np.array_equal(fn, en) and np.array_equal(fo, eo) and np.array_equal(fi, ei)
            fvs.append((fn, fo, fi))
        mp = _mp_ids(len(A.keys), 77)
        m = ORBmatcher(0.7, True)
        ng, mg = m.SearchByBoWFrame(A, mp, fvs[0], B, fvs[1])
        nr, mr = oracle.search_by_bow_frame(A, mp, fvs[0], B, fvs[1], 0.7, True)
        assert ng == nr and np.array_equal(mg, mr)
        assert nr > 30


def _contended_view(seed, n, pool, flips, level0_frac=0.8, W=640, H=480):
    """Keypoints at random positions whose descriptors are noisy copies of a few
    prototypes: many queries compete for the same candidates (claims, steals and list
    exhaustion on every path)."""
    from orbslam2commentedbyxcm_amd import KEYPOINT_DTYPE
    from orbslam2commentedbyxcm_amd.matcher import FrameView

    rng = np.random.default_rng(seed)
    keys = np.zeros(n, KEYPOINT_DTYPE)
    keys["x"] = rng.uniform(0, W - 1, n)
    keys["y"] = rng.uniform(0, H - 1, n)
    keys["size"] = 31
    keys["angle"] = rng.choice([10.0, 11.0, 200.0, 350.0], n) + rng.uniform(0, 6, n)
    keys["octave"] = np.where(rng.random(n) < level0_frac, 0, rng.integers(1, 8, n))
    keys["class_id"] = -1
    bits = np.unpackbits(pool[rng.integers(0, len(pool), n)], axis=1)
    bits ^= (rng.random(bits.shape) < flips).astype(np.uint8)
    desc = np.packbits(bits, axis=1)
    sf = (1.2 ** np.arange(8)).astype(np.float32)
    return FrameView(keys=keys, desc=desc, fx=500.0, fy=500.0, cx=320.0, cy=240.0, max_x=float(W), max_y=float(H),
                     scale_factors=sf, level_sigma2=sf * sf, Tcw=np.eye(4, dtype=np.float32))


@pytest.mark.parametrize("seed,n,window,flips", [(0, 1500, 100, 0.03), (1, 3000, 60, 0.05), (2, 800, 300, 0.02)])
def test_search_for_initialization_contended(oracle, orbx_built, seed, n, window, flips):
    rng = np.random.default_rng(seed)
    pool = rng.integers(0, 256, (6, 32), dtype=np.uint8)
    A = _contended_view(seed + 1, n, pool, flips)
    B = _contended_view(seed + 2, n + 37, pool, flips)
    m = ORBmatcher(0.9, True)
    prev_g = np.ascontiguousarray(np.stack([A.keys["x"], A.keys["y"]], 1).astype(np.float32))
    prev_r = prev_g.copy()
    ng, mg = m.SearchForInitialization(A, B, prev_g, window)
    nr, mr, prev_r = oracle.search_for_initialization(A, B, prev_r, window, 0.9, True)
    assert ng == nr and np.array_equal(mg, mr), (ng, nr, np.nonzero(mg != mr)[0][:10])
    assert np.array_equal(prev_g.view(np.uint32), prev_r.view(np.uint32))


@pytest.mark.parametrize("seed,nnodes", [(0, 3), (1, 30)])
def test_search_by_bow_contended(oracle, orbx_built, seed, nnodes):
    rng = np.random.default_rng(seed + 5)
    pool = rng.integers(0, 256, (4, 32), dtype=np.uint8)
    A = _contended_view(seed + 1, 2000, pool, 0.04)
    B = _contended_view(seed + 2, 2100, pool, 0.04)
    fv1 = feature_vector_csr(rng.integers(0, nnodes, len(A.keys)))
    fv2 = feature_vector_csr(rng.integers(0, nnodes, len(B.keys)))
    mp1 = _mp_ids(len(A.keys), seed + 8, 0.1)
    mp2 = _mp_ids(len(B.keys), seed + 9, 0.1, base=9000)
    m = ORBmatcher(0.9, True)
    ng, mg = m.SearchByBoWFrame(A, mp1, fv1, B, fv2)
    nr, mr = oracle.search_by_bow_frame(A, mp1, fv1, B, fv2, 0.9, True)
    assert ng == nr and np.array_equal(mg, mr)
    ng, mg = m.SearchByBoWKeyFrames(A, mp1, fv1, B, mp2, fv2)
    nr, mr = oracle.search_by_bow_keyframes(A, mp1, fv1, B, mp2, fv2, 0.9, True)
    assert ng == nr and np.array_equal(mg, mr)
