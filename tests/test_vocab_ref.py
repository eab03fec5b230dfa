"""The oracle's DBoW2 frame transform against the reference's own compiled code.

DBoW2's BowVector.cpp and FeatureVector.cpp are the only part of the reference path that
builds without OpenCV: oracle/ref_dbow2.mk compiles them where they lie under
/root/reference into oracle/_ref/libdbow2_ref.so (with the harness
oracle/ref_dbow2_capi.cpp).  The oracle's per-feature tree walk
(TemplatedVocabulary.h:1220-1259, restated: TemplatedVocabulary.h includes OpenCV) feeds
the reference containers, which accumulate (addWeight / addIfNotExist), scale and
normalise exactly as the reference binary would; the result must equal the oracle's
own BowVector / FeatureVector bit for bit (doubles included).  The GPU vocabulary tests
compare liborbx with the oracle, so this pins k_vocab_frame's double arithmetic to the
reference's code.  Skipped where neither the library nor the reference sources exist.
"""
from __future__ import annotations

import numpy as np
import pytest

import vocab_scenes as VS


@pytest.fixture(scope="module")
def ref(oracle):
    L = oracle.ref_dbow2()
    if L is None:
        pytest.skip("oracle/_ref not built and /root/reference absent")
    return L


# every (scoring, weighting) family: L1 / L2 / chi-square / KL / Bhattacharyya / dot
# product x TF-IDF / TF / IDF / BINARY, regular, irregular, tied and stopped trees
CASES = [(s, w) for s in range(6) for w in range(4)]


@pytest.mark.parametrize("scoring,weighting", CASES)
@pytest.mark.parametrize("levelsup", [0, 2, 4])
def test_oracle_frame_transform_matches_reference_containers(oracle, ref, scoring, weighting, levelsup):
    seed = 10 * scoring + weighting
    t = VS.make_vocab(seed, k=6, L=4, scoring=scoring, weighting=weighting, irregular=bool(seed % 2),
                      tie_frac=0.1, stop_frac=0.1)
    V = oracle.Vocab(t.text())
    assert V.ok
    q = VS.queries(seed + 7, t, 300)
    word, weight, node = V.transform_features(q, levelsup)
    got = V.transform(q, levelsup)
    want = oracle.ref_frame(ref, word, weight, node, weighting, scoring)
    for g, w in zip(got, want):
        assert g.dtype == w.dtype or g.dtype.kind == w.dtype.kind
        assert np.array_equal(g.view(np.uint8), w.view(np.uint8)) if g.dtype == w.dtype else np.array_equal(g, w)
    assert len(want[4]) > 100  # features kept (BINARY trees of this generator may map them to few words)


def test_reference_containers_edge_cases(oracle, ref):
    """No features; every feature stopped (weight 0); one word repeated (addWeight sums in
    feature order, addIfNotExist keeps the first)."""
    e = oracle.ref_frame(ref, np.zeros(0, np.int32), np.zeros(0), np.zeros(0, np.int32), 0, 0)
    assert len(e[0]) == 0 and len(e[2]) == 0
    s = oracle.ref_frame(ref, np.array([3, 4]), np.array([0.0, 0.0]), np.array([1, 1]), 0, 0)
    assert len(s[0]) == 0 and len(s[2]) == 0
    w = np.array([7, 7, 7], np.int32)
    v = np.array([0.1, 0.2, 0.7])
    a = oracle.ref_frame(ref, w, v, np.array([2, 2, 2]), 0, 5)  # TF-IDF, dot product: summed / size
    assert a[1][0] == (0.1 + 0.2 + 0.7) / 1.0
    b = oracle.ref_frame(ref, w, v, np.array([2, 2, 2]), 2, 5)  # IDF: first kept
    assert b[1][0] == 0.1
    assert list(a[4]) == [0, 1, 2]
