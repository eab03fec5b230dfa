"""CPU checks of the DBoW2 vocabulary oracle (oracle/orbx_oracle_vocab.c): hand-built
known answers for the reference semantics (TemplatedVocabulary.h:1127-1259,
1338-1424; BowVector.cpp; FeatureVector.cpp) and agreement with the independent
pure-Python restatement in vocab_scenes.py.  Parity unpinned: the reference ships no
vocabulary and no tests for this path."""
from __future__ import annotations

import numpy as np
import pytest

import vocab_scenes as VS
from orbslam2commentedbyxcm_amd.vocabulary import save_text


def _d(byte0: int, fill: int = 0) -> np.ndarray:
    d = np.full(32, fill, np.uint8)
    d[0] = byte0
    return d


def _tiny(scoring=0, weighting=0, wa1=1.0, wb2=2.0):
    """root -> A (0x00..), B (0xff..); A -> a1 (0x00), a2 (0x0f); B -> b1, b2 (both
    0xff..: a tie, b1 must win)."""
    parents = [0, 0, 1, 1, 2, 2]
    leaf = [0, 0, 1, 1, 1, 1]
    desc = [_d(0), _d(255, 255), _d(0), _d(0x0F), _d(255, 255), _d(255, 255)]
    weights = [0, 0, wa1, 0.5, 3.0, wb2]
    return save_text(2, 2, scoring, weighting, parents, leaf, desc, weights)


def test_known_answer_tiny(oracle):
    V = oracle.Vocab(_tiny())
    assert V.ok and V.v.nnodes == 7 and V.v.nwords == 4
    q = np.stack([_d(0), _d(0x0F), _d(0), _d(255, 255), _d(0x01)])
    bw, bv, fn, fo, fi = V.transform(q, levelsup=1)
    # words: a1=0, a2=1, b1=2 (tie with b2 resolved to the first child)
    assert bw.tolist() == [0, 1, 2]
    raw = [1.0 + 1.0 + 1.0, 0.5, 3.0]   # q0, q2, q4 -> a1 (0x01 is 1 bit from a1, 3 from a2)
    s = sum(raw)
    assert bv.tolist() == [r / s for r in raw]
    # levelsup 1 -> node at level 1: A = 1, B = 2
    assert fn.tolist() == [1, 2] and fo.tolist() == [0, 4, 5] and fi.tolist() == [0, 1, 2, 4, 3]


def test_known_answer_stopped_and_levels(oracle):
    V = oracle.Vocab(_tiny(wa1=0.0))
    q = np.stack([_d(0), _d(0x0F), _d(255, 255)])
    bw, bv, fn, fo, fi = V.transform(q, levelsup=0)  # nid at level 2 = the leaf itself
    assert bw.tolist() == [1, 2] and bv.tolist() == [0.5 / 3.5, 3.0 / 3.5]
    assert fn.tolist() == [4, 5] and fi.tolist() == [1, 2]   # stopped feature 0 is in neither
    bw, bv, fn, fo, fi = V.transform(q, levelsup=5)  # nid_level <= 0 -> root
    assert fn.tolist() == [0] and fi.tolist() == [1, 2]


@pytest.mark.parametrize("scoring,weighting,expect", [
    (5, 0, [3.0 / 3, 0.5 / 3, 3.0 / 3]),       # DotProduct + TF_IDF: / size()
    (5, 2, [1.0, 0.5, 3.0]),                   # DotProduct + IDF: first weight, no division
    (1, 3, None),                               # L2
])
def test_known_answer_weighting(oracle, scoring, weighting, expect):
    V = oracle.Vocab(_tiny(scoring, weighting))
    q = np.stack([_d(0), _d(0), _d(0), _d(0x0F), _d(255, 255)])
    bw, bv, fn, fo, fi = V.transform(q, levelsup=1)
    if expect is None:
        raw = np.array([1.0, 0.5, 3.0])
        expect = list(raw / np.sqrt(np.sum(raw * raw)))
    assert bw.tolist() == [0, 1, 2]
    assert np.allclose(bv, expect, rtol=0, atol=1e-15)


@pytest.mark.parametrize("header", ["21 2 0 0", "2 0 0 0", "2 11 0 0", "2 2 6 0", "2 2 0 4", "x"])
def test_header_rejected(oracle, header):
    assert not oracle.Vocab(header + "\n0 1 " + "0 " * 32 + " 1\n").ok


def test_empty_vocabulary(oracle):
    V = oracle.Vocab("3 2  0 0\n")
    assert V.ok and V.v.nwords == 0
    out = V.transform(np.zeros((4, 32), np.uint8))
    assert all(len(a) == 0 for a in out[:3])


@pytest.mark.parametrize("seed,kw", [
    (1, dict(k=3, L=2)),
    (2, dict(k=4, L=3, irregular=True)),
    (3, dict(k=5, L=2, tie_frac=0.3, weighting=2)),
    (4, dict(k=3, L=3, shuffle=True, scoring=1, weighting=1)),
    (5, dict(k=6, L=2, scoring=5, weighting=0, stop_frac=0.3)),
    (6, dict(k=2, L=4, irregular=True, scoring=3, weighting=3)),
])
@pytest.mark.parametrize("levelsup", [0, 1, 4])
def test_oracle_matches_python_restatement(oracle, seed, kw, levelsup):
    t = VS.make_vocab(seed, **kw)
    V = oracle.Vocab(t.text())
    assert V.ok
    q = VS.queries(seed + 100, t, 60)
    got = VS.arrays_to_maps(*V.transform(q, levelsup))
    want = VS.py_transform(t, q, levelsup)
    assert list(got[0]) == list(want[0])
    assert [got[0][w] for w in got[0]] == [want[0][w] for w in want[0]]  # bit-exact doubles
    assert got[1] == want[1]
