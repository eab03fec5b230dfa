"""The H1 allocator measurement's transcription (tests/h1_glibc/octree_glibc.cpp) agrees
with the oracle on every level whose output does not depend on the tie order, under glibc
in both arenas and both allocation modes, and on every level -- tie-deciding ones included --
under a monotonic bump allocator, whose address order is the shipped rule's
(tests/h1_glibc_measure.py)."""
import tempfile
from pathlib import Path

import pytest

import h1_glibc_measure as H


@pytest.mark.parametrize("prm", [(1000, 1.2, 8, 20, 7), (5000, 1.2, 12, 20, 7)])
def test_glibc_octree_matches_oracle_where_untied(oracle, prm):
    from orbslam2commentedbyxcm_amd import synth
    frames, _ = synth.sequence(1000, 3)
    with tempfile.TemporaryDirectory() as d:
        exe = H.build(Path(d))
        r = H.measure(frames, prm, 3, exe, Path(d))
    assert r["bump_allocator"]["mismatched_vs_shipped"] == 0, r["bump_allocator"]
    assert r["bump_allocator"]["tie_deciding_levels"] >= 1
    for k, v in r.items():
        if isinstance(v, dict) and k != "bump_allocator":
            assert v["untied_levels_mismatched"] == 0, (k, v)
            assert v["tie_deciding_levels"] + 0 >= 1
            assert (v["glibc_equals_shipped"] + v["glibc_equals_opposite"] + v["glibc_equals_neither"]
                    == v["tie_deciding_levels"])
