"""The replay's parallel forms against the sequential claim loop (tools/sim/replay_sim.py):
SearchByProjection's per-query choice (ORBmatcher.cc:61-173, 1620-1789) with blocking and
non-blocking claims (Observations() > 0 / == 0, cc:117-119), ratio test on and off, lists
that run out.  The round-4 commit (non-blocking acceptances commit with their chunk; a
keypoint keeps its last claim) must give the reference's acceptances and its final
F.mvpMapPoints.  The GPU tests check the kernels themselves against the oracle."""
import importlib.util
import random
from pathlib import Path

import pytest

_spec = importlib.util.spec_from_file_location(
    "replay_sim", Path(__file__).resolve().parent.parent / "tools" / "sim" / "replay_sim.py")
sim = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(sim)


@pytest.mark.parametrize("seed", range(4))
def test_round4_commit_equals_sequential(seed):
    rng = random.Random(100 + seed)
    for _ in range(6):
        nq = rng.choice([64, 150, 300])
        ratio = rng.random() < 0.5
        qs, bself = sim.make_scene(rng, nq, nq * rng.choice([1, 2]), ratio, rng.choice([0.0, 0.1, 0.5, 1.0]),
                                   rng.choice([4, 12, 30]))
        ref = sim.sequential(qs, bself, ratio)
        out, claims, _ = sim.chunked_nb(qs, bself, ratio)
        assert out == ref
        assert claims == sim.final_claims(qs, ref)


def test_round4_commit_needs_fewer_iterations():
    """Non-blocking acceptances were sequence points (one commit each) before round 4."""
    rng = random.Random(7)
    qs, bself = sim.make_scene(rng, 300, 300, False, 0.5, 12)
    _, it3 = sim.chunked(qs, bself, False)
    _, _, it4 = sim.chunked_nb(qs, bself, False)
    assert it4 * 3 < it3
