"""configs[3] on one GPU: the frame-sharded stereo keyframe pipeline
(orbslam2commentedbyxcm_amd/keyframes.py) -- extraction of L and R, ComputeStereoMatches,
ComputeBoW, close-point MapPoints and the batched SearchForTriangulation against stream
neighbours -- checked keyframe by keyframe and pair by pair against the oracle, including
the double-buffered (pipelined) steps."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run_snapshots(pl, steps):
    """Issue `steps` steps back to back (no host synchronisation between them); each
    step's outputs are cloned on the triangulation stream when it is enqueued (before its
    set is released), then returned as host dicts with the window each step used."""
    import torch

    snaps = []

    def grab(k):
        snaps.append((pl.window_of[k], {name: t.clone() for name, t in pl.results(k).items()}))

    pl.on_step_done = grab
    with torch.cuda.stream(pl.ts):
        pl.run(steps)
    torch.cuda.synchronize()
    assert len(snaps) == steps
    return [(w, pl.to_host(r)) for w, r in snaps]


@pytest.mark.parametrize("B,nn,steps,windows", [(8, 4, 4, 2), (12, 10, 3, 3)])
def test_keyframe_pipeline_matches_oracle(oracle, orbx_built, B, nn, steps, windows):
    """Every step (its own keyframe window: same poses, another texture), not only the
    last, against the oracle."""
    import euroc_bench as E
    from orbslam2commentedbyxcm_amd import synth
    from orbslam2commentedbyxcm_amd.keyframes import StereoKeyFramePipeline
    # a smaller tree of the same depth (k=8, L=6: FeatureVector nodes at level 2, 64 of them)
    pl = StereoKeyFramePipeline(B, 0, 1, device=0, nn=nn, vocab_text=synth.vocabulary_text(11, 8, 6, 0, 0),
                                windows=windows)
    assert len(pl.plan.pairs) > B
    snaps = _run_snapshots(pl, steps)
    assert pl.status()
    oks = {}
    for j, (w, res) in enumerate(snaps):
        assert w == j % windows
        ok = oks.setdefault(w, E.OracleKeyFrames(oracle, pl, oracle.Vocab(pl.vocab_text), window=w))
        r = E.check(pl, ok, res, B, 8)
        assert r["bit_exact"], (j, r)
        assert r["pairs_checked"] == len(pl.plan.pairs)
        assert r["mean_triangulation_matches_ref"] > 10, r
        assert (res["ur"] >= 0).sum() > 50 * B


def _rank(rank, world, port, outdir, backend="gloo", B=6, steps=4):
    import json
    import os

    import torch
    import torch.distributed as dist

    import euroc_bench as E
    from oracle import oracle as O
    from orbslam2commentedbyxcm_amd import synth
    from orbslam2commentedbyxcm_amd.keyframes import StereoKeyFramePipeline

    # several ranks on the one GPU of the test box: gloo carries the slab exchange (the
    # RCCL all_gather_into_tensor needs one GPU per rank); everything else is the N-GPU path.
    # backend "nccl" (world 1): the RCCL collective itself, forced at one rank
    kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world, **kw)
    try:
        pl = StereoKeyFramePipeline(B, rank, world, device=0, nn=4, vocab_text=synth.vocabulary_text(11, 8, 6, 0, 0),
                                    windows=2, collective=True)
        assert pl.collective and pl.gathered is not None
        snaps = _run_snapshots(pl, steps)
        O.build()
        oks = {}
        steps = []
        for j, (w, res) in enumerate(snaps):
            ok = oks.setdefault(w, E.OracleKeyFrames(O, pl, O.Vocab(pl.vocab_text), window=w))
            r = E.check(pl, ok, res, B, 4)
            r["window"] = w
            steps.append(r)
        out = {"pairs": len(pl.plan.pairs), "status": pl.status(), "steps": steps,
               "backend": dist.get_backend()}
        with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
            json.dump(out, f)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_keyframe_pipeline_world2_gloo_on_one_gpu(orbx_built, tmp_path):
    """The N-rank layout at world size 2: keyframe g on rank g % 2, neighbours read from the
    gathered slabs (the other rank's keyframes).  Four pipelined steps over two keyframe
    windows; every step's keyframes, gathered neighbours and pair lists bit-exact vs the
    oracle (a gather that overwrote neighbours still being read would mix two windows)."""
    import json
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rank, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        out = json.loads(open(tmp_path / f"r{r}.json").read())
        assert out["status"] and len(out["steps"]) == 4, out
        for j, st in enumerate(out["steps"]):
            assert st["window"] == j % 2 and st["bit_exact"], (r, j, st)
            assert st["gathered_neighbours_checked"] > 6 and st["pairs_checked"] == out["pairs"] > 6, (r, j, st)


def test_keyframe_pipeline_rccl_allgather_world1(orbx_built, tmp_path):
    """The RCCL branch of gather_slabs on hardware: a one-rank nccl (RCCL) group with the
    exchange forced (collective=True), so every step's slab goes through
    all_gather_into_tensor into that set's gathered buffer and the triangulation reads its
    neighbours from there.  Six pipelined steps over two alternating keyframe windows with
    no host synchronisation between them (the RCCL enqueue is asynchronous: it is ordered
    only by the matcher stream it is issued on, and the triangulation stream waits on that
    stream's event); every step's keyframes, gathered copies and pair lists vs the oracle."""
    import json
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_rank, args=(1, port, str(tmp_path), "nccl", 8, 6), nprocs=1, join=True)
    out = json.loads(open(tmp_path / "r0.json").read())
    assert out["backend"] == "nccl" and out["status"] and len(out["steps"]) == 6, out
    for j, st in enumerate(out["steps"]):
        assert st["window"] == j % 2 and st["bit_exact"], (j, st)
        assert st["gathered_neighbours_checked"] >= 8 and st["pairs_checked"] == out["pairs"] > 8, (j, st)
