"""GPU parity of the headline path itself: SequencePipeline (what bench.py times) over
device-resident batches, every frame's extraction and every pair's TrackWithMotionModel
matches against the oracle.

Covers the configurations the bench runs and their neighbours: B = 256 in two 128-frame
lanes (nframes % 8 == 0: the XCD-swizzled grids of orbx_extract.hip's xcd_frame_block),
pipelined (double-buffered, matching of batch j-1 beside extraction of batch j) and not;
B = 16 in one lane; B = 8 and 12 with lanes and pipelining; plus the octree status words
(orbx_extractor_status) on the device path, clean and forced to overflow.
"""
import numpy as np
import pytest

from oracle import checks
from orbslam2commentedbyxcm_amd import OrbxError, ORBextractor, synth
from orbslam2commentedbyxcm_amd.pipeline import SequencePipeline, sequence_poses

pytestmark = pytest.mark.gpu


def _run(B, lanes, pipelined, steps, seed=1000, matcher_mode=None, lane_offset=2, match_after=0, cu_stride=1,
         priority=0):
    import torch

    frames, off = synth.sequence(seed, B)
    T = sequence_poses(off)
    pl = SequencePipeline(B, 640, 480, lanes=lanes, pipelined=pipelined, matcher_mode=matcher_mode,
                          lane_offset_stage=lane_offset, match_after_stage=match_after, match_cu_stride=cu_stride,
                          match_priority=priority)
    d_frames = torch.from_numpy(frames).to(pl.dev)
    d_T = torch.from_numpy(T).to(pl.dev)
    torch.cuda.synchronize()
    pl.run(d_frames, d_T, steps)
    torch.cuda.synchronize()
    return frames, T, pl


@pytest.mark.parametrize("B,lanes,pipelined,steps,mode,offset,after",
                         [(256, 2, True, 2, None, 2, 0), (16, 1, False, 1, None, 2, 0), (8, 2, True, 3, None, 2, 0),
                          (12, 2, False, 2, None, 2, 0), (256, 2, False, 1, None, 2, 0), (256, 2, True, 2, 2, 2, 0),
                          (13, 2, True, 3, 2, 2, 0), (256, 2, True, 2, 4, 0, 0), (24, 3, True, 3, 0, 1, 0),
                          (16, 2, True, 3, None, 0, 2), (16, 2, True, 3, None, 4, 0)])
def test_sequence_pipeline_matches_oracle(oracle, orbx_built, B, lanes, pipelined, steps, mode, offset, after):
    """Every frame and pair of the newest batch == the oracle, over matcher footprints
    (None = the default lean split), lanes in step (offset 0) or out of phase, and the
    matcher started after a later extraction stage of the next batch (after > 0)."""
    frames, T, pl = _run(B, lanes, pipelined, steps, matcher_mode=mode, lane_offset=offset, match_after=after)
    res = pl.host_results()
    assert not pl.status().any()
    r = checks.check_sequence(frames, T, res, pl.sf)
    assert r["frames_mismatched"] == 0, r
    assert r["pairs_mismatched"] == 0, r
    assert r["mean_matches_per_pair_ref"] > 200
    # the lane boundary pair (last frame of lane 0 -> first frame of lane 1) is matched
    b1 = pl.bounds[0][1]
    if lanes > 1 and b1 < B:
        assert res["nm"][b1] > 200


@pytest.mark.parametrize("cu_stride,priority", [(4, 0), (1, -1)])
def test_matcher_stream_forms_match_oracle(oracle, orbx_built, cu_stride, priority):
    """The matcher on a CU-masked stream (orbx_stream_create with cu_stride 4) or on a
    high-priority one: the same output, and the pipeline releases its stream."""
    frames, T, pl = _run(24, 2, True, 3, seed=1100, cu_stride=cu_stride, priority=priority)
    res = pl.host_results()
    r = checks.check_sequence(frames, T, res, pl.sf)
    assert r["frames_mismatched"] == 0 and r["pairs_mismatched"] == 0, r
    pl.close()
    assert pl._own_ms is None


def test_device_status_reports_forced_overflow(oracle, orbx_built):
    """A node capacity below the algorithm's bound truncates the octree: the device path
    returns normally but orbx_extractor_status flags every frame; the host path fails
    with ORBX_ERR_STATE; restoring the capacity restores bit-exact output."""
    import torch

    frames, _ = synth.sequence(7, 8)
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    cap = ex.max_keypoints(640, 480)
    dev = torch.device("cuda", 0)
    d_frames = torch.from_numpy(frames).to(dev)
    kps = torch.empty((8, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.empty((8, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.empty((8,), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ex.extract_batch_device(d_frames, kps, desc, n)
    assert not ex.status().any()
    ex.set_node_capacity(40)  # below level 0's 217 + 4
    ex.extract_batch_device(d_frames, kps, desc, n)
    st = ex.status()
    assert len(st) == 8 and (st & ORBextractor.STATUS_NODE_OVERFLOW).all(), st
    with pytest.raises(OrbxError) as e:
        ex(frames[0])
    assert e.value.code == -5 and "overflow" in str(e.value)
    ex.set_node_capacity(0)
    kp, ds = ex(frames[0])
    kr, dr, _ = oracle.extract(frames[0], oracle.params(1000, 1.2, 8, 20, 7))
    assert np.array_equal(kp.view(np.uint8), kr.view(np.uint8)) and np.array_equal(ds, dr)
    assert not ex.status().any()


@pytest.mark.parametrize("B,lanes,pipelined,steps,nbuf,fip", [(16, 2, True, 5, 2, True), (24, 3, True, 4, 2, True),
                                                              (12, 1, False, 3, 2, True), (256, 2, True, 3, 2, True),
                                                              (16, 2, True, 5, 3, True), (256, 2, True, 4, 3, True),
                                                              (16, 2, True, 5, 3, False)])
def test_sequence_pipeline_distinct_batch_every_step(oracle, orbx_built, B, lanes, pipelined, steps, nbuf, fip):
    """Every step gets its own batch (its own canvas and poses) and steps are issued
    back to back with no host synchronisation; each batch's outputs are copied out on the
    matcher stream as soon as its matching is enqueued (SequencePipeline.on_matched, before
    the buffer is released), so a buffer reused too early, an event waited on the wrong
    buffer or a batch matched with another batch's poses shows up as a mismatch.  Two
    buffer sets and three (the bench's at <= 8 levels); the first batch's lanes in phase
    (the default) or offset from the start."""
    import torch

    batches = [synth.sequence(2000 + j, B) for j in range(steps)]
    snaps = []
    pl = None

    def grab(b):
        r = pl.results(b)
        snaps.append({k: v.clone() for k, v in r.items()})

    pl = SequencePipeline(B, 640, 480, lanes=lanes, pipelined=pipelined, on_matched=grab, nbuf=nbuf,
                          first_in_phase=fip)
    dev_in = [(torch.from_numpy(f).to(pl.dev), torch.from_numpy(sequence_poses(o)).to(pl.dev)) for f, o in batches]
    torch.cuda.synchronize()
    with torch.cuda.stream(pl.ms):  # the clones run on the matcher stream, after the matching
        for frames, T in dev_in:
            pl.step(frames, T)
        pl.drain()
    torch.cuda.synchronize()
    assert len(snaps) == steps
    from orbslam2commentedbyxcm_amd import _lib as L
    for j, ((frames, off), snap) in enumerate(zip(batches, snaps)):
        cap = pl.cap
        res = {"kps": snap["kps"].cpu().numpy().view(np.uint8).reshape(B, cap, 28).view(L.KEYPOINT_DTYPE)
               .reshape(B, cap), "desc": snap["desc"].cpu().numpy(), "n": snap["n"].cpu().numpy(),
               "mp": snap["mp"].cpu().numpy(), "nm": snap["nm"].cpu().numpy()}
        r = checks.check_sequence(frames, sequence_poses(off), res, pl.sf)
        assert r["frames_mismatched"] == 0 and r["pairs_mismatched"] == 0, (j, r)
        assert r["mean_matches_per_pair_ref"] > 200, (j, r)


@pytest.mark.parametrize("B,lanes,pipelined,steps,mode", [(16, 2, True, 3, None), (12, 1, False, 2, None),
                                                          (256, 2, True, 2, None), (24, 2, True, 3, 2)])
def test_sequence_pipeline_local_map_matches_oracle(oracle, orbx_built, B, lanes, pipelined, steps, mode):
    """The front end with TrackLocalMap: MapPoints of every keypoint (CreateNewKeyFrame's
    UnprojectStereo at the model depth), TrackWithMotionModel against them, then
    SearchLocalPoints against the MapPoints of the three previous frames; every frame's
    final mvpMapPoints and both match counts against the oracle, on distinct batches."""
    import torch

    batches = [synth.sequence(3000 + j, B) for j in range(steps)]
    snaps = []
    pl = None

    def grab(b):
        snaps.append({k: v.clone() for k, v in pl.results(b).items()})

    pl = SequencePipeline(B, 640, 480, lanes=lanes, pipelined=pipelined, on_matched=grab, local_map=True,
                          matcher_mode=mode)
    dev_in = [(torch.from_numpy(f).to(pl.dev), torch.from_numpy(sequence_poses(o)).to(pl.dev)) for f, o in batches]
    torch.cuda.synchronize()
    with torch.cuda.stream(pl.ms):
        for frames, T in dev_in:
            pl.step(frames, T)
        pl.drain()
    torch.cuda.synchronize()
    assert len(snaps) == steps
    from orbslam2commentedbyxcm_amd import _lib as L
    cap = pl.cap
    for j, ((frames, off), snap) in enumerate(zip(batches, snaps)):
        res = {k: v.cpu().numpy() for k, v in snap.items() if k != "kps"}
        res["kps"] = snap["kps"].cpu().numpy().view(np.uint8).reshape(B, cap, 28).view(L.KEYPOINT_DTYPE).reshape(B, cap)
        r = checks.check_sequence_local(frames, sequence_poses(off), res, pl.sf, cap)
        assert r["bit_exact"], (j, r)
        assert r["mean_matches_per_pair_ref"] > 200 and r["mean_local_matches_ref"] > 50, (j, r)


def test_sequence_pipeline_local_map_c5_large_local_map(oracle, orbx_built):
    """configs[4] (5000 features x 12 levels) with TrackLocalMap: each frame's local map
    is the MapPoints of its three predecessors, 3 x cap > 8192 entries (more than the 13-bit
    keypoint positions of the grids can name: queries are not position-encoded)."""
    import torch

    prm = (5000, 1.2, 12, 20, 7)
    B = 8
    frames, off = synth.sequence(3100, B)
    T = sequence_poses(off)
    pl = SequencePipeline(B, 640, 480, lanes=2, pipelined=True, params=prm, local_map=True)
    assert 3 * pl.cap > 8192
    d_frames = torch.from_numpy(frames).to(pl.dev)
    d_T = torch.from_numpy(T).to(pl.dev)
    torch.cuda.synchronize()
    pl.run(d_frames, d_T, 2)
    torch.cuda.synchronize()
    res = pl.host_results()
    r = checks.check_sequence_local(frames, T, res, pl.sf, pl.cap, params=prm)
    assert r["bit_exact"], r
    assert r["mean_local_matches_ref"] > 50, r
    pl.close()


def test_sequence_pipeline_configs4_bench_shape(oracle, orbx_built):
    """configs[4]'s bench shape exactly: B = 256 in two 128-frame lanes, 5000 features x 12
    levels (two pyramid segments), the default lane offset for deep pyramids (3 since round
    5: lane 1 starts after lane 0's FAST cells), the LDS-DMA describe, the lean split matcher
    with its per-window-class scoring lanes, pipelined; every frame and every pair of the
    newest batch against the oracle."""
    prm = (5000, 1.2, 12, 20, 7)
    import torch

    frames, off = synth.sequence(1000, 256)
    T = sequence_poses(off)
    pl = SequencePipeline(256, 640, 480, lanes=2, pipelined=True, params=prm)
    assert pl.lane_offset_stage == 3 and pl.lane_ev is not None and pl.S == 2
    d_frames = torch.from_numpy(frames).to(pl.dev)
    d_T = torch.from_numpy(T).to(pl.dev)
    torch.cuda.synchronize()
    pl.run(d_frames, d_T, 3)
    torch.cuda.synchronize()
    res = pl.host_results()
    assert not pl.status().any()
    r = checks.check_sequence(frames, T, res, pl.sf, params=prm)
    assert r["frames_checked"] == 256 and r["pairs_checked"] == 255
    assert r["frames_mismatched"] == 0 and r["pairs_mismatched"] == 0, r
    assert r["mean_matches_per_pair_ref"] > 1000, r
    pl.close()


def test_sequence_pipeline_posed_b256(oracle, orbx_built):
    """The headline pipeline (B = 256, two lanes, pipelined) on a posed batch: every Tcw a
    full rotation, the camera rolling 5-14 degrees between frames, so the rotation
    histogram of every pair (ORBmatcher.cc:1750-1786) has its dominant bin off zero on most
    pairs; every frame and pair against the oracle."""
    import torch

    import match_scenes as S

    imgs, _, T = S.posed_walk(40, 256)
    pl = SequencePipeline(256, 640, 480, lanes=2, pipelined=True, depth=S.Z0)
    d_frames = torch.from_numpy(imgs).to(pl.dev)
    d_T = torch.from_numpy(T).to(pl.dev)
    torch.cuda.synchronize()
    pl.run(d_frames, d_T, 2)
    torch.cuda.synchronize()
    res = pl.host_results()
    assert not pl.status().any()
    r = checks.check_sequence(imgs, T, res, pl.sf, depth=S.Z0)
    assert r["frames_mismatched"] == 0 and r["pairs_mismatched"] == 0, r
    assert r["mean_matches_per_pair_ref"] > 300, r
    dom = []
    for b in range(1, 256):
        n0, n1 = int(res["n"][b - 1]), int(res["n"][b])
        h = S.rotation_bins(res["kps"][b - 1][:n0], res["kps"][b][:n1], res["mp"][b][:n1])
        dom.append(int(np.argmax(h)))
    assert sum(d != 0 for d in dom) > 200, dom
    pl.close()


def test_sequence_pipeline_retry_below_20(oracle, orbx_built):
    """TrackWithMotionModel's second search (Tracking.cc:988-994): frame 5 keeps texture in
    one 140 px window (about a hundred keypoints) and frame 6's pose is off by 25 px, so
    pair 6's search at th = 15 finds fewer than 20 matches and the one at 30 more.  Every
    frame and pair against the oracle, which searches
    again the same way; and the same pipeline with the retry off against one search."""
    import torch

    from oracle import checks
    from orbslam2commentedbyxcm_amd import synth
    from orbslam2commentedbyxcm_amd.pipeline import SequencePipeline, sequence_poses
    frames, off = synth.sequence(3, 8)
    keep = np.zeros((480, 640), bool)
    keep[200:340, 260:400] = True
    frames[5][~keep] = 128
    T = sequence_poses(off)
    T[6, 3] += np.float32(25 * 5.0 / 500.0)
    dev = torch.device("cuda", 0)
    d_f, d_T = torch.from_numpy(frames).to(dev), torch.from_numpy(T).to(dev)
    for retry in (20, 0):
        pl = SequencePipeline(8, 640, 480, retry_below=retry)
        pl.run(d_f, d_T, 2)
        torch.cuda.synchronize(dev)
        res = pl.host_results()
        r = checks.check_sequence(frames, T, res, pl.sf, retry=bool(retry))
        assert r["bit_exact"], r
        nm = res["nm"]
        assert min(nm[b] for b in (1, 2, 3, 4, 7)) > 200, nm
        if retry:
            assert nm[6] >= 20, nm
        else:
            assert nm[6] < 20, nm
        pl.close()
