"""Multi-rank path: frame sharding, the keyframe-block all-gather over a
world-size-2 gloo group on CPU, and (GPU) triangulation against gathered neighbours
checked against the oracle."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

from orbslam2commentedbyxcm_amd import KEYPOINT_DTYPE
from orbslam2commentedbyxcm_amd.distributed import KeyFrameBlock, compute_f12, shard


def _block(seed: int, n: int, stereo: bool) -> KeyFrameBlock:
    rng = np.random.default_rng(seed)
    keys = np.zeros(n, KEYPOINT_DTYPE)
    keys["x"] = rng.uniform(20, 620, n)
    keys["y"] = rng.uniform(20, 460, n)
    keys["size"] = 31
    keys["angle"] = rng.uniform(0, 360, n)
    keys["response"] = rng.integers(1, 100, n)
    keys["octave"] = rng.integers(0, 8, n)
    keys["class_id"] = -1
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    has = (rng.random(n) < 0.3).astype(np.uint8)
    node = rng.integers(-1, 40, n).astype(np.int32)
    T = np.hstack([np.eye(3), rng.normal(0, 0.1, (3, 1))]).astype(np.float32)
    ur = rng.uniform(0, 600, n).astype(np.float32) if stereo else None
    return KeyFrameBlock(keys, desc, has, node, T, ur)


def _same(a: KeyFrameBlock, b: KeyFrameBlock) -> bool:
    ok = (np.array_equal(a.keys.view(np.uint8), b.keys.view(np.uint8)) and np.array_equal(a.desc, b.desc)
          and np.array_equal(a.has_mp, b.has_mp) and np.array_equal(a.fv_node, b.fv_node)
          and np.array_equal(a.Tcw, b.Tcw))
    if a.u_right is None or b.u_right is None:
        return ok and a.u_right is None and b.u_right is None
    return ok and np.array_equal(a.u_right, b.u_right)


@pytest.mark.parametrize("n,world", [(256, 1), (256, 2), (256, 8), (255, 8), (3, 8), (0, 4)])
def test_shard_partitions_frames(n, world):
    slices = [shard(n, r, world) for r in range(world)]
    flat = [i for s in slices for i in s]
    assert flat == list(range(n))
    sizes = [len(s) for s in slices]
    assert max(sizes) - min(sizes) <= 1


def test_shard_rejects_bad_rank():
    with pytest.raises(ValueError):
        shard(10, 2, 2)


@pytest.mark.parametrize("stereo", [False, True])
def test_block_roundtrip(stereo):
    b = _block(7, 123, stereo)
    assert _same(KeyFrameBlock.unpack(b.pack()), b)
    with pytest.raises(ValueError):
        KeyFrameBlock.unpack(np.zeros(64, np.uint8))


def test_compute_f12_epipolar_constraint():
    """x2^T F21 x1 = 0 for a point seen by both cameras (F12 maps kf2 points to kf1 lines)."""
    rng = np.random.default_rng(3)
    fx, fy, cx, cy = 500.0, 500.0, 320.0, 240.0
    T1 = np.hstack([np.eye(3), [[0.1], [0.0], [0.0]]]).astype(np.float32)
    c, s = np.cos(0.05), np.sin(0.05)
    R2 = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], np.float32)
    T2 = np.hstack([R2, [[-0.2], [0.05], [0.0]]]).astype(np.float32)
    F12 = compute_f12(T1, T2, fx, fy, cx, cy)
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float64)
    for _ in range(20):
        Xw = np.array([rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(4, 6)])
        x1 = K @ (T1[:, :3] @ Xw + T1[:, 3])
        x2 = K @ (T2[:, :3] @ Xw + T2[:, 3])
        x1, x2 = x1 / x1[2], x2 / x2[2]
        assert abs(x1 @ F12.astype(np.float64) @ x2) < 1e-3


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    from orbslam2commentedbyxcm_amd.distributed import allgather_keyframes

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        mine = _block(100 + rank, 50 + 37 * rank, stereo=(rank % 2 == 1))
        got = allgather_keyframes(mine)
        ok = len(got) == world and all(_same(g, _block(100 + r, 50 + 37 * r, r % 2 == 1)) for r, g in enumerate(got))
        mine_frames = list(shard(256, rank, world))
        with open(os.path.join(outdir, f"r{rank}"), "w") as f:
            f.write(f"{int(ok)} {mine_frames[0]} {mine_frames[-1]}\n")
    finally:
        dist.destroy_process_group()


def test_allgather_keyframes_gloo_world2(tmp_path):
    import torch.multiprocessing as mp

    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    lines = [open(tmp_path / f"r{r}").read().split() for r in range(world)]
    assert all(l[0] == "1" for l in lines), lines
    assert lines[0][1:] == ["0", "127"] and lines[1][1:] == ["128", "255"]


@pytest.mark.gpu
def test_triangulate_with_gathered_neighbours(oracle, orbx_built):
    """World size 1 on the GPU box: gather (identity) then triangulate this keyframe
    against two neighbours; every pair list equals the oracle's SearchForTriangulation."""
    import torch.distributed as dist

    import match_scenes as S
    from orbslam2commentedbyxcm_amd.distributed import allgather_keyframes, triangulate_with_neighbours
    from orbslam2commentedbyxcm_amd.matcher import ORBmatcher, feature_vector_csr

    A, B = S.two_views(oracle, 4)
    _, C = S.two_views(oracle, 4, dx=-5, dy=6)
    rng = np.random.default_rng(4)
    blocks = []
    for V in (A, B, C):
        has = (rng.random(len(V.keys)) < 0.2).astype(np.uint8)
        blocks.append(KeyFrameBlock(V.keys, V.desc, has, S.vocab_nodes(V).astype(np.int32),
                                    np.asarray(V.Tcw, np.float32)[:3, :4]))
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        got = allgather_keyframes(blocks[0])
    finally:
        dist.destroy_process_group()
    assert _same(got[0], blocks[0])
    m = ORBmatcher(0.6, False)
    pairs = triangulate_with_neighbours(m, got[0], blocks[1:], A.scale_factors, S.FX, S.FY, S.CX, S.CY, 640, 480)
    for nb, V, pg in zip(blocks[1:], (B, C), pairs):
        F12 = compute_f12(blocks[0].Tcw, nb.Tcw, S.FX, S.FY, S.CX, S.CY)
        pr = oracle.search_for_triangulation(A, blocks[0].has_mp, feature_vector_csr(blocks[0].fv_node), V,
                                             nb.has_mp, feature_vector_csr(nb.fv_node), F12, False, False)
        assert np.array_equal(pg, pr), (len(pg), len(pr))
        assert len(pr) > 20


# ---- configs[3]: keyframe slabs, the neighbour plan and the slab all-gather (keyframes.py)

def test_slab_layout_fields_disjoint_and_aligned():
    from orbslam2commentedbyxcm_amd.keyframes import SlabLayout
    lay = SlabLayout(5, 1301)
    spans = sorted((lay.offset[n], lay.offset[n] + 5 * lay.stride[n]) for n, *_ in SlabLayout.FIELDS)
    assert all(a % 256 == 0 for a, _ in spans)
    assert all(spans[i][1] <= spans[i + 1][0] for i in range(len(spans) - 1))
    assert spans[-1][1] <= lay.nbytes and lay.nbytes % 256 == 0
    assert lay.address(1000, 2, 3, "desc") == 1000 + 2 * lay.nbytes + lay.offset["desc"] + 3 * 1301 * 32


@pytest.mark.parametrize("world,batch", [(1, 16), (2, 8), (8, 4)])
def test_neighbour_plan(world, batch):
    from orbslam2commentedbyxcm_amd import synth
    from orbslam2commentedbyxcm_amd.keyframes import (EUROC, plan_neighbours, record_index, stream_poses,
                                                      window_index)
    s = EUROC
    N = world * batch
    seq = synth.StereoSequence.__new__(synth.StereoSequence)  # offsets only (no canvas needed)
    rng = np.random.default_rng(1)
    off = np.cumsum(rng.integers(-16, 17, (N, 2)), axis=0)
    depth = s["bf"] / 13
    T = stream_poses(off, s["fx"], s["fy"], depth)
    mb = s["bf"] / s["fx"]
    plans = [plan_neighbours(T, r, world, batch, 4, mb, s) for r in range(world)]
    allpairs = set()
    for r, pl in enumerate(plans):
        assert len(pl.pairs) + pl.skipped_baseline == batch * min(4, N - 1)
        for p in range(len(pl.pairs)):
            g, h = int(pl.kf1_window[p]), int(pl.kf2_window[p])
            assert g % world == r and g != h and abs(g - h) <= 4
            assert tuple(pl.pairs[p]) == (record_index(g, world, batch), record_index(h, world, batch))
            # baseline test passed: camera centres at least mb apart
            assert np.hypot(*(off[g] - off[h])) * depth / s["fx"] >= mb * (1 - 1e-5)
            assert np.allclose(pl.F12[p], compute_f12(T[g][:3], T[h][:3], s["fx"], s["fy"], s["cx"], s["cy"]))
            allpairs.add((g, h))
    # every rank plans its own keyframes: the union is the whole window's plan
    assert {g for g, _ in allpairs} <= set(range(N))
    assert all(window_index(g % world, g // world, world) == g for g in range(N))
    del seq


def _slab_worker(rank, world, port, outdir, force=False):
    import torch
    import torch.distributed as dist

    from orbslam2commentedbyxcm_amd.keyframes import SlabLayout, gather_slabs

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        lay = SlabLayout(3, 50)
        slab = torch.zeros(lay.nbytes, dtype=torch.uint8)
        v = lay.views(slab)
        for i in range(3):
            v["desc"][i].fill_(10 * rank + i)
            v["n"][i] = 100 * rank + i
            v["fv_off"][i] = torch.arange(51, dtype=torch.int32) + rank
        gathered = torch.zeros(world * lay.nbytes, dtype=torch.uint8)
        gather_slabs(slab, gathered, force=force)
        buf = gathered.numpy()
        ok = True
        for q in range(world):
            for i in range(3):
                d = buf[lay.address(0, q, i, "desc"):][:50 * 32]
                n = buf[lay.address(0, q, i, "n"):][:4].view(np.int32)[0]
                fo = buf[lay.address(0, q, i, "fv_off"):][:51 * 4].view(np.int32)
                ok &= bool((d == 10 * q + i).all()) and n == 100 * q + i and bool((fo == np.arange(51) + q).all())
        with open(os.path.join(outdir, f"s{rank}"), "w") as f:
            f.write(f"{int(ok)}\n")
    finally:
        dist.destroy_process_group()


def test_gather_slabs_gloo_world2(tmp_path):
    import torch.multiprocessing as mp

    world = 2
    mp.spawn(_slab_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert all(open(tmp_path / f"s{r}").read().strip() == "1" for r in range(world))


def test_gather_slabs_forced_world1(tmp_path):
    """collective=True at world size 1: the exchange goes through the process group's
    all_gather (gloo here; RCCL's all_gather_into_tensor on the GPU test) and lands the
    slab in the gathered buffer."""
    import torch.multiprocessing as mp

    mp.spawn(_slab_worker, args=(1, _free_port(), str(tmp_path), True), nprocs=1, join=True)
    assert open(tmp_path / "s0").read().strip() == "1"
