"""Multi-GPU layout of the hot path.

Frames are independent units of work.  One process per GPU (``torch.distributed``:
RCCL over xGMI on the GPU node, gloo on CPU for the tests) owns a contiguous slice of
the frame stream and extracts + matches it with no collective (weak scaling).

The one real exchange is cross-keyframe ``SearchForTriangulation`` (configs[3], one
keyframe per GPU): ``LocalMapping::CreateNewMapPoints`` matches a new keyframe against
its covisible neighbours (LocalMapping.cc:235-305), which live on other ranks.  Each
rank publishes its keyframe block -- keypoints, descriptors, has-MapPoint flags,
vocabulary node per keypoint (the FeatureVector), pose -- and all-gathers the
others'; the matching then runs locally on every rank.

This module is the host-staged form (numpy KeyFrameBlocks, for callers whose keyframes
live on the host).  The device-resident form -- one HBM slab per rank, all-gathered
device to device, matched by one batched launch -- is keyframes.py (configs[3]).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib as L

_MAGIC = 0x4B465842  # "BXFK"


def shard(n_frames: int, rank: int, world: int) -> range:
    """Contiguous, balanced slice of frames [0, n_frames) owned by `rank`."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_frames, world)
    lo = rank * base + min(rank, extra)
    return range(lo, lo + base + (1 if rank < extra else 0))


@dataclass
class KeyFrameBlock:
    """What SearchForTriangulation reads of one KeyFrame (ORBmatcher.cc:850-1056)."""
    keys: np.ndarray       # mvKeysUn, KEYPOINT_DTYPE (n,)
    desc: np.ndarray       # mDescriptors (n, 32) uint8
    has_mp: np.ndarray     # GetMapPoint(i) != NULL, (n,) uint8
    fv_node: np.ndarray    # vocabulary node of each keypoint (mFeatVec), (n,) int32, -1 = none
    Tcw: np.ndarray        # (3, 4) float32
    u_right: np.ndarray | None = None  # mvuRight (n,) float32 or None (monocular)

    def pack(self) -> np.ndarray:
        n = len(self.keys)
        keys = np.ascontiguousarray(self.keys, dtype=L.KEYPOINT_DTYPE)
        desc = np.ascontiguousarray(self.desc, dtype=np.uint8).reshape(n, 32)
        has = np.ascontiguousarray(self.has_mp, dtype=np.uint8).reshape(n)
        node = np.ascontiguousarray(self.fv_node, dtype=np.int32).reshape(n)
        T = np.ascontiguousarray(self.Tcw, dtype=np.float32).reshape(3, 4)
        stereo = self.u_right is not None
        head = np.array([_MAGIC, n, int(stereo), 0], dtype=np.int32)
        parts = [head.view(np.uint8), keys.view(np.uint8), desc.reshape(-1), has, node.view(np.uint8),
                 T.view(np.uint8).reshape(-1)]
        if stereo:
            parts.append(np.ascontiguousarray(self.u_right, dtype=np.float32).reshape(n).view(np.uint8))
        return np.concatenate(parts)

    @staticmethod
    def unpack(buf: np.ndarray) -> "KeyFrameBlock":
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        magic, n, stereo, _ = buf[:16].view(np.int32)
        if magic != _MAGIC:
            raise ValueError("not a keyframe block")
        o = 16

        def take(nbytes):
            nonlocal o
            v = buf[o:o + nbytes]
            o += nbytes
            return v

        keys = take(28 * n).view(L.KEYPOINT_DTYPE).copy()
        desc = take(32 * n).reshape(n, 32).copy()
        has = take(n).copy()
        node = take(4 * n).view(np.int32).copy()
        T = take(48).view(np.float32).reshape(3, 4).copy()
        ur = take(4 * n).view(np.float32).copy() if stereo else None
        if o != len(buf):
            raise ValueError("trailing bytes in keyframe block")
        return KeyFrameBlock(keys, desc, has, node, T, ur)


def allgather_keyframes(block: KeyFrameBlock, group=None, device=None) -> list[KeyFrameBlock]:
    """All-gather every rank's keyframe block (rank order).  `device`: where the
    collective runs (a CUDA device for RCCL, None / cpu for gloo)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    buf = torch.from_numpy(block.pack())
    dev = torch.device(device) if device is not None else torch.device("cpu")
    size = torch.tensor([buf.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(size) for _ in range(world)]
    dist.all_gather(sizes, size, group=group)
    cap = int(max(int(s.item()) for s in sizes))
    padded = torch.zeros(cap, dtype=torch.uint8, device=dev)
    padded[: buf.numel()] = buf.to(dev)
    outs = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(outs, padded, group=group)
    return [KeyFrameBlock.unpack(o[: int(s.item())].cpu().numpy()) for o, s in zip(outs, sizes)]


def compute_f12(T1: np.ndarray, T2: np.ndarray, fx: float, fy: float, cx: float, cy: float) -> np.ndarray:
    """LocalMapping::ComputeF12 (LocalMapping.cc:606-625) for K1 = K2 = K, float32."""
    f32 = np.float32
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], f32)
    R1, t1 = np.asarray(T1, f32)[:3, :3], np.asarray(T1, f32)[:3, 3]
    R2, t2 = np.asarray(T2, f32)[:3, :3], np.asarray(T2, f32)[:3, 3]
    R12 = R1 @ R2.T
    t12 = -R1 @ R2.T @ t2 + t1
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]], f32)
    Ki = np.linalg.inv(K).astype(f32)
    return (Ki.T @ tx @ R12 @ Ki).astype(f32)


def triangulate_with_neighbours(matcher, mine: KeyFrameBlock, neighbours: list[KeyFrameBlock], scale_factors,
                                fx: float, fy: float, cx: float, cy: float, width: int, height: int,
                                bf: float = 0.0, only_stereo: bool = False) -> list[np.ndarray]:
    """SearchForTriangulation of this rank's keyframe against each gathered neighbour
    (LocalMapping::CreateNewMapPoints' per-neighbour loop, LocalMapping.cc:247-305, with
    ORBmatcher(0.6, false), LocalMapping.cc:243).  Returns the (idx1, idx2) pairs per
    neighbour."""
    from .matcher import FrameView, feature_vector_csr

    sf = np.asarray(scale_factors, np.float32)

    def view(b: KeyFrameBlock) -> FrameView:
        return FrameView(keys=b.keys, desc=b.desc, fx=fx, fy=fy, cx=cx, cy=cy, bf=bf, max_x=float(width),
                         max_y=float(height), scale_factors=sf, level_sigma2=sf * sf,
                         Tcw=np.vstack([b.Tcw, [0, 0, 0, 1]]).astype(np.float32), u_right=b.u_right)

    v1, fv1 = view(mine), feature_vector_csr(mine.fv_node)
    out = []
    for nb in neighbours:
        F12 = compute_f12(mine.Tcw, nb.Tcw, fx, fy, cx, cy)
        out.append(matcher.SearchForTriangulation(v1, mine.has_mp, fv1, view(nb), nb.has_mp,
                                                  feature_vector_csr(nb.fv_node), F12, only_stereo))
    return out
