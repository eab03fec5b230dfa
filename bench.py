#!/usr/bin/env python3
"""bench.py -- ORB extraction throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (BASELINE.json configs[1]): a batch of B=256 synthetic 640x480 grayscale
frames, nFeatures=1000, scaleFactor 1.2, 8 levels, FAST 20/7, extract-only, with a
bit-exact descriptor check of a few frames against the CPU oracle outside the timed
region.  A "step" = ORBextractor::operator() over the whole batch (device-resident
frames in HBM -> keypoints + descriptors in HBM), one launch sequence on the
extractor's HIP stream.  N>1: one process per GPU, each rank extracts its own batch
(frames are independent: no data-path collective), "scaling": "weak".

Prints ONE JSON line on rank 0 (contract in the task statement): value = frames/s
of the whole job; roofline for the dominant kernel (HIP-event timed per stage on the
extractor's stream); cpu_baseline = the oracle (C restatement) on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def level_areas(W, H, nlevels=8, scale=1.2):
    """Level sizes as ORBextractor.cc:1641-1643 computes them (float inv scale, cvRound)."""
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(scale))))
    out = []
    for l in range(nlevels):
        inv = np.float32(1.0) / s[l]
        w = int(np.rint(np.float32(W) * inv))
        h = int(np.rint(np.float32(H) * inv))
        out.append((w, h))
    return out


def stage_bytes(W, H, n_kps, nlevels=8, scale=1.2):
    """Algorithmic bytes per frame of each stage."""
    A = [w * h for (w, h) in level_areas(W, H, nlevels, scale)]
    P = sum(A)
    return {
        # read input, write every level (level 0 copied), read levels 0..L-2 as resize sources
        "pyramid": A[0] + P + (P - A[-1]),
        # read every level once, write its Gaussian-blurred copy and its FAST strength map
        "score_blur": 3 * P,
        # read the strength map of every FAST detection window once
        "fast_cells": sum((w - 38) * (h - 38) for (w, h) in level_areas(W, H, nlevels, scale)),
        # candidates in, kept keypoints out: 4 B each, ~3x n_kps candidates per level budget
        "octree": 8 * n_kps,
        # 28 B keypoint + 32 B descriptor out per keypoint (patch reads are L2 hits)
        "describe": 60 * n_kps,
        # SURVEY.md §8(d) canonical whole-pipeline figure
        "total": A[0] + (P - A[0]) + 3 * P + 60 * n_kps,
    }


def cpu_baseline(frames_np, seconds: float, threads: int):
    """Oracle (TEST INFRASTRUCTURE) on host cores: frames/s over a bounded sample."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    O.build()
    p = O.params(1000, 1.2, 8, 20, 7)
    n = len(frames_np)
    done = [0] * threads
    stop = time.perf_counter() + seconds

    def worker(t):
        i = t
        while time.perf_counter() < stop:
            O.extract(frames_np[i % n], p)
            done[t] += 1
            i += threads

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(worker, range(threads)))
    el = time.perf_counter() - t0
    return sum(done) / el, sum(done), el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, available cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-frames", type=int, default=2)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    B, W, H = args.batch, args.width, args.height

    # Render frames before anything touches the GPU (the pool forks).
    frames_np = None
    from orbslam2commentedbyxcm_amd import synth
    frames_np = synth.frames(B, W, H, first_seed=rank * B, workers=min(16, os.cpu_count() or 1))

    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from orbslam2commentedbyxcm_amd import ORBextractor
    ex = ORBextractor(1000, 1.2, 8, 20, 7, device=local_rank)
    cap = ex.max_keypoints(W, H)
    d_frames = torch.from_numpy(frames_np).to(dev)
    d_kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
    d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.empty((B,), dtype=torch.int32, device=dev)
    sync_all = torch.cuda.synchronize
    sync_all(dev)  # frames uploaded on torch's stream before the extractor's stream reads them

    def step():
        ex.extract_batch_device(d_frames, d_kps, d_desc, d_n)

    def sync():
        torch.cuda.synchronize(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_frames = B * args.steps * world
    value = total_frames / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # keypoint statistics of this batch
    n_host = d_n.cpu().numpy()
    mean_kps = float(n_host.mean())

    # per-stage HIP-event timing on the extractor's stream (separate, untimed pass)
    ex.set_timing(True)
    reps = 5
    acc = {}
    for _ in range(reps):
        step()
        st = ex.stage_times()
        for k, v in st.items():
            acc[k] = acc.get(k, 0.0) + v
    sync()
    ex.set_timing(False)
    stage_ms = {k: v / reps for k, v in acc.items()}
    bytes_pf = stage_bytes(W, H, mean_kps)
    kernels = {k: v for k, v in stage_ms.items() if k != "total"}
    dom = max(kernels, key=kernels.get)
    achieved = bytes_pf[dom] * B / (stage_ms[dom] * 1e-3) / 1e9
    pipeline_gbs = bytes_pf["total"] * B / (stage_ms["total"] * 1e-3) / 1e9

    # bit-exact descriptor check of a few frames vs the oracle (outside the timed region)
    parity = None
    if rank == 0 and args.parity_frames > 0:
        from oracle import oracle as O
        O.build()
        p = O.params(1000, 1.2, 8, 20, 7)
        kps_all = d_kps.cpu().numpy()
        desc_all = d_desc.cpu().numpy()
        ok = True
        for b in range(min(args.parity_frames, B)):
            kr, dr, _ = O.extract(frames_np[b], p)
            n = int(n_host[b])
            kg = kps_all[b, :n].view(np.uint8).reshape(n, 28)
            kref = kr.view(np.uint8).reshape(len(kr), 28)
            ok &= n == len(kr) and np.array_equal(kg, kref) and np.array_equal(desc_all[b, :n], dr)
        parity = {"frames_checked": min(args.parity_frames, B), "bit_exact": bool(ok)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        fps, nfr, el = cpu_baseline(frames_np[:32], args.cpu_seconds, threads)
        cpu = {"value": round(fps, 2), "unit": "frames/s", "cores": threads, "kind": "port",
               "sample": f"{nfr} synthetic 640x480 frames (32 distinct) in {el:.1f}s, oracle C restatement "
                         f"of ORBextractor::operator(), -O2 scalar, {threads} threads"}

    if rank == 0:
        out = {
            "metric": "frames/s ORB extract+match, 640x480 1000-feat, 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": "configs[1]: batch of 256 synthetic 640x480 gray frames, nFeatures=1000, "
                                   "scale 1.2, 8 levels, FAST 20/7, extract-only",
                       "global_batch": B * world, "frames_per_gpu_step": B, "width": W, "height": H,
                       "parallelism": f"frame-sharded x{world}"},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                         "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
                         "pipeline_algorithmic_GBs": round(pipeline_gbs, 2)},
            "cpu_baseline": cpu,
            "parity": parity,
            "mean_keypoints_per_frame": round(mean_kps, 1),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
