#!/usr/bin/env python3
"""configs[4] throughput: TUM RGB-D frames at 5000 features x 12 levels, with tracking.

    python bench.py --workload tum5k [--gpus N] [--steps K] [--warmup W] [--batch B]

(bench.py's configs[4] leg; it runs the oracle as its parity check and CPU baseline.)

Workload: B = 256 synthetic 640x480 RGB-D frames per GPU and step
(benchmarks/tum_rgbd_scenes.py: a hand-held walk past a textured plane rendered through
TUM1's lens distortion, registered 16-bit depth images at DepthMapFactor 5000 with
Kinect-like holes, depths 1.6-3.9 m on both sides of mThDepth, motion along the optical
axis beyond mb both ways), TUM1's calibration (Camera.bf 40, ThDepth 40) and configs[4]'s
ORB settings (5000 features, scale 1.2, 12 levels, FAST 20/7).  One step
(orbslam2commentedbyxcm_amd/rgbd.py, RGBDSequencePipeline):
  1. ORBextractor::operator() on the B gray images (two lanes on two extractor streams);
  2. the RGB-D Frame constructor's UndistortKeyPoints + ComputeStereoFromRGBD with
     GrabImageRGBD's u16 -> f32 depth conversion (Frame.cc:192-264, 888-909; Tracking.cc:
     265-271), one kernel over every keypoint;
  3. Tracking::UpdateLastFrame (Tracking.cc:893-954): frame b-1's temporal MapPoints beside
     the map MapPoints it already tracks (half its keypoints with depth, set up once:
     Observations() 2);
  4. TrackWithMotionModel's SearchByProjection(frame b, frame b-1, th = 15, bMono = false)
     with the retry at 2*th below 20 matches (Tracking.cc:966-994, ORBmatcher.cc:1620-1789)
     for every b >= 1;
steps 2-4 on the matcher stream beside the next batch's extraction.  Inputs (gray and depth
images, poses) and outputs stay in HBM.  N > 1: one process per GPU, each rank its own
sequence (no data-path collective), "scaling": "weak".

Prints ONE JSON line (rank 0): value = RGB-D frames per second of the whole job; roofline of
the dominant kernel (algorithmic bytes); parity = on every rank, every
frame's keypoints, descriptors, mvKeysUn, mvuRight and mvDepth, every LastFrame's MapPoints
and every pair's mvpMapPoints / nmatches against the oracle (mismatch counts summed over
the ranks); cpu_baseline = the oracle (-O3 -march=native) doing the same per-frame work on
the host's cores (rank 0 at N = 1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for _p in (ROOT, ROOT / "benchmarks"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import numpy as np  # noqa: E402

import tum_rgbd_scenes as S  # noqa: E402

HBM_PEAK_GBS = 8000.0
SEED = 6000
WL = "tum5k"


def cpu_baseline(gray, depth, T, tracked, sf, bounds, seconds: float, threads: int):
    """Per frame: oracle extraction + UndistortKeyPoints + ComputeStereoFromRGBD, then
    UpdateLastFrame of the previous frame and TrackWithMotionModel's search against it --
    one chain of consecutive frames per thread."""
    from oracle import oracle as O
    flags = O.select("native")
    try:
        p = O.params(*S.PARAMS)
        n = len(gray)
        thd = S.th_depth()

        def chain(start, stop, counter, idx):
            i = start % n
            prev = S.oracle_frame(O, p, sf, gray[i], depth[i], T[i], bounds)
            while time.perf_counter() < stop:
                i += 1
                if i == n:  # frame 0 does not follow frame n-1: re-seed the chain
                    i = 0
                    prev = S.oracle_frame(O, p, sf, gray[0], depth[0], T[0], bounds)
                    continue
                cur = S.oracle_frame(O, p, sf, gray[i], depth[i], T[i], bounds)
                S.oracle_track(O, prev, cur, tracked[i - 1], thd)
                prev = cur
                counter[idx] += 1

        one = [0]
        t0 = time.perf_counter()
        chain(0, t0 + seconds / 3, one, 0)
        el1 = time.perf_counter() - t0
        done = [0] * threads
        stop = time.perf_counter() + seconds
        t1 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda t: chain(t * max(1, n // threads), stop, done, t), range(threads)))
        el = time.perf_counter() - t1
    finally:
        O.select("parity")
    import bench
    return {"value": round(sum(done) / el, 2), "unit": "RGB-D frames/s", "cores": threads, "kind": "port",
            "single_thread_ms_per_frame": round(el1 * 1e3 / max(one[0], 1), 3), "cpu_model": bench.cpu_model(),
            "flags": flags,
            "sample": f"{sum(done)} RGB-D frames in {el:.1f}s on {threads} threads (+{one[0]} in {el1:.1f}s on 1 "
                      f"thread), each = oracle C restatement of ORBextractor::operator() (5000 x 12) + "
                      f"UndistortKeyPoints + ComputeStereoFromRGBD (u16 depth, factor 1/5000) + "
                      f"Tracking::UpdateLastFrame of the previous frame + TrackWithMotionModel's "
                      f"SearchByProjection(th=15, RGB-D, retry at 30 below 20 matches) against it, over {n} "
                      f"consecutive synthetic 640x480 frames; scalar port built {flags}"}


def check_parity(O, gray, depth, T, h, tracked, sf, bounds, th_depth, cap, nchk, threads=16):
    """Every frame and pair of the host results `h` against the oracle -> parity dict."""
    p = O.params(*S.PARAMS)
    with ThreadPoolExecutor(threads) as pool:
        views = list(pool.map(lambda b: S.oracle_frame(O, p, sf, gray[b], depth[b], T[b], bounds), range(nchk)))
        tr = list(pool.map(lambda b: S.oracle_track(O, views[b - 1], views[b], tracked[b - 1], th_depth),
                           range(1, nchk)))
    bad, bad_pairs, fwd, bwd, retried = [], [], 0, 0, 0
    for b, v in enumerate(views):
        n = h["n"][b]
        ok = (n == len(v.keys) and np.array_equal(h["kps"][b, :n].view(np.uint8), v.kd.view(np.uint8))
              and np.array_equal(h["desc"][b, :n], v.desc)
              and np.array_equal(h["kpu"][b, :n].view(np.uint8), v.keys.view(np.uint8))
              and np.array_equal(h["ur"][b, :n], v.u_right) and np.array_equal(h["dp"][b, :n], v.depth))
        if not ok:
            bad.append(b)
    ok0 = int(h["nm"][0]) == 0 and bool((h["mp"][0] == -1).all())
    for b in range(1, nchk):
        ref, nr, obs, pos, rt = tr[b - 1]
        last, cur = views[b - 1], views[b]
        n0 = len(last.keys)
        mp = h["mp"][b, :len(cur.keys)]
        got = np.where(mp >= 0, mp - (b - 1) * cap, -1)
        ok = (h["nm"][b] == nr and np.array_equal(got, ref) and np.array_equal(h["mp_obs"][b - 1, :n0], obs)
              and np.array_equal(h["mp_pos"][b - 1, :n0][obs >= 0], pos[obs >= 0]))
        if not ok:
            bad_pairs.append(b)
        retried += int(rt)
        Tl, Tc = last.Tcw, cur.Tcw
        tlc = Tl[:3, :3] @ (-(Tc[:3, :3].T @ Tc[:3, 3])) + Tl[:3, 3]
        fwd += int(tlc[2] > last.b)
        bwd += int(-tlc[2] > last.b)
    return {"frames_checked": nchk, "frames_mismatched": len(bad), "first_bad_frames": bad[:8],
            "pairs_checked": nchk - 1, "pairs_mismatched": len(bad_pairs) + (0 if ok0 else 1),
            "first_bad_pairs": bad_pairs[:8], "pairs_forward": fwd, "pairs_backward": bwd,
            "pairs_retried_at_2th": retried,
            "mean_keypoints_with_depth": float(np.mean([(v.depth > 0).sum() for v in views])),
            "mean_track_matches": float(np.mean([t[1] for t in tr])) if tr else 0.0}


def main(argv=None):
    ap = argparse.ArgumentParser(prog="bench.py --workload tum5k")
    ap.add_argument("--workload", default=WL)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="RGB-D frames per GPU and step")
    ap.add_argument("--lanes", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-frames", type=int, default=-1, help="-1 = every frame and pair of the last step")
    args, _ = ap.parse_known_args(argv)
    B = args.batch
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    workers = min(16, len(os.sched_getaffinity(0)))
    gray, depth, T = S.sequence(SEED + rank, B, workers=max(1, workers // max(1, world)))

    import torch
    import torch.distributed as dist

    import bench
    from orbslam2commentedbyxcm_amd.extractor import device_frames
    from orbslam2commentedbyxcm_amd.rgbd import RGBDSequencePipeline
    gpu = 0 if os.environ.get("ORBX_BENCH_SHARE_GPU") == "1" else local_rank
    if world > 1:
        if os.environ.get("ORBX_BENCH_PG", "nccl") == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    pl = RGBDSequencePipeline(B, S.W, S.H, S.FX, S.FY, S.CX, S.CY, S.DIST, S.BF, params=S.PARAMS,
                              depth_map_factor=S.DEPTH_MAP_FACTOR, th_depth_factor=S.TH_DEPTH_FACTOR,
                              lanes=args.lanes, nbuf=int(os.environ.get("ORBX_PIPE_NBUF", "2")), device=gpu,
                              matcher_mode=None if "ORBX_MATCH_MODE" not in os.environ
                              else int(os.environ["ORBX_MATCH_MODE"]),
                              match_after_stage=int(os.environ.get("ORBX_MATCH_AFTER", "0")),
                              frame_on_lanes=os.environ.get("ORBX_RGBD_FRAME_LANES", "1") != "0",
                              match_priority=int(os.environ.get("ORBX_MATCH_PRIORITY", "0")),
                              first_in_phase=os.environ.get("ORBX_PIPE_FIRST_INPHASE", "1") == "1",
                              match_cu_stride=int(os.environ.get("ORBX_MATCH_CUSTRIDE", "1")),
                              **({"lane_offset_stage": int(os.environ["ORBX_LANE_OFFSET"])}
                                 if "ORBX_LANE_OFFSET" in os.environ else {}))
    sf, cap = pl.sf, pl.cap
    d_gray = device_frames(gray, dev)
    d_depth = torch.from_numpy(depth).to(dev)
    d_T = torch.from_numpy(T).to(dev)
    tracked = S.tracked_mask(SEED + rank, B, cap)
    torch.cuda.synchronize(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # setup: the map MapPoints each LastFrame already tracks (half its keypoints with a
    # depth, at UnprojectStereo, Observations() 2), made once from a first step's depths
    pl.run(d_gray, d_T, 1, d_depth)
    torch.cuda.synchronize(dev)
    pl.set_tracked(*pl.tracked_from(tracked, S.TRACKED_OBS))
    bench.source_hash()
    stages = ["pyramid", "score_blur", "fast_cells", "octree", "describe"]
    dom_trace = bench.dominant_stage_from_trace(stages, WL)
    # warmup: the first step untimed, the others with every stage's events (stage table)
    pl.run(d_gray, d_T, 1, d_depth)
    torch.cuda.synchronize(dev)
    pl.set_timing(True)
    pl.run(d_gray, d_T, max(args.warmup - 1, 1), d_depth)
    torch.cuda.synchronize(dev)
    stage_ms = pl.stage_times()
    kern = {k: v for k, v in stage_ms.items() if k in stages}
    dom = dom_trace or max(kern, key=kern.get)
    if stage_ms.get("match", 0.0) > stage_ms.get("total", 0.0):
        dom = "match"  # the matcher's launch, beside a lane's extraction, is then the critical path
    pl.set_timing(True, stage=dom)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    pl.run(d_gray, d_T, args.steps, d_depth)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    el = max_over_ranks(time.perf_counter() - t0)
    value = B * args.steps * world / el
    dom_ms = pl.stage_times()[dom]
    pl.set_timing(False)

    h = pl.host_results()
    status_ok = not bool(pl.status().any())
    parity = {"octree_status_clean": status_ok, "basis": bench.PARITY_BASIS}
    if args.parity_frames != 0:
        # every rank checks its own last batch (each renders its own sequence); the mismatch
        # counts are summed over the ranks
        from oracle import oracle as O
        O.build()
        nchk = B if args.parity_frames < 0 else min(B, max(2, args.parity_frames))
        pr = check_parity(O, gray, depth, T, h, tracked, sf, pl.image_bounds, pl.th_depth, cap, nchk,
                          threads=bench.parity_threads(world))
        parity.update(pr)
        parity["bit_exact"] = pr["frames_mismatched"] == 0 and pr["pairs_mismatched"] == 0 and status_ok
        parity = bench.reduce_parity(parity, world, dev)
    n_mean = float(h["n"].mean())
    bytes_pf = bench.stage_bytes(S.W, S.H, n_mean, nlevels=S.PARAMS[2], scale=S.PARAMS[1])
    per_launch = (B - 1) if dom == "match" else (pl.bounds[0][1] - pl.bounds[0][0])
    achieved = bytes_pf[dom] * per_launch / (dom_ms * 1e-3) / 1e9
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or workers
        cpu = cpu_baseline(gray[:32], depth[:32], T[:32], tracked[:32], sf, pl.image_bounds, args.cpu_seconds,
                           threads)
    if rank == 0:
        out = {
            "metric": "RGB-D frames/s ORB extract + RGB-D Frame + TrackWithMotionModel SearchByProjection, "
                      "640x480 5000-feat 12-level (configs[4]), MI355X",
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "source_hash": bench.source_hash(),
            "config": {"workload": f"configs[4] TUM RGB-D: {B} synthetic 640x480 gray + 16-bit depth frames per GPU "
                                   f"and step (a hand-held walk past a textured plane through TUM1's lens "
                                   f"distortion, DepthMapFactor {S.DEPTH_MAP_FACTOR:g} with holes), nFeatures=5000, "
                                   f"scale 1.2, 12 levels, FAST 20/7, bf {S.BF:g}, ThDepth {S.TH_DEPTH_FACTOR:g}; "
                                   f"step = extract + UndistortKeyPoints + ComputeStereoFromRGBD (u16 -> f32 depth) "
                                   f"+ Tracking::UpdateLastFrame + TrackWithMotionModel SearchByProjection (th 15, "
                                   f"bMono false, retry at 2*th below 20 matches) of every frame against its "
                                   f"predecessor",
                       "sensor": "RGB-D",
                       "frames_per_gpu_step": B, "global_batch": B * world, "width": S.W, "height": S.H,
                       "parallelism": f"frame-sharded x{world}", "lanes_per_gpu": pl.S,
                       "buffer_sets": len(pl.kps), "lane_offset_stage": pl.lane_offset_stage,
                       "first_batch_lanes_in_phase": pl.first_in_phase,
                       "frame_steps_on_lanes": pl.frame_on_lanes, "th_depth_m": round(pl.th_depth, 4),
                       "image_bounds": [round(float(x), 4) for x in pl.image_bounds]},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         **bench.profile_fields(dom, bytes_pf[dom] * per_launch, dom_ms, WL),
                         "algorithmic_bytes_per_launch": int(bytes_pf[dom] * per_launch),
                         "units_per_launch": per_launch,
                         "bytes_model": "SURVEY.md §8(d) per-stage algorithmic bytes per frame x frames per launch",
                         "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
                         "concurrent_launches": pl.S},
            "cpu_baseline": cpu,
            "parity": parity,
            "mean_keypoints_per_frame": round(n_mean, 1),
            "mean_keypoints_with_depth": round(float((h["dp"] > 0).sum(axis=1).mean()), 1),
            "mean_matches_per_pair": round(float(h["nm"][1:].mean()), 1),
        }
        print(json.dumps(out), flush=True)
    pl.close()
    bench.teardown(world, dev)


if __name__ == "__main__":
    main()
