#!/usr/bin/env python3
"""configs[2] throughput: KITTI-shaped stereo Frames on one MI355X, with tracking.

    python bench.py --workload kitti [--steps K] [--warmup W] [--batch B]

(bench.py's configs[2] leg; it runs the oracle as its parity check and CPU baseline.)

Workload: B = 256 rectified 1241x376 stereo frames per step: a KITTI-like walk past a
textured plane (benchmarks/kitti_scenes.py: depths 12-28 m, motion along the optical axis beyond
the baseline both ways, rolls), KITTI 00-02's calibration and ORB settings (2000
features, scale 1.2, 8 levels, FAST 20/7), all frames distinct.  One step
(orbslam2commentedbyxcm_amd/stereo.py, StereoSequencePipeline):
  1. mpORBextractorLeft on the B left images and mpORBextractorRight on the B right
     images, two extractors on two streams at once (Frame.cc:127-131);
  2. ComputeStereoMatches (Frame.cc:673-885) of every frame on a third stream;
  3. Tracking::UpdateLastFrame (Tracking.cc:893-954): frame b-1's temporal MapPoints
     (Observations() 0) at UnprojectStereo beside the map MapPoints it already tracks
     (half its keypoints with depth, set up once: Observations() 2);
  4. TrackWithMotionModel's SearchByProjection(frame b, frame b-1, th = 7, bMono = false)
     (Tracking.cc:966-994, ORBmatcher.cc:1620-1789) for every b >= 1 -- configs[2]'s
     "L<->R SearchByProjection" leg;
steps 2-4 overlapped with the next steps' extraction: four extractor pairs in rotation
(StereoSequencePipeline.nsets, reported as config.extractor_sets), step 2 on a matcher
stream and steps 3-4 on a tracking stream of their own.
Inputs and outputs stay in HBM.

Prints ONE JSON line: value = stereo frames (L+R pairs) per second, images_per_s = 2x;
roofline of the dominant extraction kernel (algorithmic bytes, SURVEY.md §8(d): C3
5,896,388 B per image); parity = every frame's keypoints, descriptors, mvuRight and
mvDepth, every LastFrame's MapPoints and every pair's mvpMapPoints / nmatches against
the oracle; cpu_baseline = the oracle (-O3 -march=native) doing the same per-frame work
on the host's cores.
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

import kitti_scenes as K  # noqa: E402

HBM_PEAK_GBS = 8000.0
SEED = 5000


def cpu_baseline(left, right, T, tracked, sf, th_depth, seconds: float, threads: int):
    """Per frame: oracle extraction of L and R, ComputeStereoMatches, then UpdateLastFrame
    of the previous frame and SearchByProjection against it -- one chain of consecutive
    frames per thread."""
    from oracle import oracle as O
    flags = O.select("native")
    try:
        p = O.params(*K.PARAMS)
        n = len(left)

        def chain(start, stop, counter, idx):
            i = start % n
            prev = K.oracle_frame(O, p, sf, left[i], right[i], T[i])
            while time.perf_counter() < stop:
                i += 1
                if i == n:  # frame 0 does not follow frame n-1: re-seed the chain
                    i = 0
                    prev = K.oracle_frame(O, p, sf, left[0], right[0], T[0])
                    continue
                cur = K.oracle_frame(O, p, sf, left[i], right[i], T[i])
                K.oracle_track(O, prev, cur, tracked[i - 1], th_depth)
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
    return {"value": round(sum(done) / el, 2), "unit": "stereo frames/s", "cores": threads, "kind": "port",
            "single_thread_ms_per_frame": round(el1 * 1e3 / max(one[0], 1), 3), "cpu_model": bench.cpu_model(),
            "flags": flags,
            "sample": f"{sum(done)} stereo frames in {el:.1f}s on {threads} threads (+{one[0]} in {el1:.1f}s on 1 "
                      f"thread), each = oracle C restatement of ORBextractor::operator() on L and R + "
                      f"Frame::ComputeStereoMatches + Tracking::UpdateLastFrame of the previous frame + "
                      f"SearchByProjection(CurrentFrame, LastFrame, th=7, stereo) against it, over {n} consecutive "
                      f"synthetic 1241x376 frames; scalar port built {flags}"}


def main(argv=None):
    ap = argparse.ArgumentParser(prog="bench.py --workload kitti")
    ap.add_argument("--workload", default="kitti")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    # 256 stereo frames per step, as configs[1]'s batch: 62.3k stereo frames/s against
    # 59.5-60.4k at 128 and 55.7-55.9k at 64 (r05cj-ck, interleaved; bit-exact on all 256
    # frames and 255 pairs)
    ap.add_argument("--batch", type=int, default=256, help="stereo frames per step")
    ap.add_argument("--no-track", action="store_true", help="extraction + stereo matching only (round-4 step)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-frames", type=int, default=-1, help="-1 = every frame and pair of the last step")
    ap.add_argument("--packed-frames", action="store_true",
                    help="frames in HBM with 1241-byte rows (level 0 then copied into the pyramids) instead of "
                         "a 1280-byte row pitch (level 0 read in place)")
    args, _ = ap.parse_known_args(argv)
    B = args.batch
    track = not args.no_track
    if args.gpus != 1:
        raise SystemExit("--workload kitti is a single-GPU configuration (configs[2])")

    left_np, right_np, T_np = K.sequence(SEED, B, workers=min(16, len(os.sched_getaffinity(0))))

    import torch

    from orbslam2commentedbyxcm_amd.stereo import StereoSequencePipeline
    dev = torch.device("cuda", 0)
    # A/B knobs of the bench (environment): extractor pairs, the right image's lane offset,
    # the separate tracking stream
    pl = StereoSequencePipeline(B, K.W, K.H, K.FX, K.FY, K.CX, K.CY, K.BF, params=K.PARAMS, track=track,
                                th_depth_factor=K.TH_DEPTH_FACTOR, nsets=int(os.environ.get("ORBX_STEREO_SETS", "4")),
                                lane_offset_stage=int(os.environ.get("ORBX_STEREO_LANE_OFFSET", "2")),
                                track_stream=os.environ.get("ORBX_STEREO_TRACK_STREAM", "1") == "1")
    sf, cap = pl.sf, pl.cap
    from orbslam2commentedbyxcm_amd.extractor import device_frames
    if args.packed_frames:
        d_left = torch.from_numpy(left_np).to(dev)
        d_right = torch.from_numpy(right_np).to(dev)
    else:  # rows 1280 bytes apart (hipMallocPitch's layout): level 0 read in place
        d_left, d_right = device_frames(left_np, dev), device_frames(right_np, dev)
    d_T = torch.from_numpy(T_np).to(dev)
    tracked = K.tracked_mask(SEED, B, cap)
    torch.cuda.synchronize(dev)
    # setup: the map MapPoints each LastFrame already tracks (half its keypoints with a
    # depth, at UnprojectStereo, Observations() 2), made once from a first step's depths
    pl.step(d_left, d_right, d_T)
    torch.cuda.synchronize(dev)
    obs_in, pos_in = pl.tracked_from(tracked, K.TRACKED_OBS) if track else (None, None)
    for _ in range(max(args.warmup, 1)):
        pl.step(d_left, d_right, d_T, obs_in, pos_in)
    torch.cuda.synchronize(dev)
    pl.set_timing(True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pl.step(d_left, d_right, d_T, obs_in, pos_in)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    value = B * args.steps / el
    stage_ms = pl.stage_times()
    pl.set_timing(False)

    h = pl.host_results()
    status_ok = pl.status_clean()
    parity = {"octree_status_clean": status_ok, "basis": __import__("bench").PARITY_BASIS}
    if args.parity_frames != 0:
        from oracle import oracle as O
        O.build()
        p = O.params(*K.PARAMS)
        nchk = B if args.parity_frames < 0 else min(B, max(2, args.parity_frames))
        with ThreadPoolExecutor(min(16, len(os.sched_getaffinity(0)))) as pool:
            views = list(pool.map(lambda b: K.oracle_frame(O, p, sf, left_np[b], right_np[b], T_np[b]), range(nchk)))
            tr = list(pool.map(lambda b: K.oracle_track(O, views[b - 1], views[b], tracked[b - 1], pl.th_depth),
                               range(1, nchk))) if track else []
        bad, bad_pairs, fwd, bwd = [], [], 0, 0
        for b, v in enumerate(views):
            nl, nr = h["nl"][b], h["nr"][b]
            ok = (nl == len(v.keys) and nr == len(v.kr)
                  and np.array_equal(h["kl"][b, :nl].view(np.uint8), v.keys.view(np.uint8))
                  and np.array_equal(h["dl"][b, :nl], v.desc)
                  and np.array_equal(h["kr"][b, :nr].view(np.uint8), v.kr.view(np.uint8))
                  and np.array_equal(h["dr"][b, :nr], v.dr) and np.array_equal(h["ur"][b, :nl], v.u_right)
                  and np.array_equal(h["dp"][b, :nl], v.depth))
            if not ok:
                bad.append(b)
        for b in range(1, nchk if track else 0):
            ref, nr, obs, pos = tr[b - 1]
            last, cur = views[b - 1], views[b]
            n0 = len(last.keys)
            mp = h["mp"][b, :len(cur.keys)]
            got = np.where(mp >= 0, mp - (b - 1) * cap, -1)
            ok = (h["nm"][b] == nr and np.array_equal(got, ref) and np.array_equal(h["mp_obs"][b - 1, :n0], obs)
                  and np.array_equal(h["mp_pos"][b - 1, :n0][obs >= 0], pos[obs >= 0]))
            if not ok:
                bad_pairs.append(b)
            Tl, Tc = last.Tcw, cur.Tcw
            tlc = Tl[:3, :3] @ (-(Tc[:3, :3].T @ Tc[:3, 3])) + Tl[:3, 3]
            fwd += int(tlc[2] > last.b)
            bwd += int(-tlc[2] > last.b)
        parity.update({"frames_checked": nchk, "frames_mismatched": len(bad), "first_bad_frames": bad[:8],
                       "bit_exact": not bad and not bad_pairs and status_ok,
                       "mean_stereo_matches": float(np.mean([(v.u_right >= 0).sum() for v in views]))})
        if track:
            parity.update({"pairs_checked": nchk - 1, "pairs_mismatched": len(bad_pairs),
                           "first_bad_pairs": bad_pairs[:8], "pairs_forward": fwd, "pairs_backward": bwd,
                           "mean_track_matches": float(np.mean([t[1] for t in tr]))})

    import bench
    n_mean = float(np.concatenate([h["nl"], h["nr"]]).mean())
    bytes_pf = bench.stage_bytes(K.W, K.H, n_mean)
    kern = {s: v for s, v in stage_ms.items() if s not in ("total", "stereo", "track")}
    dom = bench.dominant_stage(kern, "kitti")
    achieved = bytes_pf[dom] * B / (stage_ms[dom] * 1e-3) / 1e9
    cpu = None
    if not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        cpu = cpu_baseline(left_np, right_np, T_np, tracked, sf, pl.th_depth, args.cpu_seconds, threads)
    leg = (" + Tracking::UpdateLastFrame + TrackWithMotionModel stereo SearchByProjection (th 7, bMono false) of "
           "every frame against its predecessor" if track else "")
    out = {
        "metric": "stereo frames/s ORB extract (L+R) + ComputeStereoMatches" +
                  (" + stereo SearchByProjection" if track else "") + ", 1241x376 2000-feat (configs[2])",
        "value": round(value, 2),
        "unit": "stereo frames/s",
        "images_per_s": round(2 * value, 2),
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "source_hash": bench.source_hash(),
        "config": {"workload": f"configs[2]: {B} synthetic 1241x376 rectified stereo frames per step (a KITTI-like "
                               f"walk past a textured plane, depths 12-28 m), nFeatures=2000, scale 1.2, 8 levels, "
                               f"FAST 20/7, bf {K.BF}, fx {K.FX}, ThDepth {K.TH_DEPTH_FACTOR:g}; step = extract L and "
                               f"R on two extractors + Frame::ComputeStereoMatches (maxD = fx)" + leg,
                   "frames_per_step": B, "width": K.W, "height": K.H, "search_by_projection": track,
                   "th_depth_m": round(pl.th_depth, 4),
                   "frame_row_pitch": int(d_left.stride(1)), "extractor_sets": pl.nsets,
                   "right_lane_offset_stage": int(os.environ.get("ORBX_STEREO_LANE_OFFSET", "2"))},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     **bench.profile_fields(dom, bytes_pf[dom] * B, stage_ms[dom], "kitti"),
                     "algorithmic_bytes_per_launch": int(bytes_pf[dom] * B),
                     "bytes_model": "SURVEY.md §8(d) per-stage algorithmic bytes per image x B images per launch",
                     "stage_ms": {s: round(v, 4) for s, v in stage_ms.items()},
                     "concurrent_launches": 2, "frac_all_lanes": round(2 * achieved / HBM_PEAK_GBS, 5)},
        "cpu_baseline": cpu,
        "parity": parity,
        "mean_keypoints_per_image": round(n_mean, 1),
        "mean_stereo_matches_per_frame": round(float((h["ur"] >= 0).sum(axis=1).mean()), 1),
        "mean_track_matches_per_pair": round(float(h["nm"][1:].mean()), 1) if track else None,
    }
    print(json.dumps(out), flush=True)
    pl.close()


if __name__ == "__main__":
    main()
