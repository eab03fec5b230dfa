#!/usr/bin/env python3
"""configs[2] throughput: KITTI-shaped stereo Frames on one MI355X.

    python bench.py --workload kitti [--steps K] [--warmup W] [--batch B]

(Lives under tests/ because it runs the oracle as its parity check and CPU baseline;
bench.py --workload kitti is the entry point.)

Workload: B = 128 synthetic 1241x376 stereo pairs per step (right = left shifted by a
blockwise disparity field, synth.stereo_pair; all distinct by default), ORB parameters
2000 features, scale 1.2, 8 levels, FAST 20/7 (KITTI's settings).  One step = the stereo
Frame constructor's hot path for all B pairs (Frame.cc:99-178):
  1. mpORBextractorLeft on the B left images and mpORBextractorRight on the B right
     images, two extractors on two streams at once (the reference's two threads,
     Frame.cc:127-131; orbx_extract_batch_device);
  2. ComputeStereoMatches (Frame.cc:673-885) of every pair on a third stream
     (orbx_compute_stereo_matches_batch_device), overlapped with the next step's
     extraction: two extractor pairs alternate, so a pair's pyramids stay untouched
     until its matching is done.
Inputs and outputs stay in HBM.

Prints ONE JSON line: value = stereo Frames (L+R pairs) per second, images_per_s = 2x;
roofline of the dominant extraction kernel (algorithmic bytes, SURVEY.md §8(d): C3
5,896,388 B per image); parity = every pair's keypoints, descriptors, mvuRight and
mvDepth against the oracle; cpu_baseline = the oracle (-O3 -march=native) doing the
same per-pair work on the host's cores.
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
for _p in (ROOT, ROOT / "tests"):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

import numpy as np  # noqa: E402

W, H, NF = 1241, 376, 2000
FX, BF = 718.856, 386.1448  # KITTI 00-02 calibration (Camera.fx, Camera.bf)
HBM_PEAK_GBS = 8000.0


def _pair(i):
    from orbslam2commentedbyxcm_amd import synth
    return synth.stereo_pair(5000 + i, W, H, max_disp=64)[:2]


def make_pairs(n_distinct: int, workers: int = 1):
    """The distinct stereo pairs; workers > 1 renders them in a process pool (before the
    process touches the GPU)."""
    if workers > 1 and n_distinct > 1:
        import multiprocessing as mp
        pool = mp.get_context("fork").Pool(min(workers, n_distinct))
        try:
            return list(pool.imap(_pair, range(n_distinct), chunksize=2))
        finally:
            pool.close()
            pool.join()
    return [_pair(i) for i in range(n_distinct)]


def oracle_pair(O, p, left, right, sf):
    """Oracle stereo Frame: extraction of both images + ComputeStereoMatches."""
    from orbslam2commentedbyxcm_amd.matcher import FrameView
    kl, dl, _ = O.extract(left, p)
    kr, dr, _ = O.extract(right, p)
    view = FrameView(keys=kl, desc=dl, fx=FX, fy=FX, cx=W / 2, cy=H / 2, bf=BF, b=BF / FX, max_x=W, max_y=H,
                     scale_factors=sf, level_sigma2=sf * sf)
    ur, dp = O.compute_stereo_matches(view, kr, dr, O.pyramid(left, p), O.pyramid(right, p), FX)
    return (kl, dl), (kr, dr), ur, dp


def cpu_baseline(pairs, sf, seconds: float, threads: int):
    from oracle import oracle as O
    flags = O.select("native")
    try:
        p = O.params(NF, 1.2, 8, 20, 7)

        def chain(start, stop, counter, idx):
            i = start
            while time.perf_counter() < stop:
                lft, rgt = pairs[i % len(pairs)]
                oracle_pair(O, p, lft, rgt, sf)
                counter[idx] += 1
                i += 1

        one = [0]
        t0 = time.perf_counter()
        chain(0, t0 + seconds / 3, one, 0)
        el1 = time.perf_counter() - t0
        done = [0] * threads
        stop = time.perf_counter() + seconds
        t1 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda t: chain(t, stop, done, t), range(threads)))
        el = time.perf_counter() - t1
    finally:
        O.select("parity")
    import bench
    return {"value": round(sum(done) / el, 2), "unit": "stereo frames/s", "cores": threads, "kind": "port",
            "single_thread_ms_per_frame": round(el1 * 1e3 / max(one[0], 1), 3), "cpu_model": bench.cpu_model(),
            "flags": flags,
            "sample": f"{sum(done)} stereo pairs in {el:.1f}s on {threads} threads (+{one[0]} in {el1:.1f}s on 1 "
                      f"thread), each = oracle C restatement of ORBextractor::operator() on L and R + "
                      f"Frame::ComputeStereoMatches, over {len(pairs)} distinct synthetic 1241x376 pairs; scalar "
                      f"port built {flags}"}


def main(argv=None):
    ap = argparse.ArgumentParser(prog="bench.py --workload kitti")
    ap.add_argument("--workload", default="kitti")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128, help="stereo pairs per step")
    ap.add_argument("--distinct", type=int, default=0, help="distinct pairs (0 = the batch size)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-frames", type=int, default=-1, help="-1 = every pair of the last step")
    args, _ = ap.parse_known_args(argv)
    B = args.batch
    if args.gpus != 1:
        raise SystemExit("--workload kitti is a single-GPU configuration (configs[2])")

    pairs = make_pairs(min(args.distinct or B, B), workers=min(16, len(os.sched_getaffinity(0))))
    idx = [b % len(pairs) for b in range(B)]
    left_np = np.stack([pairs[i][0] for i in idx])
    right_np = np.stack([pairs[i][1] for i in idx])

    import torch

    from orbslam2commentedbyxcm_amd import ORBextractor
    from orbslam2commentedbyxcm_amd.matcher import ORBmatcher
    dev = torch.device("cuda", 0)
    # the stereo matcher's stream first: HIP assigns hardware queues in stream-creation
    # order, and a stream created after the extractors' (or from torch's pool) can share
    # one with an extraction stream
    from orbslam2commentedbyxcm_amd.extractor import stream_create
    ms = torch.cuda.ExternalStream(stream_create(0, 1), device=dev)
    sets = [(ORBextractor(NF, 1.2, 8, 20, 7), ORBextractor(NF, 1.2, 8, 20, 7)) for _ in range(2)]
    matcher = ORBmatcher(0.6, True)
    sf = sets[0][0].GetScaleFactors()
    cap = sets[0][0].max_keypoints(W, H)
    d_left = torch.from_numpy(left_np).to(dev)
    d_right = torch.from_numpy(right_np).to(dev)
    i32 = dict(dtype=torch.int32, device=dev)
    buf = [{"kl": torch.empty((B, cap, 7), **i32), "dl": torch.empty((B, cap, 32), dtype=torch.uint8, device=dev),
            "nl": torch.empty((B,), **i32), "kr": torch.empty((B, cap, 7), **i32),
            "dr": torch.empty((B, cap, 32), dtype=torch.uint8, device=dev), "nr": torch.empty((B,), **i32),
            "ur": torch.empty((B, cap), dtype=torch.float32, device=dev),
            "dp": torch.empty((B, cap), dtype=torch.float32, device=dev)} for _ in range(2)]
    streams = [(torch.cuda.ExternalStream(a.stream_handle(), device=dev),
                torch.cuda.ExternalStream(b.stream_handle(), device=dev)) for a, b in sets]
    ev_l = [torch.cuda.Event() for _ in range(2)]
    ev_r = [torch.cuda.Event() for _ in range(2)]
    ev_m = [torch.cuda.Event() for _ in range(2)]
    used = [False, False]
    state = {"it": 0, "last": 0}
    torch.cuda.synchronize(dev)

    def step():
        k = state["it"] % 2
        (exl, exr), (sl, sr), bk = sets[k], streams[k], buf[k]
        if used[k]:  # the matching that last read this set's pyramids is done
            sl.wait_event(ev_m[k])
            sr.wait_event(ev_m[k])
        exl.extract_batch_device(d_left, bk["kl"], bk["dl"], bk["nl"])
        exr.extract_batch_device(d_right, bk["kr"], bk["dr"], bk["nr"])
        ev_l[k].record(sl)
        ev_r[k].record(sr)
        ms.wait_event(ev_l[k])
        ms.wait_event(ev_r[k])
        matcher.ComputeStereoMatchesBatchDevice(exl, exr, bk["kl"], bk["dl"], bk["nl"], bk["kr"], bk["dr"], bk["nr"],
                                                BF, FX, bk["ur"], bk["dp"], stream=ms)
        ev_m[k].record(ms)
        used[k] = True
        state["last"] = k
        state["it"] += 1

    for _ in range(max(args.warmup, 2)):
        step()
    torch.cuda.synchronize(dev)
    for ex in (e for st in sets for e in st):
        ex.set_timing(True)
    matcher.set_timing(True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    value = B * args.steps / el
    per = [e.stage_times() for st in sets for e in st]  # every extractor's launches (L and R, both sets)
    stage_ms = {s: sum(p[s] for p in per) / len(per) for s in per[0]}
    stage_ms["stereo"] = matcher.last_ms()
    for ex in (e for st in sets for e in st):
        ex.set_timing(False)
    matcher.set_timing(False)

    k = state["last"]
    bk = buf[k]
    hk = bk["kl"].cpu().numpy().view(np.uint8).reshape(B, cap, 28)
    from orbslam2commentedbyxcm_amd import KEYPOINT_DTYPE
    kl = hk.view(KEYPOINT_DTYPE).reshape(B, cap)
    kr = bk["kr"].cpu().numpy().view(np.uint8).reshape(B, cap, 28).view(KEYPOINT_DTYPE).reshape(B, cap)
    dl, dr = bk["dl"].cpu().numpy(), bk["dr"].cpu().numpy()
    nl, nr = bk["nl"].cpu().numpy(), bk["nr"].cpu().numpy()
    ur, dp = bk["ur"].cpu().numpy(), bk["dp"].cpu().numpy()
    status_ok = not any(ex.status().any() for ex in sets[k])

    parity = {"octree_status_clean": status_ok}
    if args.parity_frames != 0:
        from oracle import oracle as O
        O.build()
        p = O.params(NF, 1.2, 8, 20, 7)
        nchk = min(len(pairs), B) if args.parity_frames < 0 else min(B, args.parity_frames)
        # pairs repeat every len(pairs) entries: checking the distinct ones checks them all,
        # and the repeats must equal their first copy
        with ThreadPoolExecutor(min(16, len(os.sched_getaffinity(0)))) as pool:
            refs = list(pool.map(lambda i: oracle_pair(O, p, pairs[i][0], pairs[i][1], sf), range(nchk)))
        bad = []
        for b in range(B):
            i = idx[b]
            if i >= nchk:
                continue
            (rkl, rdl), (rkr, rdr), rur, rdp = refs[i]
            ok = (nl[b] == len(rkl) and nr[b] == len(rkr)
                  and np.array_equal(kl[b, :nl[b]].view(np.uint8), rkl.view(np.uint8))
                  and np.array_equal(dl[b, :nl[b]], rdl) and np.array_equal(kr[b, :nr[b]].view(np.uint8), rkr.view(np.uint8))
                  and np.array_equal(dr[b, :nr[b]], rdr) and np.array_equal(ur[b, :nl[b]], rur)
                  and np.array_equal(dp[b, :nl[b]], rdp))
            if not ok:
                bad.append(b)
        parity.update({"pairs_checked": sum(1 for b in range(B) if idx[b] < nchk), "distinct_pairs": nchk,
                       "pairs_mismatched": len(bad), "first_bad_pairs": bad[:8],
                       "bit_exact": not bad and status_ok,
                       "mean_stereo_matches": float(np.mean([(r[2] >= 0).sum() for r in refs]))})

    import bench
    n_mean = float(np.concatenate([nl, nr]).mean())
    bytes_pf = bench.stage_bytes(W, H, n_mean)
    kern = {s: v for s, v in stage_ms.items() if s not in ("total", "stereo")}
    dom = bench.dominant_stage(kern, "kitti")
    achieved = bytes_pf[dom] * B / (stage_ms[dom] * 1e-3) / 1e9
    cpu = None
    if not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        cpu = cpu_baseline(pairs, sf, args.cpu_seconds, threads)
    out = {
        "metric": "stereo frames/s ORB extract (L+R) + ComputeStereoMatches, 1241x376 2000-feat (configs[2])",
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
        "source_hash": __import__("bench").source_hash(),
        "config": {"workload": f"configs[2]: {B} synthetic 1241x376 stereo pairs per step ({len(pairs)} distinct), "
                               f"nFeatures=2000, scale 1.2, 8 levels, FAST 20/7; step = extract L and R on two "
                               f"extractors + Frame::ComputeStereoMatches of every pair (bf {BF}, maxD = fx)",
                   "pairs_per_step": B, "width": W, "height": H},
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
        "mean_stereo_matches_per_frame": round(float((ur >= 0).sum(axis=1).mean()), 1),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
