#!/usr/bin/env python3
"""bench.py -- ORB extract + match throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (BASELINE.json configs[1], 640x480, nFeatures=1000, scale 1.2, 8 levels,
FAST 20/7): each rank holds a batch of B=256 synthetic grayscale frames in HBM -- 256
views of one textured canvas along a random camera walk (data: synthetic).  One step =
  1. ORBextractor::operator() on all 256 frames (orbx_extract_batch_device), and
  2. TrackWithMotionModel matching of every frame against its predecessor
     (SearchByProjection(CurrentFrame, LastFrame, th=15, bMono) semantics, batched:
     orbx_match_sequence_device),
both enqueued on the extractor's HIP stream; inputs and outputs stay in HBM.  N>1: one
process per GPU over RCCL, each rank its own batch (frames are independent: no
data-path collective), "scaling": "weak".

Prints ONE JSON line on rank 0: value = frames/s of the whole job; roofline for the
dominant kernel (HIP events on the extractor's stream; algorithmic bytes in
DESIGN.md §Roofline); cpu_baseline = the oracle (C restatement) on this host's cores;
parity = bit-exact check of a few frames and one matched pair against the oracle.
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

# The pipelined step keeps three HIP streams busy at once (two extraction lanes and the
# matcher) beside torch's own and the library's idle ones.  With HIP's default of 4
# hardware queues per process two busy streams can share a queue and then run in order
# (measured: 147k vs 189k frames/s at --lanes 2), so ask for 8 before HIP initialises.
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
VALU_PEAK_GIPS = 1024 * 2.4 / 2  # wave64 VALU issue: 1024 SIMDs, 2.4 GHz, 2 cycles each (same guide)
FX = FY = 500.0
CX, CY = 320.0, 240.0
DEPTH = 5.0
TH = 15.0  # Tracking.cc:985 (mono / RGB-D search radius factor)


def level_areas(W, H, nlevels=8, scale=1.2):
    """Level sizes as ORBextractor.cc:1641-1643 computes them (float inv scale, cvRound)."""
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(np.float64(s[-1]) * np.float64(np.float32(scale))))
    out = []
    for l in range(nlevels):
        inv = np.float32(1.0) / s[l]
        out.append((int(np.rint(np.float32(W) * inv)), int(np.rint(np.float32(H) * inv))))
    return out


def stage_bytes(W, H, n_kps, nlevels=8, scale=1.2):
    """Algorithmic bytes per frame of each stage."""
    lv = level_areas(W, H, nlevels, scale)
    A = [w * h for (w, h) in lv]
    P = sum(A)
    return {
        # read input, write every level (level 0 copied), read levels 0..L-2 as resize sources
        "pyramid": A[0] + P + (P - A[-1]),
        # read every level once, write its Gaussian-blurred copy and its FAST strength map
        "score_blur": 3 * P,
        # read the strength map of every FAST detection window once, write 4 B per kept candidate
        "fast_cells": sum((w - 38) * (h - 38) for (w, h) in lv),
        # candidates in, kept keypoints out (4 B each)
        "octree": 8 * n_kps,
        # 28 B keypoint + 32 B descriptor out per keypoint (patch reads hit L2)
        "describe": 60 * n_kps,
        # matching: query + candidate descriptors and keypoints read once, 4 B assignment out
        "match": (32 + 28) * 2 * n_kps + 4 * n_kps,
        # SURVEY.md §8(d) canonical whole-extraction figure
        "total": A[0] + (P - A[0]) + 3 * P + 60 * n_kps,
    }


# stage -> kernels of one launch of that stage (rocprofv3 kernel names)
STAGE_KERNELS = {"pyramid": ["orbx::k_pyramid"], "score_blur": ["orbx::k_level_tiles"],
                 "fast_cells": ["orbx::k_fast_cells"], "octree": ["orbx::k_octree"],
                 "describe": ["orbx::k_describe"], "match": ["orbx::k_seq_build", "orbx::k_proj_search"]}


def _stage_sum(ks: dict, stage: str, field: str):
    """Sum of `field` over the kernels of `stage` (a name matches its STAGE_KERNELS entry
    or that entry plus template arguments); None unless every entry matches one."""
    tot = 0
    for name in STAGE_KERNELS.get(stage, []):
        hits = [k for k in ks if k == name or k.startswith(name + "<")]
        if not hits:
            return None
        tot += sum(ks[k][field] for k in hits)
    return tot if STAGE_KERNELS.get(stage) else None


def newest_profiles(pattern: str):
    """profiles/ files matching `pattern` (vocabulary runs excluded), oldest first by the
    numbers in their tags (r01v9 < r01v10)."""
    import re
    files = [f for f in (ROOT / "profiles").glob(pattern) if "vocab" not in f.name]
    return sorted(files, key=lambda f: [int(x) for x in re.findall(r"\d+", f.name)])


def pmc_valu(stage: str):
    """VALU wave-instructions per launch of `stage` from the newest profiles/*_pmc_valu.json
    (tools/pmc_valu.sh + tools/pmc_valu.py), or (None, None)."""
    files = newest_profiles("*_pmc_valu.json")
    if not files:
        return None, None
    ks = json.loads(files[-1].read_text())["kernels"]
    tot = _stage_sum(ks, stage, "sq_insts_valu")
    return (None if tot is None else int(tot)), files[-1].name


def pmc_traffic(stage: str):
    """HBM bytes per launch of `stage` from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from separate FETCH_SIZE /
    WRITE_SIZE rocprofv3 passes of this bench), or (None, None)."""
    files = newest_profiles("*_pmc_traffic.json")
    if not files:
        return None, None
    ks = json.loads(files[-1].read_text())["kernels"]
    tot = _stage_sum(ks, stage, "traffic_bytes")
    return (None if tot is None else int(tot)), files[-1].name


def cpu_baseline(frames_np, seconds: float, threads: int):
    """Oracle (TEST INFRASTRUCTURE) on host cores: extracted frames/s over a bounded sample."""
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


def poses(off):
    """mTcw (rows 0..2) of each view: pure translation making pixel shifts consistent at DEPTH."""
    T = np.zeros((len(off), 12), np.float32)
    for b in range(len(off)):
        T[b] = [1, 0, 0, -off[b, 0] * DEPTH / FX, 0, 1, 0, -off[b, 1] * DEPTH / FY, 0, 0, 1, 0]
    return T


def check_parity(frames_np, T, kps_all, desc_all, n_host, mp_all, nm_all, nframes, sf):
    """Bit-exact check of the first frames' extraction and of pair (0 -> 1)'s matches."""
    from oracle import oracle as O
    from orbslam2commentedbyxcm_amd.matcher import FrameView, MapPoints
    O.build()
    p = O.params(1000, 1.2, 8, 20, 7)
    ok = True
    ref = []
    for b in range(nframes):
        kr, dr, _ = O.extract(frames_np[b], p)
        n = int(n_host[b])
        kg = kps_all[b, :n].view(np.uint8).reshape(n, 28)
        ok &= n == len(kr) and np.array_equal(kg, kr.view(np.uint8).reshape(len(kr), 28)) \
            and np.array_equal(desc_all[b, :n], dr)
        ref.append((kr, dr))
    F32 = np.float32
    (lk, ld), (ck, cd) = ref[0], ref[1]
    Tl = T[0]
    xc0 = (lk["x"] - F32(CX)) / F32(FX) * F32(DEPTH)
    xc1 = (lk["y"] - F32(CY)) / F32(FY) * F32(DEPTH)
    xc2 = np.full(len(lk), F32(DEPTH), np.float32)
    Xw = np.stack([Tl[c] * (xc0 - Tl[3]) + Tl[4 + c] * (xc1 - Tl[7]) + Tl[8 + c] * (xc2 - Tl[11])
                   for c in range(3)], 1).astype(np.float32)
    mps = MapPoints(desc=ld, observations=np.ones(len(lk), np.int32), pos=Xw)
    mk = lambda k, d, t: FrameView(keys=k, desc=d, fx=FX, fy=FY, cx=CX, cy=CY, max_x=640.0, max_y=480.0,  # noqa
                                   scale_factors=sf, Tcw=np.vstack([t.reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32))
    cur_ref = np.full(len(ck), -1, np.int32)
    nr = O.sbp_frame(mk(ck, cd, T[1]), cur_ref, mk(lk, ld, T[0]), np.arange(len(lk), dtype=np.int32), mps, TH,
                     True, True)
    ok &= int(nm_all[1]) == nr and np.array_equal(mp_all[1, :len(ck)], cur_ref)
    return {"frames_checked": nframes, "pairs_checked": 1, "bit_exact": bool(ok), "matches_pair0": int(nr)}



def _match_stream(dev):
    """The matcher's stream.  ORBX_MATCH_CUSTRIDE=k (tuning knob) restricts it to every
    k-th compute unit (hipExtStreamCreateWithCUMask), so the concurrent extraction keeps
    the other CUs' LDS and wave slots to itself."""
    import torch
    k = int(os.environ.get("ORBX_MATCH_CUSTRIDE", "0"))
    if k <= 1:  # ORBX_MATCH_PRIO=-1: high-priority matcher stream (tuning knob)
        return torch.cuda.Stream(device=dev, priority=int(os.environ.get("ORBX_MATCH_PRIO", "0")))
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
    for i in range(0, ncu, k):
        words[i // 32] |= 1 << (i % 32)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), words)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {rc}")
    return torch.cuda.ExternalStream(h.value, device=dev)

def main():
    # Secondary measurements (their implementations live under tests/: they run the
    # oracle as parity check and CPU baseline): the DBoW2 transform and the per-row table.
    if "--vocab" in sys.argv[1:] or "--rows" in sys.argv[1:]:
        sys.path.insert(0, str(ROOT / "tests"))
        mode = "--vocab" if "--vocab" in sys.argv[1:] else "--rows"
        rest = [a for a in sys.argv[1:] if a != mode]
        if mode == "--vocab":
            import vocab_bench
            return vocab_bench.main(rest)
        import row_bench
        return row_bench.main(rest)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--no-match", action="store_true", help="extraction only")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, available cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-frames", type=int, default=2)
    ap.add_argument("--no-pipeline", action="store_true",
                    help="do not overlap batch i's matching with batch i+1's extraction")
    ap.add_argument("--lanes", type=int, default=2,
                    help="split the batch into this many contiguous chunks, each on its own extractor/matcher "
                         "stream, so one chunk's latency-bound kernels overlap another's")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    B, W, H = args.batch, args.width, args.height
    match = not args.no_match

    from orbslam2commentedbyxcm_amd import synth
    frames_np, off = synth.sequence(1000 + rank, B, W, H)
    T = poses(off)

    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from orbslam2commentedbyxcm_amd import ORBextractor
    from orbslam2commentedbyxcm_amd.matcher import ORBmatcher
    S = max(1, min(args.lanes, B // 2))
    exs = [ORBextractor(1000, 1.2, 8, 20, 7, device=local_rank) for _ in range(S)]
    # TrackWithMotionModel, Tracking.cc:968
    matchers = [ORBmatcher(0.9, True, device=local_rank) for _ in range(S)]
    ex, matcher = exs[0], matchers[0]
    sf = ex.GetScaleFactors()
    cap = ex.max_keypoints(W, H)
    d_frames = torch.from_numpy(frames_np).to(dev)
    d_T = torch.from_numpy(T).to(dev)
    d_kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
    d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.empty((B,), dtype=torch.int32, device=dev)
    d_mp = torch.empty((B, cap), dtype=torch.int32, device=dev)
    d_nm = torch.empty((B,), dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)  # uploads on torch's stream finish before the extractor's stream reads them
    # lane c extracts frames [b0, b1) on its extractor's stream and matches pairs (b-1 -> b)
    # for b in [max(b0,1), b1); its first pair needs lane c-1's last frame (event).
    bounds = [(B * c // S, B * (c + 1) // S) for c in range(S)]
    streams = [torch.cuda.ExternalStream(e.stream_handle(), device=dev) for e in exs]
    done = [torch.cuda.Event() for _ in range(S)]
    # matches of lane c > 0 go to their own buffers (frame b0-1 is the first frame of its range)
    lane_mp = [d_mp] + [torch.empty((b1 - b0 + 1, cap), dtype=torch.int32, device=dev) for (b0, b1) in bounds[1:]]
    lane_nm = [d_nm] + [torch.empty((b1 - b0 + 1,), dtype=torch.int32, device=dev) for (b0, b1) in bounds[1:]]

    def step():
        for c in range(S):
            b0, b1 = bounds[c]
            exs[c].extract_batch_device(d_frames[b0:b1], d_kps[b0:b1], d_desc[b0:b1], d_n[b0:b1])
            if S > 1:
                done[c].record(streams[c])
        if match:
            for c in range(S):
                b0, b1 = bounds[c]
                lo = b0 if c == 0 else b0 - 1
                if c > 0:
                    streams[c].wait_event(done[c - 1])
                out_mp = d_mp[0:b1] if c == 0 else lane_mp[c]
                out_nm = d_nm[0:b1] if c == 0 else lane_nm[c]
                matchers[c].match_sequence_device(d_kps[lo:b1], d_desc[lo:b1], d_n[lo:b1], d_T[lo:b1], out_mp,
                                                  out_nm, sf, FX, FY, CX, CY, W, H, depth=DEPTH, th=TH,
                                                  stream=exs[c].stream_handle())

    # Pipelined mode (default): batch j is extracted on the extractor's stream while batch
    # j-1 is matched on a second stream (double-buffered keypoints/descriptors), so the
    # matcher's latency-bound replay overlaps the next extraction.  A timed run of K steps
    # does K extractions and K matchings, pipeline fill and drain included.
    pipeline = match and not args.no_pipeline
    if pipeline:
        kps2 = [d_kps, torch.empty_like(d_kps)]
        desc2 = [d_desc, torch.empty_like(d_desc)]
        n2 = [d_n, torch.empty_like(d_n)]
        mp2 = [d_mp, torch.empty_like(d_mp)]
        nm2 = [d_nm, torch.empty_like(d_nm)]
        ms = _match_stream(dev)
        # leave wave slots / LDS to the concurrent extraction (ORBX_MATCH_BIG=1: tuning knob)
        matcher.set_footprint(os.environ.get("ORBX_MATCH_BIG", "0") != "1")
        ev_ex = [[torch.cuda.Event() for _ in range(S)] for _ in range(2)]  # [buffer][lane]
        ev_m = [torch.cuda.Event(), torch.cuda.Event()]
        used = [False, False]
        state = {"it": 0}

        def p_extract():
            b = state["it"] % 2
            for c in range(S):
                b0, b1 = bounds[c]
                if used[b]:
                    streams[c].wait_event(ev_m[b])  # matching of the batch that last used buffer b is done
                exs[c].extract_batch_device(d_frames[b0:b1], kps2[b][b0:b1], desc2[b][b0:b1], n2[b][b0:b1])
                ev_ex[b][c].record(streams[c])
            used[b] = True
            state["it"] += 1

        def p_match(b):
            for c in range(S):
                ms.wait_event(ev_ex[b][c])
            matcher.match_sequence_device(kps2[b], desc2[b], n2[b], d_T, mp2[b], nm2[b], sf, FX, FY, CX, CY, W, H,
                                          depth=DEPTH, th=TH, stream=ms.cuda_stream)
            ev_m[b].record(ms)

        def run(k):
            for j in range(k):
                b_prev = (state["it"] - 1) % 2
                p_extract()          # batch j on the extractor stream(s)
                if j > 0:
                    p_match(b_prev)  # batch j-1 on the matcher stream
            p_match((state["it"] - 1) % 2)  # drain: the last batch

    def sync():
        torch.cuda.synchronize(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    if pipeline:
        run(max(args.warmup, 1))
    else:
        for _ in range(args.warmup):
            step()
    sync()
    # Per-stage HIP events on the extractor's stream, recorded inside the timed loop
    # (a ring of event sets; read back after the loop, no synchronisation inside it).
    ex.set_timing(True)
    matcher.set_timing(True)
    barrier()
    sync()
    t0 = time.perf_counter()
    if pipeline:
        run(args.steps)
    else:
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
    value = B * args.steps * world / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    if pipeline:  # results of the last batch
        b = (state["it"] - 1) % 2
        d_kps, d_desc, d_n, d_mp, d_nm = kps2[b], desc2[b], n2[b], mp2[b], nm2[b]
    n_host = d_n.cpu().numpy()
    mean_kps = float(n_host.mean())
    mean_matches = 0.0
    if match:
        nm_all = [d_nm[1:bounds[0][1]].cpu().numpy()] + [lane_nm[c][1:].cpu().numpy() for c in range(1, S)]
        mean_matches = float(np.concatenate(nm_all).mean())

    stage_ms = ex.stage_times()
    if match:
        stage_ms["match"] = matcher.last_ms()
    ex.set_timing(False)
    matcher.set_timing(False)
    bytes_pf = stage_bytes(W, H, mean_kps)
    # Dominant kernel: the longest stage on the critical path.  Pipelined, the matcher
    # runs beside the next batch's extraction on its own stream (its event time includes
    # that contention), so the extraction stages are the critical path.
    kernels = {k: v for k, v in stage_ms.items() if k != "total" and not (pipeline and k == "match")}
    dom = max(kernels, key=kernels.get)
    Bc = bounds[0][1] - bounds[0][0]  # frames of lane 0, whose events time the stages
    achieved = bytes_pf[dom] * Bc / (stage_ms[dom] * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic(dom)
    valu, valu_src = pmc_valu(dom)
    issue = None
    if valu:
        rate = valu / (stage_ms[dom] * 1e-3) / 1e9
        issue = {"bound": "valu", "achieved": round(rate, 1), "peak": VALU_PEAK_GIPS, "unit": "G wave-instr/s",
                 "frac": round(rate / VALU_PEAK_GIPS, 4), "valu_per_launch": valu, "source": valu_src,
                 "note": "SQ_INSTS_VALU per launch / stage time; peak = 1024 SIMDs x 2.4 GHz / 2 cycles",
                 "frac_all_lanes": round(rate * S / VALU_PEAK_GIPS, 4)}

    parity = None
    if rank == 0 and args.parity_frames > 0 and match:
        parity = check_parity(frames_np, T, d_kps.cpu().numpy(), d_desc.cpu().numpy(), n_host, d_mp.cpu().numpy(),
                              d_nm.cpu().numpy(), max(2, args.parity_frames), sf)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        fps, nfr, el = cpu_baseline(frames_np[:32], args.cpu_seconds, threads)
        cpu = {"value": round(fps, 2), "unit": "frames/s", "cores": threads, "kind": "port",
               "sample": f"{nfr} synthetic 640x480 frames (32 distinct) in {el:.1f}s: oracle C restatement of "
                         f"ORBextractor::operator() (extraction only, matching not timed), -O2 scalar, "
                         f"{threads} threads"}

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
            "config": {"workload": "configs[1]: 256 synthetic 640x480 gray frames per GPU (views of one textured canvas "
                                   "along a random walk), nFeatures=1000, scale 1.2, 8 levels, FAST 20/7; step = "
                                   "extract all frames + TrackWithMotionModel SearchByProjection of each frame "
                                   "against its predecessor" + ("" if match else " (match disabled)"),
                       "frames_per_gpu_step": B, "global_batch": B * world, "width": W, "height": H,
                       "parallelism": f"frame-sharded x{world}", "lanes_per_gpu": S,
                       "pipelined_match": pipeline},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_unit": "bytes per launch (PMC FETCH_SIZEx2 + WRITE_SIZE)",
                         "traffic_source": traffic_src, "algorithmic_bytes_per_launch": int(bytes_pf[dom] * Bc),
                         "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()}, "issue": issue,
                         # the S lanes launch the same kernel on S streams at once, so a
                         # launch's duration is shared with S - 1 concurrent launches
                         "concurrent_launches": S,
                         "achieved_all_lanes": round(achieved * S, 2),
                         "frac_all_lanes": round(achieved * S / HBM_PEAK_GBS, 5)},
            "cpu_baseline": cpu,
            "parity": parity,
            "mean_keypoints_per_frame": round(mean_kps, 1),
            "mean_matches_per_pair": round(mean_matches, 1),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
