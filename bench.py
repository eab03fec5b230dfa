#!/usr/bin/env python3
"""bench.py -- ORB extract + match throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--workload tum|kitti|euroc]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (BASELINE.json configs[1], 640x480, nFeatures=1000, scale 1.2, 8 levels,
FAST 20/7): each rank holds a batch of B=256 synthetic grayscale frames in HBM -- 256
views of one textured canvas along a random camera walk (data: synthetic).  One step =
  1. ORBextractor::operator() on all 256 frames (orbx_extract_batch_device, two
     128-frame lanes on two extractor streams), and
  2. TrackWithMotionModel matching of every frame against its predecessor
     (SearchByProjection(CurrentFrame, LastFrame, th=15, bMono) semantics, batched:
     orbx_match_sequence_device) on a third stream, overlapped with the next batch's
     extraction (orbslam2commentedbyxcm_amd/pipeline.py); inputs and outputs stay in HBM.
N>1: one process per GPU over RCCL (`--gpus N` starts the N ranks itself when no
launcher did), each rank its own batch (frames are independent: no data-path
collective), "scaling": "weak".  --workload kitti / euroc: configs[2] / configs[3]
(benchmarks/stereo_bench.py, benchmarks/euroc_bench.py).

Prints ONE JSON line on rank 0: value = frames/s of the whole job; roofline for the
dominant kernel (HIP events on the extractor's stream; algorithmic bytes in
DESIGN.md §5); cpu_baseline = the oracle (C restatement, -O3 -march=native) doing the
same extract + match work on this host's cores; parity = every frame and every matched
pair of the last batch against the oracle, plus the octree status words.
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import sys
import time
from pathlib import Path

# a fault anywhere in the run (a kernel's, a library's at exit) prints every thread's Python
# stack to stderr before the process dies
faulthandler.enable()

ROOT = Path(__file__).resolve().parent
SRC_ROOT = ROOT  # the sources source_hash() covers (ROOT may be redirected by tests)
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

# What "bit_exact" is measured against, in every bench line's parity block
PARITY_BASIS = ("oracle restatement (oracle/; the reference itself is unbuildable here -- OpenCV 3.3.1 absent -- "
                "and ships no fixtures, so parity is unpinned against its binary); H1: DistributeOctTree ties go to "
                "the later-created node (the bump-allocator order, checked by tests/h1_glibc); H4: FMA contraction "
                "where g++ -O3 -march=native contracts the reference's own C++; OpenCV 3.3.1 internals (resize, "
                "GaussianBlur, FAST, fastAtan2, Mat products) restated per SURVEY.md App. B, unpinned")


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
        # 28 B keypoint + 32 B descriptor out per keypoint, and the pixels it samples: the
        # IC_Angle disc of the level (749 px, umax of ORBextractor.cc:519-549) and the 512
        # rBRIEF points of the blurred level per keypoint, at most both images of every level
        "describe": 60 * n_kps + min(n_kps * (749 + 512), 2 * P),
        # matching: query + candidate descriptors and keypoints read once, 4 B assignment out
        "match": (32 + 28) * 2 * n_kps + 4 * n_kps,
        # SURVEY.md §8(d) canonical whole-extraction figure
        "total": A[0] + (P - A[0]) + 3 * P + 60 * n_kps,
    }


# stage -> kernels of one launch of that stage (rocprofv3 kernel names); the match stage
# is the pipeline's lean split footprint (build, sort + score, one-wave replay)
STAGE_KERNELS = {"pyramid": ["orbx::k_pyramid"], "score_blur": ["orbx::k_level_tiles"],
                 "fast_cells": ["orbx::k_fast_cells"], "octree": ["orbx::k_octree"],
                 "describe": ["orbx::k_describe"],
                 "match": ["orbx::k_seq_build", "orbx::k_proj_search", "orbx::k_seq_commit"]}


def _stage_sum(ks: dict, stage: str, field: str, count: str = None):
    """Sum of `field` over the kernels of `stage` (a name matches its STAGE_KERNELS entry
    or that entry plus template arguments); None unless every entry matches one.
    count: the per-kernel launch-count field; an extraction stage's per-launch value is
    then scaled by its launches per extraction (k_level_tiles runs once per extraction;
    k_pyramid once per pyramid segment: 2 at configs[4]'s 12 levels)."""
    def per_ex(k):
        if not count:
            return 1
        if stage == "match":
            # launches of this kernel per matcher call: the RGB-D step's retry pass adds a
            # k_seq_build and a lean k_proj_search launch to every call (mostly empty)
            com = [v for n, v in ks.items() if n.startswith("orbx::k_seq_commit")]
            if not com or not com[0].get(count) or not ks[k].get(count):
                return 1
            return ks[k][count] / com[0][count]
        anchor = [v for n, v in ks.items() if n == "orbx::k_level_tiles"]
        if not anchor or not anchor[0].get(count) or not ks[k].get(count):
            return 1
        return max(1, round(ks[k][count] / anchor[0][count]))
    tot = 0
    for name in STAGE_KERNELS.get(stage, []):
        hits = [k for k in ks if k == name or k.startswith(name + "<")]
        if not hits:
            return None
        tot += sum(ks[k][field] * per_ex(k) for k in hits)
    return tot if STAGE_KERNELS.get(stage) else None


def newest_profiles(pattern: str):
    """profiles/ files matching `pattern` (vocabulary runs excluded), oldest first: the
    ones taken at the current source_hash() last, each group by the numbers in its tags
    (r01v9 < r01v10) -- a pass at HEAD wins whatever its letter (r04f after r04n)."""
    import re
    files = [f for f in (ROOT / "profiles").glob(pattern) if "vocab" not in f.name]
    cur = _current_source_hash()
    return sorted(files, key=lambda f: (profile_hash(f) == cur, [int(x) for x in re.findall(r"\d+", f.name)], f.name))


_SRC_HASH = None


def _current_source_hash() -> str:
    global _SRC_HASH
    if _SRC_HASH is None:
        _SRC_HASH = source_hash()
    return _SRC_HASH


def rocprof_mean_ms(stage: str, workload: str):
    """Mean duration (ms) per launch of `stage`'s kernels in the newest committed kernel
    trace of this workload's bench (rocprofv3 --kernel-trace --stats of the command the
    driver runs, tools/prof_bench.sh): over the timed steps' launches
    (profiles/<tag>_<workload>_kernel_stats_timed.csv) when there is one, else over the
    whole trace (<tag>_<workload>_kernel_stats.csv) -- the profile-side check of the
    HIP-event time -- or (None, None)."""
    import csv
    # the timed steps' launches only (tools/prof_collect.py) when committed: the trace's
    # later legs (TrackLocalMap, host-fed) run the same kernels beside other work
    files = newest_profiles(f"*_{workload}_kernel_stats_timed.csv") or newest_profiles(f"*_{workload}_kernel_stats.csv")
    if not files:
        return None, None
    ks = {}
    for r in csv.DictReader(open(files[-1])):
        name = r["Name"].split("(")[0].replace("void ", "")
        ks[name] = {"avg_ns": float(r["AverageNs"]), "calls": int(r["Calls"])}
    tot = _stage_sum(ks, stage, "avg_ns", "calls")
    return (None if tot is None else tot * 1e-6), files[-1].name


def dominant_stage_from_trace(stages, workload: str):
    """The stage whose kernels run longest per launch in the committed kernel trace of this
    workload's bench, or None when the trace does not cover every stage."""
    prof = {k: rocprof_mean_ms(k, workload)[0] for k in stages}
    if all(v is not None for v in prof.values()):
        return max(prof, key=prof.get)
    return None


def dominant_stage(event_ms: dict, workload: str) -> str:
    """The stage whose kernels run longest per launch: by the committed kernel trace of
    this workload's bench when it covers every stage, else by the HIP-event times (which,
    pipelined, also hold the time a kernel waited for CUs held by other streams)."""
    return dominant_stage_from_trace(event_ms, workload) or max(event_ms, key=event_ms.get)


OTHER_WORKLOADS = ("_tum5k_", "_tum5k_mono_", "_kitti_", "_euroc_")


def workload_profiles(kind: str, workload: str):
    """profiles/*_<kind> files of this workload's bench, oldest first: configs[1] ("tum")
    files are tagged <tag>_tum_<kind> or carry no workload tag (older passes), the others
    <tag>_<workload>_<kind>."""
    if workload == "tum":
        return [f for f in newest_profiles(f"*_{kind}") if not any(w in f.name for w in OTHER_WORKLOADS)]
    return newest_profiles(f"*_{workload}_{kind}")


def source_hash() -> str:
    """Hash of the code a profile measures: the HIP / C++ sources of liborbx.so and the
    C ABI header (file names and bytes).  Every bench line carries it, so a committed
    profile (whose bench line records the hash it ran with) can be told stale."""
    import hashlib
    h = hashlib.sha256()
    csrc = SRC_ROOT / "orbslam2commentedbyxcm_amd" / "csrc"
    for f in sorted(list(csrc.iterdir()) + [SRC_ROOT / "include" / "orbx.h"]):
        if f.is_file():
            h.update(f.name.encode() + b"\0" + f.read_bytes())
    return h.hexdigest()[:16]


def profile_hash(f: Path):
    """The source_hash a committed profile summary was taken at (None: not recorded)."""
    try:
        if f.suffix == ".json":
            return json.loads(f.read_text()).get("source_hash")
        side = f.with_name(f.name.replace("_kernel_stats_timed.csv", "_prof_bench.json")
                           .replace("_kernel_stats.csv", "_prof_bench.json"))
        return json.loads(side.read_text()).get("source_hash") if side.exists() else None
    except (OSError, ValueError):
        return None


def pmc_valu(stage: str, workload: str = "tum"):
    """VALU wave-instructions per launch of `stage` from the newest VALU summary of this
    workload's bench (profiles/<tag>_<workload>_pmc_valu.json, tools/pmc_valu.sh +
    tools/pmc_valu.py), or (None, None)."""
    files = workload_profiles("pmc_valu.json", workload)
    if not files:
        return None, None
    ks = json.loads(files[-1].read_text())["kernels"]
    tot = _stage_sum(ks, stage, "sq_insts_valu", "dispatches")
    return (None if tot is None else int(tot)), files[-1].name


def pmc_traffic(stage: str, workload: str = "tum"):
    """HBM bytes per launch of `stage` from the newest committed PMC summary of this
    workload's bench (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from
    separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes), or (None, None)."""
    files = workload_profiles("pmc_traffic.json", workload)
    if not files:
        return None, None
    ks = json.loads(files[-1].read_text())["kernels"]
    tot = _stage_sum(ks, stage, "traffic_bytes", "dispatches")
    return (None if tot is None else int(tot)), files[-1].name


def profile_fields(dom: str, algorithmic_bytes: float, event_ms: float, workload: str) -> dict:
    """Roofline fields that come from the committed profiles of this workload's bench:
    the PMC traffic per launch and the kernel-trace mean duration, with the fraction of
    HBM peak recomputed from that mean (the profile-side check of the HIP-event `frac`)."""
    traffic, traffic_src = pmc_traffic(dom, workload)
    prof_ms, prof_src = rocprof_mean_ms(dom, workload)
    cur = source_hash()
    src_hash = {n: profile_hash(ROOT / "profiles" / n) for n in (traffic_src, prof_src) if n}
    return {"traffic": traffic, "traffic_unit": "bytes per launch (PMC FETCH_SIZEx2 + WRITE_SIZE)",
            "traffic_source": traffic_src, "kernels": STAGE_KERNELS.get(dom),
            # a profile taken at other sources than this run's (or with no hash recorded)
            # may not describe the code measured here
            "profile_source_hash": src_hash,
            "profiles_stale": any(h != cur for h in src_hash.values()),
            "event_ms": round(event_ms, 4),
            "rocprof_mean_ms": None if prof_ms is None else round(prof_ms, 4), "rocprof_source": prof_src,
            "frac_rocprof": None if not prof_ms else
            round(algorithmic_bytes / (prof_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(frames_np, T, sf, seconds: float, threads: int, W=640, H=480, params=(1000, 1.2, 8, 20, 7)):
    """The oracle (C restatement, TEST INFRASTRUCTURE) on this host's cores doing the same
    work as one step's unit: extract frame i and match it against frame i-1
    (SearchByProjection(CurrentFrame, LastFrame, th=15, bMono), ORBmatcher.cc:1620-1789),
    built with the reference's -O3 -march=native (CMakeLists.txt:10-19).  Bounded sample:
    a contiguous run of the bench's frames, ~seconds/3 on one thread (latency) then
    ~seconds on `threads` threads (throughput, one chain of consecutive frames each)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import checks
    from oracle import oracle as O
    from orbslam2commentedbyxcm_amd.matcher import FrameView, MapPoints

    flags = O.select("native")
    try:
        n = len(frames_np)
        p = O.params(*params)
        F32 = np.float32

        def view(k, d, t):
            return FrameView(keys=k, desc=d, fx=FX, fy=FY, cx=CX, cy=CY, max_x=float(W), max_y=float(H),
                             scale_factors=sf, Tcw=np.vstack([t.reshape(3, 4), [0, 0, 0, 1]]).astype(np.float32))

        def match(prev, cur, i):
            (lk, ld), (ck, cd) = prev, cur
            Tl = T[i - 1]
            xc0 = (lk["x"] - F32(CX)) / F32(FX) * F32(DEPTH)
            xc1 = (lk["y"] - F32(CY)) / F32(FY) * F32(DEPTH)
            xc2 = np.full(len(lk), F32(DEPTH), np.float32)
            Xw = np.stack([Tl[c] * (xc0 - Tl[3]) + Tl[4 + c] * (xc1 - Tl[7]) + Tl[8 + c] * (xc2 - Tl[11])
                           for c in range(3)], 1).astype(np.float32)
            mps = MapPoints(desc=ld, observations=np.ones(len(lk), np.int32), pos=Xw)
            out = np.full(len(ck), -1, np.int32)
            # TrackWithMotionModel's search: again at 2*th below 20 matches (Tracking.cc:988-994)
            return O.track_motion_model(view(ck, cd, T[i]), out, view(lk, ld, Tl), np.arange(len(lk), dtype=np.int32),
                                        mps, TH, True, True)[0]

        # same sources, other flags: the baseline build must reproduce the checker exactly
        k0, d0, _ = O.extract(frames_np[0], p)
        k1, d1, _ = O.extract(frames_np[1], p)
        nm_native = match((k0, d0), (k1, d1), 1)
        O.select("parity")
        ref = checks.extract_all(frames_np[:2], params=params, threads=1)
        same = all(np.array_equal(a[0].view(np.uint8), b[0].view(np.uint8)) and np.array_equal(a[1], b[1])
                   for a, b in zip(ref, [(k0, d0), (k1, d1)]))
        same = same and nm_native == match(ref[0], ref[1], 1)
        O.select("native")

        def chain(start, stop_at, counter, idx):
            i = start % n
            prev = O.extract(frames_np[i], p)[:2]
            while time.perf_counter() < stop_at:
                i += 1
                if i == n:  # wrap: frame 0 does not follow frame n-1, re-seed the chain
                    i = 0
                    prev = O.extract(frames_np[0], p)[:2]
                    continue
                cur = O.extract(frames_np[i], p)[:2]
                match(prev, cur, i)
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
    host = len(os.sched_getaffinity(0))
    return {"value": round(sum(done) / el, 2), "unit": "frames/s", "cores": threads, "kind": "port",
            "single_thread_ms_per_frame": round(el1 * 1e3 / max(one[0], 1), 3),
            "single_thread_frames_per_s": round(one[0] / el1, 2),
            # the GPU box allots 16 of its host CPUs to a one-GPU job (its process guard
            # counts the rest as other jobs'), so `value` is measured at <= 16 threads; the
            # host-wide figure is that rate scaled linearly to every visible CPU -- an
            # upper bound (no memory-bandwidth or SMT loss), not a measurement
            "per_thread_frames_per_s": round(sum(done) / el / threads, 2),
            "linear_estimate_at_host_cpus": {"cpus": host, "value": round(sum(done) / el / threads * host, 1),
                                             "measured": False},
            "cpu_model": cpu_model(), "host_cpus_visible": host, "flags": flags,
            "baseline_build_matches_checker": bool(same),
            "sample": f"{sum(done)} frames in {el:.1f}s on {threads} threads (+{one[0]} in {el1:.1f}s on 1 thread), "
                      f"each = oracle C restatement of ORBextractor::operator() + TrackWithMotionModel's "
                      f"SearchByProjection(CurrentFrame, LastFrame, th={TH:g}, mono; again at {2 * TH:g} below 20 "
                      f"matches) against the previous frame, over {n} consecutive bench frames; "
                      f"scalar port built {flags} (no OpenCV / IPP SIMD)"}

def _match_stream(dev):
    """ORBX_MATCH_PRIO=p (tuning knob): the matcher on a torch stream of priority p over
    every CU instead of the pipeline's own stream (ORBX_MATCH_CUSTRIDE=k: on CUs 0, k,
    2k, ... only; default 1 = every CU)."""
    import torch
    if "ORBX_MATCH_PRIO" not in os.environ:
        return None
    return torch.cuda.Stream(device=dev, priority=int(os.environ["ORBX_MATCH_PRIO"]))


def parity_threads(world: int) -> int:
    """Oracle threads per rank for the parity check: the host's CPUs shared by the ranks."""
    return max(2, min(16, len(os.sched_getaffinity(0)) // max(1, world)))


def reduce_parity(parity: dict, world: int, dev) -> dict:
    """Every rank checks its own last batch; the counts are summed over the ranks and the
    line's verdict is the job's: parity.ranks_checked = the ranks that checked."""
    keys = ("frames_checked", "frames_mismatched", "pairs_checked", "pairs_mismatched")
    counts = [int(parity.get(k, 0)) for k in keys] + [int(not parity.get("octree_status_clean", True)),
                                                     int("frames_checked" in parity)]
    if world > 1:
        import torch
        import torch.distributed as dist
        t = torch.tensor(counts, dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        counts = [int(x) for x in t.tolist()]
    out = dict(parity)
    out.update({f"{k}_all_ranks": c for k, c in zip(keys, counts)})
    out["ranks_checked"] = counts[5]
    if "bit_exact" in parity:
        out["bit_exact"] = counts[1] == 0 and counts[3] == 0 and counts[4] == 0 and counts[5] == world
    return out


def teardown(world: int, dev=None) -> None:
    """The run's explicit, ordered teardown (DESIGN.md §1 "Teardown"): every liborbx handle
    owner still alive is closed, pipelines first (liborbx's handle registry), the device is
    synchronised, and only then is the process group destroyed -- nothing of liborbx or of
    RCCL is left for the C runtime's exit-time destructors."""
    import torch
    from orbslam2commentedbyxcm_amd import _lib
    _lib.release_all()
    if dev is not None:
        torch.cuda.synchronize(dev)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


def launch_ranks(n: int, argv) -> int:
    """bench.py --gpus N without a launcher: start N ranks of this script as child processes
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, 127.0.0.1 rendezvous) before this
    process touches the GPU, wait for all, return the worst exit code.  Rank 0 prints the
    JSON line."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *argv], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def selftest_launch(args, rank, world, local_rank):
    """--selftest-launch: the launcher path on CPU (gloo): every rank joins the group, the
    world size is checked against --gpus, rank 0 prints one JSON line."""
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo")
    try:
        t = torch.tensor([rank + 1], dtype=torch.int64)
        dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"selftest_launch": True, "world": dist.get_world_size(), "gpus": args.gpus,
                              "rank_sum": int(t.item()), "local_rank0": local_rank}), flush=True)
    finally:
        dist.destroy_process_group()


def main():
    # Secondary workloads and measurements (their implementations live under tests/: they
    # run the oracle as parity check and CPU baseline).
    for flag, mod in (("--vocab", "vocab_bench"), ("--rows", "row_bench"), ("--dropin", "dropin_bench")):
        if flag in sys.argv[1:]:
            sys.path.insert(0, str(ROOT / "benchmarks"))
            return __import__(mod).main([a for a in sys.argv[1:] if a != flag])
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)  # ~60 ms timed at C1: pipeline fill/drain < 1 %
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--workload", default="tum", choices=["tum", "tum5k", "tum5k_mono", "kitti", "euroc"],
                    help="tum: configs[1] (default, the headline); tum5k: configs[4], the TUM RGB-D step (5000 "
                         "features x 12 levels, benchmarks/rgbd_bench.py); tum5k_mono: the same extraction with "
                         "the monocular search (round 5's configs[4] step); kitti: configs[2] stereo; euroc: "
                         "configs[3]")
    ap.add_argument("--no-match", action="store_true", help="extraction only")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, available cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--parity-frames", type=int, default=-1, help="-1 = every frame and pair of the last batch")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="do not overlap batch i's matching with batch i+1's extraction")
    ap.add_argument("--lanes", type=int, default=2,
                    help="split the batch into this many contiguous chunks, each on its own extractor stream, so "
                         "one chunk's latency-bound kernels overlap another's")
    ap.add_argument("--no-host-fed", action="store_true",
                    help="skip the host-fed leg (frames uploaded from pinned host memory every step)")
    ap.add_argument("--no-local-map", action="store_true",
                    help="skip the second measurement of the step with TrackLocalMap's SearchLocalPoints")
    ap.add_argument("--no-exchange", action="store_true",
                    help="at --gpus > 1, skip the configs[3] keyframe-exchange leg (RCCL all-gather between ranks)")
    ap.add_argument("--track-retry", type=int, default=20,
                    help="TrackWithMotionModel's second search at 2*th below this many matches (Tracking.cc:988-994; "
                         "0 = one search, for pricing it)")
    ap.add_argument("--selftest-launch", action="store_true", help=argparse.SUPPRESS)
    args, _ = ap.parse_known_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, sys.argv[1:])  # nothing here has touched the GPU
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    if args.selftest_launch:
        return selftest_launch(args, rank, world, local_rank)
    if args.workload not in ("tum", "tum5k_mono"):
        sys.path.insert(0, str(ROOT / "benchmarks"))
        mod = {"kitti": "stereo_bench", "euroc": "euroc_bench", "tum5k": "rgbd_bench"}[args.workload]
        return __import__(mod).main([a for a in sys.argv[1:]])

    B, W, H = args.batch, args.width, args.height
    # configs[1] (the headline), or configs[4]'s extraction shape (5000 features x 12 levels)
    # with the monocular search (tum5k_mono; the RGB-D step itself is --workload tum5k)
    c5 = args.workload == "tum5k_mono"
    prm = (5000, 1.2, 12, 20, 7) if c5 else (1000, 1.2, 8, 20, 7)
    match = not args.no_match
    from orbslam2commentedbyxcm_amd import synth
    from orbslam2commentedbyxcm_amd.pipeline import SequencePipeline, sequence_poses
    frames_np, off = synth.sequence(1000 + rank, B, W, H)
    T = sequence_poses(off, FX, FY, DEPTH)

    import torch
    import torch.distributed as dist

    # Rehearsal of the N-rank run on a one-GPU box (never the driver's run):
    # ORBX_BENCH_SHARE_GPU=1 puts every rank on GPU 0 and ORBX_BENCH_PG=gloo carries the
    # barriers, the max-over-ranks time and the slab exchange (staged through host memory),
    # since RCCL needs one GPU per rank.
    gpu = 0 if os.environ.get("ORBX_BENCH_SHARE_GPU") == "1" else local_rank
    if world > 1:
        if os.environ.get("ORBX_BENCH_PG", "nccl") == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)

    pipeline = match and not args.no_pipeline
    pl = SequencePipeline(B, W, H, lanes=args.lanes, pipelined=pipeline, match=match, device=gpu,
                          params=prm, fx=FX, fy=FY, cx=CX, cy=CY, depth=DEPTH, th=TH,
                          match_stream=_match_stream(dev) if match else None,
                          # three buffer sets at <= 8 levels: extraction j + 2 need not wait for
                          # matching j (configs[1] +0.6 %, 7 of 8 interleaved pairs at 20 / 50 steps,
                          # r05bs-bt; configs[4] -0.3 %, two)
                          nbuf=int(os.environ.get("ORBX_PIPE_NBUF", "3" if prm[2] <= 8 else "2")),
                          matcher_mode=None if "ORBX_MATCH_MODE" not in os.environ
                          else int(os.environ["ORBX_MATCH_MODE"]),
                          match_after_stage=int(os.environ.get("ORBX_MATCH_AFTER", "0")),
                          lane_offset_stage=int(os.environ["ORBX_LANE_OFFSET"]) if "ORBX_LANE_OFFSET" in os.environ else None,
                          match_cu_stride=int(os.environ.get("ORBX_MATCH_CUSTRIDE", "1")),
                          match_priority=int(os.environ.get("ORBX_MATCH_STREAM_PRIO", "0")),
                          level0_in_place=os.environ.get("ORBX_L0_COPY") != "1",
                          first_in_phase=os.environ.get("ORBX_PIPE_FIRST_INPHASE", "1") == "1",
                          retry_below=args.track_retry)
    first_in_phase = bool(pl.first_in_phase)
    S = pl.S
    nbufs = len(pl.kps)  # output buffer sets in rotation
    lane_off = pl.lane_offset_stage if pl.lane_ev is not None else None  # None: no offset applied
    d_frames = torch.from_numpy(frames_np).to(dev)
    d_T = torch.from_numpy(T).to(dev)
    torch.cuda.synchronize(dev)  # uploads on torch's stream finish before the extractor streams read them

    def sync():
        torch.cuda.synchronize(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    # The warmup steps record every stage boundary (HIP events on each lane's stream and
    # the matcher's): the stage table and the dominant stage come from them.  The timed
    # steps then record only the dominant stage's two events per launch (a ring of event
    # sets, read back after the loop, no synchronisation inside it): every recorded event
    # costs the pipelined step ~0.2 % (tools/timing_ab.py: all stages' events 1.3-1.6 %).
    wl = "tum5k_mono" if c5 else "tum"
    # the committed trace's choice of the dominant stage is read (files, hashes) before the
    # warmup, not between the warmup and the timed region: ~13 ms of host work there left
    # the GPU idle right before the timed steps
    # (ORBX_BENCH_DOM_LATE=1, A/B knob: read it after the warmup as until round 4)
    late = os.environ.get("ORBX_BENCH_DOM_LATE") == "1"
    if not late:
        source_hash()
    dom_trace = None if late else \
        dominant_stage_from_trace(["pyramid", "score_blur", "fast_cells", "octree", "describe"], wl)
    # the first warmup step (first-call costs) is not recorded: the stage table comes from
    # the W - 1 after it (one step when W <= 2)
    if args.warmup >= 2:
        pl.run(d_frames, d_T, 1)
        sync()
    pl.set_timing(True)
    pl.run(d_frames, d_T, max(args.warmup - 1, 1))
    sync()
    stage_ms = pl.stage_times()  # warmup steps after the first, every stage
    kernels = {k: v for k, v in stage_ms.items() if k not in ("total", "match")}
    # Dominant kernel: the longest stage on the critical path.  Pipelined, the matcher
    # runs beside the next batch's extraction on its own stream, so the step is set by
    # whichever is longer: a lane's extraction (its longest stage is reported) or the
    # matcher (configs[4]: its launch is then the critical path).
    dom = dominant_stage(kernels, wl) if late else (dom_trace or max(kernels, key=kernels.get))
    if match and pipeline and stage_ms.get("match", 0.0) > stage_ms.get("total", 0.0):
        dom = "match"
    # ORBX_BENCH_ALL_EVENTS=1 (A/B knob): every stage's events in the timed steps too
    pl.set_timing(True, stage=None if os.environ.get("ORBX_BENCH_ALL_EVENTS") else dom)
    barrier()
    sync()
    t0 = time.perf_counter()
    pl.run(d_frames, d_T, args.steps)
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

    res = pl.host_results()
    status = pl.status()
    n_host = res["n"]
    mean_kps = float(n_host.mean())
    mean_matches = float(res["nm"][1:].mean()) if match and B > 1 else 0.0

    dom_ms = pl.stage_times()[dom]  # HIP events over the timed steps, mean over the lanes' launches
    pl.set_timing(False)
    bytes_pf = stage_bytes(W, H, mean_kps, nlevels=prm[2], scale=prm[1])
    # frames per launch: a lane's batch for extraction stages, every pair for the matcher
    per_launch = (B - 1) if dom == "match" else (pl.bounds[0][1] - pl.bounds[0][0])
    achieved = bytes_pf[dom] * per_launch / (dom_ms * 1e-3) / 1e9
    prof = profile_fields(dom, bytes_pf[dom] * per_launch, dom_ms, wl)
    valu, valu_src = pmc_valu(dom, wl)
    issue = None
    if valu:
        rate = valu / (dom_ms * 1e-3) / 1e9
        issue = {"bound": "valu", "achieved": round(rate, 1), "peak": VALU_PEAK_GIPS, "unit": "G wave-instr/s",
                 "frac": round(rate / VALU_PEAK_GIPS, 4), "valu_per_launch": valu, "source": valu_src,
                 "source_stale": profile_hash(ROOT / "profiles" / valu_src) != source_hash(),
                 "note": "SQ_INSTS_VALU per launch / stage time; peak = 1024 SIMDs x 2.4 GHz / 2 cycles",
                 "frac_all_lanes": round(rate * S / VALU_PEAK_GIPS, 4)}

    parity = {"octree_status_clean": not bool(status.any()), "basis": PARITY_BASIS}
    if args.parity_frames != 0:
        # every rank checks its own last batch (each extracts its own frames), counts summed
        from oracle import checks
        nchk = B if args.parity_frames < 0 else min(B, max(2, args.parity_frames))
        sub = {k: v[:nchk] for k, v in res.items()}
        if not match:
            sub.pop("mp"), sub.pop("nm")
        parity.update(checks.check_sequence(frames_np[:nchk], T[:nchk], sub, pl.sf, params=prm, fx=FX, fy=FY, cx=CX,
                                            cy=CY, W=W, H=H, depth=DEPTH, th=TH, threads=parity_threads(world),
                                            retry=pl.retry_below > 0))
        parity["bit_exact"] = parity["bit_exact"] and parity["octree_status_clean"]
        parity = reduce_parity(parity, world, dev)

    # The same step fed from host memory: every step's 256 frames are uploaded from pinned
    # host memory (double-buffered, on a copy stream beside the previous step's work) and
    # the extraction lanes wait for their upload -- the PCIe-inclusive rate a caller whose
    # frames arrive in host memory would see.  Not `value`.
    host_fed = None
    if match and not args.no_host_fed:
        pl.set_timing(False)
        h_frames = torch.from_numpy(frames_np).pin_memory()
        nb = len(pl.kps)
        d_buf = [torch.empty_like(d_frames) for _ in range(nb)]
        cs = torch.cuda.Stream(device=dev)
        ev_up = [torch.cuda.Event() for _ in range(nb)]

        def hf_step(j):
            b = pl.it % nb  # the pipeline's buffer of this step = the upload buffer
            with torch.cuda.stream(cs):
                if j >= nb:  # the extraction nb steps back (pipeline buffer b) read d_buf[b]
                    for c in range(pl.S):
                        cs.wait_event(pl.ev_ex[b][c])
                d_buf[b].copy_(h_frames, non_blocking=True)
                ev_up[b].record(cs)
            for c in range(pl.S):
                pl.streams[c].wait_event(ev_up[b])
            pl.step(d_buf[b], d_T)

        for j in range(max(args.warmup, 1)):
            hf_step(j)
        pl.drain(d_T)
        sync()
        barrier()
        sync()
        t0 = time.perf_counter()
        for j in range(args.steps):
            hf_step(j + nb)  # d_buf[b] was read by an extraction nb steps back
        pl.drain(d_T)
        sync()
        barrier()
        sync()
        el3 = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el3], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el3 = float(t.item())
        host_fed = {"value": round(B * args.steps * world / el3, 2), "unit": "frames/s",
                    "ms_per_step": round(el3 / args.steps * 1e3, 4),
                    "upload_bytes_per_step": int(frames_np.nbytes),
                    "upload_GBps": round(frames_np.nbytes * args.steps / el3 / 1e9, 2),
                    "note": f"frames uploaded from pinned host memory every step (copy stream, {nb} buffers, "
                            "overlapped with the previous step's extraction and matching); results stay in HBM"}

    # The same step with TrackLocalMap (SearchLocalPoints against the MapPoints of the three
    # previous frames, after TrackWithMotionModel against the previous frame's MapPoints):
    # a second pipeline, timed the same way, checked the same way.
    local = None
    sf_main = pl.sf
    match_cu = None if (not match or pl._own_ms is None) else int(os.environ.get("ORBX_MATCH_CUSTRIDE", "1"))
    if match and not args.no_local_map:
        pl.close()
        del pl
        pl2 = SequencePipeline(B, W, H, lanes=args.lanes, pipelined=pipeline, device=gpu, params=prm, fx=FX,
                               fy=FY, cx=CX, cy=CY, depth=DEPTH, th=TH, local_map=True)
        pl2.run(d_frames, d_T, max(args.warmup, 1))
        sync()
        pl2.set_timing(True)
        barrier()
        sync()
        t0 = time.perf_counter()
        pl2.run(d_frames, d_T, args.steps)
        sync()
        barrier()
        sync()
        el2 = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el2], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el2 = float(t.item())
        st2 = pl2.stage_times()
        pl2.set_timing(False)
        res2 = pl2.host_results()
        local = {"value": round(B * args.steps * world / el2, 2), "unit": "frames/s",
                 "ms_per_step": round(el2 / args.steps * 1e3, 4),
                 "step": "extract + MapPoints of every keypoint (CreateNewKeyFrame's UnprojectStereo at the model "
                         "depth) + TrackWithMotionModel SearchByProjection vs the previous frame's MapPoints + "
                         "TrackLocalMap SearchLocalPoints (IsInFrustum + SearchByProjection(F, vpLocalMapPoints, "
                         "th=1), ORBmatcher(0.8)) vs the MapPoints of the 3 previous frames",
                 "stage_ms": {k: round(v, 4) for k, v in st2.items()},
                 "mean_matches_per_pair": round(float(res2["nm"][1:].mean()), 1),
                 "mean_local_matches_per_frame": round(float(res2["nm_local"][1:].mean()), 1)}
        if args.parity_frames != 0:
            from oracle import checks
            nchk = B if args.parity_frames < 0 else min(B, max(2, args.parity_frames))
            sub = {k: v[:nchk] for k, v in res2.items()}
            pr = checks.check_sequence_local(frames_np[:nchk], T[:nchk], sub, pl2.sf, pl2.cap, params=prm, fx=FX,
                                             fy=FY, cx=CX, cy=CY, W=W, H=H, depth=DEPTH, th=TH,
                                             threads=parity_threads(world))
            pr["octree_status_clean"] = not bool(pl2.status().any())
            pr["bit_exact"] = pr["bit_exact"] and pr["octree_status_clean"]
            local["parity"] = reduce_parity(pr, world, dev)
        pl2.close()

    # At world size > 1 the node's GPUs also run configs[3]'s step with its one real
    # exchange -- the keyframe slabs all-gathered over RCCL between the ranks (DESIGN.md
    # section 6) -- for a few timed steps, rank 0 checking its keyframes, the neighbours it
    # received from the other ranks and its triangulation pairs against the oracle.  Not
    # `value`; the headline step itself has no collective.
    exchange = None
    if world > 1 and not args.no_exchange:
        sys.path.insert(0, str(ROOT / "benchmarks"))
        import euroc_bench
        eargs = euroc_bench.parse(["--steps", "10", "--warmup", "3", "--no-cpu-baseline"])
        line = euroc_bench.run(eargs, rank, world, gpu, True)
        if line is not None:
            c, pr = line["config"], line["parity"]
            exchange = {"value": line["value"], "unit": line["unit"], "ms_per_step": line["ms_per_step"],
                        "steps": line["steps"], "slab_exchange": c["slab_exchange"],
                        "slab_mb_per_rank": c["slab_mb_per_rank"],
                        "allgather_mb_per_rank_step": c["allgather_mb_per_rank_step"],
                        "parity": {k: pr.get(k) for k in ("bit_exact", "ranks_checked", "keyframes_checked_all_ranks",
                                                          "keyframes_mismatched_all_ranks",
                                                          "gathered_neighbours_checked_all_ranks",
                                                          "gathered_mismatched_all_ranks", "pairs_checked_all_ranks",
                                                          "pairs_mismatched_all_ranks")},
                        "step": "configs[3] (bench.py --workload euroc): extract L+R, ComputeStereoMatches, "
                                "ComputeBoW, close-point MapPoints, RCCL all_gather_into_tensor of the keyframe "
                                "slabs, SearchForTriangulation against the gathered neighbours"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        cpu = cpu_baseline(frames_np[:32], T[:32], sf_main, args.cpu_seconds, threads, W, H, params=prm)

    if rank == 0:
        out = {
            "metric": ("frames/s ORB extract+match, 640x480 5000-feat 12-level monocular (configs[4] shape), MI355X"
                       if c5 else
                       "frames/s ORB extract+match, 640x480 1000-feat, 1/2/4/8 MI355X"),
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
            "source_hash": source_hash(),
            "config": {"workload": f"{'configs[4] extraction shape, monocular search' if c5 else 'configs[1]'}: {B} "
                                   f"synthetic 640x480 gray frames per GPU "
                                   f"(views of one textured canvas along a random walk), nFeatures={prm[0]}, scale 1.2, "
                                   f"{prm[2]} levels, FAST 20/7; step = "
                                   "extract all frames + TrackWithMotionModel SearchByProjection of each frame "
                                   "against its predecessor" + ("" if match else " (match disabled)"),
                       "frames_per_gpu_step": B, "global_batch": B * world, "width": W, "height": H,
                       "parallelism": f"frame-sharded x{world}", "lanes_per_gpu": S,
                       "lane_offset_stage": lane_off,
                       "pipelined_match": pipeline, "buffer_sets": nbufs,
                       "first_batch_lanes_in_phase": first_in_phase,
                       "match_cu_stride": match_cu},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), **prof,
                         "algorithmic_bytes_per_launch": int(bytes_pf[dom] * per_launch),
                         "units_per_launch": per_launch,
                         "event_ms_note": "HIP events on the launching stream around the stage, mean over the timed "
                                          "steps and the lanes (the timed steps record only this stage's events)",
                         "stage_ms": {k: round(v, 4) for k, v in stage_ms.items()},
                         "stage_ms_note": "every stage's HIP-event ms over the warmup steps after the first (all "
                                          "boundaries recorded there; used to pick the dominant stage when no kernel "
                                          "trace is committed)",
                         "issue": issue,
                         # the S lanes launch the same kernel on S streams at once, so a
                         # launch's duration is shared with S - 1 concurrent launches
                         "concurrent_launches": S,
                         "achieved_all_lanes": round(achieved * S, 2),
                         "frac_all_lanes": round(achieved * S / HBM_PEAK_GBS, 5)},
            "cpu_baseline": cpu,
            "parity": parity,
            "with_local_map": local,
            "host_fed": host_fed,
            "keyframe_exchange": exchange,
            "mean_keypoints_per_frame": round(mean_kps, 1),
            "mean_matches_per_pair": round(mean_matches, 1),
        }
        print(json.dumps(out), flush=True)
    teardown(world, dev)


if __name__ == "__main__":
    sys.exit(main() or 0)

