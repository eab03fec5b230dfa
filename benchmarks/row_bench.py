"""Per-row measurement of SURVEY.md §8's matcher / frame / map rows (a11-a18, f2-f4):
one drop-in call through liborbx.so's host API on the GPU vs the same call of the CPU
oracle (the C restatement, single thread), on C1-sized synthetic scenes, with the
results compared byte for byte.

    python bench.py --rows [--reps 20]

The GPU figure is the wall time of the reference-shaped host call (arguments in host
memory, as Tracking / LocalMapping would pass them): upload, kernels, download.  It is
dominated by launch and PCIe latency at these sizes; the throughput paths are the
batched device calls (bench.py for a1-a12, bench.py --vocab for f1).  bench.py --rows
runs it; it runs the oracle too (parity check and CPU baseline).
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "benchmarks"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

import numpy as np  # noqa: E402


def _time(fn, reps):
    """Median wall time (ms) of fn() over reps calls; fn returns the result to check."""
    out, ts = None, []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    return statistics.median(ts), out


def _eq(a, b) -> bool:
    if isinstance(a, tuple):
        return len(a) == len(b) and all(_eq(x, y) for x, y in zip(a, b))
    if isinstance(a, np.ndarray):
        return a.shape == b.shape and np.array_equal(a.view(np.uint8), np.asarray(b).view(np.uint8))
    return a == b


def rows(O, reps: int, only=None):
    import match_scenes as S
    from orbslam2commentedbyxcm_amd import ORBextractor, synth
    from orbslam2commentedbyxcm_amd import frame as FR
    from orbslam2commentedbyxcm_amd.matcher import ComputeDistinctiveDescriptors, FrameView, ORBmatcher

    cpu_reps = max(3, reps // 4)
    out = []

    def add(row, ref, size, gpu_fn, cpu_fn, lib=None):
        """lib: the ORBmatcher / ORBextractor the GPU call runs on -- its in-library wall time
        per call (orbx_matcher_last_call_us / orbx_extractor_last_call_us: what a C++ caller
        pays, without the ctypes binding) is reported beside the Python-side time."""
        if only and row not in only:
            return
        gpu_fn()  # warm-up (device init, first allocation)
        lib_us = []

        def g_fn():
            r = gpu_fn()
            if lib is not None:
                lib_us.append(lib.last_call_us())
            return r
        g_ms, g = _time(g_fn, reps)
        c_ms, c = _time(cpu_fn, cpu_reps)
        rec = {"row": row, "reference": ref, "size": size, "gpu_ms": round(g_ms, 4), "cpu_ms": round(c_ms, 4),
               "speedup": round(c_ms / g_ms, 2) if g_ms > 0 else None, "bit_exact": bool(_eq(g, c))}
        if lib_us:
            lib_ms = statistics.median(lib_us) / 1e3
            rec.update({"lib_ms": round(lib_ms, 4), "speedup_lib": round(c_ms / lib_ms, 2) if lib_ms > 0 else None})
        out.append(rec)

    # a1-a8 ORBextractor::operator(): one frame per call (host image in, keypoints and
    # descriptors out), the BASELINE configs C1, C3 (KITTI), C5 (5000 features, 12 levels)
    for (W, H, nf, L, tag) in ((640, 480, 1000, 8, "C1"), (1241, 376, 2000, 8, "C3"), (640, 480, 5000, 12, "C5")):
        img = synth.frame(11, W, H)
        ex = ORBextractor(nf, 1.2, L, 20, 7)
        p = O.params(nf, 1.2, L, 20, 7)

        def ex_g(ex=ex, img=img):
            k, d = ex(img)
            return k.view(np.uint8).copy(), d.copy()

        def ex_c(p=p, img=img):
            k, d, _ = O.extract(img, p)
            return k.view(np.uint8).copy(), d.copy()
        add("a2", "ORBextractor::operator() ORBextractor.cc:1513-1629 (a1-a8)",
            f"{tag}: {W}x{H}, {nf} features, {L} levels, one frame", ex_g, ex_c, lib=ex)

    A, B = S.two_views(O, 0)
    As, Bs = S.two_views(O, 2, stereo=True)
    nA, nB = len(A.keys), len(B.keys)
    size = f"{nA} x {nB} keypoints, 640x480"
    rng = np.random.default_rng(0)

    # a11 SearchByProjection(Frame&, vector<MapPoint*>, th) -- Tracking::SearchLocalPoints
    mps = S.mappoints_from(A, 0)
    trk = S.local_track(A, B, mps, 0)
    queries = rng.permutation(nA).astype(np.int32)
    f0 = np.full(nB, -1, np.int32)
    m = ORBmatcher(0.8, False)

    def a11_g():
        f = f0.copy()
        return m.SearchByProjectionLocal(B, f, queries, mps, trk, 3.0), f

    def a11_c():
        f = f0.copy()
        return O.sbp_local(B, f, queries, mps, trk, 3.0, 0.8), f
    add("a11", "ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, float) ORBmatcher.cc:61-173",
        size, a11_g, a11_c, lib=m)

    # a12 SearchByProjection(Frame& cur, const Frame& last, th, bMono) -- TrackWithMotionModel
    last_mp = np.arange(nA, dtype=np.int32)
    cur0 = np.full(nB, -1, np.int32)
    m12 = ORBmatcher(0.9, True)

    def a12_g():
        c = cur0.copy()
        return m12.SearchByProjectionFrame(B, c, A, last_mp, mps, 15.0, True), c

    def a12_c():
        c = cur0.copy()
        return O.sbp_frame(B, c, A, last_mp, mps, 15.0, True, True), c
    add("a12", "ORBmatcher::SearchByProjection(Frame&, const Frame&, float, bool) ORBmatcher.cc:1620-1789",
        size, a12_g, a12_c, lib=m12)

    # a13 SearchByProjection(Frame&, KeyFrame*, set<MapPoint*>, th, ORBdist) -- relocalisation
    mpsd = S.with_depth_info(S.mappoints_from(A, 1), A, 1)
    kf_mp = np.arange(nA, dtype=np.int32)

    def a13_g():
        c = cur0.copy()
        return m12.SearchByProjectionKeyFrame(B, c, A, kf_mp, mpsd, 10.0, 100), c

    def a13_c():
        c = cur0.copy()
        return O.sbp_keyframe(B, c, A, kf_mp, mpsd, 10.0, 100, True), c
    add("a13", "ORBmatcher::SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, float, int) "
        "ORBmatcher.cc:1792-1924", size, a13_g, a13_c, lib=m12)

    # a14 SearchByProjection(KeyFrame*, Scw, vpPoints, vpMatched, th) -- loop closing
    Scw = np.asarray(B.Tcw, np.float32)[:3, :4].copy()
    points = rng.permutation(nA)[: int(0.9 * nA)].astype(np.int32)
    m14 = ORBmatcher(0.75, False)

    def a14_g():
        c = cur0.copy()
        return m14.SearchByProjectionSim3(B, Scw, points, c, mpsd, 10), c

    def a14_c():
        c = cur0.copy()
        return O.sbp_sim3(B, Scw, points, c, mpsd, 10), c
    add("a14", "ORBmatcher::SearchByProjection(KeyFrame*, cv::Mat, const vector<MapPoint*>&, "
        "vector<MapPoint*>&, int) ORBmatcher.cc:398-520", size, a14_g, a14_c, lib=m14)

    # a15 SearchForTriangulation -- LocalMapping::CreateNewMapPoints
    has1 = (rng.random(nA) < 0.2).astype(np.uint8)
    has2 = (rng.random(nB) < 0.2).astype(np.uint8)
    fv1, fv2 = S.fv(A), S.fv(B)
    F12 = S.fundamental(A, B)
    m15 = ORBmatcher(0.6, False)
    add("a15", "ORBmatcher::SearchForTriangulation ORBmatcher.cc:850-1056", size,
        lambda: m15.SearchForTriangulation(A, has1, fv1, B, has2, fv2, F12, False),
        lambda: O.search_for_triangulation(A, has1, fv1, B, has2, fv2, F12, False, False), lib=m15)

    # a18 Frame::ComputeStereoMatches, 640x480 and KITTI 1241x376
    for W, H, nf in ((640, 480, 1000), (1241, 376, 2000)):
        left, right, _ = synth.stereo_pair(3, W, H, max_disp=48)
        ex = ORBextractor(nf, 1.2, 8, 20, 7)
        kps, desc, n = ex.extract_batch(np.stack([left, right]))
        kl, dl, kr, dr = kps[0][: n[0]], desc[0][: n[0]], kps[1][: n[1]], desc[1][: n[1]]
        p = O.params(nf, 1.2, 8, 20, 7)
        sf = np.array(p.scale[:8], np.float32)
        fx, bf = 718.856, 386.1448
        view = FrameView(keys=kl, desc=dl, fx=fx, fy=fx, cx=W / 2, cy=H / 2, bf=bf, b=bf / fx, max_x=W, max_y=H,
                         scale_factors=sf, level_sigma2=sf * sf)
        pl, pr = O.pyramid(left, p), O.pyramid(right, p)
        ms = ORBmatcher(0.6, True)
        add("a18", "Frame::ComputeStereoMatches Frame.cc:673-885", f"{len(kl)} x {len(kr)} keypoints, {W}x{H}",
            lambda: ms.ComputeStereoMatches(ex, 0, ex, 1, view, kr, dr, maxD=fx),
            lambda: O.compute_stereo_matches(view, kr, dr, pl, pr, fx), lib=ms)

    # f2 SearchByBoW (KF -> F, KF -> KF), SearchForInitialization
    mpb = np.arange(1000, 1000 + nA, dtype=np.int32)
    mpb[rng.random(nA) < 0.2] = -1
    mpb2 = np.arange(5000, 5000 + nB, dtype=np.int32)
    mpb2[rng.random(nB) < 0.3] = -1
    mb = ORBmatcher(0.7, True)
    add("f2", "ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) ORBmatcher.cc:228-392", size,
        lambda: mb.SearchByBoWFrame(A, mpb, fv1, B, fv2),
        lambda: O.search_by_bow_frame(A, mpb, fv1, B, fv2, 0.7, True), lib=mb)
    mk = ORBmatcher(0.75, True)
    add("f2", "ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&) ORBmatcher.cc:696-839", size,
        lambda: mk.SearchByBoWKeyFrames(A, mpb, fv1, B, mpb2, fv2),
        lambda: O.search_by_bow_keyframes(A, mpb, fv1, B, mpb2, fv2, 0.75, True), lib=mk)
    prev0 = np.ascontiguousarray(np.stack([A.keys["x"], A.keys["y"]], 1).astype(np.float32))
    mi = ORBmatcher(0.9, True)

    def init_g():
        prev = prev0.copy()
        n, mt = mi.SearchForInitialization(A, B, prev, 100)
        return n, mt, prev

    def init_c():
        return O.search_for_initialization(A, B, prev0.copy(), 100, 0.9, True)
    add("f2", "ORBmatcher::SearchForInitialization ORBmatcher.cc:539-683", size, init_g, init_c, lib=mi)

    # f3 UndistortKeyPoints + ComputeImageBounds + AssignFeaturesToGrid (TUM1 calibration)
    K = [517.306408, 516.469215, 318.643040, 255.313989]
    D = [0.262383, -0.953104, -0.005358, 0.002628, 1.163314]
    cam = FR.camera(*K, *D)
    keys = B.keys

    def f3_g():
        ku = FR.UndistortKeyPoints(cam, keys)
        b = FR.ComputeImageBounds(cam, 640, 480)
        s, i = FR.AssignFeaturesToGrid(ku, b)
        return ku, b, s, i

    def f3_c():
        kr_ = O.undistort_keypoints(K, D, keys)
        br = O.compute_image_bounds(K, D, 640, 480)
        s, i = O.assign_features_to_grid(kr_, br)
        return kr_, br, s, i
    add("f3", "Frame::UndistortKeyPoints + ComputeImageBounds + AssignFeaturesToGrid Frame.cc:351-370, 586-665",
        f"{len(keys)} keypoints", f3_g, f3_c)

    # f4 Fuse (both overloads), SearchBySim3, ComputeDistinctiveDescriptors
    mpf = S.mappoints_from(A, 4)
    mpf.pos = (mpf.pos - np.asarray(A.Tcw, np.float32)[:3, 3][None, :]).astype(np.float32)
    mpf = S.with_depth_info(mpf, A, 4)
    fpoints = rng.permutation(nA).astype(np.int32)
    skip = (rng.random(nA) < 0.1).astype(np.uint8)
    mf = ORBmatcher(0.6, True)
    add("f4", "ORBmatcher::Fuse(KeyFrame*, const vector<MapPoint*>&, float) ORBmatcher.cc:1067-1221", size,
        lambda: mf.Fuse(B, fpoints, skip, mpf, 3.0), lambda: O.fuse(B, fpoints, skip, mpf, 3.0), lib=mf)
    add("f4", "ORBmatcher::Fuse(KeyFrame*, cv::Mat Scw, ..., vector<MapPoint*>&) ORBmatcher.cc:1226-1352", size,
        lambda: mf.FuseSim3(B, Scw, fpoints, skip, mpf, 4.0), lambda: O.fuse_sim3(B, Scw, fpoints, skip, mpf, 4.0),
        lib=mf)
    counts = rng.integers(1, 12, 1000)
    base = rng.integers(0, 256, (len(counts), 32), dtype=np.uint8)
    descs = []
    for k, c in enumerate(counts):
        bits = np.unpackbits(np.repeat(base[k:k + 1], c, 0), axis=1)
        bits ^= (rng.random(bits.shape) < 0.15).astype(np.uint8)
        descs.append(np.packbits(bits, axis=1))
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    dd = np.concatenate(descs)
    add("f4", "MapPoint::ComputeDistinctiveDescriptors MapPoint.cc:295-360", f"{len(counts)} MapPoints",
        lambda: ComputeDistinctiveDescriptors(off, dd)[0], lambda: O.distinctive_descriptors(off, dd))
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(prog="bench.py --rows")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--steps", type=int, default=None, help="alias of --reps (profiling scripts)")
    ap.add_argument("--warmup", type=int, default=None, help="ignored")
    ap.add_argument("--no-cpu-baseline", action="store_true", help="ignored (the CPU leg is the comparison)")
    ap.add_argument("--only", default="", help="comma-separated row ids (e.g. a2,a12); default every row")
    args = ap.parse_args(argv)
    reps = args.steps if args.steps else args.reps
    from oracle import oracle as O
    O.build()
    res = rows(O, reps, set(args.only.split(",")) if args.only else None)
    print(json.dumps({"metric": "per-row drop-in call latency (host API, GPU) vs CPU oracle", "unit": "ms",
                      "reps": reps, "rows": res,
                      "all_bit_exact": all(r["bit_exact"] for r in res)}), flush=True)


if __name__ == "__main__":
    main()
