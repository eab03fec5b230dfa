"""Concurrent drop-in calls: T host threads, each with its own ORBextractor and ORBmatchers
(each instance has its own stream and pinned staging), run the per-frame work an
unchanged Tracking thread does through the reference-shaped host API --
ORBextractor::operator() on a C1 frame (ORBextractor.cc:1513-1629), TrackWithMotionModel's
SearchByProjection(Frame&, const Frame&, th, bMono) (a12, ORBmatcher.cc:1620-1789) and
TrackLocalMap's SearchByProjection(Frame&, vector<MapPoint*>, th) (a11, cc:61-173) -- in
a loop, and report the aggregate frames/s for each T.

One Tracking thread is latency-bound: it hands over one frame at a time, so its rate is
1 / (the three calls' latency).  Several Tracking threads (a multi-camera rig, several
sequences, a tracking server) share the GPU through the same drop-in calls; this
measures how far that goes without the batched API.

    python bench.py --dropin [--threads 1,2,4,8,16] [--seconds 3]

Lives in benchmarks/ (bench.py --dropin); it checks every frame's results against the oracle
(test infrastructure), and builds the matching scene with it."""
from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "benchmarks"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

import numpy as np  # noqa: E402


def write_scene(path, imgs, A, B, mps, trk, queries, last_mp, n12, c_ref, n11, f_ref, refs, nlevels):
    """The C++ driver's input (tests/cpp/dropin_mt.cpp, Scene / load): little-endian int32 /
    float32 / uint8 arrays in a fixed order; the images and the oracle's (keypoints,
    descriptors) of each last."""
    from match_scenes import CX, CY, FX, FY
    i32 = lambda *v: np.asarray(v, np.int32).tobytes()  # noqa: E731
    f32 = lambda a: np.ascontiguousarray(a, np.float32).tobytes()  # noqa: E731
    u8 = lambda a: np.ascontiguousarray(a).view(np.uint8).tobytes()  # noqa: E731
    h, w = imgs[0].shape
    parts = [i32(w, h, len(A.keys), len(B.keys), nlevels, len(queries)), f32([FX, FY, CX, CY]),
             u8(A.keys), u8(A.desc), f32(np.asarray(A.Tcw, np.float32)[:3].reshape(-1)),
             u8(B.keys), u8(B.desc), f32(np.asarray(B.Tcw, np.float32)[:3].reshape(-1)),
             f32(A.scale_factors), f32(A.level_sigma2),
             f32(mps.pos), u8(mps.desc), i32(*mps.observations), u8(mps.bad),
             u8(trk.in_view), f32(trk.proj_x), f32(trk.proj_y), f32(trk.proj_xr), i32(*trk.scale_level),
             f32(trk.view_cos), i32(*queries), i32(*last_mp),
             i32(n12), i32(*c_ref), i32(n11), i32(*f_ref), i32(len(imgs))]
    for img, (k_ref, d_ref) in zip(imgs, refs):
        parts += [u8(img), i32(len(k_ref)), u8(k_ref), u8(d_ref)]
    Path(path).write_bytes(b"".join(parts))


def build_driver(out: Path) -> Path:
    """tests/cpp/dropin_mt.cpp against include/orbx.hpp and the in-tree liborbx.so."""
    import subprocess
    lib = ROOT / "orbslam2commentedbyxcm_amd"
    cmd = ["g++", "-O2", "-std=c++17", "-pthread", f"-I{ROOT / 'include'}", str(ROOT / "tests" / "cpp" / "dropin_mt.cpp"),
           "-o", str(out), f"-L{lib}", "-lorbx", f"-Wl,-rpath,{lib}"]
    subprocess.run(cmd, check=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(prog="bench.py --dropin")
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--images", type=int, default=8, help="distinct C1 images cycled through (each frame checked)")
    ap.add_argument("--cpp", action="store_true",
                    help="run the threads in a C++ program (tests/cpp/dropin_mt.cpp) instead of Python threads")
    args, _ = ap.parse_known_args(argv)
    counts = [int(t) for t in args.threads.split(",") if t]

    from oracle import oracle as O
    O.build()
    import match_scenes as S
    from orbslam2commentedbyxcm_amd import ORBextractor, synth
    from orbslam2commentedbyxcm_amd.matcher import ORBmatcher

    prm = (1000, 1.2, 8, 20, 7)
    imgs = [synth.frame(11 + j, 640, 480) for j in range(max(1, args.images))]
    A, B = S.two_views(O, 0)
    mps = S.mappoints_from(A, 0)
    trk = S.local_track(A, B, mps, 0)
    nA, nB = len(A.keys), len(B.keys)
    queries = np.random.default_rng(0).permutation(nA).astype(np.int32)
    last_mp = np.arange(nA, dtype=np.int32)
    cur0 = np.full(nB, -1, np.int32)
    f0 = np.full(nB, -1, np.int32)

    # the oracle's answers for the three calls (the extraction per image)
    refs = [O.extract(im, O.params(*prm))[:2] for im in imgs]
    c_ref = cur0.copy()
    n12_ref = O.sbp_frame(B, c_ref, A, last_mp, mps, 15.0, True, True)
    f_ref = f0.copy()
    n11_ref = O.sbp_local(B, f_ref, queries, mps, trk, 3.0, 0.8)

    if args.cpp:
        import subprocess
        import tempfile
        tmp = Path(tempfile.mkdtemp(prefix="orbx_dropin_"))
        scene = tmp / "scene.bin"
        write_scene(scene, imgs, A, B, mps, trk, queries, last_mp, n12_ref, c_ref, n11_ref, f_ref, refs,
                    len(A.scale_factors))
        exe = build_driver(tmp / "dropin_mt")
        rows = []
        for T in counts:
            r = subprocess.run([str(exe), str(scene), str(T), str(args.seconds)], capture_output=True, text=True,
                               timeout=120 + 4 * args.seconds)
            if r.returncode:
                raise SystemExit(f"dropin_mt: {r.stderr[-500:]}")
            rec = json.loads(r.stdout.strip().splitlines()[-1])
            rec["ms_per_frame_per_thread"] = round(1e3 * T / rec["frames_per_s"], 4)
            rows.append(rec)
            print(json.dumps(rec), file=sys.stderr, flush=True)
        print(json.dumps({"metric": "frames/s of the per-frame drop-in host calls (ORBextractor::operator() C1 + "
                                    "SearchByProjection a12 + a11) from C++ threads (include/orbx.hpp), one MI355X",
                          "unit": "frames/s", "rows": rows, "all_bit_exact": all(r["bit_exact"] for r in rows),
                          "frames_run": sum(r["frames"] + 2 * r["threads"] for r in rows),
                          "frames_checked": sum(r["frames_checked"] for r in rows),
                          "frames_mismatched": sum(r["frames_mismatched"] for r in rows),
                          "note": f"tests/cpp/dropin_mt.cpp: each thread its own ORBextractor / ORBmatcher instances "
                                  f"(own streams); host images and host arrays in and out; frame k of thread t "
                                  f"extracts image (k + t) % {len(imgs)}, and every frame (warm-up and timed) is "
                                  f"compared with the oracle's results"}), flush=True)
        return

    def one_frame(ex, m12, m11, j):
        k, d = ex(imgs[j])
        c = cur0.copy()
        n12 = m12.SearchByProjectionFrame(B, c, A, last_mp, mps, 15.0, True)
        f = f0.copy()
        n11 = m11.SearchByProjectionLocal(B, f, queries, mps, trk, 3.0)
        return k, d, n12, c, n11, f, j

    def exact(r) -> bool:
        k, d, n12, c, n11, f, j = r
        k_ref, d_ref = refs[j]
        return (np.array_equal(k.view(np.uint8), k_ref.view(np.uint8)) and np.array_equal(d, d_ref)
                and n12 == n12_ref and np.array_equal(c, c_ref) and n11 == n11_ref and np.array_equal(f, f_ref))

    rows, all_exact = [], True
    for T in counts:
        ready = threading.Barrier(T + 1)
        go = threading.Event()
        done = [0] * T
        bad = [0] * T
        spans = [None] * T
        errors = []
        deadline = [0.0]

        def worker(i):
            try:
                ex = ORBextractor(*prm)
                m12, m11 = ORBmatcher(0.9, True), ORBmatcher(0.8, False)
                bad[i] += not exact(one_frame(ex, m12, m11, i % len(imgs)))  # warm-up (checked too)
                bad[i] += not exact(one_frame(ex, m12, m11, (i + 1) % len(imgs)))
            except Exception as e:  # reported, and the run fails below
                errors.append(repr(e))
                ex = None
            ready.wait()
            go.wait()
            if ex is None:
                return
            t0 = time.perf_counter()
            n = 0
            while time.perf_counter() < deadline[0]:
                bad[i] += not exact(one_frame(ex, m12, m11, (i + 2 + n) % len(imgs)))  # every frame compared
                n += 1
            spans[i] = (t0, time.perf_counter())
            done[i] = n

        threads = [threading.Thread(target=worker, args=(i,)) for i in range(T)]
        for t in threads:
            t.start()
        ready.wait()
        deadline[0] = time.perf_counter() + args.seconds
        go.set()
        for t in threads:
            t.join()
        if errors:
            raise SystemExit(f"dropin: {errors[0]}")
        start = min(s[0] for s in spans)
        end = max(s[1] for s in spans)
        frames = sum(done)
        rate = frames / (end - start)
        all_exact = all_exact and not any(bad)
        rows.append({"threads": T, "frames_per_s": round(rate, 1), "frames": frames,
                     "ms_per_frame_per_thread": round(1e3 * T / rate, 4), "frames_checked": frames + 2 * T,
                     "frames_mismatched": sum(bad), "bit_exact": not any(bad)})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    out = {"metric": "frames/s of the per-frame drop-in host calls (ORBextractor::operator() C1 + "
                     "SearchByProjection a12 + a11), T Tracking threads on one MI355X",
           "unit": "frames/s", "rows": rows, "all_bit_exact": all_exact,
           "frames_checked": sum(r["frames_checked"] for r in rows),
           "frames_mismatched": sum(r["frames_mismatched"] for r in rows),
           "note": "each thread: its own ORBextractor / ORBmatcher instances (own streams); host images and "
                   "host arrays in and out, as Tracking passes them; every frame (warm-up and timed) compared "
                   "with the oracle's results"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
