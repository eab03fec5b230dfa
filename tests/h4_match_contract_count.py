"""H4 in the matchers: how many outputs the reference build's FMA contraction would change.

g++ -O3 -march=native (the reference's flags) contracts the matchers' projection and
epipolar expressions -- u = fx*xc*invzc + cx, ur = u - mbf*invzc, CheckDistEpipolarLine's
a*x + b*y + c, the epipole test and Fuse's chi-square -- and the shipped restatement
(oracle and liborbx) fuses them the same way.  This script runs
the oracle's matchers fused and unfused (ora_set_match_contract_mode(0)) on the same
scenes and counts the outputs that differ -- what the choice decides: the bench's 255 TrackWithMotionModel pairs, and the general-pose
scenes of the GPU tests for a11, a12 (mono, stereo), a13, a14, a15 and Fuse.

    python tests/h4_match_contract_count.py [--out profiles/r03_h4_match_contract.json]

TEST INFRASTRUCTURE: runs only the CPU oracle.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def both(O, fn):
    """fn() unfused and fused -> (unfused result, fused result)."""
    L = O.lib()
    L.ora_set_match_contract_mode.argtypes = [__import__("ctypes").c_int]
    L.ora_set_match_contract_mode(0)
    a = fn()
    L.ora_set_match_contract_mode(1)
    try:
        b = fn()
    finally:
        L.ora_set_match_contract_mode(1)  # the shipped (fused) form
    return a, b


def diff(a, b) -> int:
    """Differing entries of two (count, array) or array results."""
    if isinstance(a, tuple):
        return sum(diff(x, y) for x, y in zip(a, b))
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return max(a.size, b.size)
    return int((a != b).sum())


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--frames", type=int, default=256)
    args = ap.parse_args(argv)
    import match_scenes as S
    from oracle import checks
    from oracle import oracle as O
    from orbslam2commentedbyxcm_amd import synth
    from orbslam2commentedbyxcm_amd.matcher import Track
    from orbslam2commentedbyxcm_amd.pipeline import sequence_poses
    O.build()
    out = {"model": "fused: u = fma(fx*xc, invzc, cx), ur = fma(-mbf, invzc, u), epipolar a = fma(x, F00, y*F10) + F20 "
                    "etc., den = fma(a, a, b*b), chi2 e2 = fma(ex, ex, ey*ey) (shipped); compared: unfused"}
    # the bench's sequence (configs[1]): every pair's matches
    frames, off = synth.sequence(1000, args.frames)
    T = sequence_poses(off)
    ref = checks.extract_all(frames)
    sf = np.array(O.params(1000, 1.2, 8, 20, 7).scale[:8], np.float32)
    u, f = both(O, lambda: checks.sequence_matches(ref, T, sf, threads=8))
    pairs = [b for b in range(1, len(ref)) if u[b][0] != f[b][0] or not np.array_equal(u[b][1], f[b][1])]
    out["configs[1] a12 pairs"] = {"pairs": len(ref) - 1, "pairs_differing": len(pairs),
                                   "matches": int(sum(u[b][0] for b in range(1, len(ref)))),
                                   "assignments_differing": int(sum((u[b][1] != f[b][1]).sum()
                                                                    for b in range(1, len(ref))))}
    rows = {}

    def add(name, fn):
        a, b = both(O, fn)
        rows.setdefault(name, [0, 0])
        rows[name][0] += 1
        rows[name][1] += diff(a, b)

    for scene in S.POSED:
        for stereo in (False, True):
            A, B = S.posed_views(O, 1, scene, stereo=stereo)
            mps = S.posed_mappoints(A, 1)
            lm = np.arange(len(A.keys), dtype=np.int32)
            for co in (False, True):
                def a12(A=A, B=B, mps=mps, lm=lm, co=co, stereo=stereo):
                    c = np.full(len(B.keys), -1, np.int32)
                    return O.sbp_frame(B, c, A, lm, mps, 7.0 if stereo else 15.0, not stereo, co), c
                add("a12 SearchByProjection(Frame, LastFrame)", a12)
        A, B = S.posed_views(O, 4, scene, stereo=scene in ("forward", "tilt"))
        mps = S.with_depth_info(S.posed_mappoints(A, 4), A, 4)
        q = np.random.default_rng(5).permutation(len(A.keys)).astype(np.int32)

        def a11(A=A, B=B, mps=mps, q=q):
            t = O.is_in_frustum(B, mps)
            tr = Track(in_view=t.in_view, proj_x=t.proj_x, proj_y=t.proj_y, proj_xr=t.proj_xr,
                       scale_level=t.scale_level, view_cos=t.view_cos)
            fr = np.full(len(B.keys), -1, np.int32)
            return O.sbp_local(B, fr, q, mps, tr, 1.0, 0.8), fr
        add("a11 SearchByProjection(Frame, vpMapPoints) + IsInFrustum", a11)
        A, B = S.posed_views(O, 6, scene)
        mps6 = S.with_depth_info(S.posed_mappoints(A, 6), A, 6)
        km = np.arange(len(A.keys), dtype=np.int32)

        def a13(A=A, B=B, mps=mps6, km=km):
            c = np.full(len(B.keys), -1, np.int32)
            return O.sbp_keyframe(B, c, A, km, mps, 10.0, 100, True), c
        add("a13 SearchByProjection(Frame, KeyFrame, set)", a13)
        Scw = np.asarray(B.Tcw, np.float32)[:3, :4].copy()
        pts = np.arange(len(A.keys), dtype=np.int32)

        def a14(B=B, Scw=Scw, pts=pts, mps=mps6):
            c = np.full(len(B.keys), -1, np.int32)
            return O.sbp_sim3(B, Scw, pts, c, mps, 10), c
        add("a14 SearchByProjection(KeyFrame, Scw)", a14)

        def fuse(B=B, pts=pts, mps=mps6):
            return O.fuse(B, pts, np.zeros(len(pts), np.uint8), mps, 3.0)
        add("f4 Fuse(KeyFrame, vpMapPoints)", fuse)
        for stereo in (False, True):
            A, B = S.posed_views(O, 9, scene, stereo=stereo)
            rng = np.random.default_rng(9)
            h1 = (rng.random(len(A.keys)) < 0.2).astype(np.uint8)
            h2 = (rng.random(len(B.keys)) < 0.2).astype(np.uint8)
            fv1, fv2, F12 = S.fv(A), S.fv(B), S.fundamental(A, B)
            add("a15 SearchForTriangulation",
                lambda A=A, B=B, h1=h1, h2=h2, fv1=fv1, fv2=fv2, F12=F12:
                O.search_for_triangulation(A, h1, fv1, B, h2, fv2, F12, False, False))
    out["posed scenes"] = {k: {"calls": v[0], "outputs_differing": v[1]} for k, v in rows.items()}
    print(json.dumps(out, indent=1))
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
