"""H1 against a real allocator: DistributeOctTree's final-phase tie order as glibc malloc
decides it, compared with the shipped rule (later-created node first) and the opposite
one, on the bench frames.

ORBextractor.cc:899-913 sorts (size, ExtractorNode*) pairs, so equal-size nodes split in
heap-address order.  tests/h1_glibc/octree_glibc.cpp runs the octree's list and sort
under glibc (its node and vector allocations sized like the reference's), one process per
frame sequence, all frames and levels in order; this script feeds it the oracle's FAST
candidates of each level (the input the reference's DistributeOctTree sees) and compares
its kept keypoints per level with the oracle's under both tie rules.

A level is *tie-deciding* when the two rules give different outputs; elsewhere all three
must agree (a check of the transcription).  Modes: "octree" (the octree's own
allocations only) and "frame" (plus the surrounding per-frame allocations of
ORBextractor::operator()), each in the main thread and in a second thread (a non-main
malloc arena, like ORB-SLAM2's Tracking thread).

    python tests/h1_glibc_measure.py [--frames 256] [--out profiles/r04_h1_glibc.json] [--bump-only]

"bump_allocator": the same transcription with the octree's allocations from a monotonic
bump allocator (mode 2): nodes created later have higher addresses, the order H1's shipped
rule names, so it must equal the oracle on every level -- tie-deciding ones included.

TEST INFRASTRUCTURE: the CPU oracle and a host C++ program only.
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

SRC = Path(__file__).resolve().parent / "h1_glibc" / "octree_glibc.cpp"
EDGE = 19


def build(out_dir: Path) -> Path:
    exe = out_dir / "octree_glibc"
    subprocess.run(["g++", "-O3", "-std=c++11", "-Wall", "-pthread", "-o", str(exe), str(SRC)], check=True)
    return exe


def level_inputs(frames, prm, threads):
    """Per frame and level: (minX, maxX, minY, maxY, N, cell counts, candidates, w, h)."""
    from oracle import oracle as O
    O.build()
    p = O.params(*prm)

    def one(img):
        lv = O.pyramid(img, p)
        out = []
        for l, level in enumerate(lv):
            h, w = level.shape
            cand, cells = O.level_candidates_cells(level, p)
            out.append((EDGE - 3, w - EDGE + 3, EDGE - 3, h - EDGE + 3, int(p.features_per_level[l]), cells, cand,
                        w, h))
        return out

    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(one, frames))


def write_input(path: Path, levels, nfeatures: int, mode: int, thread: int):
    with open(path, "wb") as f:
        f.write(struct.pack("<5i", len(levels), len(levels[0]), nfeatures, mode, thread))
        for fr in levels:
            for (x0, x1, y0, y1, N, cells, cand, w, h) in fr:
                f.write(struct.pack("<9i", x0, x1, y0, y1, N, len(cells), len(cand), w, h))
                cc = np.zeros((len(cells), 2), np.int32)
                cc[:, 0] = cells
                f.write(cc.tobytes())
                f.write(np.stack([cand["x"], cand["y"], cand["response"]], 1).astype(np.float32).tobytes())


def read_output(path: Path, nframes: int, nlevels: int):
    buf = path.read_bytes()
    o = 0
    res = []
    for _ in range(nframes):
        fr = []
        for _ in range(nlevels):
            n = struct.unpack_from("<i", buf, o)[0]
            o += 4
            fr.append(np.frombuffer(buf, np.float32, 3 * n, o).reshape(n, 3).copy())
            o += 12 * n
        res.append(fr)
    return res


def oracle_rules(levels, threads):
    """The oracle's kept (x, y, response) per frame and level under tie rules 0 and 1."""
    from oracle import oracle as O
    L = O.lib()
    out = {}
    for mode in (0, 1):
        L.ora_set_octree_tie_mode(mode)
        res = []
        for fr in levels:
            r = []
            for (x0, x1, y0, y1, N, _, cand, _, _) in fr:
                k = O.distribute_octree(cand, x0, x1, y0, y1, N)
                r.append(np.stack([k["x"], k["y"], k["response"]], 1).astype(np.float32))
            res.append(r)
        out[mode] = res
    L.ora_set_octree_tie_mode(0)
    return out


def compare(glibc, rules):
    same = lambda a, b: a.shape == b.shape and np.array_equal(a, b)  # noqa: E731
    tie_levels = agree_shipped = agree_opposite = neither = 0
    set_shipped = set_opposite = 0
    untied_mismatch = 0
    per_level = {}
    for f, fr in enumerate(glibc):
        for l, g in enumerate(fr):
            a, b = rules[0][f][l], rules[1][f][l]
            if same(a, b):
                untied_mismatch += not same(g, a)
                continue
            tie_levels += 1
            pl = per_level.setdefault(l, [0, 0, 0])
            pl[0] += 1
            if same(g, a):
                agree_shipped += 1
                pl[1] += 1
            elif same(g, b):
                agree_opposite += 1
                pl[2] += 1
            else:
                neither += 1
            gs = {tuple(r) for r in g.tolist()}
            set_shipped += gs == {tuple(r) for r in a.tolist()}
            set_opposite += gs == {tuple(r) for r in b.tolist()}
    return {"tie_deciding_levels": tie_levels, "glibc_equals_shipped": agree_shipped,
            "glibc_equals_opposite": agree_opposite, "glibc_equals_neither": neither,
            "glibc_keypoint_set_equals_shipped": set_shipped, "glibc_keypoint_set_equals_opposite": set_opposite,
            "fraction_equal_shipped": round(agree_shipped / tie_levels, 4) if tie_levels else None,
            "untied_levels_mismatched": untied_mismatch,
            "by_level_tied_shipped_opposite": {str(k): v for k, v in sorted(per_level.items())}}


def compare_bump(bump, rules):
    """The bump-allocator run against the shipped rule on every level (tied or not)."""
    same = lambda a, b: a.shape == b.shape and np.array_equal(a, b)  # noqa: E731
    levels = tied = mism = mism_tied = 0
    for f, fr in enumerate(bump):
        for l, g in enumerate(fr):
            a, b = rules[0][f][l], rules[1][f][l]
            t = not same(a, b)
            levels += 1
            tied += t
            if not same(g, a):
                mism += 1
                mism_tied += t
    return {"levels": levels, "tie_deciding_levels": tied, "mismatched_vs_shipped": mism,
            "tie_deciding_mismatched_vs_shipped": mism_tied}


def measure(frames, prm, threads, exe, tmp: Path, bump_only: bool = False) -> dict:
    levels = level_inputs(frames, prm, threads)
    rules = oracle_rules(levels, threads)
    out = {"frames": len(frames), "levels": len(levels[0])}
    fin, fout = tmp / "in_bump.bin", tmp / "out_bump.bin"
    write_input(fin, levels, prm[0], 2, 0)
    subprocess.run([str(exe), str(fin), str(fout)], check=True)
    out["bump_allocator"] = compare_bump(read_output(fout, len(frames), len(levels[0])), rules)
    if bump_only:
        return out
    for mode, mname in ((0, "octree"), (1, "frame")):
        for thread in (0, 1):
            fin, fout = tmp / f"in_{mode}{thread}.bin", tmp / f"out_{mode}{thread}.bin"
            write_input(fin, levels, prm[0], mode, thread)
            subprocess.run([str(exe), str(fin), str(fout)], check=True)
            g = read_output(fout, len(frames), len(levels[0]))
            out[f"{mname}_{'worker_thread' if thread else 'main_thread'}"] = compare(g, rules)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--out", default="")
    ap.add_argument("--bump-only", action="store_true", help="only the monotonic bump-allocator check")
    a = ap.parse_args(argv)
    from orbslam2commentedbyxcm_amd import synth
    frames, _ = synth.sequence(1000, a.frames)  # bench.py's rank-0 batch
    th = min(16, len(os.sched_getaffinity(0)))
    import platform
    libc = " ".join(platform.libc_ver())
    with tempfile.TemporaryDirectory() as d:
        tmp = Path(d)
        exe = build(tmp)
        what = ("DistributeOctTree final-phase tie order under glibc malloc (tests/h1_glibc/octree_glibc.cpp, "
                "one process per 256-frame sequence) vs the shipped rule (later-created node first) and the "
                "opposite (earlier-created first), per level of the bench frames")
        if a.bump_only:
            what = ("the same transcription (tests/h1_glibc/octree_glibc.cpp mode 2) with the octree's allocations "
                    "from a monotonic bump allocator (global operator new replaced, reset per level), against the "
                    "shipped rule on every level of the bench frames: 0 mismatches means the transcription is right "
                    "on the tie-deciding levels too and the shipped rule is the bump-allocator order H1 names")
        res = {"what": what,
               "libc": libc, "compiler": subprocess.run(["g++", "--version"], capture_output=True,
                                                         text=True).stdout.splitlines()[0],
               "workload": f"bench.py configs[1] batch (synth.sequence(1000, {a.frames})), 640x480"}
        res["configs[1] C1 1000 x 8"] = measure(frames, (1000, 1.2, 8, 20, 7), th, exe, tmp, a.bump_only)
        res["configs[4] C5 5000 x 12"] = measure(frames, (5000, 1.2, 12, 20, 7), th, exe, tmp, a.bump_only)
    print(json.dumps(res, indent=1))
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
