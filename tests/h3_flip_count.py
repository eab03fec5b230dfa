"""H3 at descriptor level: how far the shipped restatement's rBRIEF rotation is from the
reference's literal arithmetic.

ORBextractor.cc:123-125 computes `float a = (float)cos(angle), b = (float)sin(angle)` on
a float radian under `using namespace std`, i.e. glibc cosf / sinf.  The oracle and the
GPU use the correctly rounded (float)cos((double)r) instead, because
cosf is a library-version-dependent approximation (glibc 2.23 in the reference's build
environment, 2.35 here).  This script extracts the same frames both ways (the oracle's
ora_set_trig_mode) and counts frames, descriptors and bits that differ.  Keypoints,
angles and order cannot differ: cos / sin feed only the descriptor sample positions.

    python tests/h3_flip_count.py [--frames 256] [--out profiles/r02_h3_flips.json]

TEST INFRASTRUCTURE: runs only the CPU oracle.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def count_flips(frames: np.ndarray, nfeatures=1000, scale=1.2, nlevels=8, threads: int = 8) -> dict:
    from oracle import oracle as O
    O.build()
    p = O.params(nfeatures, scale, nlevels, 20, 7)

    def one(img):
        k0, d0, _ = O.extract(img, p, trig_mode=0)
        k1, d1, _ = O.extract(img, p, trig_mode=1)
        same_kps = len(k0) == len(k1) and np.array_equal(k0.view(np.uint8), k1.view(np.uint8))
        rows = np.nonzero((d0 != d1).any(axis=1))[0] if same_kps else np.arange(len(k0))
        bits = int(np.unpackbits(d0 ^ d1).sum()) if same_kps else -1
        return len(k0), len(rows), bits, same_kps

    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(one, frames))
    nk = sum(r[0] for r in res)
    nd = sum(r[1] for r in res)
    return {
        "frames": len(frames),
        "keypoints_identical_all_frames": all(r[3] for r in res),
        "frames_with_a_differing_descriptor": sum(1 for r in res if r[1]),
        "keypoints": nk,
        "descriptors_differing": nd,
        "descriptor_bits_differing": sum(r[2] for r in res),
        "descriptor_diff_rate": nd / max(nk, 1),
        "glibc": " ".join(platform.libc_ver()),
    }


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    from orbslam2commentedbyxcm_amd import synth
    frames, _ = synth.sequence(1000, a.frames)  # bench.py's rank-0 batch
    r = count_flips(frames, threads=min(16, len(os.sched_getaffinity(0))))
    r["workload"] = f"bench.py configs[1] batch (synth.sequence(1000, {a.frames})), 640x480, 1000 features"
    print(json.dumps(r))
    if a.out:
        Path(a.out).write_text(json.dumps(r, indent=1) + "\n")


if __name__ == "__main__":
    main()
