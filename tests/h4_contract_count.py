"""H4 at descriptor level: the reference's build contracts a*b + c*d into FMA.

The reference is compiled by g++ with -O3 -march=native (CMakeLists.txt:10-19), and g++
contracts floating-point expressions in C++ even under -std=c++11 (GCC keeps contraction
off by default only for ISO C): the reference's own BowVector.cpp, built with DBoW2's
flags, holds a vfmadd (tests/test_vocab_ref.py).  The rBRIEF sample offsets
x*b + y*a and x*a - y*b (ORBextractor.cc:136-138) are contractible, so the reference
binary rounds them fused, fma(x, b, y*a) and fma(x, a, -(y*b)) (GCC's FMA pass fuses the
first product into the add), and so do the shipped oracle and k_describe.  This script
extracts the same frames fused and unfused (the oracle's ora_set_contract_mode(0)) and
counts frames, descriptors and bits that differ: what the choice decides.  Keypoints and
angles cannot differ.

    python tests/h4_contract_count.py [--frames 256] [--out profiles/r03_h4_contract.json]

TEST INFRASTRUCTURE: runs only the CPU oracle.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def count(frames: np.ndarray, nfeatures: int, nlevels: int, threads: int) -> dict:
    from oracle import oracle as O
    O.build()
    p = O.params(nfeatures, 1.2, nlevels, 20, 7)

    def one(img):
        k0, d0, _ = O.extract(img, p)  # shipped: fused
        k1, d1, _ = O.extract(img, p, contract_mode=0)
        same_kps = len(k0) == len(k1) and np.array_equal(k0.view(np.uint8), k1.view(np.uint8))
        rows = np.nonzero((d0 != d1).any(axis=1))[0] if same_kps else np.arange(len(k0))
        bits = int(np.unpackbits(d0 ^ d1).sum()) if same_kps else -1
        return len(k0), len(rows), bits, same_kps

    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(one, frames))
    nk = sum(r[0] for r in res)
    nd = sum(r[1] for r in res)
    return {"frames": len(frames), "keypoints_identical_all_frames": all(r[3] for r in res),
            "frames_with_a_differing_descriptor": sum(1 for r in res if r[1]), "keypoints": nk,
            "descriptors_differing": nd, "descriptor_bits_differing": sum(r[2] for r in res),
            "descriptor_diff_rate": nd / max(nk, 1)}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    from orbslam2commentedbyxcm_amd import synth
    frames, _ = synth.sequence(1000, a.frames)  # bench.py's rank-0 batch
    th = min(16, len(os.sched_getaffinity(0)))
    out = {"model": "shipped: rBRIEF offsets fused as g++ -O3 -march=native builds the reference, "
                    "fma(x, b, y*a), fma(x, a, -(y*b)) (ORBextractor.cc:136-138); compared: unfused",
           "workload": f"bench.py configs[1] batch (synth.sequence(1000, {a.frames})), 640x480",
           "configs[1] C1 1000 x 8": count(frames, 1000, 8, th),
           "configs[4] C5 5000 x 12": count(frames, 5000, 12, th)}
    print(json.dumps(out))
    if a.out:
        Path(a.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
