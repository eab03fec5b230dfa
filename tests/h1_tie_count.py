"""H1 at keypoint level: how often DistributeOctTree's heap-address tie-break decides the
output.

ORBextractor.cc:899-913 sorts the final phase's (size, ExtractorNode*) pairs with
std::sort and splits from the back, so nodes of equal size are taken in heap-address
order -- whatever glibc malloc returned in the reference's process.  The oracle and the GPU
fix the order to allocation order (later-created node first: a monotonic allocator,
DESIGN.md §2).  This script extracts the same frames with that rule and with the opposite
one (earlier-created first; the oracle's tie mode 1) and counts the frames and levels whose
keypoints differ, plus the final-phase passes in which a split node shared its size with
another node (the passes where any address order could matter).  A level that differs
between the two extremes is one where the reference's output depends on its heap.

    python tests/h1_tie_count.py [--frames 256] [--out profiles/r03_h1_ties.json]

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


def count_ties(frames: np.ndarray, prm=(1000, 1.2, 8, 20, 7), threads: int = 8) -> dict:
    from oracle import oracle as O
    O.build()
    p = O.params(*prm)
    L = O.lib()

    def one(img):
        L.ora_octree_ties(1)
        k0, d0, c0 = O.extract(img, p, tie_mode=0)
        ties = int(L.ora_octree_ties(1))
        k1, d1, c1 = O.extract(img, p, tie_mode=1)
        L.ora_octree_ties(1)
        levels_order, levels_set = [], []
        o0 = np.concatenate([[0], np.cumsum(c0)])
        o1 = np.concatenate([[0], np.cumsum(c1)])
        for lv in range(p.nlevels):
            a = k0[o0[lv]:o0[lv + 1]].view(np.uint8).reshape(-1, 28)
            b = k1[o1[lv]:o1[lv + 1]].view(np.uint8).reshape(-1, 28)
            if len(a) == len(b) and np.array_equal(a, b):
                continue
            levels_order.append(lv)
            sa = {bytes(r) for r in a}
            sb = {bytes(r) for r in b}
            if sa != sb:
                levels_set.append(lv)
        return ties, levels_order, levels_set, len(k0)

    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(one, frames))
    per_level_order = np.zeros(p.nlevels, int)
    per_level_set = np.zeros(p.nlevels, int)
    for _, lo, ls, _ in res:
        per_level_order[lo] += 1
        per_level_set[ls] += 1
    return {
        "frames": len(frames),
        "levels_per_frame": p.nlevels,
        "keypoints": int(sum(r[3] for r in res)),
        "final_phase_passes_with_a_deciding_tie": int(sum(r[0] for r in res)),
        "frames_with_a_tie_pass": int(sum(1 for r in res if r[0])),
        "frames_output_differs": int(sum(1 for r in res if r[1])),
        "frames_keypoint_set_differs": int(sum(1 for r in res if r[2])),
        "levels_output_differs": int(per_level_order.sum()),
        "levels_keypoint_set_differs": int(per_level_set.sum()),
        "levels_output_differs_by_level": per_level_order.tolist(),
        "levels_keypoint_set_differs_by_level": per_level_set.tolist(),
    }


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    from orbslam2commentedbyxcm_amd import synth
    frames, _ = synth.sequence(1000, a.frames)  # bench.py's rank-0 batch
    th = min(16, len(os.sched_getaffinity(0)))
    out = {"rule_shipped": "later-created node first (allocation order, ORBextractor.cc:899-913 with a monotonic "
                           "allocator)", "rule_opposite": "earlier-created node first"}
    out["configs[1] C1 1000 x 8"] = count_ties(frames, (1000, 1.2, 8, 20, 7), th)
    out["configs[4] C5 5000 x 12"] = count_ties(frames, (5000, 1.2, 12, 20, 7), th)
    out["workload"] = f"bench.py configs[1] batch (synth.sequence(1000, {a.frames})), 640x480"
    print(json.dumps(out))
    if a.out:
        Path(a.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
