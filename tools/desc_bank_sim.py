"""LDS bank-conflict model of k_describe's steered-BRIEF sampling.

Each pair step of k_describe is two ds_read_u8 gathers per lane: lane ql of quarter qt
reads one rotated pattern point of keypoint 4 * wave + qt from that keypoint's staged
37-row patch (orbx_extract.hip, `sample`).  A gather over 32 lanes costs as many LDS
cycles as the most distinct dwords any one bank receives (same-dword reads broadcast).
The 16 points of a quarter are fixed pattern points turned by the keypoint's own angle,
so their dwords fall on banks like random draws whatever the patch layout: this script
measures the expected cycles per 32-lane gather over random angles and sub-dword offsets
for the shipped layout (10-dword rows, 370-dword patches) and for padded / swizzled
alternatives, against the 1-cycle conflict-free ideal.

usage: python tools/desc_bank_sim.py [--trials N] [--out profiles/r06_desc_bank_sim.json]
"""
import argparse
import json
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def pattern():
    txt = open(os.path.join(ROOT, "orbslam2commentedbyxcm_amd", "csrc", "orb_pattern.inc")).read()
    body = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return np.array([int(v) for v in re.findall(r"-?\d+", body)], dtype=np.int32).reshape(256, 4)


def gather_cycles(pat, rng, row_dw, patch_dw, trials, banks=32, group=32, swz=False):
    """Mean cycles per `group`-lane gather (dwords bank-mapped mod `banks`)."""
    tot = n = 0
    for _ in range(trials):
        th = rng.uniform(0, 2 * np.pi, 4)
        d = rng.integers(0, 4, 4)
        slot = rng.integers(0, 4)  # the wave's first patch
        a = np.cos(th).astype(np.float32)
        b = np.sin(th).astype(np.float32)
        for w in range(16):
            for side in (0, 1):
                dws = []
                for q in range(4):
                    pr = np.arange(16) + 16 * w
                    px = pat[pr, 2 * side].astype(np.float32)
                    py = pat[pr, 2 * side + 1].astype(np.float32)
                    rx = np.rint(px * a[q] - py * b[q]).astype(int)
                    ry = np.rint(px * b[q] + py * a[q]).astype(int)
                    row, col = 18 + ry, 18 + d[q] + rx
                    cdw = col // 4
                    if swz:
                        cdw = cdw ^ (row & 7)
                    dws.append((4 * slot + q) * patch_dw + row * row_dw + cdw)
                lanes = np.concatenate(dws)
                for h in range(64 // group):
                    u = np.unique(lanes[h * group:(h + 1) * group])
                    tot += np.bincount(u % banks, minlength=banks).max()
                    n += 1
    return tot / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=400)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_desc_bank_sim.json"))
    args = ap.parse_args()
    pat = pattern()
    rows = []
    for row_dw, patch_dw, swz in [(10, 370, False), (10, 372, False), (10, 378, False), (11, 407, False),
                                  (12, 444, False), (13, 481, False), (16, 592, True), (16, 600, True)]:
        rng = np.random.default_rng(7)
        c32 = gather_cycles(pat, rng, row_dw, patch_dw, args.trials)
        rng = np.random.default_rng(7)
        c64 = gather_cycles(pat, rng, row_dw, patch_dw, args.trials, banks=64, group=64)
        rows.append({"row_dwords": row_dw, "patch_dwords": patch_dw, "xor_swizzle": swz,
                     "cycles_per_gather_32lanes_32banks": round(c32, 3),
                     "conflict_share_32": round(1 - 1 / c32, 3),
                     "cycles_per_gather_64lanes_64banks": round(c64, 3)})
        print(rows[-1], flush=True)
    out = {"what": "k_describe rotated-pattern gathers: expected LDS cycles per gather (1 = conflict-free)",
           "trials": args.trials, "layouts": rows,
           "shipped": "row_dwords 10, patch_dwords 370 (40-byte rows, STAGE 2 LDS-DMA)"}
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print("->", args.out)


if __name__ == "__main__":
    main()
