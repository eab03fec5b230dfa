"""Minimal extraction loop to run under rocprofv3 (kernel trace / PMC passes).

    rocprofv3 --kernel-trace --stats -d gpurun_out/p -- python tools/prof_driver.py --steps 5
    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/p -- python tools/prof_driver.py --steps 3
"""
import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--nlevels", type=int, default=8)
    args = ap.parse_args()
    from orbslam2commentedbyxcm_amd import synth
    frames = synth.frames(args.batch, args.width, args.height, workers=min(16, os.cpu_count() or 1))
    import torch
    from orbslam2commentedbyxcm_amd import ORBextractor
    dev = torch.device("cuda", 0)
    ex = ORBextractor(args.nfeatures, 1.2, args.nlevels, 20, 7)
    cap = ex.max_keypoints(args.width, args.height)
    d_frames = torch.from_numpy(frames).to(dev)
    d_kps = torch.empty((args.batch, cap, 7), dtype=torch.int32, device=dev)
    d_desc = torch.empty((args.batch, cap, 32), dtype=torch.uint8, device=dev)
    d_n = torch.empty((args.batch,), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    for _ in range(args.steps):
        ex.extract_batch_device(d_frames, d_kps, d_desc, d_n)
    torch.cuda.synchronize()
    print("mean keypoints", float(d_n.float().mean()))


if __name__ == "__main__":
    main()
