"""Does recording the per-stage HIP events inside the timed loop cost throughput?  The
bench's configs[1] pipeline timed K steps after W warmup with stage events on and off,
interleaved.  usage: python tools/timing_ab.py [rounds] [steps] [warmup]"""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")


def main():
    rounds, steps, warm = (int(a) for a in (sys.argv[1:] + ["3", "20", "5"][len(sys.argv) - 1:])[:3])
    import torch

    import bench
    from orbslam2commentedbyxcm_amd import synth
    from orbslam2commentedbyxcm_amd.pipeline import SequencePipeline, sequence_poses
    frames, off = synth.sequence(1000, 256)
    T = sequence_poses(off, bench.FX, bench.FY, bench.DEPTH)
    dev = torch.device("cuda", 0)
    d_f = torch.from_numpy(frames).to(dev)
    d_T = torch.from_numpy(T).to(dev)
    for r in range(rounds):
        for timing in (True, False):
            pl = SequencePipeline(256, 640, 480, lanes=2, pipelined=True, params=(1000, 1.2, 8, 20, 7))
            pl.run(d_f, d_T, warm)
            torch.cuda.synchronize()
            pl.set_timing(timing)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pl.run(d_f, d_T, steps)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            print(f"round {r} events {'on ' if timing else 'off'}: {256 * steps / el:10.1f} frames/s "
                  f"({el / steps * 1e3:.4f} ms/step)", flush=True)
            pl.set_timing(False)
            pl.close()
            del pl


if __name__ == "__main__":
    main()
