"""k_octree phase times of the single-frame host call (ORBX_OCT_STAMPS=1: the library
prints per-level gather / full passes / final phase / output times to stderr) at C1, C3 and
C5 frame sizes, plus the in-library time of the call with the stamps off.
usage: python tools/oct_stamps.py   (GPU)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {"C1": (640, 480, 1000, 8), "C3": (1241, 376, 2000, 8), "C5": (640, 480, 5000, 12)}


def child(case: str, stamps: bool) -> None:
    sys.path.insert(0, ROOT)
    import numpy as np
    from orbslam2commentedbyxcm_amd import synth
    from orbslam2commentedbyxcm_amd.extractor import ORBextractor
    W, H, nf, nl = CASES[case]
    img = synth.frame(7, W, H)
    ex = ORBextractor(nf, 1.2, nl, 20, 7)
    for _ in range(3):
        ex(img)
    if stamps:
        return
    t = []
    for _ in range(30):
        ex(img)
        t.append(ex.last_call_us())
    print(f"{case} in-library median {float(np.median(t)):.1f} us", flush=True)


def main():
    if len(sys.argv) > 2:
        child(sys.argv[1], sys.argv[2] == "1")
        return
    for case in CASES:
        for stamps in (False, True):
            env = dict(os.environ)
            if stamps:
                env["ORBX_OCT_STAMPS"] = "1"
            r = subprocess.run([sys.executable, __file__, case, "1" if stamps else "0"], env=env,
                               capture_output=True, text=True, timeout=300)
            if r.returncode:
                print(r.stderr[-2000:])
                sys.exit(r.returncode)
            out = r.stdout.strip()
            if stamps:
                lines = [x for x in r.stderr.splitlines() if x.startswith("[orbx oct]")]
                L = CASES[case][3]
                out = f"{case} octree stamps (last call):\n" + "\n".join(lines[-L:])
            print(out, flush=True)


if __name__ == "__main__":
    main()
