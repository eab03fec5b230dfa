"""k_pyramid's tiling (make_plan, orbx_geometry.cpp) on the host: for every level the
tiles' owned rectangles partition the level exactly, every needed rectangle contains
the tile's owned pixels and the resize source footprint of its needed rectangle one
level up, and the LDS buffers fit.  These are the invariants that make the one-launch
cascade produce every pyramid pixel once and read only staged pixels."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "orbslam2commentedbyxcm_amd" / "csrc"


@pytest.fixture(scope="module")
def plan_exe(tmp_path_factory):
    exe = tmp_path_factory.mktemp("pz") / "pyramid_plan"
    subprocess.run(["g++", "-O1", "-std=c++17", f"-I{CSRC}", f"-I{ROOT / 'include'}",
                    str(ROOT / "tests" / "cpp" / "pyramid_plan.cpp"), str(CSRC / "orbx_geometry.cpp"), "-o", str(exe)],
                   check=True)
    return exe


def _plan(exe, W, H, nf, L):
    out = subprocess.run([str(exe), str(W), str(H), str(nf), str(L)], capture_output=True, text=True, check=True)
    lines = out.stdout.split("\n")
    L_, nx, ny, lds_a, lds_b = map(int, lines[0].split())
    i, levels = 1, []
    for l in range(L_):
        w, h = map(int, lines[i].split())
        i += 1
        xt = yt = None
        if l > 0:
            xt = np.array(lines[i].split(), dtype=np.int64).reshape(-1, 2)
            yt = np.array(lines[i + 1].split(), dtype=np.int64).reshape(-1, 2)
            i += 2
        levels.append((w, h, xt, yt))
    rects = np.array([list(map(int, lines[i + k].split())) for k in range(nx * ny * L_)]).reshape(nx * ny, L_, 8)
    return levels, rects, lds_a, lds_b


@pytest.mark.parametrize("W,H,nf,L", [(640, 480, 1000, 8), (1241, 376, 2000, 8), (752, 480, 1200, 8),
                                      (640, 480, 5000, 12), (320, 240, 500, 4), (1023, 767, 1000, 8)])
def test_pyramid_tiling_invariants(plan_exe, W, H, nf, L):
    levels, rects, lds_a, lds_b = _plan(plan_exe, W, H, nf, L)
    assert lds_a + lds_b <= 150 * 1024
    for l, (w, h, xt, yt) in enumerate(levels):
        cover = np.zeros((h, w), np.int32)
        for t in range(rects.shape[0]):
            x0, y0, x1, y1, ox0, oy0, ox1, oy1 = rects[t, l]
            cover[oy0:oy1, ox0:ox1] += 1
            if ox1 > ox0 and oy1 > oy0:  # needed contains owned
                assert x0 <= ox0 and x1 >= ox1 and y0 <= oy0 and y1 >= oy1
            assert 0 <= x0 and x1 <= w and 0 <= y0 and y1 <= h
            if l + 1 < len(levels):  # needed contains the source footprint of the level above
                u0, v0, u1, v1 = rects[t, l + 1][:4]
                if u1 > u0 and v1 > v0:
                    uxt, uyt = levels[l + 1][2], levels[l + 1][3]
                    assert x0 <= uxt[u0:u1, 0].min() and uxt[u0:u1, 1].max() < x1
                    assert y0 <= uyt[v0:v1, 0].min() and uyt[v0:v1, 1].max() < y1
        assert (cover == 1).all(), f"level {l}: owned rectangles do not partition the level"
