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
    # a debug build of the planner (-DORBX_DEBUG=1): it reads ORBX_PZ_SEG from the environment
    subprocess.run(["g++", "-O1", "-std=c++17", "-DORBX_DEBUG=1", f"-I{CSRC}", f"-I{ROOT / 'include'}",
                    str(ROOT / "tests" / "cpp" / "pyramid_plan.cpp"), str(CSRC / "orbx_geometry.cpp"),
                    str(CSRC / "orbx_runtime.cpp"), "-o", str(exe)], check=True)
    return exe


def _plan(exe, W, H, nf, L, env=None):
    import os
    out = subprocess.run([str(exe), str(W), str(H), str(nf), str(L)], capture_output=True, text=True, check=True,
                         env=dict(os.environ, **(env or {})))
    lines = out.stdout.split("\n")
    L_, nseg = map(int, lines[0].split())
    segs = [tuple(map(int, lines[1 + s].split())) for s in range(nseg)]
    i, levels = 1 + nseg, []
    for l in range(L_):
        w, h = map(int, lines[i].split())
        i += 1
        xt = yt = None
        if l > 0:
            xt = np.array(lines[i].split(), dtype=np.int64).reshape(-1, 2)
            yt = np.array(lines[i + 1].split(), dtype=np.int64).reshape(-1, 2)
            i += 2
        levels.append((w, h, xt, yt))
    out_segs = []
    for (l0, nl, nx, ny, lds_a, lds_b) in segs:
        n = nx * ny * nl
        rects = np.array([list(map(int, lines[i + k].split())) for k in range(n)]).reshape(nx * ny, nl, 8)
        i += n
        out_segs.append((l0, nl, rects, lds_a, lds_b))
    return levels, out_segs


@pytest.mark.parametrize("W,H,nf,L,env", [(640, 480, 1000, 8, None), (1241, 376, 2000, 8, None),
                                          (752, 480, 1200, 8, None), (640, 480, 5000, 12, None),
                                          (640, 480, 5000, 12, {"ORBX_PZ_SEG": "0"}),
                                          (640, 480, 5000, 12, {"ORBX_PZ_SEG": "4"}),
                                          (1241, 376, 2000, 10, {"ORBX_PZ_SEG": "3"}),
                                          (320, 240, 500, 4, None), (1023, 767, 1000, 8, None)])
def test_pyramid_tiling_invariants(plan_exe, W, H, nf, L, env):
    """Per segment (orbx_geometry.h): needed rectangles hold the owned pixels and the next
    level's source footprint; over all segments every pixel of every level is owned once
    (a later segment's input level is owned by the segment before it)."""
    levels, segs = _plan(plan_exe, W, H, nf, L, env)
    seg_levels = env and int(env["ORBX_PZ_SEG"]) or 8
    if seg_levels < 2 or seg_levels > L:
        seg_levels = L
    assert segs[0][0] == 0 and segs[-1][0] + segs[-1][1] == L
    for (a0, an, *_), (b0, _bn, *_) in zip(segs, segs[1:]):
        assert b0 == a0 + an - 1 and an == seg_levels  # each later segment starts at the previous one's last level
    cover = [np.zeros((h, w), np.int32) for (w, h, _, _) in levels]
    for l0, nl, rects, lds_a, lds_b in segs:
        assert lds_a + lds_b <= 150 * 1024
        for k in range(nl):
            l = l0 + k
            w, h = levels[l][:2]
            for t in range(rects.shape[0]):
                x0, y0, x1, y1, ox0, oy0, ox1, oy1 = rects[t, k]
                cover[l][oy0:oy1, ox0:ox1] += 1
                if k == 0 and l0 > 0:
                    assert ox1 <= ox0 or oy1 <= oy0  # the input level is not owned again
                if ox1 > ox0 and oy1 > oy0:  # needed contains owned
                    assert x0 <= ox0 and x1 >= ox1 and y0 <= oy0 and y1 >= oy1
                assert 0 <= x0 and x1 <= w and 0 <= y0 and y1 <= h
                if k + 1 < nl:  # needed contains the source footprint of the level above
                    u0, v0, u1, v1 = rects[t, k + 1][:4]
                    if u1 > u0 and v1 > v0:
                        uxt, uyt = levels[l + 1][2], levels[l + 1][3]
                        assert x0 <= uxt[u0:u1, 0].min() and uxt[u0:u1, 1].max() < x1
                        assert y0 <= uyt[v0:v1, 0].min() and uyt[v0:v1, 1].max() < y1
    for l in range(L):
        assert (cover[l] == 1).all(), f"level {l}: owned rectangles do not partition the level"
