"""orbx_sincos.h (the steered-BRIEF rotation, hazard H3) against glibc.

k_describe computes (float)cos((double)r) / (float)sin((double)r) for r = fastAtan2 * pi/180
with a one-step reduction + fdlibm kernels instead of the library's double cos/sin.  The
header's claim -- equal to glibc after rounding to float for every float in [0, 6.2832] --
was checked exhaustively once (1,086,918,650 inputs); this keeps every 61st float of that
range plus the quadrant boundaries, compiled from the same header with g++ -ffp-contract=off.
"""
import subprocess
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

SRC = textwrap.dedent(r"""
    #include "orbx_sincos.h"
    #include <cmath>
    #include <cstdint>
    #include <cstdio>
    #include <cstring>
    static long bad = 0, n = 0;
    static void check(float r) {
        double c, s;
        orbx::sincos_0_2pi((double)r, c, s);
        if ((float)c != (float)std::cos((double)r) || (float)s != (float)std::sin((double)r)) bad++;
        n++;
    }
    int main() {
        float lo = 0.f, hi = 6.2832f;
        uint32_t a, b;
        std::memcpy(&a, &lo, 4);
        std::memcpy(&b, &hi, 4);
        for (uint32_t u = a; u <= b; u += 61) { float r; std::memcpy(&r, &u, 4); check(r); }
        for (int q = 0; q <= 4; q++) {  // around k * pi/4
            float m = (float)(q * 0.78539816339744830962);
            for (int d = -64; d <= 64; d++) check(std::nextafter(m, d < 0 ? 0.f : 10.f) + 0.f * d);
            float x = m;
            for (int d = 0; d < 64; d++) { check(x); x = std::nextafter(x, 10.f); }
            x = m;
            for (int d = 0; d < 64 && x > 0; d++) { check(x); x = std::nextafter(x, 0.f); }
        }
        std::printf("%ld %ld\n", n, bad);
        return 0;
    }
""")


def test_sincos_matches_glibc(tmp_path):
    src = tmp_path / "sc.cpp"
    src.write_text(SRC)
    exe = tmp_path / "sc"
    r = subprocess.run(["g++", "-O2", "-ffp-contract=off", f"-I{ROOT / 'orbslam2commentedbyxcm_amd' / 'csrc'}",
                        str(src), "-o", str(exe)], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(r.stderr)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120).stdout.split()
    n, bad = int(out[0]), int(out[1])
    assert n > 17_000_000
    assert bad == 0
