"""The C++ host mirror (include/orbx.hpp) builds with g++ against liborbx.so and,
on the GPU, extracts exactly what the oracle extracts."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from orbslam2commentedbyxcm_amd import synth

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "cpp" / "extract_cli.cpp"


def _build(tmp_path, orbx_built):
    exe = tmp_path / "extract_cli"
    lib_dir = Path(orbx_built).parent
    cmd = ["g++", "-O2", "-std=c++17", f"-I{ROOT / 'include'}", str(SRC), "-o", str(exe),
           f"-L{lib_dir}", "-lorbx", f"-Wl,-rpath,{lib_dir}"]
    subprocess.run(cmd, check=True)
    return exe


def test_cpp_mirror_builds(tmp_path, orbx_built):
    assert _build(tmp_path, orbx_built).exists()


@pytest.mark.gpu
def test_cpp_mirror_extracts_like_oracle(tmp_path, orbx_built, oracle):
    exe = _build(tmp_path, orbx_built)
    img = synth.frame(42)
    (tmp_path / "img.raw").write_bytes(img.tobytes())
    out = tmp_path / "out.bin"
    r = subprocess.run([str(exe), str(tmp_path / "img.raw"), "640", "480", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    raw = out.read_bytes()
    n = int(np.frombuffer(raw[:4], np.int32)[0])
    kps = np.frombuffer(raw[4:4 + 28 * n], np.uint8).reshape(n, 28)
    desc = np.frombuffer(raw[4 + 28 * n:], np.uint8).reshape(n, 32)
    kr, dr, _ = oracle.extract(img)
    assert np.array_equal(kps, kr.view(np.uint8).reshape(-1, 28))
    assert np.array_equal(desc, dr)
