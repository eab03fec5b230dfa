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


@pytest.mark.gpu
def test_cpp_threads_dropin_calls_like_oracle(tmp_path, orbx_built, oracle):
    # four C++ threads, each with its own extractor and matchers, calling extract + a12 + a11
    # at once (tests/cpp/dropin_mt.cpp) over three images: every frame's results equal the
    # oracle's
    import json
    import sys
    sys.path.insert(0, str(ROOT / "benchmarks"))
    import dropin_bench as D
    import match_scenes as S
    imgs = [synth.frame(11 + j, 640, 480) for j in range(3)]
    A, B = S.two_views(oracle, 0)
    mps = S.mappoints_from(A, 0)
    trk = S.local_track(A, B, mps, 0)
    nA, nB = len(A.keys), len(B.keys)
    queries = np.random.default_rng(0).permutation(nA).astype(np.int32)
    last_mp = np.arange(nA, dtype=np.int32)
    refs = [oracle.extract(im, oracle.params(1000, 1.2, 8, 20, 7))[:2] for im in imgs]
    c = np.full(nB, -1, np.int32)
    n12 = oracle.sbp_frame(B, c, A, last_mp, mps, 15.0, True, True)
    f = np.full(nB, -1, np.int32)
    n11 = oracle.sbp_local(B, f, queries, mps, trk, 3.0, 0.8)
    D.write_scene(tmp_path / "scene.bin", imgs, A, B, mps, trk, queries, last_mp, n12, c, n11, f, refs,
                  len(A.scale_factors))
    exe = D.build_driver(tmp_path / "dropin_mt")
    r = subprocess.run([str(exe), str(tmp_path / "scene.bin"), "4", "0.5"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["bit_exact"] and rec["frames"] > 4 and rec["images"] == 3
    assert rec["frames_checked"] == rec["frames"] + 2 * 4 and rec["frames_mismatched"] == 0

    # a wrong expectation for one image is caught on the frames that extract it
    bad = [refs[0], (refs[1][0], refs[1][1] ^ 1), refs[2]]
    D.write_scene(tmp_path / "bad.bin", imgs, A, B, mps, trk, queries, last_mp, n12, c, n11, f, bad,
                  len(A.scale_factors))
    r = subprocess.run([str(exe), str(tmp_path / "bad.bin"), "2", "0.2"], capture_output=True, text=True, timeout=120)
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert not rec["bit_exact"] and 0 < rec["frames_mismatched"] < rec["frames_checked"]


RGBD_SRC = ROOT / "tests" / "cpp" / "rgbd_cli.cpp"


def _build_rgbd(tmp_path, orbx_built):
    exe = tmp_path / "rgbd_cli"
    lib_dir = Path(orbx_built).parent
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT / 'include'}", str(RGBD_SRC), "-o", str(exe),
                    f"-L{lib_dir}", "-lorbx", f"-Wl,-rpath,{lib_dir}"], check=True)
    return exe


def test_cpp_rgbd_mirror_builds(tmp_path, orbx_built):
    assert _build_rgbd(tmp_path, orbx_built).exists()


@pytest.mark.gpu
def test_cpp_rgbd_frame_like_oracle(tmp_path, orbx_built, oracle):
    """orbx::ComputeStereoFromRGBD from C++ (the RGB-D Frame constructor's steps after
    ExtractORB, Frame.cc:217-230, on a TUM-like 16-bit depth image with holes): mvKeys,
    mvKeysUn, mvuRight and mvDepth equal the oracle's."""
    import tum_rgbd_scenes as S
    gray, depth, _ = S.sequence(4100, 1)
    (tmp_path / "g.raw").write_bytes(gray[0].tobytes())
    (tmp_path / "d.raw").write_bytes(np.ascontiguousarray(depth[0], np.uint16).tobytes())
    out = tmp_path / "out.bin"
    f32 = lambda x: "%.9g" % float(np.float32(x))  # noqa: E731 -- exact float32 through strtof
    cam = [f32(x) for x in (*S.K, *S.DIST)]
    exe = _build_rgbd(tmp_path, orbx_built)
    r = subprocess.run([str(exe), str(tmp_path / "g.raw"), str(tmp_path / "d.raw"), str(S.W), str(S.H), *cam,
                        f32(S.DEPTH_MAP_FACTOR), f32(S.BF), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    raw = out.read_bytes()
    n = int(np.frombuffer(raw[:4], np.int32)[0])
    o = 4
    kd = np.frombuffer(raw[o:o + 28 * n], np.uint8).reshape(n, 28)
    o += 28 * n
    ku = np.frombuffer(raw[o:o + 28 * n], np.uint8).reshape(n, 28)
    o += 28 * n
    ur = np.frombuffer(raw[o:o + 4 * n], np.float32)
    dp = np.frombuffer(raw[o + 4 * n:o + 8 * n], np.float32)
    p = oracle.params(*S.PARAMS)
    kr, _, _ = oracle.extract(gray[0], p)
    kur = oracle.undistort_keypoints(S.K, S.DIST, kr)
    urr, dpr = oracle.compute_stereo_from_rgbd(kr, kur, depth[0], S.BF, S.M_DEPTH_MAP_FACTOR)
    assert n == len(kr) and n > 3000
    assert np.array_equal(kd, kr.view(np.uint8).reshape(-1, 28))
    assert np.array_equal(ku, kur.view(np.uint8).reshape(-1, 28))
    assert np.array_equal(ur, urr) and np.array_equal(dp, dpr)
    assert (dp > 0).sum() > n // 2 and (dp == -1).any()
