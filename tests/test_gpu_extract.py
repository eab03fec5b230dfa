"""GPU parity: liborbx.so (HIP, gfx950) vs the CPU oracle, bit-exact.

Every keypoint field (x, y, size, angle, response, octave, class_id), the keypoint
order and all 256 descriptor bits must match the oracle's restatement of
ORBextractor::operator() (ORBextractor.cc:1513-1629) on the same seeded frames.
"""
import numpy as np
import pytest

from orbslam2commentedbyxcm_amd import ORBextractor, synth

pytestmark = pytest.mark.gpu


@pytest.fixture
def switch():
    """orbx_debug_set for one test: every switch back to its default afterwards."""
    from orbslam2commentedbyxcm_amd import _lib as L
    yield L.debug_set
    L.debug_set(None)


def _cmp(kp_gpu, desc_gpu, kp_ref, desc_ref):
    assert len(kp_gpu) == len(kp_ref), (len(kp_gpu), len(kp_ref))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        a, b = kp_gpu[f], kp_ref[f]
        bad = np.nonzero(a != b)[0]
        assert bad.size == 0, f"field {f}: {bad.size} mismatches, first {bad[:5]} gpu={a[bad[:5]]} ref={b[bad[:5]]}"
    bad = np.nonzero((desc_gpu != desc_ref).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} descriptor mismatches, first {bad[:5]}"


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_extract_640x480_matches_oracle(oracle, orbx_built, seed):
    img = synth.frame(seed)
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    kps, desc = ex(img)
    kr, dr, _ = oracle.extract(img, oracle.params(1000, 1.2, 8, 20, 7))
    _cmp(kps, desc, kr, dr)


def test_pyramid_matches_oracle(oracle, orbx_built):
    img = synth.frame(11)
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    ex(img)
    ref = oracle.pyramid(img, oracle.params(1000, 1.2, 8, 20, 7))
    for lv, (a, b) in enumerate(zip(ex.mvImagePyramid, ref)):
        assert a.shape == b.shape
        assert np.array_equal(a, b), f"level {lv}: {(a != b).sum()} pixels differ"


@pytest.mark.parametrize("sf,nl,byte", [(1.2, 8, True), (1.5, 6, False), (2.0, 3, False), (2.5, 3, False)])
def test_pyramid_forms_match_oracle(oracle, orbx_built, switch, sf, nl, byte):
    """Both k_pyramid forms: the dword-window one (any 4 columns' resize taps within 8
    source bytes, scale factors up to 2) and the byte-read one (switch pz_byte = 1, or a
    larger scale factor such as 2.5)."""
    if byte:
        switch("pz_byte", 1)
    img = synth.frame(12)
    ex = ORBextractor(1000, sf, nl, 20, 7)
    kps, desc = ex(img)
    p = oracle.params(1000, sf, nl, 20, 7)
    ref = oracle.pyramid(img, p)
    for lv, (a, b) in enumerate(zip(ex.mvImagePyramid, ref)):
        assert a.shape == b.shape
        assert np.array_equal(a, b), f"level {lv}: {(a != b).sum()} pixels differ"
    kr, dr, _ = oracle.extract(img, p)
    _cmp(kps, desc, kr, dr)


def test_batch_matches_single(oracle, orbx_built):
    imgs = synth.frames(6, first_seed=100)
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    kps, desc, n = ex.extract_batch(imgs)
    p = oracle.params(1000, 1.2, 8, 20, 7)
    for b in range(len(imgs)):
        kr, dr, _ = oracle.extract(imgs[b], p)
        _cmp(kps[b][: n[b]], desc[b][: n[b]], kr, dr)


@pytest.mark.parametrize("cfg", [(1241, 376, 2000, 1.2, 8), (752, 480, 1200, 1.2, 8), (640, 480, 5000, 1.2, 12)])
def test_other_configs_match_oracle(oracle, orbx_built, cfg):
    W, H, nf, sf, nl = cfg
    img = synth.frame(7, W, H)
    ex = ORBextractor(nf, sf, nl, 20, 7)
    kps, desc = ex(img)
    kr, dr, _ = oracle.extract(img, oracle.params(nf, sf, nl, 20, 7))
    _cmp(kps, desc, kr, dr)


@pytest.mark.parametrize("prm,size,B", [((1000, 1.2, 8, 20, 7), (640, 480), 8), ((5000, 1.2, 12, 20, 7), (640, 480), 8),
                                        ((2000, 1.2, 8, 20, 7), (1241, 376), 4)])
def test_describe_tiles_form_matches_oracle(oracle, orbx_built, switch, prm, size, B):
    """The tile-major describe (switch desc_tiles = 1: k_octree bins the kept slots by level
    tile, k_describe_tiles stages each tile once) gives the same keypoints and
    descriptors; the setting is read when an extractor plans a frame size."""
    import torch

    from oracle import checks
    switch("desc_tiles", 1)
    W, H = size
    frames = synth.frames(B, W, H, first_seed=40)
    ex = ORBextractor(*prm)
    cap = ex.max_keypoints(W, H)
    dev = torch.device("cuda", 0)
    kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.empty((B,), dtype=torch.int32, device=dev)
    ex.extract_batch_device(torch.from_numpy(frames).to(dev), kps, desc, n)
    torch.cuda.synchronize()
    assert not ex.status().any()
    from orbslam2commentedbyxcm_amd import _lib as L
    k = kps.cpu().numpy().view(np.uint8).reshape(B, cap, 28).view(L.KEYPOINT_DTYPE).reshape(B, cap)
    ref = checks.extract_all(frames, params=prm)
    assert checks.compare_extraction(ref, k, desc.cpu().numpy(), n.cpu().numpy()) == []


def test_level0_in_place(oracle, orbx_built):
    """orbx_extractor_set_level0_in_place: the device batch reads level 0 from the caller's
    frames (bit-exact output; mvImagePyramid level 0 is then the caller's frame, the other
    levels the extractor's own), and ComputeStereoMatches over extractors that read level 0
    in place (its octave-0 SAD windows then read the caller's frames) gives the results of
    extractors that copied it."""
    import torch

    from oracle import checks
    from orbslam2commentedbyxcm_amd.matcher import ORBmatcher
    B = 4
    frames = synth.frames(B, 640, 480, first_seed=60)
    ex = ORBextractor(1000, 1.2, 8, 20, 7)
    ex.set_level0_in_place(True)
    cap = ex.max_keypoints(640, 480)
    dev = torch.device("cuda", 0)
    d_frames = torch.from_numpy(frames).to(dev)
    kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.empty((B,), dtype=torch.int32, device=dev)
    ex.extract_batch_device(d_frames, kps, desc, n)
    torch.cuda.synchronize()
    from orbslam2commentedbyxcm_amd import _lib as L
    k = kps.cpu().numpy().view(np.uint8).reshape(B, cap, 28).view(L.KEYPOINT_DTYPE).reshape(B, cap)
    ref = checks.extract_all(frames)
    assert checks.compare_extraction(ref, k, desc.cpu().numpy(), n.cpu().numpy()) == []
    pyr = oracle.pyramid(frames[0], oracle.params(1000, 1.2, 8, 20, 7))
    for lv in (0, 3):
        assert np.array_equal(ex.pyramid_level(lv, frame=0), pyr[lv])
    # a stereo pair: the right views are the left shifted 9 px (disparity 9 everywhere)
    right = np.ascontiguousarray(np.roll(frames, -9, axis=2))
    d_right = torch.from_numpy(right).to(dev)
    out = []
    for in_place in (True, False):
        exl, exr = ORBextractor(1000, 1.2, 8, 20, 7), ORBextractor(1000, 1.2, 8, 20, 7)
        exl.set_level0_in_place(in_place)
        exr.set_level0_in_place(in_place)
        t = [torch.empty((B, cap, 7), dtype=torch.int32, device=dev), torch.empty((B, cap, 32), dtype=torch.uint8,
             device=dev), torch.empty((B,), dtype=torch.int32, device=dev)]
        r = [torch.empty_like(x) for x in t]
        exl.extract_batch_device(d_frames, *t)
        exr.extract_batch_device(d_right, *r)
        torch.cuda.synchronize()
        import ctypes as C
        from orbslam2commentedbyxcm_amd import _lib as L
        ptr = C.c_void_p()
        L.check(L.lib().orbx_pyramid_level_device(exl._h, 1, 0, C.byref(ptr), None, None, None))
        assert (ptr.value == d_frames.data_ptr() + d_frames.stride(0)) == in_place  # frame 1's level 0
        ur = torch.full((B, cap), -2.0, dtype=torch.float32, device=dev)
        dp = torch.full((B, cap), -2.0, dtype=torch.float32, device=dev)
        ORBmatcher(0.6, True).ComputeStereoMatchesBatchDevice(exl, exr, *t, *r, 100.0, 500.0, ur, dp)
        torch.cuda.synchronize()
        out.append((ur.cpu().numpy(), dp.cpu().numpy(), t[2].cpu().numpy()))
    (u1, d1, n1), (u2, d2, n2) = out
    assert np.array_equal(n1, n2)
    for b in range(B):
        assert np.array_equal(u1[b, :n1[b]], u2[b, :n1[b]]) and np.array_equal(d1[b, :n1[b]], d2[b, :n1[b]]), b
    assert (u1[0, :n1[0]] >= 0).sum() > 100


@pytest.mark.parametrize("dma", [0, 1])
@pytest.mark.parametrize("W,H,prm", [(640, 480, (1000, 1.2, 8, 20, 7)), (1241, 376, (2000, 1.2, 8, 20, 7))])
def test_host_call_paths_match_oracle(oracle, orbx_built, switch, dma, W, H, prm):
    """The single / batched host calls through mapped memory (the default: the pyramid
    reads the frames from pinned host memory, the describe kernel writes into it) and
    through DMA copies (switch extract_dma = 1), at a packed 1241-px width too."""
    switch("extract_dma", dma)
    imgs = synth.frames(3, W, H, first_seed=70)
    ex = ORBextractor(*prm)
    p = oracle.params(*prm)
    kps, desc = ex(imgs[0])
    kr, dr, _ = oracle.extract(imgs[0], p)
    _cmp(kps, desc, kr, dr)
    kb, db, nb = ex.extract_batch(imgs)
    for b in range(len(imgs)):
        kr, dr, _ = oracle.extract(imgs[b], p)
        _cmp(kb[b][: nb[b]], db[b][: nb[b]], kr, dr)

