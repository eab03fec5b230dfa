"""ORBextractor -- host-side mirror of ORB_SLAM2::ORBextractor over liborbx.so.

Same constructor arguments, call operator, getters and public ``mvImagePyramid`` as
include/ORBextractor.h:76-220; every call runs on the MI355X through the C ABI.
Keypoints come back as a structured array with cv::KeyPoint's fields
(x, y, size, angle, response, octave, class_id) in the reference order
(level-major, octree-list order within a level, ORBextractor.cc:1573-1628).
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np

from . import _lib as L


class ORBextractor:
    HARRIS_SCORE = 0
    FAST_SCORE = 1

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int,
                 device: int = 0):
        self._h = None
        prm = L.ExtractorParams(int(nfeatures), float(scaleFactor), int(nlevels), int(iniThFAST), int(minThFAST))
        h = C.c_void_p()
        L.check(L.lib().orbx_extractor_create(C.byref(prm), int(device), C.byref(h)))
        self._destroy = L.lib().orbx_extractor_destroy  # held: module globals may be gone at exit
        self._h = h
        L.track(self)
        self.nfeatures = int(nfeatures)
        self.scaleFactor = float(scaleFactor)
        self.nlevels = int(nlevels)
        self.iniThFAST = int(iniThFAST)
        self.minThFAST = int(minThFAST)
        self.device = int(device)
        self._last_batch = 0
        self._pyr_cache = None

    def close(self) -> None:
        """Release the extractor (orbx_extractor_destroy: waits for its stream); idempotent."""
        if getattr(self, "_h", None):
            self._destroy(self._h)
            self._h = None

    def __del__(self, _finalizing=sys.is_finalizing):
        if not _finalizing():  # at interpreter exit the atexit hook has closed it already
            self.close()

    # ---- getters (ORBextractor.h:119-159)
    def _levels(self):
        n = self.nlevels
        arrs = [np.zeros(n, dtype=np.float32) for _ in range(4)]
        ptrs = [a.ctypes.data_as(C.POINTER(C.c_float)) for a in arrs]
        L.check(L.lib().orbx_extractor_levels(self._h, None, *ptrs))
        return arrs

    def GetLevels(self) -> int:
        return self.nlevels

    def GetScaleFactor(self) -> float:
        return self.scaleFactor

    def GetScaleFactors(self) -> np.ndarray:
        return self._levels()[0]

    def GetInverseScaleFactors(self) -> np.ndarray:
        return self._levels()[1]

    def GetScaleSigmaSquares(self) -> np.ndarray:
        return self._levels()[2]

    def GetInverseScaleSigmaSquares(self) -> np.ndarray:
        return self._levels()[3]

    def features_per_level(self) -> np.ndarray:
        out = np.zeros(self.nlevels, dtype=np.int32)
        L.check(L.lib().orbx_extractor_features_per_level(self._h, out.ctypes.data_as(C.POINTER(C.c_int))))
        return out

    def max_keypoints(self, width: int, height: int) -> int:
        n = C.c_int()
        L.check(L.lib().orbx_extractor_max_keypoints(self._h, width, height, C.byref(n)))
        return n.value

    # ---- operator() (ORBextractor.cc:1513-1629)
    def __call__(self, image: np.ndarray, mask=None):
        """Returns (keypoints, descriptors); an empty image returns (None, None) untouched."""
        img = np.asarray(image)
        if img.size == 0:
            return None, None
        if img.dtype != np.uint8 or img.ndim != 2:
            raise TypeError("ORBextractor expects a single-channel uint8 image (CV_8UC1)")
        kps, desc, n = self.extract_batch(img[None])
        return kps[0][: n[0]].copy(), desc[0][: n[0]].copy()

    def extract_batch(self, images: np.ndarray, cap: int | None = None):
        """B host frames (B, H, W) uint8 -> (kps[B, cap], desc[B, cap, 32], n[B])."""
        imgs = np.asarray(images)
        if imgs.dtype != np.uint8 or imgs.ndim != 3:
            raise TypeError("expected (B, H, W) uint8 frames")
        B, H, W = imgs.shape
        cap = cap or self.max_keypoints(W, H)
        kps = np.zeros((B, cap), dtype=L.KEYPOINT_DTYPE)
        desc = np.zeros((B, cap, 32), dtype=np.uint8)
        n = np.zeros(B, dtype=np.int32)
        rows = [np.ascontiguousarray(imgs[b]) for b in range(B)]
        ptrs = (C.POINTER(C.c_uint8) * B)(*[L.u8ptr(r) for r in rows])
        rc = L.lib().orbx_extract_batch(self._h, B, ptrs, W, H, W, kps.ctypes.data, L.u8ptr(desc), cap,
                                        n.ctypes.data_as(C.POINTER(C.c_int)))
        L.check(rc)
        self._last_batch = B
        self._pyr_cache = None
        return kps, desc, n

    def extract_batch_device(self, frames, kps_out, desc_out, n_out, stream=None):
        """Device-resident path.  frames: CUDA/HIP uint8 tensor (B, H, W) (any object with
        data_ptr()/shape/stride()); outputs: preallocated device tensors
        kps_out (B, cap, 7) 4-byte words, desc_out (B, cap, 32) uint8, n_out (B,) int32.
        Enqueued on `stream` (a torch.cuda.Stream or raw handle) or the extractor's own."""
        B, H, W = frames.shape
        cap = desc_out.shape[1]
        s = None
        if stream is not None:
            s = C.c_void_p(getattr(stream, "cuda_stream", stream))
        rc = L.lib().orbx_extract_batch_device(self._h, B, C.c_void_p(frames.data_ptr()), frames.stride(0), W, H,
                                               frames.stride(1), C.c_void_p(kps_out.data_ptr()),
                                               C.c_void_p(desc_out.data_ptr()), cap, C.c_void_p(n_out.data_ptr()), s)
        L.check(rc)
        self._last_batch = B
        self._pyr_cache = None

    def stream_handle(self) -> int:
        return L.lib().orbx_extractor_stream(self._h) or 0

    def last_call_us(self) -> float:
        """orbx_extractor_last_call_us: in-library wall time of the newest host-API call."""
        return L.lib().orbx_extractor_last_call_us(self._h)

    def set_stage_event(self, stage: int) -> int:
        """orbx_extractor_set_stage_event: every extraction records the returned hipEvent_t
        right after stage `stage` (1 pyramid, 2 blur + FAST strength, 3 FAST cells,
        4 octree; 0 = off).  Wait on it with stream_wait_event."""
        ev = C.c_void_p()
        L.check(L.lib().orbx_extractor_set_stage_event(self._h, int(stage), C.byref(ev)))
        return ev.value or 0

    # ---- kernel status of the last extraction (orbx_extractor_status)
    STATUS_NODE_OVERFLOW = 1
    STATUS_ITERATIONS = 2

    def status(self, batch: int | None = None) -> np.ndarray:
        """Per-frame octree status words of the last extraction (0 = complete; see
        include/orbx.h).  Synchronises with that extraction's stream."""
        b = self._last_batch if batch is None else int(batch)
        flags = np.zeros(max(b, 1), dtype=np.int32)
        anyf = C.c_int()
        L.check(L.lib().orbx_extractor_status(self._h, b, flags.ctypes.data_as(C.POINTER(C.c_int)), C.byref(anyf)))
        return flags[:b]

    def status_device_ptr(self) -> int:
        """Device address of the per-frame status words (int32[last batch]), no sync."""
        p = C.c_void_p()
        L.check(L.lib().orbx_extractor_status_device(self._h, C.byref(p)))
        return p.value or 0

    def set_node_capacity(self, cap: int) -> None:
        """Test hook: cap the octree node capacity per level (0 = the guaranteed bound)."""
        L.check(L.lib().orbx_extractor_set_node_capacity(self._h, int(cap)))

    def set_level0_in_place(self, enable: bool = True) -> None:
        """orbx_extractor_set_level0_in_place: level 0 read from the caller's device frames
        when their rows are 64-byte aligned (device_frames); the frames must stay unchanged
        while the pyramid is used (the stereo matchers read level 0 from them)."""
        L.check(L.lib().orbx_extractor_set_level0_in_place(self._h, 1 if enable else 0))

    STAGES = ("pyramid", "score_blur", "fast_cells", "octree", "describe")

    def set_timing(self, enable: bool = True, stage: str | None = None) -> None:
        """HIP-event stage timing of the following calls (all stage boundaries, or only
        `stage`'s two when given: fewer events in a timed loop)."""
        v = 0 if not enable else (1 if stage is None else 2 + self.STAGES.index(stage))
        L.check(L.lib().orbx_extractor_set_timing(self._h, v))

    def stage_times(self) -> dict:
        names = (C.c_char_p * 16)()
        ms = (C.c_float * 16)()
        n = C.c_int()
        L.check(L.lib().orbx_extractor_stage_times(self._h, 16, names, ms, C.byref(n)))
        return {names[i].decode(): float(ms[i]) for i in range(n.value)}

    # ---- mvImagePyramid (ORBextractor.h:162)
    def pyramid_level(self, level: int, frame: int = 0) -> np.ndarray:
        w, h = C.c_int(), C.c_int()
        L.check(L.lib().orbx_pyramid_level(self._h, frame, level, None, 0, C.byref(w), C.byref(h)))
        out = np.zeros((h.value, w.value), dtype=np.uint8)
        L.check(L.lib().orbx_pyramid_level(self._h, frame, level, L.u8ptr(out), w.value, None, None))
        return out

    @property
    def mvImagePyramid(self):
        if self._last_batch == 0:
            return []
        if self._pyr_cache is None:
            self._pyr_cache = [self.pyramid_level(lv) for lv in range(self.nlevels)]
        return self._pyr_cache


def device_frames(frames, device, align: int = 64):
    """(B, H, W) u8 frames copied into HBM with rows `align` bytes apart (a pitched layout,
    as hipMallocPitch gives): a (B, H, W) view whose row stride is a multiple of 64, so an
    extractor with set_level0_in_place reads level 0 from it in place whatever W is
    (KITTI's 1241-byte and EuRoC's 752-byte rows included)."""
    import torch

    a = np.ascontiguousarray(frames, dtype=np.uint8)
    B, H, W = a.shape
    P = (W + align - 1) // align * align
    buf = torch.zeros((B, H, P), dtype=torch.uint8, device=device)
    view = buf[:, :, :W]
    view.copy_(torch.from_numpy(a))
    return view


def stream_wait_event(stream: int, event: int) -> None:
    """hipStreamWaitEvent(stream, event) through the library (orbx_stream_wait_event)."""
    L.check(L.lib().orbx_stream_wait_event(C.c_void_p(stream), C.c_void_p(event)))


def stream_create(device: int, cu_stride: int = 1, priority: int = 0) -> int:
    """orbx_stream_create: a non-blocking hipStream_t, on CUs 0, k, 2k, ... only when
    k = cu_stride > 1, else of HIP priority `priority`; release it with stream_destroy."""
    s = C.c_void_p()
    L.check(L.lib().orbx_stream_create(int(device), int(cu_stride), int(priority), C.byref(s)))
    return s.value or 0


def stream_destroy(stream: int) -> None:
    L.check(L.lib().orbx_stream_destroy(C.c_void_p(stream)))


def release_owned(obj, streams, owners, own_streams) -> None:
    """A pipeline's close(): wait for its streams (torch stream objects, None skipped), close
    the handle owners it holds (extractors, matchers, vocabularies: each waits for its own
    stream), then destroy the streams it created (the attributes named in own_streams,
    raw hipStream_t values, set to None).  Idempotent."""
    if getattr(obj, "_released", False):
        return
    obj._released = True
    for s in streams:
        if s is not None:
            s.synchronize()
    for o in owners:
        if o is not None:
            o.close()
    for a in own_streams:
        h = getattr(obj, a, None)
        if h:
            setattr(obj, a, None)
            stream_destroy(h)
