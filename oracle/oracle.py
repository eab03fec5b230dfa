"""ctypes binding of the CPU parity oracle (liborbx_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the orbslam2commentedbyxcm_amd product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liborbx_oracle.so"

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
MAX_LEVELS = 32


class Params(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("nlevels", C.c_int), ("ini_th_fast", C.c_int),
                ("min_th_fast", C.c_int), ("scale_factor", C.c_double),
                ("scale", C.c_float * MAX_LEVELS), ("inv_scale", C.c_float * MAX_LEVELS),
                ("sigma2", C.c_float * MAX_LEVELS), ("inv_sigma2", C.c_float * MAX_LEVELS),
                ("features_per_level", C.c_int * MAX_LEVELS), ("umax", C.c_int * 16)]


def build() -> Path:
    """Compile the oracle with its Makefile (gcc); returns the .so path."""
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
        u8p = C.POINTER(C.c_uint8)
        _lib.ora_params_init.argtypes = [C.POINTER(Params), C.c_int, C.c_float, C.c_int, C.c_int, C.c_int]
        _lib.ora_extract.argtypes = [C.POINTER(Params), u8p, C.c_int, C.c_int, C.c_size_t,
                                     C.c_void_p, u8p, C.c_int, C.POINTER(C.c_int)]
        _lib.ora_fast_atan2.argtypes = [C.c_float, C.c_float]
        _lib.ora_fast_atan2.restype = C.c_float
        _lib.ora_descriptor_distance.argtypes = [u8p, u8p]
        _lib.ora_resize_linear_u8.argtypes = [u8p, C.c_int, C.c_int, C.c_size_t, u8p, C.c_int, C.c_int, C.c_size_t]
        _lib.ora_gaussian_blur7_u8.argtypes = [u8p, C.c_int, C.c_int, C.c_size_t, u8p, C.c_size_t]
        _lib.ora_fast_corner_score.argtypes = [u8p, C.c_int, C.c_int]
        _lib.ora_fast_detect.argtypes = [u8p, C.c_int, C.c_int, C.c_size_t, C.c_int, C.c_void_p, C.c_int]
        _lib.ora_ic_angle.argtypes = [u8p, C.c_size_t, C.c_float, C.c_float, C.POINTER(C.c_int)]
        _lib.ora_ic_angle.restype = C.c_float
        _lib.ora_cos_sin.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        _lib.ora_orb_descriptor.argtypes = [u8p, C.c_size_t, C.c_float, C.c_float, C.c_float, u8p]
        _lib.ora_distribute_octree.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                               C.c_int, C.c_void_p, C.c_int]
        _lib.ora_pyramid.argtypes = [C.POINTER(Params), u8p, C.c_int, C.c_int, C.c_size_t, C.POINTER(u8p)]
        _lib.ora_level_candidates.argtypes = [C.POINTER(Params), u8p, C.c_int, C.c_int, C.c_void_p, C.c_int]
        _lib.ora_level_size.argtypes = [C.POINTER(Params), C.c_int, C.c_int, C.c_int,
                                        C.POINTER(C.c_int), C.POINTER(C.c_int)]
    return _lib


def _u8(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def params(nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th_fast=20, min_th_fast=7) -> Params:
    p = Params()
    rc = lib().ora_params_init(C.byref(p), nfeatures, scale_factor, nlevels, ini_th_fast, min_th_fast)
    if rc != 0:
        raise ValueError("bad ORB parameters")
    return p


def level_sizes(p: Params, width: int, height: int):
    out = []
    for lv in range(p.nlevels):
        w, h = C.c_int(), C.c_int()
        lib().ora_level_size(C.byref(p), width, height, lv, C.byref(w), C.byref(h))
        out.append((w.value, h.value))
    return out


def extract(img: np.ndarray, p: Params | None = None, cap: int = 1 << 16):
    """ORBextractor::operator() on one u8 image -> (keypoints[n], descriptors[n,32], level_counts)."""
    p = p or params()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    kps = np.zeros(cap, dtype=KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), dtype=np.uint8)
    counts = (C.c_int * MAX_LEVELS)()
    n = lib().ora_extract(C.byref(p), _u8(img), img.shape[1], img.shape[0], img.strides[0],
                          kps.ctypes.data, _u8(desc), cap, counts)
    if n < 0:
        raise RuntimeError("oracle capacity exceeded")
    return kps[:n].copy(), desc[:n].copy(), np.array(counts[:p.nlevels], dtype=np.int32)


def pyramid(img: np.ndarray, p: Params | None = None):
    p = p or params()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    sizes = level_sizes(p, img.shape[1], img.shape[0])
    levels = [np.zeros((h, w), dtype=np.uint8) for (w, h) in sizes]
    arr = (C.POINTER(C.c_uint8) * p.nlevels)(*[_u8(lv) for lv in levels])
    lib().ora_pyramid(C.byref(p), _u8(img), img.shape[1], img.shape[0], img.strides[0], arr)
    return levels


def level_candidates(level: np.ndarray, p: Params | None = None, cap: int = 1 << 18):
    p = p or params()
    level = np.ascontiguousarray(level)
    out = np.zeros(cap, dtype=KEYPOINT_DTYPE)
    n = lib().ora_level_candidates(C.byref(p), _u8(level), level.shape[1], level.shape[0], out.ctypes.data, cap)
    if n < 0:
        raise RuntimeError("capacity")
    return out[:n].copy()


def distribute_octree(keys: np.ndarray, minX, maxX, minY, maxY, N):
    keys = np.ascontiguousarray(keys, dtype=KEYPOINT_DTYPE)
    out = np.zeros(max(len(keys), 1) + 8, dtype=KEYPOINT_DTYPE)
    n = lib().ora_distribute_octree(keys.ctypes.data, len(keys), minX, maxX, minY, maxY, N,
                                    out.ctypes.data, len(out))
    return out[:n].copy()


def resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    src = np.ascontiguousarray(src)
    dst = np.zeros((dh, dw), dtype=np.uint8)
    lib().ora_resize_linear_u8(_u8(src), src.shape[1], src.shape[0], src.strides[0], _u8(dst), dw, dh, dw)
    return dst


def gaussian_blur(src: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(src)
    dst = np.zeros_like(src)
    lib().ora_gaussian_blur7_u8(_u8(src), src.shape[1], src.shape[0], src.strides[0], _u8(dst), dst.strides[0])
    return dst


def fast_detect(img: np.ndarray, threshold: int, cap: int = 1 << 16):
    img = np.ascontiguousarray(img)
    out = np.zeros(cap, dtype=KEYPOINT_DTYPE)
    n = lib().ora_fast_detect(_u8(img), img.shape[0], img.shape[1], img.strides[0], threshold, out.ctypes.data, cap)
    return out[:n].copy()


def fast_atan2(y: float, x: float) -> float:
    return lib().ora_fast_atan2(y, x)


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    a = np.ascontiguousarray(a, dtype=np.uint8)
    b = np.ascontiguousarray(b, dtype=np.uint8)
    return lib().ora_descriptor_distance(_u8(a), _u8(b))


def ic_angle(img: np.ndarray, x: float, y: float, p: Params | None = None) -> float:
    p = p or params()
    img = np.ascontiguousarray(img)
    return lib().ora_ic_angle(_u8(img), img.strides[0], x, y, p.umax)


def orb_descriptor(img: np.ndarray, x: float, y: float, angle: float) -> np.ndarray:
    img = np.ascontiguousarray(img)
    out = np.zeros(32, dtype=np.uint8)
    lib().ora_orb_descriptor(_u8(img), img.strides[0], x, y, angle, _u8(out))
    return out


def cos_sin(angle_deg: float):
    c, s = C.c_float(), C.c_float()
    lib().ora_cos_sin(angle_deg, C.byref(c), C.byref(s))
    return c.value, s.value


def cpu_threads() -> int:
    return len(os.sched_getaffinity(0))
