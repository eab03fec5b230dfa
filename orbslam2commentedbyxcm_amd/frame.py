"""Frame-side steps between extraction and matching (Frame.cc), on the GPU:
``UndistortKeyPoints`` (Frame.cc:586-628), ``ComputeImageBounds`` (636-665) and
``AssignFeaturesToGrid`` (351-370), host-buffer and batched-device forms."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L

I32P = C.POINTER(C.c_int32)
F32P = C.POINTER(C.c_float)
FRAME_GRID_COLS, FRAME_GRID_ROWS = 64, 48


def camera(fx, fy, cx, cy, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0) -> L.Camera:
    return L.Camera(fx, fy, cx, cy, k1, k2, p1, p2, k3)


def UndistortKeyPoints(cam: L.Camera, keys: np.ndarray, device: int = 0) -> np.ndarray:
    k = np.ascontiguousarray(keys, dtype=L.KEYPOINT_DTYPE)
    out = np.empty_like(k)
    L.check(L.lib().orbx_undistort_keypoints(device, C.byref(cam), k.ctypes.data, len(k), out.ctypes.data))
    return out


def ComputeImageBounds(cam: L.Camera, cols: int, rows: int, device: int = 0) -> np.ndarray:
    """-> float32 [mnMinX, mnMaxX, mnMinY, mnMaxY]."""
    b = np.zeros(4, np.float32)
    L.check(L.lib().orbx_compute_image_bounds(device, C.byref(cam), int(cols), int(rows), b.ctypes.data_as(F32P)))
    return b


def AssignFeaturesToGrid(keys_un: np.ndarray, bounds, device: int = 0):
    """-> (cell_start int32[3073], cell_idx int32[...]) with cell c = ix * 48 + iy."""
    k = np.ascontiguousarray(keys_un, dtype=L.KEYPOINT_DTYPE)
    bd = np.ascontiguousarray(bounds, np.float32)
    start = np.zeros(FRAME_GRID_COLS * FRAME_GRID_ROWS + 1, np.int32)
    idx = np.zeros(max(len(k), 1), np.int32)
    L.check(L.lib().orbx_assign_features_to_grid(device, k.ctypes.data, len(k), bd.ctypes.data_as(F32P),
                                                 start.ctypes.data_as(I32P), idx.ctypes.data_as(I32P)))
    return start, idx[:start[-1]].copy()


def undistort_device(cam: L.Camera, d_keys, d_n, cap: int, d_keys_un, stream=None):
    """Batched undistortion over torch tensors ([B, cap, 7] int32 keypoint rows)."""
    L.check(L.lib().orbx_undistort_keypoints_device(C.byref(cam), int(d_n.numel()), C.c_void_p(d_keys.data_ptr()),
                                                    C.c_void_p(d_n.data_ptr()), int(cap),
                                                    C.c_void_p(d_keys_un.data_ptr()), C.c_void_p(stream) if stream else None))


def grid_device(d_keys_un, d_n, cap: int, bounds, d_cell_start, d_cell_idx, stream=None):
    bd = np.ascontiguousarray(bounds, np.float32)
    L.check(L.lib().orbx_assign_features_to_grid_device(int(d_n.numel()), C.c_void_p(d_keys_un.data_ptr()),
                                                        C.c_void_p(d_n.data_ptr()), int(cap), bd.ctypes.data_as(F32P),
                                                        C.c_void_p(d_cell_start.data_ptr()),
                                                        C.c_void_p(d_cell_idx.data_ptr()),
                                                        C.c_void_p(stream) if stream else None))
