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


def ComputeStereoFromRGBD(keys: np.ndarray, depth: np.ndarray, bf: float, depth_map_factor: float,
                          cam: L.Camera | None = None, keys_un: np.ndarray | None = None, device: int = 0):
    """The RGB-D Frame constructor's steps after ExtractORB (Frame.cc:227-230) for one frame
    (orbx_compute_stereo_from_rgbd): UndistortKeyPoints when `cam` is given (else keys_un is
    mvKeysUn), then ComputeStereoFromRGBD (Frame.cc:888-909) on the depth image (H, W)
    uint16 or float32 converted as Tracking::GrabImageRGBD does (Tracking.cc:265-271, scale
    depth_map_factor = mDepthMapFactor).  -> (mvKeysUn, mvuRight, mvDepth)."""
    k = np.ascontiguousarray(keys, dtype=L.KEYPOINT_DTYPE)
    img = np.ascontiguousarray(depth)
    if img.dtype not in (np.uint16, np.float32):
        raise ValueError("depth image must be uint16 or float32")
    if cam is None:
        if keys_un is None:
            raise ValueError("keys_un is needed without a camera")
        ku = np.array(keys_un, dtype=L.KEYPOINT_DTYPE, copy=True)
    else:
        ku = np.empty_like(k)
    n = len(k)
    ur = np.zeros(max(n, 1), np.float32)
    dp = np.zeros(max(n, 1), np.float32)
    L.check(L.lib().orbx_compute_stereo_from_rgbd(
        device, C.byref(cam) if cam is not None else None, k.ctypes.data, n, img.ctypes.data,
        L.ORBX_DEPTH_F32 if img.dtype == np.float32 else L.ORBX_DEPTH_U16, img.shape[1], img.shape[0],
        img.strides[0], float(depth_map_factor), float(bf), ku.ctypes.data, ur.ctypes.data_as(F32P),
        dp.ctypes.data_as(F32P)))
    return ku, ur[:n].copy(), dp[:n].copy()


def rgbd_device(cam, d_kps, d_n, d_depth, bf: float, depth_map_factor: float, d_kps_un, d_u_right, d_depth_out,
                stream=None):
    """Batched RGB-D Frame steps (orbx_compute_stereo_from_rgbd_device) over torch tensors:
    d_kps / d_kps_un (B, cap, 7) int32 keypoint rows, d_n (B,), d_depth (B, H, W) uint16 or
    float32 depth images (any row pitch), outputs d_u_right / d_depth_out (B, cap) float32.
    cam None: d_kps_un already holds mvKeysUn.  Asynchronous."""
    import torch
    rb = L.RgbdBatch()
    rb.batch, rb.cap = int(d_n.numel()), int(d_kps.shape[1])
    rb.kps, rb.kps_un, rb.n = d_kps.data_ptr(), d_kps_un.data_ptr(), d_n.data_ptr()
    rb.depth = d_depth.data_ptr()
    rb.depth_type = L.ORBX_DEPTH_F32 if d_depth.dtype == torch.float32 else L.ORBX_DEPTH_U16
    if d_depth.dtype not in (torch.float32, torch.uint16) or d_depth.stride(2) != 1:
        raise ValueError("depth images must be uint16 or float32 with unit column stride")
    es = d_depth.element_size()
    rb.height, rb.width = int(d_depth.shape[1]), int(d_depth.shape[2])
    rb.row_bytes, rb.frame_bytes = int(d_depth.stride(1)) * es, int(d_depth.stride(0)) * es
    rb.depth_map_factor, rb.bf = float(depth_map_factor), float(bf)
    rb.u_right, rb.depth_out = d_u_right.data_ptr(), d_depth_out.data_ptr()
    L.check(L.lib().orbx_compute_stereo_from_rgbd_device(C.byref(cam) if cam is not None else None, C.byref(rb),
                                                         C.c_void_p(getattr(stream, "cuda_stream", stream))
                                                         if stream else None))
