"""ctypes binding of liborbx.so (include/orbx.h).

The HIP library is the product: if it is missing this module raises instead of
falling back to any CPU path.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

import os

# ORBX_LIB: alternative build of the library (A/B measurements of kernel variants)
LIB_PATH = Path(os.environ.get("ORBX_LIB", str(Path(__file__).resolve().parent / "liborbx.so")))

ORBX_OK = 0
ORBX_EMPTY = 1
ORBX_ERR_ARG = -1
ORBX_ERR_HIP = -2
ORBX_ERR_CAPACITY = -3
ORBX_ERR_UNSUPPORTED = -4
ORBX_ERR_STATE = -5

# == cv::KeyPoint / orbx_keypoint (28 bytes)
KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])

EXPORTED = [
    "orbx_extractor_create", "orbx_extractor_destroy", "orbx_extractor_levels",
    "orbx_extractor_features_per_level", "orbx_extractor_max_keypoints", "orbx_extract",
    "orbx_extract_batch", "orbx_extract_batch_device", "orbx_extractor_stream", "orbx_extractor_set_stage_event",
    "orbx_stream_wait_event", "orbx_stream_create", "orbx_stream_destroy",
    "orbx_extractor_set_timing", "orbx_extractor_stage_times", "orbx_pyramid_level",
    "orbx_pyramid_level_device", "orbx_hamming", "orbx_hamming_matrix_device",
    "orbx_window_match_device", "orbx_window_match", "orbx_version", "orbx_device_count",
    "orbx_last_error", "orbx_matcher_create", "orbx_matcher_destroy", "orbx_search_by_projection_local",
    "orbx_search_by_projection_frame", "orbx_search_for_triangulation", "orbx_compute_stereo_matches",
    "orbx_match_sequence_device", "orbx_matcher_set_timing", "orbx_matcher_last_ms", "orbx_matcher_last_call_us",
    "orbx_search_by_projection_keyframe", "orbx_search_by_projection_sim3", "orbx_matcher_set_footprint",
    "orbx_vocabulary_load_text_file", "orbx_vocabulary_load_text", "orbx_vocabulary_destroy",
    "orbx_vocabulary_info", "orbx_vocabulary_stream", "orbx_vocabulary_transform_features",
    "orbx_vocabulary_transform", "orbx_vocabulary_transform_batch_device", "orbx_vocabulary_set_timing",
    "orbx_vocabulary_stage_times", "orbx_search_by_bow_frame", "orbx_search_by_bow_keyframes",
    "orbx_search_for_initialization", "orbx_undistort_keypoints", "orbx_undistort_keypoints_device",
    "orbx_compute_image_bounds", "orbx_assign_features_to_grid", "orbx_assign_features_to_grid_device",
    "orbx_fuse", "orbx_fuse_sim3", "orbx_search_by_sim3", "orbx_compute_distinctive_descriptors",
    "orbx_compute_distinctive_descriptors_device", "orbx_extractor_status", "orbx_extractor_status_device",
    "orbx_extractor_set_node_capacity", "orbx_extractor_set_level0_in_place", "orbx_compute_stereo_matches_batch_device",
    "orbx_search_for_triangulation_batch_device", "orbx_match_sequence_device_ex",
    "orbx_search_local_points_device", "orbx_create_mappoints_device", "orbx_update_last_frame_device",
    "orbx_extractor_last_call_us", "orbx_compute_stereo_from_rgbd", "orbx_compute_stereo_from_rgbd_device",
    "orbx_debug_set",
]

ORBX_DEPTH_U16 = 0
ORBX_DEPTH_F32 = 1


class Camera(C.Structure):
    _fields_ = [("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float), ("k1", C.c_float),
                ("k2", C.c_float), ("p1", C.c_float), ("p2", C.c_float), ("k3", C.c_float)]


class ExtractorParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scale_factor", C.c_float), ("nlevels", C.c_int),
                ("ini_th_fast", C.c_int), ("min_th_fast", C.c_int)]


class Sequence(C.Structure):
    """orbx_sequence (include/orbx.h)."""
    _fields_ = [("batch", C.c_int), ("kps", C.c_void_p), ("desc", C.c_void_p), ("n", C.c_void_p), ("cap", C.c_int),
                ("Tcw", C.c_void_p), ("u_right", C.c_void_p), ("mp_pos", C.c_void_p), ("has_mp", C.c_void_p),
                ("depth", C.c_float), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("bf", C.c_float), ("b", C.c_float), ("min_x", C.c_float), ("max_x", C.c_float),
                ("min_y", C.c_float), ("max_y", C.c_float), ("nlevels", C.c_int),
                ("scale_factors", C.POINTER(C.c_float)), ("th", C.c_float), ("mono", C.c_int),
                ("global_ids", C.c_int), ("cur_mp", C.c_void_p), ("nmatches", C.c_void_p), ("mp_obs", C.c_void_p),
                ("retry_below", C.c_int)]


class RgbdBatch(C.Structure):
    """orbx_rgbd_batch (include/orbx.h)."""
    _fields_ = [("batch", C.c_int), ("kps", C.c_void_p), ("kps_un", C.c_void_p), ("n", C.c_void_p), ("cap", C.c_int),
                ("depth", C.c_void_p), ("depth_type", C.c_int), ("width", C.c_int), ("height", C.c_int),
                ("row_bytes", C.c_longlong), ("frame_bytes", C.c_longlong), ("depth_map_factor", C.c_float),
                ("bf", C.c_float), ("u_right", C.c_void_p), ("depth_out", C.c_void_p)]


class MapPointsDevice(C.Structure):
    """orbx_mappoints_device."""
    _fields_ = [("n", C.c_int), ("pos", C.c_void_p), ("desc", C.c_void_p), ("normal", C.c_void_p),
                ("max_distance", C.c_void_p), ("min_distance", C.c_void_p), ("observations", C.c_void_p),
                ("bad", C.c_void_p)]


class LocalMapBatch(C.Structure):
    """orbx_local_map_batch."""
    _fields_ = [("batch", C.c_int), ("kps", C.c_void_p), ("desc", C.c_void_p), ("n", C.c_void_p), ("cap", C.c_int),
                ("u_right", C.c_void_p), ("Tcw", C.c_void_p), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float), ("min_x", C.c_float),
                ("max_x", C.c_float), ("min_y", C.c_float), ("max_y", C.c_float), ("nlevels", C.c_int),
                ("scale_factors", C.POINTER(C.c_float)), ("local_off", C.POINTER(C.c_int32)),
                ("local_ids", C.c_void_p), ("th", C.c_float), ("viewing_cos_limit", C.c_float),
                ("frame_mp", C.c_void_p), ("nmatches", C.c_void_p)]


# ---- handle lifetime (DESIGN.md §1 "Teardown") ------------------------------------
# Every object that owns liborbx handles or HIP streams registers here.  At interpreter
# exit the atexit hook synchronises the devices and closes them newest first -- while the
# HIP runtime, RCCL and any profiler are still fully alive -- so no HIP object is left for
# the C runtime's static destructors (HIP's own, RCCL's, a profiler tool's) to tear down in
# whatever order they run.  __del__ does nothing once the interpreter is finalizing.
_handles: list = []
_hook = False


def track(obj) -> None:
    """Register a handle owner (it has close(): idempotent, synchronising what it frees)."""
    global _hook
    import weakref
    if len(_handles) > 4096:  # drop the owners already freed
        _handles[:] = [r for r in _handles if r() is not None]
    _handles.append(weakref.ref(obj))
    if not _hook:
        # registered after torch's own exit hooks (lib() imports torch first), so it runs
        # before them
        import atexit
        atexit.register(release_all)
        _hook = True


def release_all() -> int:
    """Synchronise the devices the process used and close every live handle owner,
    newest first; returns how many were closed."""
    live = [o for o in (r() for r in reversed(_handles)) if o is not None]
    _handles.clear()
    if not live:
        return 0
    try:
        import torch
        if torch.cuda.is_initialized():
            for d in range(torch.cuda.device_count()):
                with torch.cuda.device(d):
                    torch.cuda.synchronize()
    except Exception:
        pass
    for o in live:
        try:
            o.close()
        except Exception:
            pass
    return len(live)


class OrbxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"orbx error {code}: {msg}")
        self.code = code


_lib = None


def lib() -> C.CDLL:
    """Load liborbx.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} not built: run `python -m orbslam2commentedbyxcm_amd.build`")
    # torch bundles its own libamdhip64.so.7 (and HSA runtime).  Two HIP runtimes in one
    # process cannot both open the GPU, so when torch is installed it is loaded first and
    # liborbx.so binds to the same runtime (same SONAME); without torch liborbx.so uses
    # the system ROCm runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(str(LIB_PATH))
    vp, ip, u8p = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_uint8)
    fp = C.POINTER(C.c_float)
    L.orbx_extractor_create.argtypes = [C.POINTER(ExtractorParams), C.c_int, C.POINTER(vp)]
    L.orbx_extractor_destroy.argtypes = [vp]
    L.orbx_extractor_destroy.restype = None
    L.orbx_extractor_levels.argtypes = [vp, ip, fp, fp, fp, fp]
    L.orbx_extractor_features_per_level.argtypes = [vp, ip]
    L.orbx_extractor_max_keypoints.argtypes = [vp, C.c_int, C.c_int, ip]
    L.orbx_extract.argtypes = [vp, u8p, C.c_int, C.c_int, C.c_size_t, vp, u8p, C.c_int, ip]
    L.orbx_extract_batch.argtypes = [vp, C.c_int, C.POINTER(u8p), C.c_int, C.c_int, C.c_size_t, vp, u8p,
                                     C.c_int, ip]
    L.orbx_extract_batch_device.argtypes = [vp, C.c_int, vp, C.c_size_t, C.c_int, C.c_int, C.c_size_t, vp, vp,
                                            C.c_int, vp, vp]
    L.orbx_extractor_stream.argtypes = [vp]
    L.orbx_extractor_stream.restype = vp
    L.orbx_extractor_set_stage_event.argtypes = [vp, C.c_int, C.POINTER(vp)]
    L.orbx_stream_wait_event.argtypes = [vp, vp]
    L.orbx_stream_create.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(vp)]
    L.orbx_stream_destroy.argtypes = [vp]
    L.orbx_extractor_status.argtypes = [vp, C.c_int, ip, ip]
    L.orbx_extractor_status_device.argtypes = [vp, C.POINTER(vp)]
    L.orbx_extractor_set_node_capacity.argtypes = [vp, C.c_int]
    L.orbx_extractor_set_level0_in_place.argtypes = [vp, C.c_int]
    L.orbx_extractor_set_timing.argtypes = [vp, C.c_int]
    L.orbx_extractor_stage_times.argtypes = [vp, C.c_int, C.POINTER(C.c_char_p), fp, ip]
    L.orbx_pyramid_level.argtypes = [vp, C.c_int, C.c_int, u8p, C.c_size_t, ip, ip]
    L.orbx_pyramid_level_device.argtypes = [vp, C.c_int, C.c_int, C.POINTER(vp), C.POINTER(C.c_size_t), ip, ip]
    L.orbx_hamming.argtypes = [u8p, u8p]
    L.orbx_hamming_matrix_device.argtypes = [vp, C.c_int, vp, C.c_int, vp, vp]
    L.orbx_window_match_device.argtypes = [vp, C.c_int, vp, vp, vp, vp, C.c_int, vp, vp, vp, vp, vp, vp]
    i32p = C.POINTER(C.c_int32)
    L.orbx_window_match.argtypes = [C.c_int, u8p, C.c_int, u8p, C.c_int, i32p, i32p, i32p, C.c_int, i32p, i32p,
                                    i32p, i32p, i32p]
    L.orbx_matcher_create.argtypes = [C.c_int, C.c_float, C.c_int, C.POINTER(vp)]
    L.orbx_matcher_destroy.argtypes = [vp]
    L.orbx_matcher_destroy.restype = None
    L.orbx_search_by_projection_local.argtypes = [vp, vp, i32p, i32p, C.c_int, vp, vp, C.c_float, ip]
    L.orbx_search_by_projection_frame.argtypes = [vp, vp, i32p, vp, i32p, u8p, vp, C.c_float, C.c_int, ip]
    L.orbx_search_for_triangulation.argtypes = [vp, vp, u8p, i32p, i32p, i32p, C.c_int, vp, u8p, i32p, i32p, i32p,
                                                C.c_int, fp, C.c_int, i32p, ip]
    L.orbx_compute_stereo_matches.argtypes = [vp, vp, C.c_int, vp, C.c_int, vp, vp, u8p, C.c_int, C.c_float, fp, fp]
    L.orbx_compute_stereo_matches_batch_device.argtypes = [vp, vp, C.c_int, vp, C.c_int, C.c_int, vp, vp, vp, vp, vp,
                                                           vp, C.c_int, C.c_float, C.c_float, vp, vp, vp]
    L.orbx_search_for_triangulation_batch_device.argtypes = [vp, C.c_int, vp, vp, C.c_int, i32p, fp, C.c_int,
                                                             C.c_int, vp, vp, vp, vp]
    L.orbx_match_sequence_device.argtypes = [vp, C.c_int, vp, vp, vp, C.c_int, vp, C.c_float, C.c_float, C.c_float,
                                             C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, fp, C.c_int,
                                             C.c_float, C.c_float, vp, vp, vp]
    L.orbx_match_sequence_device_ex.argtypes = [vp, C.POINTER(Sequence), vp]
    L.orbx_search_local_points_device.argtypes = [vp, C.POINTER(MapPointsDevice), C.POINTER(LocalMapBatch), vp]
    L.orbx_create_mappoints_device.argtypes = [C.c_int, vp, vp, C.c_int, vp, C.c_float, vp, C.c_float, C.c_float,
                                               C.c_float, C.c_float, fp, C.c_int, vp, vp, vp, vp, vp, vp, vp]
    L.orbx_update_last_frame_device.argtypes = [C.c_int, vp, vp, C.c_int, vp, vp, C.c_float, C.c_float, C.c_float,
                                                C.c_float, C.c_float, vp, vp, vp, vp, vp, vp]
    L.orbx_search_by_projection_keyframe.argtypes = [vp, vp, i32p, vp, i32p, u8p, vp, C.c_float, C.c_int, ip]
    L.orbx_search_by_projection_sim3.argtypes = [vp, vp, fp, i32p, C.c_int, i32p, vp, C.c_int, ip]
    L.orbx_search_by_bow_frame.argtypes = [vp, vp, i32p, i32p, i32p, i32p, C.c_int, vp, i32p, i32p, i32p, C.c_int,
                                           i32p, ip]
    L.orbx_search_by_bow_keyframes.argtypes = [vp, vp, i32p, i32p, i32p, i32p, C.c_int, vp, i32p, i32p, i32p, i32p,
                                               C.c_int, i32p, ip]
    L.orbx_search_for_initialization.argtypes = [vp, vp, vp, fp, i32p, C.c_int, ip]
    cp = C.POINTER(Camera)
    L.orbx_undistort_keypoints.argtypes = [C.c_int, cp, vp, C.c_int, vp]
    L.orbx_undistort_keypoints_device.argtypes = [cp, C.c_int, vp, vp, C.c_int, vp, vp]
    L.orbx_compute_image_bounds.argtypes = [C.c_int, cp, C.c_int, C.c_int, fp]
    L.orbx_compute_stereo_from_rgbd_device.argtypes = [cp, C.POINTER(RgbdBatch), vp]
    L.orbx_compute_stereo_from_rgbd.argtypes = [C.c_int, cp, vp, C.c_int, vp, C.c_int, C.c_int, C.c_int, C.c_size_t,
                                                C.c_float, C.c_float, vp, fp, fp]
    L.orbx_assign_features_to_grid.argtypes = [C.c_int, vp, C.c_int, fp, i32p, i32p]
    L.orbx_assign_features_to_grid_device.argtypes = [C.c_int, vp, vp, C.c_int, fp, vp, vp, vp]
    L.orbx_fuse.argtypes = [vp, vp, i32p, C.c_int, u8p, vp, C.c_float, i32p]
    L.orbx_fuse_sim3.argtypes = [vp, vp, fp, i32p, C.c_int, u8p, vp, C.c_float, i32p]
    L.orbx_search_by_sim3.argtypes = [vp, vp, i32p, u8p, vp, i32p, u8p, vp, C.c_float, fp, fp, C.c_float, i32p, ip]
    L.orbx_compute_distinctive_descriptors.argtypes = [C.c_int, C.c_int, i32p, u8p, i32p, u8p]
    L.orbx_compute_distinctive_descriptors_device.argtypes = [C.c_int, vp, vp, vp, vp, vp]
    L.orbx_matcher_set_timing.argtypes = [vp, C.c_int]
    L.orbx_matcher_set_footprint.argtypes = [vp, C.c_int]
    L.orbx_matcher_last_ms.argtypes = [vp, fp]
    L.orbx_matcher_last_call_us.argtypes = [vp]
    L.orbx_matcher_last_call_us.restype = C.c_double
    L.orbx_extractor_last_call_us.argtypes = [vp]
    L.orbx_extractor_last_call_us.restype = C.c_double
    dp = C.POINTER(C.c_double)
    L.orbx_vocabulary_load_text_file.argtypes = [C.c_char_p, C.c_int, C.POINTER(vp)]
    L.orbx_vocabulary_load_text.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.POINTER(vp)]
    L.orbx_vocabulary_destroy.argtypes = [vp]
    L.orbx_vocabulary_destroy.restype = None
    L.orbx_vocabulary_info.argtypes = [vp, ip, ip, ip, ip, ip, ip]
    L.orbx_vocabulary_stream.argtypes = [vp]
    L.orbx_vocabulary_stream.restype = vp
    L.orbx_vocabulary_transform_features.argtypes = [vp, u8p, C.c_int, C.c_int, i32p, dp, i32p]
    L.orbx_vocabulary_transform.argtypes = [vp, u8p, C.c_int, C.c_int, i32p, dp, ip, i32p, i32p, i32p, ip]
    L.orbx_vocabulary_transform_batch_device.argtypes = [vp, C.c_int, vp, vp, C.c_int, C.c_int] + [vp] * 9 + [vp]
    L.orbx_vocabulary_set_timing.argtypes = [vp, C.c_int]
    L.orbx_vocabulary_stage_times.argtypes = [vp, fp, fp]
    L.orbx_debug_set.argtypes = [C.c_char_p, C.c_int]
    L.orbx_version.restype = C.c_char_p
    L.orbx_device_count.argtypes = [ip]
    L.orbx_last_error.restype = C.c_char_p
    _lib = L
    return L


def debug_set(name: str | None, value: int = -1) -> None:
    """orbx_debug_set: select an alternative kernel form or a diagnostics switch
    (value < 0: the default; name None: every default).  Tests and A/B tools only."""
    check(lib().orbx_debug_set(None if name is None else name.encode(), int(value)))


def check(rc: int, allow=(ORBX_OK,)) -> int:
    if rc in allow:
        return rc
    msg = lib().orbx_last_error().decode(errors="replace")
    raise OrbxError(rc, msg)


def u8ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def i32ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int32))
