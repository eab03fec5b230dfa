"""orbslam2commentedbyxcm_amd -- MI355X-native ORB extraction + Hamming matching.

Drop-in for ORB-SLAM2's per-frame hot path (ORBextractor::operator(),
ORBmatcher::DescriptorDistance / SearchByProjection / SearchForTriangulation),
implemented as hand-written HIP kernels for gfx950 behind the C ABI in
include/orbx.h (liborbx.so).  This package is the host-side mirror of the
reference's ORBextractor / ORBmatcher interface.
"""
from ._lib import KEYPOINT_DTYPE, OrbxError, lib  # noqa: F401
from .extractor import ORBextractor  # noqa: F401

__all__ = ["ORBextractor", "KEYPOINT_DTYPE", "OrbxError", "lib"]
