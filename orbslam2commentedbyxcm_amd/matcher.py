"""ORBmatcher -- host-side mirror of ORB_SLAM2::ORBmatcher over liborbx.so.

Constructor (nnratio, checkOri), the TH_HIGH / TH_LOW / HISTO_LENGTH constants and
DescriptorDistance as in include/ORBmatcher.h:57-228; the search functions take the
Frame / KeyFrame / MapPoint state as arrays (FrameView, MapPoints, Track) because
the object graph stays with the caller.  MapPoint* pointers are integer ids and
mvpMapPoints arrays hold ids (-1 = NULL).  Every call runs on the MI355X.
"""
from __future__ import annotations

import ctypes as C
import sys
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L

F32P = C.POINTER(C.c_float)
I32P = C.POINTER(C.c_int32)
U8P = C.POINTER(C.c_uint8)


class _FrameViewC(C.Structure):
    _fields_ = [("n", C.c_int), ("keys", C.c_void_p), ("desc", U8P), ("u_right", F32P),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("bf", C.c_float), ("b", C.c_float), ("min_x", C.c_float), ("max_x", C.c_float),
                ("min_y", C.c_float), ("max_y", C.c_float), ("nlevels", C.c_int),
                ("scale_factors", F32P), ("level_sigma2", F32P), ("Tcw", C.c_float * 12)]


class _KeyFrameDeviceC(C.Structure):
    """orbx_keyframe_device: device pointers + the host pose."""
    _fields_ = [("keys", C.c_void_p), ("desc", C.c_void_p), ("n", C.c_void_p), ("u_right", C.c_void_p),
                ("has_mp", C.c_void_p), ("fv_node", C.c_void_p), ("fv_off", C.c_void_p), ("fv_idx", C.c_void_p),
                ("nfv", C.c_void_p), ("Tcw", C.c_float * 12)]


def keyframe_device(keys, desc, n, has_mp, fv_node, fv_off, fv_idx, nfv, Tcw, u_right=None) -> _KeyFrameDeviceC:
    """One orbx_keyframe_device record from device tensors (or raw device addresses) of
    one keyframe: keys (cap, 7) int32 words, desc (cap, 32) u8, n / nfv 1-element int32,
    has_mp (cap,) u8, fv_node / fv_idx (cap,) int32, fv_off (cap + 1,) int32, u_right
    (cap,) f32 or None; Tcw a host 3x4 (or 4x4) pose."""
    def a(t):
        return None if t is None else (int(t) if isinstance(t, int) else t.data_ptr())

    r = _KeyFrameDeviceC()
    r.keys, r.desc, r.n, r.u_right = a(keys), a(desc), a(n), a(u_right)
    r.has_mp, r.fv_node, r.fv_off, r.fv_idx, r.nfv = a(has_mp), a(fv_node), a(fv_off), a(fv_idx), a(nfv)
    r.Tcw[:] = list(_f32(Tcw)[:3, :4].reshape(-1))
    return r


def keyframe_table(records):
    """A ctypes array of keyframe_device records (build once, pass to every call)."""
    return (_KeyFrameDeviceC * max(len(records), 1))(*records)


class _MapPointsC(C.Structure):
    _fields_ = [("n", C.c_int), ("pos", F32P), ("desc", U8P), ("observations", I32P), ("bad", U8P),
                ("max_distance", F32P), ("min_distance", F32P), ("normal", F32P)]


class _TrackC(C.Structure):
    _fields_ = [("in_view", U8P), ("proj_x", F32P), ("proj_y", F32P), ("proj_xr", F32P),
                ("scale_level", I32P), ("view_cos", F32P)]


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


@dataclass
class FrameView:
    """The Frame / KeyFrame members the matcher reads (include/Frame.h)."""
    keys: np.ndarray                   # mvKeysUn, KEYPOINT_DTYPE
    desc: np.ndarray                   # mDescriptors (n, 32) uint8
    fx: float = 500.0
    fy: float = 500.0
    cx: float = 320.0
    cy: float = 240.0
    bf: float = 0.0                    # mbf
    b: float = 0.0                     # mb
    min_x: float = 0.0
    max_x: float = 640.0
    min_y: float = 0.0
    max_y: float = 480.0
    scale_factors: np.ndarray = None   # mvScaleFactors
    level_sigma2: np.ndarray = None    # mvLevelSigma2
    Tcw: np.ndarray = None             # 3x4 (or 4x4) float
    u_right: np.ndarray | None = None  # mvuRight
    _keep: list = field(default_factory=list, repr=False)

    def c(self) -> _FrameViewC:
        keys = np.ascontiguousarray(self.keys, dtype=L.KEYPOINT_DTYPE)
        desc = np.ascontiguousarray(self.desc, dtype=np.uint8)
        sf = _f32(self.scale_factors)
        sg = _f32(self.level_sigma2 if self.level_sigma2 is not None else sf * sf)
        ur = None if self.u_right is None else _f32(self.u_right)
        T = np.eye(4, dtype=np.float32) if self.Tcw is None else _f32(self.Tcw)
        self._keep = [keys, desc, sf, sg, ur]
        v = _FrameViewC()
        v.n = len(keys)
        v.keys = keys.ctypes.data
        v.desc = desc.ctypes.data_as(U8P)
        v.u_right = ur.ctypes.data_as(F32P) if ur is not None else None
        v.fx, v.fy, v.cx, v.cy, v.bf, v.b = self.fx, self.fy, self.cx, self.cy, self.bf, self.b
        v.min_x, v.max_x, v.min_y, v.max_y = self.min_x, self.max_x, self.min_y, self.max_y
        v.nlevels = len(sf)
        v.scale_factors = sf.ctypes.data_as(F32P)
        v.level_sigma2 = sg.ctypes.data_as(F32P)
        v.Tcw[:] = list(T[:3, :4].reshape(-1))
        return v


@dataclass
class MapPoints:
    desc: np.ndarray                       # GetDescriptor() (m, 32)
    observations: np.ndarray               # Observations() (m,)
    pos: np.ndarray | None = None          # GetWorldPos() (m, 3)
    bad: np.ndarray | None = None          # isBad() (m,)
    max_distance: np.ndarray | None = None  # mfMaxDistance (m,)
    min_distance: np.ndarray | None = None  # mfMinDistance (m,)
    normal: np.ndarray | None = None        # GetNormal() (m, 3)
    _keep: list = field(default_factory=list, repr=False)

    def c(self) -> _MapPointsC:
        d = np.ascontiguousarray(self.desc, dtype=np.uint8)
        o = np.ascontiguousarray(self.observations, dtype=np.int32)
        p = None if self.pos is None else _f32(self.pos)
        b = None if self.bad is None else np.ascontiguousarray(self.bad, dtype=np.uint8)
        mx, mn, nr = (None if a is None else _f32(a) for a in (self.max_distance, self.min_distance, self.normal))
        self._keep = [d, o, p, b, mx, mn, nr]
        v = _MapPointsC()
        v.n = len(d)
        v.pos = p.ctypes.data_as(F32P) if p is not None else None
        v.desc = d.ctypes.data_as(U8P)
        v.observations = o.ctypes.data_as(I32P)
        v.bad = b.ctypes.data_as(U8P) if b is not None else None
        v.max_distance = mx.ctypes.data_as(F32P) if mx is not None else None
        v.min_distance = mn.ctypes.data_as(F32P) if mn is not None else None
        v.normal = nr.ctypes.data_as(F32P) if nr is not None else None
        return v


@dataclass
class Track:
    """Frame::IsInFrustum outputs per MapPoint id (Frame.cc:412-477)."""
    in_view: np.ndarray
    proj_x: np.ndarray
    proj_y: np.ndarray
    proj_xr: np.ndarray
    scale_level: np.ndarray
    view_cos: np.ndarray
    _keep: list = field(default_factory=list, repr=False)

    def c(self) -> _TrackC:
        a = [np.ascontiguousarray(self.in_view, np.uint8), _f32(self.proj_x), _f32(self.proj_y),
             _f32(self.proj_xr), np.ascontiguousarray(self.scale_level, np.int32), _f32(self.view_cos)]
        self._keep = a
        v = _TrackC()
        v.in_view = a[0].ctypes.data_as(U8P)
        v.proj_x, v.proj_y, v.proj_xr = (x.ctypes.data_as(F32P) for x in a[1:4])
        v.scale_level = a[4].ctypes.data_as(I32P)
        v.view_cos = a[5].ctypes.data_as(F32P)
        return v


def feature_vector_csr(nodes_per_kp: np.ndarray):
    """DBoW2::FeatureVector (node -> ascending keypoint indices, FeatureVector.cpp:31-45)
    as CSR (node ids, offsets, indices) from each keypoint's node id (-1 = none)."""
    nodes_per_kp = np.asarray(nodes_per_kp)
    valid = np.nonzero(nodes_per_kp >= 0)[0]
    order = valid[np.lexsort((valid, nodes_per_kp[valid]))]
    node_ids, starts = np.unique(nodes_per_kp[order], return_index=True)
    off = np.append(starts, len(order)).astype(np.int32)
    return node_ids.astype(np.int32), off, order.astype(np.int32)


class ORBmatcher:
    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self.device = int(device)
        self._h = None
        h = C.c_void_p()
        L.check(L.lib().orbx_matcher_create(self.device, self.mfNNratio, 1 if checkOri else 0, C.byref(h)))
        self._destroy = L.lib().orbx_matcher_destroy  # held: module globals may be gone at exit
        self._h = h
        L.track(self)

    def close(self) -> None:
        """Release the matcher (orbx_matcher_destroy: waits for its stream); idempotent."""
        if getattr(self, "_h", None):
            self._destroy(self._h)
            self._h = None

    def __del__(self, _finalizing=sys.is_finalizing):
        if not _finalizing():
            self.close()

    def last_call_us(self) -> float:
        """Wall time (us) of this matcher's newest host call inside liborbx (no binding
        overhead): what a C++ caller pays per call."""
        return float(L.lib().orbx_matcher_last_call_us(self._h))

    @staticmethod
    def DescriptorDistance(a: np.ndarray, b: np.ndarray) -> int:
        """ORBmatcher::DescriptorDistance (ORBmatcher.cc:1983-2003)."""
        a = np.ascontiguousarray(a, dtype=np.uint8)
        b = np.ascontiguousarray(b, dtype=np.uint8)
        return L.lib().orbx_hamming(L.u8ptr(a), L.u8ptr(b))

    # SearchByProjection(Frame&, const vector<MapPoint*>&, th)  ORBmatcher.cc:61-173
    def SearchByProjectionLocal(self, F: FrameView, frame_mp: np.ndarray, queries, mps: MapPoints, track: Track,
                                th: float = 1.0) -> int:
        q = np.ascontiguousarray(queries, dtype=np.int32)
        assert frame_mp.dtype == np.int32 and frame_mp.flags.c_contiguous
        fv, mv, tv = F.c(), mps.c(), track.c()
        n = C.c_int()
        L.check(L.lib().orbx_search_by_projection_local(self._h, C.addressof(fv), frame_mp.ctypes.data_as(I32P),
                                                        q.ctypes.data_as(I32P), len(q), C.addressof(mv), C.addressof(tv),
                                                        float(th), C.byref(n)))
        return n.value

    # SearchByProjection(Frame& Cur, const Frame& Last, th, bMono)  ORBmatcher.cc:1620-1789
    def SearchByProjectionFrame(self, cur: FrameView, cur_mp: np.ndarray, last: FrameView, last_mp: np.ndarray,
                                mps: MapPoints, th: float, bMono: bool, last_outlier=None) -> int:
        assert cur_mp.dtype == np.int32 and cur_mp.flags.c_contiguous
        lm = np.ascontiguousarray(last_mp, dtype=np.int32)
        lo = None if last_outlier is None else np.ascontiguousarray(last_outlier, dtype=np.uint8)
        cv_, lv, mv = cur.c(), last.c(), mps.c()
        n = C.c_int()
        L.check(L.lib().orbx_search_by_projection_frame(self._h, C.addressof(cv_), cur_mp.ctypes.data_as(I32P),
                                                        C.addressof(lv), lm.ctypes.data_as(I32P),
                                                        lo.ctypes.data_as(U8P) if lo is not None else None,
                                                        C.addressof(mv), float(th), 1 if bMono else 0, C.byref(n)))
        return n.value

    # SearchByProjection(Frame&, KeyFrame*, const set<MapPoint*>&, th, ORBdist)  ORBmatcher.cc:1792-1924
    def SearchByProjectionKeyFrame(self, cur: FrameView, cur_mp: np.ndarray, kf: FrameView, kf_mp: np.ndarray,
                                   mps: MapPoints, th: float, ORBdist: int, already_found=None) -> int:
        assert cur_mp.dtype == np.int32 and cur_mp.flags.c_contiguous
        km = np.ascontiguousarray(kf_mp, dtype=np.int32)
        af = None if already_found is None else np.ascontiguousarray(already_found, dtype=np.uint8)
        cv_, kv, mv = cur.c(), kf.c(), mps.c()
        n = C.c_int()
        L.check(L.lib().orbx_search_by_projection_keyframe(
            self._h, C.addressof(cv_), cur_mp.ctypes.data_as(I32P), C.addressof(kv), km.ctypes.data_as(I32P),
            af.ctypes.data_as(U8P) if af is not None else None, C.addressof(mv), float(th), int(ORBdist),
            C.byref(n)))
        return n.value

    # SearchByProjection(KeyFrame*, cv::Mat Scw, vpPoints, vpMatched, th)  ORBmatcher.cc:398-520
    def SearchByProjectionSim3(self, kf: FrameView, Scw, points, matched: np.ndarray, mps: MapPoints, th: int) -> int:
        assert matched.dtype == np.int32 and matched.flags.c_contiguous and len(matched) == len(kf.keys)
        S = np.ascontiguousarray(np.asarray(Scw, dtype=np.float32)[:3, :4])
        pts = np.ascontiguousarray(points, dtype=np.int32)
        kv, mv = kf.c(), mps.c()
        n = C.c_int()
        L.check(L.lib().orbx_search_by_projection_sim3(self._h, C.addressof(kv), S.ctypes.data_as(F32P),
                                                       pts.ctypes.data_as(I32P), len(pts),
                                                       matched.ctypes.data_as(I32P), C.addressof(mv), int(th),
                                                       C.byref(n)))
        return n.value

    # Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, th)  ORBmatcher.cc:1067-1221 (search part)
    def Fuse(self, kf: FrameView, points, skip, mps: MapPoints, th: float = 3.0) -> np.ndarray:
        """-> best[k]: the KF keypoint MapPoint points[k] fuses with, or -1."""
        pts = np.ascontiguousarray(points, dtype=np.int32)
        sk = np.ascontiguousarray(skip, dtype=np.uint8)
        best = np.full(max(len(pts), 1), -1, np.int32)
        kv, mv = kf.c(), mps.c()
        L.check(L.lib().orbx_fuse(self._h, C.addressof(kv), pts.ctypes.data_as(I32P), len(pts), sk.ctypes.data_as(U8P),
                                  C.addressof(mv), float(th), best.ctypes.data_as(I32P)))
        return best[:len(pts)].copy()

    # Fuse(KeyFrame* pKF, cv::Mat Scw, vpPoints, th, vpReplacePoint)  ORBmatcher.cc:1226-1352 (search part)
    def FuseSim3(self, kf: FrameView, Scw, points, skip, mps: MapPoints, th: float = 4.0) -> np.ndarray:
        S = np.ascontiguousarray(np.asarray(Scw, dtype=np.float32)[:3, :4])
        pts = np.ascontiguousarray(points, dtype=np.int32)
        sk = np.ascontiguousarray(skip, dtype=np.uint8)
        best = np.full(max(len(pts), 1), -1, np.int32)
        kv, mv = kf.c(), mps.c()
        L.check(L.lib().orbx_fuse_sim3(self._h, C.addressof(kv), S.ctypes.data_as(F32P), pts.ctypes.data_as(I32P),
                                       len(pts), sk.ctypes.data_as(U8P), C.addressof(mv), float(th),
                                       best.ctypes.data_as(I32P)))
        return best[:len(pts)].copy()

    # SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)  ORBmatcher.cc:1361-1602
    def SearchBySim3(self, kf1: FrameView, mp1, kf2: FrameView, mp2, matches12: np.ndarray, mps: MapPoints,
                     s12: float, R12, t12, th: float = 7.5, already1=None, already2=None) -> int:
        """matches12 (int32, KF2 MapPoint ids) updated in place; returns nFound."""
        assert matches12.dtype == np.int32 and matches12.flags.c_contiguous and len(matches12) == len(kf1.keys)
        a1 = np.ascontiguousarray(mp1, dtype=np.int32)
        a2 = np.ascontiguousarray(mp2, dtype=np.int32)
        al1 = None if already1 is None else np.ascontiguousarray(already1, dtype=np.uint8)
        al2 = None if already2 is None else np.ascontiguousarray(already2, dtype=np.uint8)
        R = _f32(R12).reshape(9)
        t = _f32(t12).reshape(3)
        k1, k2, mv = kf1.c(), kf2.c(), mps.c()
        n = C.c_int()
        L.check(L.lib().orbx_search_by_sim3(
            self._h, C.addressof(k1), a1.ctypes.data_as(I32P), None if al1 is None else al1.ctypes.data_as(U8P),
            C.addressof(k2), a2.ctypes.data_as(I32P), None if al2 is None else al2.ctypes.data_as(U8P),
            C.addressof(mv), float(s12), R.ctypes.data_as(F32P), t.ctypes.data_as(F32P), float(th),
            matches12.ctypes.data_as(I32P), C.byref(n)))
        return n.value

    # SearchForTriangulation(KF1, KF2, F12, vMatchedPairs, bOnlyStereo)  ORBmatcher.cc:850-1056
    def SearchForTriangulation(self, kf1: FrameView, kf1_has_mp, fv1, kf2: FrameView, kf2_has_mp, fv2, F12,
                               bOnlyStereo: bool = False):
        m1 = np.ascontiguousarray(kf1_has_mp, dtype=np.uint8)
        m2 = np.ascontiguousarray(kf2_has_mp, dtype=np.uint8)
        n1, o1, i1 = (np.ascontiguousarray(x, dtype=np.int32) for x in fv1)
        n2, o2, i2 = (np.ascontiguousarray(x, dtype=np.int32) for x in fv2)
        F = _f32(F12).reshape(9)
        v1, v2 = kf1.c(), kf2.c()
        pairs = np.zeros((max(len(kf1.keys), 1), 2), dtype=np.int32)
        npairs = C.c_int()
        L.check(L.lib().orbx_search_for_triangulation(
            self._h, C.addressof(v1), m1.ctypes.data_as(U8P), n1.ctypes.data_as(I32P), o1.ctypes.data_as(I32P),
            i1.ctypes.data_as(I32P), len(n1), C.addressof(v2), m2.ctypes.data_as(U8P), n2.ctypes.data_as(I32P),
            o2.ctypes.data_as(I32P), i2.ctypes.data_as(I32P), len(n2), F.ctypes.data_as(F32P),
            1 if bOnlyStereo else 0, pairs.ctypes.data_as(I32P), C.byref(npairs)))
        return pairs[: npairs.value].copy()

    def SearchForTriangulationBatchDevice(self, kfs, cam: FrameView, pairs, F12, cap: int, d_matches12, d_pairs,
                                          d_npairs, bOnlyStereo: bool = False, stream=None) -> None:
        """LocalMapping::CreateNewMapPoints' SearchForTriangulation loop over keyframes in
        HBM (orbx_search_for_triangulation_batch_device): kfs = list of keyframe_device
        records, pairs (P, 2) (KF1, KF2) indices into kfs, F12 (P, 3, 3) host floats,
        cam the shared intrinsics + level tables.  Device outputs d_matches12 (P, cap),
        d_pairs (P, cap, 2), d_npairs (P,) int32; asynchronous."""
        pr = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
        F = _f32(F12).reshape(-1, 9)
        if len(F) != len(pr):
            raise ValueError("one F12 per pair")
        tab = kfs if isinstance(kfs, C.Array) else keyframe_table(kfs)
        cv = cam.c()
        s = None if stream is None else C.c_void_p(getattr(stream, "cuda_stream", stream))
        p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        L.check(L.lib().orbx_search_for_triangulation_batch_device(
            self._h, len(tab) if len(kfs) else 0, C.addressof(tab), C.addressof(cv), len(pr), pr.ctypes.data_as(I32P),
            F.ctypes.data_as(F32P), 1 if bOnlyStereo else 0, int(cap), p(d_matches12), p(d_pairs), p(d_npairs), s))

    # SearchByBoW(KeyFrame* pKF, Frame& F, vpMapPointMatches)  ORBmatcher.cc:228-392
    def SearchByBoWFrame(self, kf: FrameView, kf_mp, kf_fv, f: FrameView, f_fv):
        """-> (nmatches, matches[f.n]: KF MapPoint id per frame keypoint or -1).  kf_mp:
        MapPoint id per KF keypoint, -1 for NULL / isBad().  FeatureVectors as CSR."""
        mp = np.ascontiguousarray(kf_mp, dtype=np.int32)
        n1, o1, i1 = (np.ascontiguousarray(x, dtype=np.int32) for x in kf_fv)
        n2, o2, i2 = (np.ascontiguousarray(x, dtype=np.int32) for x in f_fv)
        v1, v2 = kf.c(), f.c()
        out = np.full(max(len(f.keys), 1), -1, dtype=np.int32)
        nm = C.c_int()
        L.check(L.lib().orbx_search_by_bow_frame(
            self._h, C.addressof(v1), mp.ctypes.data_as(I32P), n1.ctypes.data_as(I32P), o1.ctypes.data_as(I32P),
            i1.ctypes.data_as(I32P), len(n1), C.addressof(v2), n2.ctypes.data_as(I32P), o2.ctypes.data_as(I32P),
            i2.ctypes.data_as(I32P), len(n2), out.ctypes.data_as(I32P), C.byref(nm)))
        return nm.value, out[:len(f.keys)].copy()

    # SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vpMatches12)  ORBmatcher.cc:696-839
    def SearchByBoWKeyFrames(self, kf1: FrameView, mp1, fv1, kf2: FrameView, mp2, fv2):
        """-> (nmatches, matches12[kf1.n]: KF2 MapPoint id per KF1 keypoint or -1)."""
        a1 = np.ascontiguousarray(mp1, dtype=np.int32)
        a2 = np.ascontiguousarray(mp2, dtype=np.int32)
        n1, o1, i1 = (np.ascontiguousarray(x, dtype=np.int32) for x in fv1)
        n2, o2, i2 = (np.ascontiguousarray(x, dtype=np.int32) for x in fv2)
        v1, v2 = kf1.c(), kf2.c()
        out = np.full(max(len(kf1.keys), 1), -1, dtype=np.int32)
        nm = C.c_int()
        L.check(L.lib().orbx_search_by_bow_keyframes(
            self._h, C.addressof(v1), a1.ctypes.data_as(I32P), n1.ctypes.data_as(I32P), o1.ctypes.data_as(I32P),
            i1.ctypes.data_as(I32P), len(n1), C.addressof(v2), a2.ctypes.data_as(I32P), n2.ctypes.data_as(I32P),
            o2.ctypes.data_as(I32P), i2.ctypes.data_as(I32P), len(n2), out.ctypes.data_as(I32P), C.byref(nm)))
        return nm.value, out[:len(kf1.keys)].copy()

    # SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)  ORBmatcher.cc:539-683
    def SearchForInitialization(self, f1: FrameView, f2: FrameView, prev_matched: np.ndarray, windowSize: int = 10):
        """prev_matched: float32 [f1.n, 2], updated in place.  -> (nmatches, vnMatches12)."""
        assert prev_matched.dtype == np.float32 and prev_matched.flags.c_contiguous
        v1, v2 = f1.c(), f2.c()
        out = np.full(max(len(f1.keys), 1), -1, dtype=np.int32)
        nm = C.c_int()
        L.check(L.lib().orbx_search_for_initialization(self._h, C.addressof(v1), C.addressof(v2),
                                                       prev_matched.ctypes.data_as(F32P), out.ctypes.data_as(I32P),
                                                       int(windowSize), C.byref(nm)))
        return nm.value, out[:len(f1.keys)].copy()

    # Frame::ComputeStereoMatches  Frame.cc:673-885
    def ComputeStereoMatches(self, ex_left, left_frame: int, ex_right, right_frame: int, left: FrameView, keys_r,
                             desc_r, maxD: float):
        """mvuRight, mvDepth of a stereo Frame whose left image is frame `left_frame` of
        ex_left's last extraction (mpORBextractorLeft) and right image frame `right_frame`
        of ex_right's (mpORBextractorRight); both pyramids are read (Frame.cc:782-818)."""
        kr = np.ascontiguousarray(keys_r, dtype=L.KEYPOINT_DTYPE)
        dr = np.ascontiguousarray(desc_r, dtype=np.uint8)
        lv = left.c()
        n = len(left.keys)
        ur = np.zeros(max(n, 1), dtype=np.float32)
        dp = np.zeros(max(n, 1), dtype=np.float32)
        L.check(L.lib().orbx_compute_stereo_matches(self._h, ex_left._h, int(left_frame), ex_right._h,
                                                    int(right_frame), C.addressof(lv), kr.ctypes.data,
                                                    dr.ctypes.data_as(U8P), len(kr), float(maxD),
                                                    ur.ctypes.data_as(F32P), dp.ctypes.data_as(F32P)))
        return ur[:n].copy(), dp[:n].copy()

    def ComputeStereoMatchesBatchDevice(self, ex_left, ex_right, d_kps_l, d_desc_l, d_n_l, d_kps_r, d_desc_r, d_n_r,
                                        bf: float, maxD: float, d_u_right, d_depth, left_frame0: int = 0,
                                        right_frame0: int = 0, stream=None) -> None:
        """ComputeStereoMatches for B pairs in HBM (device tensors in the
        orbx_extract_batch_device layout; outputs (B, cap) float32), asynchronous."""
        B, cap = d_desc_l.shape[0], d_desc_l.shape[1]
        s = None if stream is None else C.c_void_p(getattr(stream, "cuda_stream", stream))
        p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        L.check(L.lib().orbx_compute_stereo_matches_batch_device(
            self._h, ex_left._h, int(left_frame0), ex_right._h, int(right_frame0), int(B), p(d_kps_l), p(d_desc_l),
            p(d_n_l), p(d_kps_r), p(d_desc_r), p(d_n_r), int(cap), float(bf), float(maxD), p(d_u_right), p(d_depth),
            s))

    def match_sequence_device(self, d_kps, d_desc, d_n, d_Tcw, d_cur_mp, d_nmatches, scale_factors, fx, fy, cx, cy,
                              width, height, depth: float = 5.0, th: float = 15.0, stream=None) -> None:
        """Batched TrackWithMotionModel matching of frame b against b-1 (device tensors:
        kps (B, cap, 7) int32 words, desc (B, cap, 32) u8, n (B,), Tcw (B, 12) f32,
        outputs cur_mp (B, cap) int32 and nmatches (B,) int32)."""
        B, cap = d_desc.shape[0], d_desc.shape[1]
        sf = _f32(scale_factors)
        s = None if stream is None else C.c_void_p(getattr(stream, "cuda_stream", stream))
        L.check(L.lib().orbx_match_sequence_device(
            self._h, B, C.c_void_p(d_kps.data_ptr()), C.c_void_p(d_desc.data_ptr()), C.c_void_p(d_n.data_ptr()),
            cap, C.c_void_p(d_Tcw.data_ptr()), fx, fy, cx, cy, 0.0, float(width), 0.0, float(height),
            sf.ctypes.data_as(F32P), len(sf), depth, th, C.c_void_p(d_cur_mp.data_ptr()),
            C.c_void_p(d_nmatches.data_ptr()), s))

    def match_sequence_device_ex(self, d_kps, d_desc, d_n, d_Tcw, d_cur_mp, d_nmatches, scale_factors, fx, fy, cx,
                                 cy, width, height, th: float = 15.0, mono: bool = True, bf: float = 0.0,
                                 b: float = 0.0, d_u_right=None, d_mp_pos=None, d_has_mp=None, depth: float = 5.0,
                                 global_ids: bool = False, d_mp_obs=None, retry_below: int = 0,
                                 bounds=None, stream=None) -> None:
        """orbx_match_sequence_device_ex: TrackWithMotionModel's SearchByProjection(frame b,
        frame b-1, th, mono) for every b >= 1 of a device sequence, stereo included
        (d_u_right (B, cap) f32), LastFrame MapPoints at d_mp_pos (B, cap, 3) f32 (or at
        `depth` on the keypoint rays), d_has_mp (B, cap) u8 masking keypoints without one,
        d_mp_obs (B, cap) i32 their Observations() (global ids; default: all > 0);
        retry_below: TrackWithMotionModel's retry at 2*th of the pairs with fewer matches
        (Tracking.cc:988-994: 20; 0 = none); bounds: (mnMinX, mnMaxX, mnMinY, mnMaxY)
        (default: the image, 0..width x 0..height)."""
        B, cap = d_desc.shape[0], d_desc.shape[1]
        sf = _f32(scale_factors)
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        q = L.Sequence()
        q.batch, q.cap = B, cap
        q.kps, q.desc, q.n, q.Tcw = ptr(d_kps), ptr(d_desc), ptr(d_n), ptr(d_Tcw)
        q.u_right, q.mp_pos, q.has_mp = ptr(d_u_right), ptr(d_mp_pos), ptr(d_has_mp)
        q.depth, q.fx, q.fy, q.cx, q.cy, q.bf, q.b = depth, fx, fy, cx, cy, bf, b
        q.min_x, q.max_x, q.min_y, q.max_y = (0.0, float(width), 0.0, float(height)) if bounds is None \
            else tuple(float(x) for x in bounds)
        q.nlevels = len(sf)
        q.scale_factors = sf.ctypes.data_as(F32P)
        q.th, q.mono, q.global_ids = th, 1 if mono else 0, 1 if global_ids else 0
        q.cur_mp, q.nmatches = ptr(d_cur_mp), ptr(d_nmatches)
        q.mp_obs = ptr(d_mp_obs)
        q.retry_below = int(retry_below)
        s = None if stream is None else C.c_void_p(getattr(stream, "cuda_stream", stream))
        L.check(L.lib().orbx_match_sequence_device_ex(self._h, C.byref(q), s))

    def search_local_points_device(self, mps: dict, d_kps, d_desc, d_n, d_Tcw, local_off, d_local_ids, d_frame_mp,
                                   d_nmatches, scale_factors, fx, fy, cx, cy, width, height, th: float = 1.0,
                                   viewing_cos_limit: float = 0.5, bf: float = 0.0, d_u_right=None,
                                   stream=None) -> None:
        """orbx_search_local_points_device: Tracking::SearchLocalPoints (IsInFrustum +
        SearchByProjection(F, vpLocalMapPoints, th)) for every frame of a device batch.
        mps: device tensors pos (n, 3) f32, desc (n, 32) u8, normal (n, 3) f32,
        max_distance / min_distance (n,) f32, observations (n,) i32, optional bad (n,) u8;
        local_off (B + 1) host ints, d_local_ids device i32; d_frame_mp (B, cap) i32 in/out,
        d_nmatches (B,) i32 out.  Asynchronous."""
        B, cap = d_desc.shape[0], d_desc.shape[1]
        ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
        mv = L.MapPointsDevice()
        mv.n = int(mps["pos"].shape[0])
        mv.pos, mv.desc, mv.normal = ptr(mps["pos"]), ptr(mps["desc"]), ptr(mps["normal"])
        mv.max_distance, mv.min_distance = ptr(mps["max_distance"]), ptr(mps["min_distance"])
        mv.observations, mv.bad = ptr(mps["observations"]), ptr(mps.get("bad"))
        sf = _f32(scale_factors)
        off = np.ascontiguousarray(local_off, dtype=np.int32)
        if len(off) != B + 1:
            raise ValueError("local_off needs batch + 1 entries")
        q = L.LocalMapBatch()
        q.batch, q.cap = B, cap
        q.kps, q.desc, q.n, q.u_right, q.Tcw = ptr(d_kps), ptr(d_desc), ptr(d_n), ptr(d_u_right), ptr(d_Tcw)
        q.fx, q.fy, q.cx, q.cy, q.bf = fx, fy, cx, cy, bf
        q.min_x, q.max_x, q.min_y, q.max_y = 0.0, float(width), 0.0, float(height)
        q.nlevels = len(sf)
        q.scale_factors = sf.ctypes.data_as(F32P)
        q.local_off = off.ctypes.data_as(I32P)
        q.local_ids = ptr(d_local_ids)
        q.th, q.viewing_cos_limit = th, viewing_cos_limit
        q.frame_mp, q.nmatches = ptr(d_frame_mp), ptr(d_nmatches)
        s = None if stream is None else C.c_void_p(getattr(stream, "cuda_stream", stream))
        L.check(L.lib().orbx_search_local_points_device(self._h, C.byref(mv), C.byref(q), s))

    def set_timing(self, enable: bool = True) -> None:
        L.check(L.lib().orbx_matcher_set_timing(self._h, 1 if enable else 0))

    def set_footprint(self, mode) -> None:
        """Search-kernel footprint of match_sequence_device (orbx_matcher_set_footprint):
        0 / False = one 1024-thread workgroup per problem, 1 / True = 256 threads with
        global query state, 2 = split into grid / score / commit launches, 3 = one wave
        per problem, 4 = lean (1024 threads, only the grid and the claims in LDS)."""
        L.check(L.lib().orbx_matcher_set_footprint(self._h, int(mode)))

    def last_ms(self) -> float:
        t = C.c_float()
        L.check(L.lib().orbx_matcher_last_ms(self._h, C.byref(t)))
        return t.value

    def score_windows(self, qdesc, tdesc, tlevel, cand_off, cand, tie_last: bool = False) -> dict:
        """Batched candidate scoring (best / second-best Hamming) on the GPU."""
        q = np.ascontiguousarray(qdesc, dtype=np.uint8)
        t = np.ascontiguousarray(tdesc, dtype=np.uint8)
        lv = np.ascontiguousarray(tlevel, dtype=np.int32)
        off = np.ascontiguousarray(cand_off, dtype=np.int32)
        c = np.ascontiguousarray(cand, dtype=np.int32)
        nq = len(off) - 1
        out = {k: np.zeros(nq, dtype=np.int32) for k in
               ("best_idx", "best_dist", "best_level", "second_dist", "second_level")}
        L.check(L.lib().orbx_window_match(self.device, L.u8ptr(q), nq, L.u8ptr(t), len(t), L.i32ptr(lv),
                                          L.i32ptr(off), L.i32ptr(c), 1 if tie_last else 0,
                                          *(L.i32ptr(out[k]) for k in ("best_idx", "best_dist", "best_level",
                                                                       "second_dist", "second_level"))))
        return out


def create_mappoints_device(d_kps, d_n, d_Tcw, scale_factors, fx, fy, cx, cy, out: dict, d_depth=None,
                            const_depth: float = 0.0, stream=None) -> None:
    """orbx_create_mappoints_device: the MapPoints of B frames (id b*cap + i) into the device
    tensors of `out` -- pos / normal (B*cap, 3) f32, max_distance / min_distance (B*cap,)
    f32, observations (B*cap,) i32, bad (B*cap,) u8.  Asynchronous."""
    B, cap = d_kps.shape[0], d_kps.shape[1]
    sf = _f32(scale_factors)
    ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
    s = None if stream is None else C.c_void_p(getattr(stream, "cuda_stream", stream))
    L.check(L.lib().orbx_create_mappoints_device(
        B, ptr(d_kps), ptr(d_n), cap, ptr(d_depth), float(const_depth), ptr(d_Tcw), fx, fy, cx, cy,
        sf.ctypes.data_as(F32P), len(sf), ptr(out["pos"]), ptr(out["normal"]), ptr(out["max_distance"]),
        ptr(out["min_distance"]), ptr(out["observations"]), ptr(out["bad"]), s))


def update_last_frame_device(d_kps, d_n, d_depth, d_Tcw, fx, fy, cx, cy, th_depth, out: dict, d_obs_in=None,
                             d_pos_in=None, stream=None) -> None:
    """orbx_update_last_frame_device: Tracking::UpdateLastFrame's temporal MapPoints for B
    stereo LastFrames (device tensors; out: mp_obs (B, cap) i32, mp_pos (B, cap, 3) f32,
    has_mp (B, cap) u8, e.g. from last_frame_table).  Asynchronous."""
    B, cap = d_kps.shape[0], d_kps.shape[1]
    ptr = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
    s = None if stream is None else C.c_void_p(getattr(stream, "cuda_stream", stream))
    L.check(L.lib().orbx_update_last_frame_device(
        B, ptr(d_kps), ptr(d_n), cap, ptr(d_depth), ptr(d_Tcw), fx, fy, cx, cy, float(th_depth), ptr(d_obs_in),
        ptr(d_pos_in), ptr(out["mp_obs"]), ptr(out["mp_pos"]), ptr(out["has_mp"]), s))


def last_frame_table(B: int, cap: int, device) -> dict:
    """Device tensors for update_last_frame_device's outputs."""
    import torch
    return {"mp_obs": torch.empty((B, cap), dtype=torch.int32, device=device),
            "mp_pos": torch.empty((B, cap, 3), dtype=torch.float32, device=device),
            "has_mp": torch.empty((B, cap), dtype=torch.uint8, device=device)}


def mappoint_table(B: int, cap: int, device) -> dict:
    """Device tensors for create_mappoints_device / search_local_points_device (id b*cap + i)."""
    import torch
    f32 = dict(dtype=torch.float32, device=device)
    N = B * cap
    return {"pos": torch.empty((N, 3), **f32), "normal": torch.empty((N, 3), **f32),
            "max_distance": torch.empty((N,), **f32), "min_distance": torch.empty((N,), **f32),
            "observations": torch.empty((N,), dtype=torch.int32, device=device),
            "bad": torch.empty((N,), dtype=torch.uint8, device=device)}


def ComputeDistinctiveDescriptors(off, desc, device: int = 0):
    """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:295-360) for many MapPoints:
    MapPoint k's observation descriptors are desc[off[k]:off[k+1]].  -> (best index per
    MapPoint or -1, chosen descriptors (nmp, 32))."""
    o = np.ascontiguousarray(off, dtype=np.int32)
    d = np.ascontiguousarray(desc, dtype=np.uint8).reshape(-1, 32)
    nmp = len(o) - 1
    best = np.full(max(nmp, 1), -1, np.int32)
    out = np.zeros((max(nmp, 1), 32), np.uint8)
    L.check(L.lib().orbx_compute_distinctive_descriptors(device, nmp, o.ctypes.data_as(I32P), d.ctypes.data_as(U8P),
                                                         best.ctypes.data_as(I32P), out.ctypes.data_as(U8P)))
    return best[:nmp].copy(), out[:nmp].copy()
