"""DBoW2 vocabulary mirror: ``ORBVocabulary`` (= ``DBoW2::TemplatedVocabulary<FORB::
TDescriptor, FORB>``, include/ORBVocabulary.h) on the HIP tree walk in liborbx.so.

Method names follow the reference: ``loadFromTextFile`` (TemplatedVocabulary.h:
1338-1424), ``transform`` (1127-1186 for a frame, 1220-1259 per feature), ``size``,
``getBranchingFactor``, ``getDepthLevels``, ``getScoringType``, ``getWeightingType``.
``BowVector`` / ``FeatureVector`` come back as dicts ordered by key, like the
reference's ``std::map`` s.
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np

from . import _lib as L

I32P = C.POINTER(C.c_int32)
DP = C.POINTER(C.c_double)

# BowVector.h enums
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = range(6)
TF_IDF, TF, IDF, BINARY = range(4)

MAX_FEATURES = 8192  # per frame in one transform call


class ORBVocabulary:
    def __init__(self, device: int = 0):
        self.device = int(device)
        self._h = None
        self._destroy = L.lib().orbx_vocabulary_destroy  # held: module globals may be gone at exit
        L.track(self)

    def close(self) -> None:
        """Release the vocabulary (orbx_vocabulary_destroy); idempotent."""
        self._release()

    def __del__(self, _finalizing=sys.is_finalizing):
        if not _finalizing():
            self._release()

    def _release(self):
        if getattr(self, "_h", None):
            self._destroy(self._h)
            self._h = None

    # -- loading ------------------------------------------------------------------
    def loadFromTextFile(self, filename: str) -> bool:
        """True on success; False (the reference's return) on a rejected file."""
        self._release()
        h = C.c_void_p()
        rc = L.lib().orbx_vocabulary_load_text_file(str(filename).encode(), self.device, C.byref(h))
        if rc == L.ORBX_ERR_ARG:
            return False
        L.check(rc)
        self._h = h
        return True

    def loadFromText(self, text: str | bytes) -> bool:
        self._release()
        b = text.encode() if isinstance(text, str) else bytes(text)
        h = C.c_void_p()
        rc = L.lib().orbx_vocabulary_load_text(b, len(b), self.device, C.byref(h))
        if rc == L.ORBX_ERR_ARG:
            return False
        L.check(rc)
        self._h = h
        return True

    def _info(self):
        if not self._h:
            raise L.OrbxError(L.ORBX_ERR_STATE, "vocabulary not loaded")
        v = [C.c_int() for _ in range(6)]
        L.check(L.lib().orbx_vocabulary_info(self._h, *[C.byref(x) for x in v]))
        return [x.value for x in v]

    def getBranchingFactor(self) -> int:
        return self._info()[0]

    def getDepthLevels(self) -> int:
        return self._info()[1]

    def getScoringType(self) -> int:
        return self._info()[2]

    def getWeightingType(self) -> int:
        return self._info()[3]

    def nodes(self) -> int:
        return self._info()[4]

    def size(self) -> int:
        return self._info()[5]

    def empty(self) -> bool:
        return self.size() == 0

    @property
    def stream(self) -> int:
        return L.lib().orbx_vocabulary_stream(self._h)

    # -- transform ----------------------------------------------------------------
    def transform_features(self, desc: np.ndarray, levelsup: int = 0):
        """Per-descriptor transform(feature, word_id, weight, nid, levelsup): returns
        (word int32, weight float64, node int32) arrays."""
        d = np.ascontiguousarray(desc, dtype=np.uint8).reshape(-1, 32)
        n = len(d)
        w = np.zeros(n, np.int32)
        wt = np.zeros(n, np.float64)
        nd = np.zeros(n, np.int32)
        L.check(L.lib().orbx_vocabulary_transform_features(self._h, L.u8ptr(d), n, int(levelsup), w.ctypes.data_as(I32P),
                                                           wt.ctypes.data_as(DP), nd.ctypes.data_as(I32P)))
        return w, wt, nd

    def transform_arrays(self, desc: np.ndarray, levelsup: int = 4):
        """transform(features, BowVector, FeatureVector, levelsup) as flat arrays:
        (bow_word, bow_value, fv_node, fv_off, fv_idx)."""
        d = np.ascontiguousarray(desc, dtype=np.uint8).reshape(-1, 32)
        n = len(d)
        cap = max(n, 1)
        bw = np.zeros(cap, np.int32)
        bv = np.zeros(cap, np.float64)
        fn = np.zeros(cap, np.int32)
        fo = np.zeros(cap + 1, np.int32)
        fi = np.zeros(cap, np.int32)
        nb, nf = C.c_int(), C.c_int()
        L.check(L.lib().orbx_vocabulary_transform(self._h, L.u8ptr(d), n, int(levelsup), bw.ctypes.data_as(I32P),
                                                  bv.ctypes.data_as(DP), C.byref(nb), fn.ctypes.data_as(I32P),
                                                  fo.ctypes.data_as(I32P), fi.ctypes.data_as(I32P), C.byref(nf)))
        nb, nf = nb.value, nf.value
        return bw[:nb], bv[:nb], fn[:nf], fo[:nf + 1], fi[:fo[nf]]

    def transform(self, desc: np.ndarray, levelsup: int = 4):
        """-> (BowVector {word: value}, FeatureVector {node: [feature indices]})."""
        bw, bv, fn, fo, fi = self.transform_arrays(desc, levelsup)
        bow = {int(w): float(v) for w, v in zip(bw, bv)}
        fv = {int(nd): fi[fo[j]:fo[j + 1]].tolist() for j, nd in enumerate(fn)}
        return bow, fv

    def transform_batch_device(self, desc, n, cap: int, levelsup: int, out: dict, stream=None,
                               feat_word=None, feat_node=None):
        """Batched device transform over torch tensors (layout of
        orbx_extract_batch_device).  `out` holds bow_word, bow_value, nbow, fv_node,
        fv_off, fv_idx, nfv device tensors (see include/orbx.h)."""
        def p(t):
            return C.c_void_p(t.data_ptr()) if t is not None else None

        B = int(n.numel())
        L.check(L.lib().orbx_vocabulary_transform_batch_device(
            self._h, B, p(desc), p(n), int(cap), int(levelsup), p(feat_word), p(feat_node), p(out["bow_word"]),
            p(out["bow_value"]), p(out["nbow"]), p(out["fv_node"]), p(out["fv_off"]), p(out["fv_idx"]),
            p(out["nfv"]), C.c_void_p(stream) if stream else None))

    @staticmethod
    def alloc_batch_outputs(batch: int, cap: int, device="cuda"):
        import torch

        i32 = dict(dtype=torch.int32, device=device)
        return {"bow_word": torch.empty(batch, cap, **i32),
                "bow_value": torch.empty(batch, cap, dtype=torch.float64, device=device),
                "nbow": torch.empty(batch, **i32), "fv_node": torch.empty(batch, cap, **i32),
                "fv_off": torch.empty(batch, cap + 1, **i32), "fv_idx": torch.empty(batch, cap, **i32),
                "nfv": torch.empty(batch, **i32)}

    def set_timing(self, enable: bool = True):
        L.check(L.lib().orbx_vocabulary_set_timing(self._h, 1 if enable else 0))

    def stage_times(self):
        a, b = C.c_float(), C.c_float()
        L.check(L.lib().orbx_vocabulary_stage_times(self._h, C.byref(a), C.byref(b)))
        return {"vocab_walk": a.value, "vocab_frame": b.value}


def save_text(k: int, L_: int, scoring: int, weighting: int, parents, is_leaf, desc, weights) -> str:
    """Text in the saveToTextFile / loadFromTextFile format (TemplatedVocabulary.h:
    1427-1470): header, then one line per non-root node."""
    lines = [f"{k} {L_}  {scoring} {weighting}"]
    for p, lf, d, w in zip(parents, is_leaf, desc, weights):
        # FORB::toString ends with a space; weights print at ostream precision 6 (%g)
        lines.append(f"{int(p)} {int(lf)} " + " ".join(str(int(x)) for x in d) + f"  {float(w):g}")
    return "\n".join(lines) + "\n"
