"""Host-side mirror of the reference's feature-matching plugin interface.

Reference (paths relative to brunothg/sfm-mvs-pipeline/src/photogrammetrie):
  * ``IFeatureMatchingStrategy::calculateShotMatches(scene, matcher, out)``  sfm/IFeatureMatchingStrategy.h:45-46
  * ``UnorderedFeatureMatchingStrategy``   sfm/UnorderedFeatureMatchingStrategy.cpp:27-90
  * ``VideoFeatureMatchingStrategy(seq)``  sfm/VideoFeatureMatchingStrategy.cpp:27-100 (seq < 2 -> invalid_argument, :32-35)
  * ``GridFeatureMatchingStrategy(seq, rowLength)`` sfm/GridFeatureMatchingStrategy.cpp:24-144 (:32-44)
  * ``ShotMatches`` (left, right, DMatch list, homographyInlierRatio = -1)   common/Scene.h:35-58
  * ``SfM::calculateShotMatches`` filters (distinct, min match count)       sfm/SfM.cpp:542-575
  * ``cv::BFMatcher::create(NORM_L2 | NORM_HAMMING)`` -> :class:`BFMatcher`  cli/PhotogrammetrieCli.cpp:359-392

Same names, argument meaning and error behaviour (``std::invalid_argument`` ->
``ValueError``).  All matching arithmetic runs in the HIP kernels behind the C
ABI (libsfmx.so); this module only marshals buffers.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import lib, check, sfmx_desc, SFMX_NORM_L2, SFMX_NORM_HAMMING, SFMX_32F, SFMX_8U

NORM_L2 = SFMX_NORM_L2            # == cv::NORM_L2
NORM_HAMMING = SFMX_NORM_HAMMING  # == cv::NORM_HAMMING
LOWE_RATIO = 0.7                  # UnorderedFeatureMatchingStrategy.cpp:55 (hard-coded, not a flag)

DMATCH_DTYPE = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"), ("distance", "<f4")])


def _i32p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def _i64p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int64))


# ---- a1: pair enumeration -------------------------------------------------

def _pairs(fn, *args) -> np.ndarray:
    n = check(fn(*args, None, 0), fn.__name__)
    out = np.empty((n, 2), dtype=np.int32)
    if n:
        check(fn(*args, _i32p(out), n), fn.__name__)
    return out


def pairs_unordered(n_images: int) -> np.ndarray:
    return _pairs(lib.sfmx_pairs_unordered, n_images)


def pairs_video(n_images: int, sequence_length: int) -> np.ndarray:
    return _pairs(lib.sfmx_pairs_video, n_images, sequence_length)


def pairs_grid(n_images: int, sequence_length: int, row_length: int, grid_mode: int = 1) -> np.ndarray:
    return _pairs(lib.sfmx_pairs_grid, n_images, sequence_length, row_length, grid_mode)


# ---- matcher (cv::DescriptorMatcher stand-in) -------------------------------

class BFMatcher:
    """Exact brute-force 2-NN matcher on one MI355X (``cv::BFMatcher::create(norm)``)."""

    def __init__(self, norm: int = NORM_L2, device: int = 0):
        if norm not in (NORM_L2, NORM_HAMMING):
            raise ValueError("norm must be NORM_L2 or NORM_HAMMING")
        self.norm = norm
        self.device = device
        h = C.c_void_p()
        check(lib.sfmx_matcher_create(device, C.byref(h)), "sfmx_matcher_create")
        self._h = h
        self._n_pairs = 0
        self._keep_alive: list = []

    def close(self):
        if getattr(self, "_h", None):
            lib.sfmx_matcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # descriptors --------------------------------------------------------
    def _descs(self, mats, device_ptrs: bool):
        arr = (sfmx_desc * max(len(mats), 1))()
        keep = []
        for i, m in enumerate(mats):
            if device_ptrs:
                rows, cols = int(m.shape[0]), int(m.shape[1]) if m.dim() == 2 else 0
                typ = SFMX_32F if str(m.dtype) == "torch.float32" else SFMX_8U
                if not m.is_contiguous():
                    raise ValueError("device descriptor tensors must be contiguous")
                arr[i] = sfmx_desc(m.data_ptr() if rows else None, rows, cols, typ, 0)
            else:
                want = np.float32 if self.norm == NORM_L2 else np.uint8
                m = np.ascontiguousarray(m, dtype=want)
                if m.ndim != 2:
                    raise ValueError("descriptor matrices must be 2-D (rows x cols)")
                keep.append(m)
                arr[i] = sfmx_desc(m.ctypes.data if m.shape[0] else None, m.shape[0], m.shape[1],
                                   SFMX_32F if want is np.float32 else SFMX_8U, 0)
        return arr, keep

    def set_images(self, mats: Sequence[np.ndarray], stream: int = 0):
        arr, keep = self._descs(mats, False)
        check(lib.sfmx_matcher_set_images(self._h, arr, len(mats), self.norm, C.c_void_p(stream)),
              "sfmx_matcher_set_images")
        self._n_images = len(mats)

    def set_images_device(self, tensors, stream: int = 0):
        arr, _ = self._descs(tensors, True)
        check(lib.sfmx_matcher_set_images_device(self._h, arr, len(tensors), self.norm, C.c_void_p(stream)),
              "sfmx_matcher_set_images_device")
        self._n_images = len(tensors)

    # matching -----------------------------------------------------------
    def run(self, pairs: np.ndarray, ratio: float = LOWE_RATIO, distinct: bool = False, min_count: int = 0,
            stream: int = 0):
        pairs = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
        self._pairs_buf = pairs
        check(lib.sfmx_matcher_run(self._h, _i32p(pairs), len(pairs), float(ratio), int(bool(distinct)),
                                   int(min_count), C.c_void_p(stream)), "sfmx_matcher_run")
        self._n_pairs = len(pairs)

    def device_results(self):
        """-> (matches_ptr, pair_offsets_ptr, keep_ptr): the packed results left in
        HBM by the last run (sfmx_matcher_device_results), valid until the next run."""
        mp, op, kp = C.c_void_p(), C.c_void_p(), C.c_void_p()
        check(lib.sfmx_matcher_device_results(self._h, C.byref(mp), C.byref(op), C.byref(kp)),
              "sfmx_matcher_device_results")
        return mp.value, op.value, kp.value

    def fetch(self, stream: int = 0):
        """-> (matches[DMATCH_DTYPE], pair_offsets[int64, n_pairs+1], keep[int32, n_pairs])"""
        req = np.zeros(1, np.int64)
        off = np.zeros(self._n_pairs + 1, np.int64)
        keep = np.zeros(max(self._n_pairs, 1), np.int32)
        check(lib.sfmx_matcher_fetch(self._h, None, 0, _i64p(req), _i64p(off), _i32p(keep), C.c_void_p(stream)),
              "sfmx_matcher_fetch")
        out = np.zeros(int(req[0]), DMATCH_DTYPE)
        if len(out):
            check(lib.sfmx_matcher_fetch(self._h, C.c_void_p(out.ctypes.data), len(out), _i64p(req), None, None,
                                         C.c_void_p(stream)), "sfmx_matcher_fetch")
        return out, off, keep[: self._n_pairs]

    def stats(self, stream: int = 0):
        slow = np.zeros(1, np.int64)
        f32 = np.zeros(1, np.int64)
        check(lib.sfmx_matcher_stats(self._h, _i64p(slow), _i64p(f32), C.c_void_p(stream)), "sfmx_matcher_stats")
        return int(slow[0]), int(f32[0])

    def timing(self):
        """-> (main 2-NN kernel ms, whole-run ms) of the last run (HIP events on its stream)."""
        a, b = C.c_float(), C.c_float()
        check(lib.sfmx_matcher_timing(self._h, C.byref(a), C.byref(b)), "sfmx_matcher_timing")
        return a.value, b.value

    def timing_history(self, n):
        """-> (main 2-NN kernel ms, screen ms) arrays of the last min(n, runs, 32) runs, oldest first
        (HIP events of each run; read without a host sync inside the loop that made them)."""
        a = np.zeros(max(n, 1), np.float32)
        b = np.zeros(max(n, 1), np.float32)
        k = check(lib.sfmx_matcher_timing_history(self._h, a.ctypes.data_as(C.POINTER(C.c_float)),
                                                  b.ctypes.data_as(C.POINTER(C.c_float)), int(n)),
                  "sfmx_matcher_timing_history")
        return a[:k].astype(float), b[:k].astype(float)

    def pass_timing(self):
        """-> (screen ms, pass-2 ms) of the last run's two-pass 2-NN launch (screen 0 when single pass)."""
        a, b = C.c_float(), C.c_float()
        check(lib.sfmx_matcher_pass_timing(self._h, C.byref(a), C.byref(b)), "sfmx_matcher_pass_timing")
        return a.value, b.value

    def match_pairs(self, mats, pairs, ratio=LOWE_RATIO, distinct=False, min_count=0):
        self.set_images(mats)
        self.run(pairs, ratio, distinct, min_count)
        return self.fetch()


def match_pairs(mats: Sequence[np.ndarray], pairs: np.ndarray, norm: int = NORM_L2, ratio: float = LOWE_RATIO,
                distinct: bool = False, min_count: int = 0, n_gpus: int = 1):
    """One-shot ``sfmx_match_pairs`` (multi-device capable)."""
    m = BFMatcher.__new__(BFMatcher)
    m.norm = norm
    arr, keep_alive = BFMatcher._descs(m, mats, False)
    pairs = np.ascontiguousarray(pairs, dtype=np.int32).reshape(-1, 2)
    req = np.zeros(1, np.int64)
    off = np.zeros(len(pairs) + 1, np.int64)
    keep = np.zeros(max(len(pairs), 1), np.int32)
    args = (arr, len(mats), _i32p(pairs), len(pairs), norm, float(ratio), int(bool(distinct)), int(min_count),
            int(n_gpus))
    # one call: each query yields at most one match, so sum(rows(left)) always suffices
    cap = int(sum(len(mats[l]) for l in pairs[:, 0])) if len(pairs) else 0
    out = np.zeros(max(cap, 1), DMATCH_DTYPE)
    check(lib.sfmx_match_pairs(*args, C.c_void_p(out.ctypes.data), cap, _i64p(req), _i64p(off), _i32p(keep)),
          "sfmx_match_pairs")
    return out[: int(req[0])], off, keep[: len(pairs)]


# ---- reference plugin interface -------------------------------------------

@dataclass
class Shot:
    """Minimal CameraShot: its image path, the descriptor matrix of its Features
    and (for the homography step) their keypoint positions (n x 2 float32,
    cv::KeyPoint::pt) and the image size (width, height) (CameraShot.h:39-54, :174)."""
    path: str
    descriptors: np.ndarray
    keypoints: Optional[np.ndarray] = None
    image_size: tuple = (0, 0)

    def getImageSize(self):
        return self.image_size


@dataclass
class Scene:
    shots: List[Shot] = field(default_factory=list)

    def getShots(self):
        return self.shots


@dataclass
class ShotMatches:
    """Scene.h:35-58 — left -> queryIdx, right -> trainIdx."""
    left: int
    right: int
    matches: np.ndarray
    homographyInlierRatio: float = -1.0

    def getMatches(self):
        return self.matches

    def getHomographyInlierRatio(self):
        return self.homographyInlierRatio

    def setHomographyInlierRatio(self, r: float):
        self.homographyInlierRatio = r


class IFeatureMatchingStrategy:
    def pairs(self, n_images: int) -> np.ndarray:
        raise NotImplementedError

    def calculateShotMatches(self, scene: Scene, matcher: BFMatcher) -> List[ShotMatches]:
        """One batched GPU pass over every pair of the strategy.  Result order is
        the pair-enumeration order (the reference's order is nondeterministic,
        UnorderedFeatureMatchingStrategy.cpp:76-79)."""
        shots = scene.getShots()
        pairs = self.pairs(len(shots))
        matcher.set_images([s.descriptors for s in shots])
        matcher.run(pairs, LOWE_RATIO)
        m, off, _ = matcher.fetch()
        return [ShotMatches(int(l), int(r), m[off[p]:off[p + 1]].copy()) for p, (l, r) in enumerate(pairs)]


class UnorderedFeatureMatchingStrategy(IFeatureMatchingStrategy):
    def pairs(self, n_images):
        return pairs_unordered(n_images)


class VideoFeatureMatchingStrategy(IFeatureMatchingStrategy):
    def __init__(self, sequenceLength: int):
        self.setSequenceLength(sequenceLength)

    def setSequenceLength(self, n: int):
        if n < 2:
            raise ValueError("sequence length must be >= 2 (self plus one successor)")
        self.sequenceLength = n

    def pairs(self, n_images):
        return pairs_video(n_images, self.sequenceLength)


class GridFeatureMatchingStrategy(IFeatureMatchingStrategy):
    def __init__(self, sequenceLength: int, rowLength: int, grid_mode: int = 1):
        self.setSequenceLength(sequenceLength)
        self.setRowLength(rowLength)
        self.grid_mode = grid_mode

    def setSequenceLength(self, n: int):
        if n < 2:
            raise ValueError("sequence length must be >= 2 (self plus one successor)")
        self.sequenceLength = n

    def setRowLength(self, n: int):
        if n < 1:
            raise ValueError("row length must be >= 1")
        self.rowLength = n

    def pairs(self, n_images):
        return pairs_grid(n_images, self.sequenceLength, self.rowLength, self.grid_mode)


def calculate_shot_matches(scene: Scene, strategy: IFeatureMatchingStrategy, matcher: BFMatcher,
                           distinct: bool = False, min_match_count: int = 20) -> List[ShotMatches]:
    """SfM::calculateShotMatches (SfM.cpp:542-575): strategy pass, optional
    distinct-trainIdx filter, drop pairs with < min_match_count matches
    (setMinMatchCount rejects < 4, SfM.cpp:74-79).  Filters run on the GPU."""
    if min_match_count < 4:
        raise ValueError("minimum match count must be >= 4")
    shots = scene.getShots()
    pairs = strategy.pairs(len(shots))
    matcher.set_images([s.descriptors for s in shots])
    matcher.run(pairs, LOWE_RATIO, distinct, min_match_count)
    m, off, keep = matcher.fetch()
    return [ShotMatches(int(l), int(r), m[off[p]:off[p + 1]].copy())
            for p, (l, r) in enumerate(pairs) if keep[p]]
