"""Per-pair homography RANSAC over the match graph — host mirror of
``SfM::calculateHomography(Scene&)`` (src/photogrammetrie/sfm/SfM.cpp:599-637),
SURVEY.md §8 row f1.  All arithmetic runs in the HIP kernel behind
``sfmx_homography_ratios`` (include/sfmx_homography.h); this module only
marshals buffers.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence

import numpy as np

from ._lib import lib, check
from .matching import DMATCH_DTYPE, Scene, ShotMatches

RANSAC_MAX_ITERS = 2000            # cv::findHomography default
RANSAC_CONFIDENCE = 0.995          # cv::findHomography default
RANSAC_MATCHING_THRESHOLD = -3.0   # SfM.h:50 (negative: absolute pixels)


def _i32(a):
    return np.ascontiguousarray(a, np.int32)


def homography_ratios(keypoints: Sequence[np.ndarray], image_sizes, pairs: np.ndarray, matches: np.ndarray,
                      offsets: np.ndarray, threshold: float = RANSAC_MATCHING_THRESHOLD,
                      max_iters: int = RANSAC_MAX_ITERS, confidence: float = RANSAC_CONFIDENCE,
                      device: int = 0, stream: int = 0) -> np.ndarray:
    """Inlier ratio of cv::findHomography(RANSAC) for every pair (-1: < 4 matches).
    keypoints[i]: (n_i x 2) float32 host array; matches/offsets: packed DMatch
    lists as BFMatcher.fetch returns them."""
    kps = [np.ascontiguousarray(k, np.float32).reshape(-1, 2) for k in keypoints]
    nkp = _i32([len(k) for k in kps])
    sizes = _i32(np.asarray(image_sizes).reshape(-1, 2))
    pairs = _i32(pairs).reshape(-1, 2)
    m = np.ascontiguousarray(matches, DMATCH_DTYPE)
    off = np.ascontiguousarray(offsets, np.int64)
    if len(off) != len(pairs) + 1:
        raise ValueError("offsets must have n_pairs + 1 entries")
    ptrs = (C.c_void_p * max(len(kps), 1))(*[k.ctypes.data for k in kps])
    out = np.full(len(pairs), -1.0)
    check(lib.sfmx_homography_ratios(ptrs, nkp.ctypes.data_as(C.POINTER(C.c_int32)), len(kps),
                                     sizes.ctypes.data_as(C.POINTER(C.c_int32)),
                                     pairs.ctypes.data_as(C.POINTER(C.c_int32)), len(pairs),
                                     m.ctypes.data if len(m) else None, off.ctypes.data, float(threshold),
                                     int(max_iters), float(confidence), 0, int(device), stream or None,
                                     out.ctypes.data_as(C.POINTER(C.c_double))), "sfmx_homography_ratios")
    return out


def homography_ratios_device(keypoint_ptrs: Sequence[int], n_keypoints, image_sizes, pairs: np.ndarray,
                             matches_ptr: int, offsets_ptr: int, threshold: float = RANSAC_MATCHING_THRESHOLD,
                             max_iters: int = RANSAC_MAX_ITERS, confidence: float = RANSAC_CONFIDENCE,
                             device: int = 0, stream: int = 0) -> np.ndarray:
    """Same, with keypoints and match lists already resident on `device`
    (e.g. torch tensors' data_ptr() and sfmx_matcher_device_results)."""
    nkp = _i32(n_keypoints)
    sizes = _i32(np.asarray(image_sizes).reshape(-1, 2))
    pairs = _i32(pairs).reshape(-1, 2)
    ptrs = (C.c_void_p * max(len(nkp), 1))(*keypoint_ptrs)
    out = np.full(len(pairs), -1.0)
    check(lib.sfmx_homography_ratios(ptrs, nkp.ctypes.data_as(C.POINTER(C.c_int32)), len(nkp),
                                     sizes.ctypes.data_as(C.POINTER(C.c_int32)),
                                     pairs.ctypes.data_as(C.POINTER(C.c_int32)), len(pairs), matches_ptr, offsets_ptr,
                                     float(threshold), int(max_iters), float(confidence), 1, int(device),
                                     stream or None, out.ctypes.data_as(C.POINTER(C.c_double))),
          "sfmx_homography_ratios")
    return out


def last_kernel_ms() -> float:
    return float(lib.sfmx_homography_last_kernel_ms())


def calculateHomography(scene: Scene, shot_matches: List[ShotMatches],
                        ransacReprojectionMatchingThreshold: float = RANSAC_MATCHING_THRESHOLD) -> None:
    """SfM::calculateHomography (SfM.cpp:599-637): sets every ShotMatches'
    homographyInlierRatio (pairs with < 4 matches keep -1)."""
    shots = scene.getShots()
    if not shot_matches:
        return
    pairs = np.array([[s.left, s.right] for s in shot_matches], np.int32)
    counts = np.array([len(s.getMatches()) for s in shot_matches], np.int64)
    off = np.concatenate([[0], np.cumsum(counts)])
    m = np.concatenate([np.asarray(s.getMatches(), DMATCH_DTYPE) for s in shot_matches]) if off[-1] else \
        np.zeros(0, DMATCH_DTYPE)
    r = homography_ratios([sh.keypoints for sh in shots], [sh.getImageSize() for sh in shots], pairs, m, off,
                          ransacReprojectionMatchingThreshold)
    for s, v in zip(shot_matches, r):
        if v >= 0:
            s.setHomographyInlierRatio(float(v))
