"""Scene bookkeeping around bundle adjustment — host
mirror over include/sfmx_scene.h:

* ``find_3d2d_matches``: ``Scene::find3d2dMatches`` (common/Scene.cpp:369-424),
  a GPU hash join (csrc/scene.hip) instead of the reference's nested scans;
* ``ba_observations_from_origins``: the Ceres problem's observation arrays
  (BundleAdjustment.cpp:50-91), O(n) native host code.

Point-cloud origins are flattened per point (PointcloudElement::getOriginPoints,
Scene.cpp:162-185): ``origin_offsets[n_points+1]``, ``origin_shot``,
``origin_xy`` (n x 2 float64, cv::Point2d).
"""
from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from ._lib import lib, check
from .matching import DMATCH_DTYPE


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def find_3d2d_matches(keypoints: Sequence[np.ndarray], pairs, matches, offsets, origin_offsets, origin_shot,
                      origin_xy, shot: int, device: int = 0, stream: int = 0):
    """-> (keypoint index in `shot` per origin record or -1, pair index or -1,
    matched keypoint positions n x 2 float32 (NaN where none))."""
    kps = [np.ascontiguousarray(k, np.float32).reshape(-1, 2) for k in keypoints]
    nkp = np.array([len(k) for k in kps], np.int32)
    ptrs = (C.c_void_p * max(len(kps), 1))(*[k.ctypes.data for k in kps])
    pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
    m = np.ascontiguousarray(matches, DMATCH_DTYPE)
    off = np.ascontiguousarray(offsets, np.int64)
    oo = np.ascontiguousarray(origin_offsets, np.int64)
    os_ = np.ascontiguousarray(origin_shot, np.int32)
    oxy = np.ascontiguousarray(origin_xy, np.float64).reshape(-1, 2)
    n = int(oo[-1])
    okp = np.zeros(max(n, 1), np.int32)
    opr = np.zeros(max(n, 1), np.int32)
    oxy_out = np.zeros((max(n, 1), 2), np.float32)
    check(lib.sfmx_find_3d2d_matches(ptrs, _p(nkp, C.c_int32), len(kps), _p(pairs, C.c_int32), len(pairs),
                                     m.ctypes.data if len(m) else None, off.ctypes.data, oo.ctypes.data, len(oo) - 1,
                                     os_.ctypes.data if n else None, oxy.ctypes.data if n else None, int(shot), 0,
                                     int(device), stream or None, okp.ctypes.data, opr.ctypes.data, oxy_out.ctypes.data),
          "sfmx_find_3d2d_matches")
    return okp[:n], opr[:n], oxy_out[:n]


def find_3d2d_matches_device(keypoint_ptrs, n_keypoints, pairs, matches_ptr, offsets_ptr, origin_offsets_ptr,
                             n_points, origin_shot_ptr, origin_xy_ptr, shot, out_kp_ptr, out_pair_ptr, out_xy_ptr=0,
                             device: int = 0, stream: int = 0):
    """Same with every array resident on `device` (pairs stays host)."""
    nkp = np.ascontiguousarray(n_keypoints, np.int32)
    ptrs = (C.c_void_p * max(len(nkp), 1))(*keypoint_ptrs)
    pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
    check(lib.sfmx_find_3d2d_matches(ptrs, _p(nkp, C.c_int32), len(nkp), _p(pairs, C.c_int32), len(pairs), matches_ptr,
                                     offsets_ptr, origin_offsets_ptr, int(n_points), origin_shot_ptr, origin_xy_ptr,
                                     int(shot), 1, int(device), stream or None, out_kp_ptr, out_pair_ptr,
                                     out_xy_ptr or None), "sfmx_find_3d2d_matches")


def last_kernel_ms() -> float:
    return float(lib.sfmx_find_3d2d_last_kernel_ms())


def ba_observations_from_origins(origin_offsets, origin_shot, origin_xy, n_shots: int):
    """-> dict(obs_point, obs_cam, obs_xy, pose_of_shot, shot_of_pose): the
    sfmx_ba_problem observation arrays in AddResidualBlock order
    (BundleAdjustment.cpp:50-91), poses in first-appearance order."""
    oo = np.ascontiguousarray(origin_offsets, np.int64)
    os_ = np.ascontiguousarray(origin_shot, np.int32)
    oxy = np.ascontiguousarray(origin_xy, np.float64).reshape(-1, 2)
    n = int(oo[-1])
    op = np.zeros(max(n, 1), np.int32)
    oc = np.zeros(max(n, 1), np.int32)
    ox = np.zeros((max(n, 1), 2))
    pos = np.zeros(max(n_shots, 1), np.int32)
    sop = np.zeros(max(n_shots, 1), np.int32)
    npose = C.c_int32(0)
    check(lib.sfmx_ba_observations_from_origins(_p(oo, C.c_int64), len(oo) - 1, _p(os_, C.c_int32),
                                                _p(oxy, C.c_double), int(n_shots), _p(op, C.c_int32), _p(oc, C.c_int32),
                                                _p(ox, C.c_double), _p(pos, C.c_int32), _p(sop, C.c_int32),
                                                C.byref(npose)), "sfmx_ba_observations_from_origins")
    return dict(obs_point=op[:n], obs_cam=oc[:n], obs_xy=ox[:n], pose_of_shot=pos[:n_shots],
                shot_of_pose=sop[:npose.value])
