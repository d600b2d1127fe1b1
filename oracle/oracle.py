"""sfmx ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper over liboracle.so (oracle/match_oracle.cpp, flann_oracle.cpp, ba_oracle.cpp):
the CPU restatement of the reference's matching / bundle-adjustment semantics.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / CPU baseline — never as the
thing measured or shipped.  Parity status: unpinned against the reference
itself (it cannot be built here and ships no fixtures).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

DMATCH_DTYPE = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"), ("distance", "<f4")])


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load():
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    vp, i32p, i64p = C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int64)
    f32p = C.POINTER(C.c_float)
    lib.orc_knn2_l2.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, i32p, f32p]
    lib.orc_knn2_hamming.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, i32p, f32p]
    lib.orc_match_pair.restype = C.c_int64
    lib.orc_match_pair.argtypes = [C.c_int, vp, C.c_int, vp, C.c_int, C.c_int, C.c_double, vp]
    lib.orc_match_pairs.argtypes = [C.c_int, C.POINTER(vp), i32p, C.c_int, i32p, C.c_int, C.c_double, vp, i64p,
                                    i64p, C.c_int]
    for n in ("orc_pairs_unordered",):
        getattr(lib, n).restype = C.c_int64
        getattr(lib, n).argtypes = [C.c_int, i32p]
    lib.orc_pairs_video.restype = C.c_int64
    lib.orc_pairs_video.argtypes = [C.c_int, C.c_int, i32p]
    lib.orc_pairs_grid.restype = C.c_int64
    lib.orc_pairs_grid.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, i32p]
    lib.orc_filter_matches.argtypes = [vp, i64p, i64p, C.c_int, C.c_int, C.c_int, i32p]
    lib.orc_flann_match_pairs.argtypes = [C.c_int, C.POINTER(vp), i32p, C.c_int, i32p, C.c_int, C.c_double, vp,
                                          i64p, i64p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64]
    lib.orc_homography_ratios.argtypes = [C.POINTER(vp), i32p, i32p, C.c_int, vp, i64p, C.c_double, C.c_int,
                                          C.c_double, C.POINTER(C.c_double), C.c_int]
    lib.orc_find_3d2d_matches.argtypes = [C.POINTER(vp), i32p, C.c_int, vp, i64p, i64p, C.c_int, i32p,
                                          C.POINTER(C.c_double), C.c_int, i32p, i32p, C.c_int]
    lib.orc_ba_observations.argtypes = [i64p, C.c_int, i32p, C.POINTER(C.c_double), C.c_int, i32p, i32p,
                                        C.POINTER(C.c_double), i32p]
    lib.orc_undistort.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.orc_undistort_batch.argtypes = [C.POINTER(vp), C.POINTER(vp), i32p, i32p, i32p, C.POINTER(C.c_double),
                                        C.POINTER(C.c_double), C.c_int, C.c_int]
    lib.orc_sift.argtypes = [vp, C.c_int, C.c_int, C.c_int64, C.c_int, C.c_int, C.c_double, C.c_double, C.c_double,
                             vp, vp, C.c_int]
    lib.orc_sift_batch.argtypes = [C.POINTER(vp), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_double, C.c_double,
                                   C.c_double, vp, vp, C.c_int, i32p, C.c_int]
    lib.orc_sift_set_arith.restype = C.c_int
    lib.orc_sift_set_arith.argtypes = [C.c_int]
    lib.orc_homography_set_arith.restype = C.c_int
    lib.orc_homography_set_arith.argtypes = [C.c_int]
    lib.orc_orb.restype = C.c_int
    lib.orc_orb.argtypes = [vp, C.c_int, C.c_int, C.c_int64, C.c_int, C.c_float, C.c_int, C.c_int, C.c_int, vp, vp,
                            C.c_int]
    lib.orc_orb_batch.restype = None
    lib.orc_orb_batch.argtypes = [C.POINTER(vp), C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, C.c_int, i32p, C.c_int]
    lib.orc_orb_stage.restype = C.c_int64
    lib.orc_orb_stage.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_float, C.c_int, C.c_int, vp, i32p]
    lib.orc_first_sqrt_collision.restype = C.c_int64
    lib.orc_first_sqrt_collision.argtypes = [C.c_int64]
    return lib


lib = _load()


def _ptr(a, t=C.c_int32):
    return a.ctypes.data_as(C.POINTER(t))


def knn2(q: np.ndarray, t: np.ndarray):
    """cv::BFMatcher knnMatch(q, t, k=2) restated: -> (idx[nq,2], dist[nq,2], n_neighbours)."""
    l2 = q.dtype == np.float32
    q = np.ascontiguousarray(q)
    t = np.ascontiguousarray(t)
    nq, nt = q.shape[0], t.shape[0]
    dim = q.shape[1] if q.ndim == 2 else t.shape[1]
    idx = np.empty((nq, 2), np.int32)
    dist = np.empty((nq, 2), np.float32)
    fn = lib.orc_knn2_l2 if l2 else lib.orc_knn2_hamming
    nn = fn(q.ctypes.data, nq, t.ctypes.data, nt, dim, _ptr(idx), _ptr(dist, C.c_float))
    return idx, dist, nn


def match_pair(q: np.ndarray, t: np.ndarray, ratio: float = 0.7) -> np.ndarray:
    l2 = q.dtype == np.float32
    q = np.ascontiguousarray(q)
    t = np.ascontiguousarray(t)
    dim = q.shape[1] if q.ndim == 2 and q.shape[0] else t.shape[1]
    out = np.zeros(max(q.shape[0], 1), DMATCH_DTYPE)
    n = lib.orc_match_pair(0 if l2 else 1, q.ctypes.data, q.shape[0], t.ctypes.data, t.shape[0], dim, ratio,
                           out.ctypes.data)
    return out[:n].copy()


def _pair_batch(imgs, pairs, call):
    """Shared packing of the pair-parallel batch entry points: per-pair output
    slots at the cumulative left-image row counts, then compacted in pair order
    -> (matches, pair_offsets[n+1]) packed like sfmx_matcher_fetch."""
    l2 = imgs[0].dtype == np.float32
    imgs = [np.ascontiguousarray(m) for m in imgs]
    dim = imgs[0].shape[1]
    pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
    rows = np.array([m.shape[0] for m in imgs], np.int32)
    ptrs = (C.c_void_p * len(imgs))(*[m.ctypes.data for m in imgs])
    base = np.zeros(len(pairs), np.int64)
    if len(pairs):
        base[1:] = np.cumsum(rows[pairs[:-1, 0]])
    cap = int(rows[pairs[:, 0]].sum()) if len(pairs) else 0
    tmp = np.zeros(max(cap, 1), DMATCH_DTYPE)
    counts = np.zeros(max(len(pairs), 1), np.int64)
    call(0 if l2 else 1, ptrs, _ptr(rows), dim, _ptr(pairs), len(pairs), tmp.ctypes.data,
         _ptr(base, C.c_int64), _ptr(counts, C.c_int64))
    off = np.zeros(len(pairs) + 1, np.int64)
    off[1:] = np.cumsum(counts[: len(pairs)])
    out = np.concatenate([tmp[base[p]: base[p] + counts[p]] for p in range(len(pairs))]) if len(pairs) else tmp[:0]
    return out, off


def match_pairs(imgs, pairs: np.ndarray, ratio: float = 0.7, nthreads: int = 0):
    """Pair-parallel exact BF (OpenMP over pairs, as the reference) ->
    (matches, pair_offsets[n+1]) packed like sfmx_matcher_fetch."""
    return _pair_batch(imgs, pairs, lambda t, ptrs, rows, dim, pr, n, out, base, counts: lib.orc_match_pairs(
        t, ptrs, rows, dim, pr, n, ratio, out, base, counts, nthreads))


def flann_match_pairs(imgs, pairs: np.ndarray, ratio: float = 0.7, nthreads: int = 0, trees: int = 5,
                      checks: int = 100, tables: int = 6, key_size: int = 12, seed: int = 0x5F3D):
    """FLANN-style approximate matcher (oracle/flann_oracle.cpp): per-pair
    KDTreeIndex(trees) + SearchParams(checks) for f32 rows, LshIndex(tables,
    key_size, 1) for u8 rows, index rebuilt per pair as the reference's
    2-argument knnMatch does (PhotogrammetrieCli.cpp:371-384).  CPU baseline +
    recall reference only; not a parity oracle (FLANN is RNG-driven)."""
    return _pair_batch(imgs, pairs, lambda t, ptrs, rows, dim, pr, n, out, base, counts: lib.orc_flann_match_pairs(
        t, ptrs, rows, dim, pr, n, ratio, out, base, counts, nthreads, trees, checks, tables, key_size, seed))


def recall(exact: np.ndarray, exact_off: np.ndarray, approx: np.ndarray, approx_off: np.ndarray):
    """(recall, precision) of an approximate match list against the exact one:
    a match is the (pair, queryIdx, trainIdx) triple."""
    def keys(m, off):
        p = np.repeat(np.arange(len(off) - 1, dtype=np.int64), np.diff(off))
        return (p << 40) | (m["queryIdx"].astype(np.int64) << 20) | m["trainIdx"].astype(np.int64)
    a, b = keys(exact, exact_off), keys(approx, approx_off)
    hit = np.intersect1d(a, b).size
    return hit / max(a.size, 1), hit / max(b.size, 1)


def homography_ratios(keypoints, image_sizes, pairs, matches, offsets, threshold=-3.0, max_iters=2000,
                      confidence=0.995, nthreads: int = 0):
    """SfM::calculateHomography (SfM.cpp:599-637) restated with OpenCV 4.5.1's
    findHomography RANSAC (oracle/homography_oracle.cpp) -> ratio per pair."""
    kps = [np.ascontiguousarray(k, np.float32).reshape(-1, 2) for k in keypoints]
    ptrs = (C.c_void_p * max(len(kps), 1))(*[k.ctypes.data for k in kps])
    sizes = np.ascontiguousarray(np.asarray(image_sizes).reshape(-1, 2), np.int32)
    pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
    m = np.ascontiguousarray(matches, DMATCH_DTYPE)
    off = np.ascontiguousarray(offsets, np.int64)
    out = np.zeros(len(pairs))
    lib.orc_homography_ratios(ptrs, _ptr(sizes), _ptr(pairs), len(pairs), m.ctypes.data if len(m) else None,
                              _ptr(off, C.c_int64), threshold, max_iters, confidence,
                              out.ctypes.data_as(C.POINTER(C.c_double)), nthreads)
    return out


def find_3d2d_matches(keypoints, pairs, matches, offsets, origin_offsets, origin_shot, origin_xy, shot, nthreads=0):
    """Scene::find3d2dMatches (Scene.cpp:369-424) as the reference's literal loops
    -> (keypoint index in `shot` per origin record or -1, pair index or -1)."""
    kps = [np.ascontiguousarray(k, np.float32).reshape(-1, 2) for k in keypoints]
    ptrs = (C.c_void_p * max(len(kps), 1))(*[k.ctypes.data for k in kps])
    pairs = np.ascontiguousarray(pairs, np.int32).reshape(-1, 2)
    m = np.ascontiguousarray(matches, DMATCH_DTYPE)
    off = np.ascontiguousarray(offsets, np.int64)
    oo = np.ascontiguousarray(origin_offsets, np.int64)
    os_ = np.ascontiguousarray(origin_shot, np.int32)
    oxy = np.ascontiguousarray(origin_xy, np.float64)
    n = int(oo[-1])
    kp_out = np.zeros(max(n, 1), np.int32)
    pr_out = np.zeros(max(n, 1), np.int32)
    lib.orc_find_3d2d_matches(ptrs, _ptr(pairs), len(pairs), m.ctypes.data if len(m) else None, _ptr(off, C.c_int64),
                              _ptr(oo, C.c_int64), len(oo) - 1, _ptr(os_), oxy.ctypes.data_as(C.POINTER(C.c_double)),
                              int(shot), _ptr(kp_out), _ptr(pr_out), nthreads)
    return kp_out[:n], pr_out[:n]


def ba_observations(origin_offsets, origin_shot, origin_xy, n_shots):
    """BundleAdjustment.cpp:50-91 problem assembly -> (obs_point, obs_cam, obs_xy, shot_of_pose)."""
    oo = np.ascontiguousarray(origin_offsets, np.int64)
    os_ = np.ascontiguousarray(origin_shot, np.int32)
    oxy = np.ascontiguousarray(origin_xy, np.float64)
    n = int(oo[-1])
    op = np.zeros(max(n, 1), np.int32)
    oc = np.zeros(max(n, 1), np.int32)
    ox = np.zeros(max(2 * n, 1))
    sp = np.zeros(max(n_shots, 1), np.int32)
    npose = lib.orc_ba_observations(_ptr(oo, C.c_int64), len(oo) - 1, _ptr(os_), oxy.ctypes.data_as(C.POINTER(C.c_double)),
                                    n_shots, _ptr(op), _ptr(oc), ox.ctypes.data_as(C.POINTER(C.c_double)), _ptr(sp))
    return op[:n], oc[:n], ox[:2 * n].reshape(-1, 2), sp[:npose]


KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                           ("octave", "<i4"), ("class_id", "<i4")])


def sift(image: np.ndarray, nfeatures: int = 0, n_octave_layers: int = 3, contrast_threshold: float = 0.09,
         edge_threshold: float = 10.0, sigma: float = 1.6, descriptors: bool = True):
    """SIFT::detectAndCompute restated (oracle/sift_oracle.cpp) on an H x W uint8
    grayscale image -> (keypoints (KEYPOINT_DTYPE), n x 128 float32 descriptors)."""
    img = np.ascontiguousarray(image, np.uint8)
    H, W = img.shape
    cap = 4096
    while True:
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 128), np.float32) if descriptors else None
        n = lib.orc_sift(img.ctypes.data, W, H, W, nfeatures, n_octave_layers, contrast_threshold, edge_threshold, sigma,
                         kps.ctypes.data, desc.ctypes.data if descriptors else None, cap)
        if n <= cap:
            return kps[:n], (desc[:n] if descriptors else None)
        cap = n


# OpenCV-arithmetic model of the SIFT restatement (oracle/sift_oracle.cpp AR_* flags).  0 is the
# arithmetic the GPU kernels share; SIFT_OPENCV_AVX2 models OpenCV 4.5.1 on an AVX2/FMA3 host.
SIFT_EXP32F, SIFT_TRIG, SIFT_POWF, SIFT_FLOATHIST, SIFT_FMAVEC, SIFT_FMAFILT = 1, 2, 4, 8, 16, 32
SIFT_OPENCV_SSE2 = SIFT_EXP32F | SIFT_TRIG | SIFT_POWF | SIFT_FLOATHIST
SIFT_OPENCV_AVX2 = SIFT_OPENCV_SSE2 | SIFT_FMAVEC | SIFT_FMAFILT


class arith:
    """with oracle.arith(sift=flags, homography=flags): ... selects the oracle's arithmetic model
    for the block (measurement of the deviations from OpenCV's own arithmetic; tests only)."""

    def __init__(self, sift: int = 0, homography: int = 0):
        self.flags = (sift, homography)

    def __enter__(self):
        self.old = (lib.orc_sift_set_arith(self.flags[0]), lib.orc_homography_set_arith(self.flags[1]))
        return self

    def __exit__(self, *exc):
        lib.orc_sift_set_arith(self.old[0])
        lib.orc_homography_set_arith(self.old[1])
        return False


def sift_batch(images, nfeatures=0, contrast_threshold=0.09, cap=16384, nthreads=0):
    """sift() over equally sized images, OpenMP over images -> (counts, keypoints
    (n_images x cap), descriptors (n_images x cap x 128))."""
    n = len(images)
    H, W = images[0].shape
    imgs = [np.ascontiguousarray(a, np.uint8) for a in images]
    ptrs = (C.c_void_p * n)(*[a.ctypes.data for a in imgs])
    kps = np.zeros((n, cap), KEYPOINT_DTYPE)
    desc = np.zeros((n, cap, 128), np.float32)
    cnt = np.zeros(n, np.int32)
    lib.orc_sift_batch(ptrs, n, W, H, nfeatures, 3, contrast_threshold, 10.0, 1.6, kps.ctypes.data, desc.ctypes.data,
                       cap, _ptr(cnt), nthreads or os.cpu_count())
    return cnt, kps, desc


def orb(image: np.ndarray, nfeatures: int = 500, scale_factor: float = 1.2, nlevels: int = 8, edge_threshold: int = 31,
        fast_threshold: int = 20):
    """ORB detect() then compute() restated (oracle/orb_oracle.cpp) on an H x W uint8
    image -> (keypoints (KEYPOINT_DTYPE), n x 32 uint8 descriptors)."""
    img = np.ascontiguousarray(image, np.uint8)
    H, W = img.shape
    cap = 4096
    while True:
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = lib.orc_orb(img.ctypes.data, W, H, W, nfeatures, scale_factor, nlevels, edge_threshold, fast_threshold,
                        kps.ctypes.data, desc.ctypes.data, cap)
        if n <= cap:
            return kps[:n], desc[:n]
        cap = n


def orb_batch(images, nfeatures=30000, cap=32768, nthreads=0):
    """orb() over equally sized images, OpenMP over images -> (counts, keypoints
    (n_images x cap), descriptors (n_images x cap x 32))."""
    n = len(images)
    H, W = images[0].shape
    imgs = [np.ascontiguousarray(a, np.uint8) for a in images]
    ptrs = (C.c_void_p * n)(*[a.ctypes.data for a in imgs])
    kps = np.zeros((n, cap), KEYPOINT_DTYPE)
    desc = np.zeros((n, cap, 32), np.uint8)
    cnt = np.zeros(n, np.int32)
    lib.orc_orb_batch(ptrs, n, W, H, nfeatures, kps.ctypes.data, desc.ctypes.data, cap, _ptr(cnt),
                      nthreads or os.cpu_count())
    return cnt, kps, desc


def orb_stage(image: np.ndarray, stage: int, nlevels: int = 8, scale_factor: float = 1.2, fast_threshold: int = 20):
    """Per-level intermediate of the ORB restatement: stage 0 = pyramid, 1 = FAST score
    maps, 2 = blurred levels -> list of H_l x W_l uint8 arrays."""
    img = np.ascontiguousarray(image, np.uint8)
    H, W = img.shape
    sizes = np.zeros(2 * nlevels, np.int32)
    n = lib.orc_orb_stage(img.ctypes.data, W, H, nlevels, scale_factor, fast_threshold, stage, None, _ptr(sizes))
    out = np.zeros(n, np.uint8)
    lib.orc_orb_stage(img.ctypes.data, W, H, nlevels, scale_factor, fast_threshold, stage, out.ctypes.data, _ptr(sizes))
    res, off = [], 0
    for l in range(nlevels):
        w, h = int(sizes[2 * l]), int(sizes[2 * l + 1])
        res.append(out[off:off + w * h].reshape(h, w))
        off += w * h
    return res


def _dist5(dist):
    d = np.zeros(5)
    d[:len(dist)] = np.asarray(dist, np.float64).ravel()[:5]
    return d


def undistort(img: np.ndarray, K, dist) -> np.ndarray:
    """cv::undistort(img, out, K, dist) (ICamera.cpp:72-80; OpenCV 4.5.1 restated in
    oracle/mvs_oracle.cpp) for an H x W [x C] uint8 image."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape[:2]
    cn = 1 if img.ndim == 2 else img.shape[2]
    out = np.empty_like(img)
    Kd = np.ascontiguousarray(K, np.float64).reshape(9)
    d = _dist5(dist)
    lib.orc_undistort(img.ctypes.data, out.ctypes.data, W, H, cn, Kd.ctypes.data_as(C.POINTER(C.c_double)),
                      d.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def undistort_batch(imgs, Ks, dists, outs, nthreads=0):
    """undistort() over a list of images into preallocated outs (OpenMP over images,
    as the reference's omp loop, OpenMvsUtils.cpp:141)."""
    n = len(imgs)
    sp = (C.c_void_p * n)(*[a.ctypes.data for a in imgs])
    dp = (C.c_void_p * n)(*[a.ctypes.data for a in outs])
    W = np.array([a.shape[1] for a in imgs], np.int32)
    H = np.array([a.shape[0] for a in imgs], np.int32)
    cn = np.array([1 if a.ndim == 2 else a.shape[2] for a in imgs], np.int32)
    Kd = np.ascontiguousarray(np.stack([np.asarray(k, np.float64).reshape(9) for k in Ks]))
    dd = np.ascontiguousarray(np.stack([_dist5(d) for d in dists]))
    lib.orc_undistort_batch(sp, dp, _ptr(W), _ptr(H), _ptr(cn), Kd.ctypes.data_as(C.POINTER(C.c_double)),
                            dd.ctypes.data_as(C.POINTER(C.c_double)), n, nthreads or os.cpu_count())


def openmvs_interface(cameras, shots, points, origin_offsets, origin_shot):
    """OpenMvsUtils::toOpenMVS's Interface assembly (OpenMvsUtils.cpp:44-133), restated
    in plain Python.  cameras: [(width, height, K 3x3)]; shots: [(camera index or -1,
    recovered, pose 3x4, image name)]; origins: CSR of origin shot indices per point.
    Returns a dict mirroring openMVS::Interface."""
    platforms = [{"name": "", "cameras": [{"name": "", "width": int(w), "height": int(h),
                                           "K": np.asarray(K, np.float64).reshape(3, 3),
                                           "R": np.eye(3), "C": np.zeros(3)}], "poses": []}
                 for (w, h, K) in cameras]
    images, shot_to_id = [], {}
    for s, (cam, rec, pose, name) in enumerate(shots):
        if not rec or cam < 0 or cam >= len(cameras):                       # :76-78
            continue
        P = np.asarray(pose, np.float64).reshape(3, 4)
        R, t = P[:, :3], P[:, 3]
        C_ = np.array([-sum(R[k, i] * t[k] for k in range(3)) for i in range(3)])   # -R^T t
        images.append({"name": name, "platformID": cam, "cameraID": 0,
                       "poseID": len(platforms[cam]["poses"])})
        platforms[cam]["poses"].append({"R": R.copy(), "C": C_})
        shot_to_id[s] = len(images) - 1
    vertices = []
    pts = np.asarray(points, np.float64).reshape(-1, 3)
    for p in range(len(pts)):
        shots_p = set(int(x) for x in origin_shot[origin_offsets[p]:origin_offsets[p + 1]])   # getOriginShots
        views = sorted(shot_to_id[s] for s in shots_p if s in shot_to_id)
        if len(views) < 2:                                                   # :122-124
            continue
        vertices.append({"X": pts[p].astype(np.float32), "views": [(v, 0.0) for v in views]})
    return {"platforms": platforms, "images": images, "vertices": vertices}


def openmvs_serialize(iface, version=1) -> bytes:
    """openMVS ARCHIVE::SerializeSave of an Interface dict (openMVS v1.1.1 stream:
    'MVSI', uint32 version, uint32 0; uint64 counts; raw Matx / Point3; serialize()
    field order with its version gates)."""
    import struct
    out = [b"MVSI", struct.pack("<II", version, 0)]
    cnt = lambda n: out.append(struct.pack("<Q", n))

    def st(s):
        b = s.encode()
        cnt(len(b))
        out.append(b)
    cnt(len(iface["platforms"]))
    for pf in iface["platforms"]:
        st(pf["name"])
        cnt(len(pf["cameras"]))
        for c in pf["cameras"]:
            st(c["name"])
            if version > 0:
                out.append(struct.pack("<II", c["width"], c["height"]))
            out.append(np.asarray(c["K"], "<f8").tobytes() + np.asarray(c["R"], "<f8").tobytes()
                       + np.asarray(c["C"], "<f8").tobytes())
        cnt(len(pf["poses"]))
        for q in pf["poses"]:
            out.append(np.asarray(q["R"], "<f8").tobytes() + np.asarray(q["C"], "<f8").tobytes())
    cnt(len(iface["images"]))
    for im in iface["images"]:
        st(im["name"])
        out.append(struct.pack("<III", im["platformID"], im["cameraID"], im["poseID"]))
        if version > 2:
            out.append(struct.pack("<I", 0xFFFFFFFF))
    cnt(len(iface["vertices"]))
    for v in iface["vertices"]:
        out.append(np.asarray(v["X"], "<f4").tobytes())
        cnt(len(v["views"]))
        for (i, c) in v["views"]:
            out.append(struct.pack("<If", i, c))
    cnt(0)
    cnt(0)
    if version > 0:
        cnt(0)
        cnt(0)
        cnt(0)
        if version > 1:
            out.append(np.eye(4, dtype="<f8").tobytes())
    return b"".join(out)


def openmvs_parse(buf: bytes) -> dict:
    """Inverse of openmvs_serialize (what openMVS's SerializeLoad reads)."""
    import struct
    pos = 0

    def take(fmt):
        nonlocal pos
        v = struct.unpack_from(fmt, buf, pos)
        pos += struct.calcsize(fmt)
        return v

    def arr(n, dt):
        nonlocal pos
        a = np.frombuffer(buf, dt, n, pos).copy()
        pos += n * np.dtype(dt).itemsize
        return a

    def st():
        nonlocal pos
        (n,) = take("<Q")
        s = buf[pos:pos + n].decode()
        pos += n
        return s
    assert buf[:4] == b"MVSI"
    pos = 4
    version, _ = take("<II")
    pfs = []
    for _ in range(take("<Q")[0]):
        pf = {"name": st(), "cameras": [], "poses": []}
        for _ in range(take("<Q")[0]):
            c = {"name": st()}
            if version > 0:
                c["width"], c["height"] = take("<II")
            c["K"], c["R"], c["C"] = arr(9, "<f8").reshape(3, 3), arr(9, "<f8").reshape(3, 3), arr(3, "<f8")
            pf["cameras"].append(c)
        for _ in range(take("<Q")[0]):
            pf["poses"].append({"R": arr(9, "<f8").reshape(3, 3), "C": arr(3, "<f8")})
        pfs.append(pf)
    imgs = []
    for _ in range(take("<Q")[0]):
        im = {"name": st()}
        im["platformID"], im["cameraID"], im["poseID"] = take("<III")
        if version > 2:
            im["ID"] = take("<I")[0]
        imgs.append(im)
    verts = []
    for _ in range(take("<Q")[0]):
        X = arr(3, "<f4")
        verts.append({"X": X, "views": [take("<If") for _ in range(take("<Q")[0])]})
    rest = {"verticesNormal": take("<Q")[0], "verticesColor": take("<Q")[0]}
    if version > 0:
        rest.update(lines=take("<Q")[0], linesNormal=take("<Q")[0], linesColor=take("<Q")[0])
        if version > 1:
            rest["transform"] = arr(16, "<f8").reshape(4, 4)
    assert pos == len(buf), "trailing bytes"
    return {"version": version, "platforms": pfs, "images": imgs, "vertices": verts, **rest}


def filter_matches(matches: np.ndarray, offsets: np.ndarray, distinct: bool, min_count: int):
    """SfM.cpp:547-570 restated -> (matches, offsets, keep) with the same packing."""
    n = len(offsets) - 1
    m = matches.copy()
    base = offsets[:-1].astype(np.int64).copy()
    counts = np.diff(offsets).astype(np.int64)
    keep = np.zeros(max(n, 1), np.int32)
    lib.orc_filter_matches(m.ctypes.data, _ptr(base, C.c_int64), _ptr(counts, C.c_int64), n, int(distinct),
                           int(min_count), _ptr(keep))
    out = np.concatenate([m[base[p]: base[p] + counts[p]] for p in range(n)]) if n else m[:0]
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(counts[:n])
    return out, off, keep[:n]


def pairs_unordered(n):
    k = lib.orc_pairs_unordered(n, None)
    out = np.empty((k, 2), np.int32)
    lib.orc_pairs_unordered(n, _ptr(out))
    return out


def pairs_video(n, seq):
    k = lib.orc_pairs_video(n, seq, None)
    if k < 0:
        raise ValueError("sequence length < 2")
    out = np.empty((k, 2), np.int32)
    lib.orc_pairs_video(n, seq, _ptr(out))
    return out


def pairs_grid(n, seq, row_len, mode=1):
    k = lib.orc_pairs_grid(n, seq, row_len, mode, None)
    if k < 0:
        raise ValueError("bad grid parameters")
    out = np.empty((k, 2), np.int32)
    lib.orc_pairs_grid(n, seq, row_len, mode, _ptr(out))
    return out


def first_sqrt_collision(limit: int = 1 << 24) -> int:
    return int(lib.orc_first_sqrt_collision(limit))


# ---- bundle adjustment (oracle/ba_oracle.cpp) --------------------------------

class _BAProblem(C.Structure):
    _fields_ = [("n_points", C.c_int32), ("n_cams", C.c_int32), ("n_obs", C.c_int32), ("cam_model", C.c_int32),
                ("points", C.c_void_p), ("poses", C.c_void_p), ("intr", C.c_void_p),
                ("obs_point", C.c_void_p), ("obs_cam", C.c_void_p), ("obs_xy", C.c_void_p),
                ("cx", C.c_double), ("cy", C.c_double),
                ("n_intr", C.c_int32), ("_reserved", C.c_int32), ("intr_model", C.c_void_p),
                ("pose_intr", C.c_void_p), ("intr_center", C.c_void_p)]


class _BAOptions(C.Structure):
    _fields_ = [("max_num_iterations", C.c_int32), ("max_num_consecutive_invalid_steps", C.c_int32),
                ("jacobi_scaling", C.c_int32), ("device", C.c_int32),
                ("function_tolerance", C.c_double), ("gradient_tolerance", C.c_double),
                ("parameter_tolerance", C.c_double), ("initial_trust_region_radius", C.c_double),
                ("max_trust_region_radius", C.c_double), ("min_trust_region_radius", C.c_double),
                ("min_lm_diagonal", C.c_double), ("max_lm_diagonal", C.c_double),
                ("min_relative_decrease", C.c_double)]


class _BASummary(C.Structure):
    _fields_ = [("initial_cost", C.c_double), ("final_cost", C.c_double),
                ("num_successful_steps", C.c_int32), ("num_unsuccessful_steps", C.c_int32),
                ("num_invalid_steps", C.c_int32), ("termination_type", C.c_int32),
                ("total_ms", C.c_double), ("ms_per_iteration", C.c_double),
                ("final_gradient_max_norm", C.c_double), ("final_radius", C.c_double)]


CERES_DEFAULTS = dict(max_num_iterations=5000, max_num_consecutive_invalid_steps=5, jacobi_scaling=1, device=0,
                      function_tolerance=1e-6, gradient_tolerance=1e-10, parameter_tolerance=1e-8,
                      initial_trust_region_radius=1e4, max_trust_region_radius=1e16, min_trust_region_radius=1e-32,
                      min_lm_diagonal=1e-6, max_lm_diagonal=1e32, min_relative_decrease=1e-3)

lib.orc_ba_solve.argtypes = [C.POINTER(_BAProblem), C.POINTER(_BAOptions), C.POINTER(_BASummary), C.c_void_p,
                             C.c_int, C.c_int]
lib.orc_ba_cost.restype = C.c_double
lib.orc_ba_cost.argtypes = [C.POINTER(_BAProblem)]
lib.orc_ba_jacobian.argtypes = [C.POINTER(_BAProblem), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]


def _ba_struct(p: dict):
    keep = {   # parameter blocks are copied: the solver writes its result into them
        "points": np.array(p["points"], np.float64, copy=True).reshape(-1, 3),
        "poses": np.array(p["poses"], np.float64, copy=True).reshape(-1, 6),
        "intr": np.array(p["intr"], np.float64, copy=True).reshape(-1),
        "obs_point": np.ascontiguousarray(p["obs_point"], np.int32).reshape(-1),
        "obs_cam": np.ascontiguousarray(p["obs_cam"], np.int32).reshape(-1),
        "obs_xy": np.ascontiguousarray(p["obs_xy"], np.float64).reshape(-1, 2),
    }
    s = _BAProblem(len(keep["points"]), len(keep["poses"]), len(keep["obs_point"]), int(p["cam_model"]),
                   keep["points"].ctypes.data, keep["poses"].ctypes.data, keep["intr"].ctypes.data,
                   keep["obs_point"].ctypes.data, keep["obs_cam"].ctypes.data, keep["obs_xy"].ctypes.data,
                   float(p.get("cx", 0.0)), float(p.get("cy", 0.0)))
    if p.get("intr_models") is not None:   # several cameras (BundleAdjustment.cpp:45-48, 81-89)
        keep["intr_models"] = np.ascontiguousarray(p["intr_models"], np.int32).reshape(-1)
        keep["pose_intr"] = np.ascontiguousarray(p["pose_intr"], np.int32).reshape(-1)
        keep["centers"] = np.ascontiguousarray(p["centers"], np.float64).reshape(-1, 2)
        s.n_intr = len(keep["intr_models"])
        s.intr_model = keep["intr_models"].ctypes.data
        s.pose_intr = keep["pose_intr"].ctypes.data
        s.intr_center = keep["centers"].ctypes.data
    return s, keep


def ba_cost(p: dict) -> float:
    s, keep = _ba_struct(p)
    return float(lib.orc_ba_cost(C.byref(s)))


def ba_jacobian(p: dict):
    s, keep = _ba_struct(p)
    O, k = len(keep["obs_point"]), len(keep["intr"])
    r = np.zeros((O, 2)); Je = np.zeros((O, 2, 3)); Jc = np.zeros((O, 2, 6)); Ji = np.zeros((O, 2, k))
    lib.orc_ba_jacobian(C.byref(s), r.ctypes.data, Je.ctypes.data, Jc.ctypes.data, Ji.ctypes.data)
    return r, Je, Jc, Ji


def ba_solve(p: dict, nthreads: int = 0, trace_cap: int = 0, **options):
    """LM + DENSE_SCHUR restatement of Ceres 1.14 -> (solution dict, summary dict, trace[n,3])."""
    s, keep = _ba_struct(p)
    o = dict(CERES_DEFAULTS)
    o.update(options)
    opt = _BAOptions(**o)
    sm = _BASummary()
    tr = np.zeros((max(trace_cap, 1), 3))
    n = lib.orc_ba_solve(C.byref(s), C.byref(opt), C.byref(sm), tr.ctypes.data if trace_cap else None, trace_cap,
                         nthreads)
    summary = {f: getattr(sm, f) for f, _ in sm._fields_}
    sol = dict(p)
    sol.update(points=keep["points"], poses=keep["poses"], intr=keep["intr"])
    return sol, summary, tr[:max(n, 0)]
