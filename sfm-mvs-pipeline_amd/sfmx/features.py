"""Feature extraction — host mirror over
include/sfmx_features.h of the reference's

    featureDetector = cv::SIFT::create(featureLimit, 3, 0.09)   (cli/PhotogrammetrieCli.cpp:354)
    featureDetector->detect(image, keypoints); descriptorExtractor->compute(...)
                                                                (sfm/SfM.cpp:577-597)

``SIFT.create(...).detectAndCompute(image)`` runs csrc/sift_features.hip on the
GPU (OpenCV 4.5.1 SIFT semantics restated; see DESIGN.md for the documented
deviations).  Descriptors are n x 128 float32 with integer values, ready for
``sfmx.BFMatcher``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import lib, check

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"), ("response", "<f4"),
                           ("octave", "<i4"), ("class_id", "<i4")])   # cv::KeyPoint


class sfmx_sift_params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("n_octave_layers", C.c_int32), ("contrast_threshold", C.c_double),
                ("edge_threshold", C.c_double), ("sigma", C.c_double)]


class SIFT:
    """cv::SIFT::create(nfeatures, nOctaveLayers, contrastThreshold, edgeThreshold, sigma);
    the reference passes (featureLimit, 3, 0.09)."""

    def __init__(self, nfeatures: int = 0, nOctaveLayers: int = 3, contrastThreshold: float = 0.09,
                 edgeThreshold: float = 10.0, sigma: float = 1.6, device: int = 0):
        self.params = sfmx_sift_params(int(nfeatures), int(nOctaveLayers), float(contrastThreshold),
                                       float(edgeThreshold), float(sigma))
        self.device = device

    @classmethod
    def create(cls, nfeatures: int = 0, nOctaveLayers: int = 3, contrastThreshold: float = 0.09,
               edgeThreshold: float = 10.0, sigma: float = 1.6, device: int = 0) -> "SIFT":
        return cls(nfeatures, nOctaveLayers, contrastThreshold, edgeThreshold, sigma, device)

    def detectAndCompute(self, image: np.ndarray, capacity: int = 1 << 16, stream: int = 0):
        """H x W uint8 grayscale -> (keypoints (KEYPOINT_DTYPE), n x 128 float32 descriptors)."""
        img = np.ascontiguousarray(image, np.uint8)
        if img.ndim != 2:
            raise ValueError("grayscale H x W uint8 image expected (CameraShot::loadImage default)")
        n = C.c_int32(0)
        while True:
            kps = np.zeros(capacity, KEYPOINT_DTYPE)
            desc = np.zeros((capacity, 128), np.float32)
            rc = lib.sfmx_sift_detect_compute(img.ctypes.data, img.shape[1], img.shape[0], img.strides[0],
                                              C.byref(self.params), 0, self.device, stream or None, kps.ctypes.data,
                                              desc.ctypes.data, capacity, C.byref(n))
            if rc == -4 and n.value > capacity:
                capacity = n.value
                continue
            check(rc, "sfmx_sift_detect_compute")
            return kps[:n.value], desc[:n.value]

    def detect(self, image):
        return self.detectAndCompute(image)[0]

    def detectAndCompute_device(self, image_t, keypoints_t, descriptors_t, stream: int = 0) -> int:
        """Resident torch tensors: image (H x W uint8), keypoints (cap x 7 int32 view of
        KEYPOINT_DTYPE rows), descriptors (cap x 128 float32) -> keypoint count."""
        n = C.c_int32(0)
        cap = int(keypoints_t.shape[0])
        check(lib.sfmx_sift_detect_compute(image_t.data_ptr(), image_t.shape[1], image_t.shape[0], image_t.stride(0),
                                           C.byref(self.params), 1, self.device, stream or None, keypoints_t.data_ptr(),
                                           descriptors_t.data_ptr(), cap, C.byref(n)), "sfmx_sift_detect_compute")
        return n.value

    def detectAndCompute_batch_device(self, images, keypoints, descriptors, n_streams: int = 4):
        """SfM::extractFeatures over shots (SfM.cpp:577-597): lists of resident torch
        tensors as for detectAndCompute_device, run by n_streams workers with one HIP
        stream each (sfmx_sift_detect_compute_batch) -> list of keypoint counts.
        Results equal the one-image call's."""
        n = len(images)
        if not (len(keypoints) == len(descriptors) == n):
            raise ValueError("images, keypoints and descriptors must have the same length")
        imgs = (sfmx_gray_image * max(n, 1))()
        for i, t in enumerate(images):
            if t.dim() != 2:
                raise ValueError("grayscale H x W uint8 image expected (CameraShot::loadImage default)")
            imgs[i] = sfmx_gray_image(t.data_ptr(), t.shape[1], t.shape[0], t.stride(0))
        kp = (C.c_void_p * max(n, 1))(*[k.data_ptr() for k in keypoints])
        dd = (C.c_void_p * max(n, 1))(*[d.data_ptr() for d in descriptors])
        caps = np.array([k.shape[0] for k in keypoints] or [0], np.int32)
        cnt = np.zeros(max(n, 1), np.int32)
        st = np.zeros(max(n, 1), np.int32)
        i32p = C.POINTER(C.c_int32)
        check(lib.sfmx_sift_detect_compute_batch(imgs, n, C.byref(self.params), 1, self.device, int(n_streams), kp, dd,
                                                 caps.ctypes.data_as(i32p), cnt.ctypes.data_as(i32p),
                                                 st.ctypes.data_as(i32p)), "sfmx_sift_detect_compute_batch")
        return [int(c) for c in cnt[:n]]


class sfmx_orb_params(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("n_levels", C.c_int32),
                ("edge_threshold", C.c_int32), ("first_level", C.c_int32), ("wta_k", C.c_int32),
                ("score_type", C.c_int32), ("patch_size", C.c_int32), ("fast_threshold", C.c_int32)]


class ORB:
    """cv::ORB::create(nfeatures, scaleFactor, nlevels, edgeThreshold, firstLevel, WTA_K,
    scoreType, patchSize, fastThreshold); the reference passes only nfeatures =
    featureLimit (cli/PhotogrammetrieCli.cpp:347-348).  detectAndCompute runs
    csrc/orb_features.hip: detect() then compute(), as SfM.cpp:586-587 calls them."""

    def __init__(self, nfeatures: int = 500, scaleFactor: float = 1.2, nlevels: int = 8, edgeThreshold: int = 31,
                 firstLevel: int = 0, WTA_K: int = 2, scoreType: int = 0, patchSize: int = 31,
                 fastThreshold: int = 20, device: int = 0):
        self.params = sfmx_orb_params(int(nfeatures), float(scaleFactor), int(nlevels), int(edgeThreshold),
                                      int(firstLevel), int(WTA_K), int(scoreType), int(patchSize), int(fastThreshold))
        self.device = device

    @classmethod
    def create(cls, nfeatures: int = 500, *args, **kw) -> "ORB":
        return cls(nfeatures, *args, **kw)

    def detectAndCompute(self, image: np.ndarray, capacity: int = 1 << 15, stream: int = 0):
        """H x W uint8 grayscale -> (keypoints (KEYPOINT_DTYPE), n x 32 uint8 descriptors)."""
        img = np.ascontiguousarray(image, np.uint8)
        if img.ndim != 2:
            raise ValueError("grayscale H x W uint8 image expected (CameraShot::loadImage default)")
        n = C.c_int32(0)
        while True:
            kps = np.zeros(capacity, KEYPOINT_DTYPE)
            desc = np.zeros((capacity, 32), np.uint8)
            rc = lib.sfmx_orb_detect_compute(img.ctypes.data, img.shape[1], img.shape[0], img.strides[0],
                                             C.byref(self.params), 0, self.device, stream or None, kps.ctypes.data,
                                             desc.ctypes.data, capacity, C.byref(n))
            if rc == -4 and n.value > capacity:
                capacity = n.value
                continue
            check(rc, "sfmx_orb_detect_compute")
            return kps[:n.value], desc[:n.value]

    def detect(self, image):
        return self.detectAndCompute(image)[0]

    def detectAndCompute_device(self, image_t, keypoints_t, descriptors_t, stream: int = 0) -> int:
        """Resident torch tensors: image (H x W uint8), keypoints (cap x 7 int32 view of
        KEYPOINT_DTYPE rows), descriptors (cap x 32 uint8) -> keypoint count."""
        n = C.c_int32(0)
        check(lib.sfmx_orb_detect_compute(image_t.data_ptr(), image_t.shape[1], image_t.shape[0], image_t.stride(0),
                                          C.byref(self.params), 1, self.device, stream or None, keypoints_t.data_ptr(),
                                          descriptors_t.data_ptr(), int(keypoints_t.shape[0]), C.byref(n)),
              "sfmx_orb_detect_compute")
        return n.value

    def detectAndCompute_batch_device(self, images, keypoints, descriptors, n_streams: int = 4):
        """SfM::extractFeatures over shots with resident torch tensors (image H x W uint8,
        keypoints cap x 7 int32, descriptors cap x 32 uint8) -> list of keypoint counts."""
        n = len(images)
        if not (len(keypoints) == len(descriptors) == n):
            raise ValueError("images, keypoints and descriptors must have the same length")
        imgs = (sfmx_gray_image * max(n, 1))()
        for i, t in enumerate(images):
            if t.dim() != 2:
                raise ValueError("grayscale H x W uint8 image expected (CameraShot::loadImage default)")
            imgs[i] = sfmx_gray_image(t.data_ptr(), t.shape[1], t.shape[0], t.stride(0))
        kp = (C.c_void_p * max(n, 1))(*[k.data_ptr() for k in keypoints])
        dd = (C.c_void_p * max(n, 1))(*[d.data_ptr() for d in descriptors])
        caps = np.array([k.shape[0] for k in keypoints] or [0], np.int32)
        cnt = np.zeros(max(n, 1), np.int32)
        st = np.zeros(max(n, 1), np.int32)
        i32p = C.POINTER(C.c_int32)
        check(lib.sfmx_orb_detect_compute_batch(imgs, n, C.byref(self.params), 1, self.device, int(n_streams), kp, dd,
                                                caps.ctypes.data_as(i32p), cnt.ctypes.data_as(i32p),
                                                st.ctypes.data_as(i32p)), "sfmx_orb_detect_compute_batch")
        return [int(c) for c in cnt[:n]]

    def detectAndCompute_batch(self, images, capacity: int = 1 << 15, n_streams: int = 4):
        """Host images -> list of (keypoints, descriptors), n_streams workers
        (sfmx_orb_detect_compute_batch).  Results equal the one-image call's."""
        imgs = [np.ascontiguousarray(im, np.uint8) for im in images]
        n = len(imgs)
        arr = (sfmx_gray_image * max(n, 1))()
        for i, im in enumerate(imgs):
            arr[i] = sfmx_gray_image(im.ctypes.data, im.shape[1], im.shape[0], im.strides[0])
        kps = [np.zeros(capacity, KEYPOINT_DTYPE) for _ in range(n)]
        desc = [np.zeros((capacity, 32), np.uint8) for _ in range(n)]
        kp = (C.c_void_p * max(n, 1))(*[k.ctypes.data for k in kps])
        dd = (C.c_void_p * max(n, 1))(*[d.ctypes.data for d in desc])
        caps = np.full(max(n, 1), capacity, np.int32)
        cnt = np.zeros(max(n, 1), np.int32)
        st = np.zeros(max(n, 1), np.int32)
        i32p = C.POINTER(C.c_int32)
        check(lib.sfmx_orb_detect_compute_batch(arr, n, C.byref(self.params), 0, self.device, int(n_streams), kp, dd,
                                                caps.ctypes.data_as(i32p), cnt.ctypes.data_as(i32p),
                                                st.ctypes.data_as(i32p)), "sfmx_orb_detect_compute_batch")
        return [(kps[i][:cnt[i]], desc[i][:cnt[i]]) for i in range(n)]


def orb_last_kernel_ms() -> float:
    return float(lib.sfmx_orb_last_kernel_ms())


class sfmx_gray_image(C.Structure):
    _fields_ = [("data", C.c_void_p), ("width", C.c_int32), ("height", C.c_int32), ("pitch", C.c_int64)]


def last_kernel_ms() -> float:
    return float(lib.sfmx_sift_last_kernel_ms())


__all__ = ["SIFT", "KEYPOINT_DTYPE", "last_kernel_ms"]
