"""The openMVS export seam — host mirror over
include/sfmx_mvs.h of ``OpenMvsUtils::toOpenMVS`` (util/OpenMvsUtils.cpp:31-154):

* ``undistort`` / ``undistort_device``: the per-shot ``cv::undistort`` of
  :142-150 (``ICamera::undistort``, common/ICamera.cpp:72-80), all images in one
  gfx950 launch (csrc/mvs.hip);
* ``serialize`` / ``toOpenMVS``: the ``openMVS::Interface`` assembly (:44-133)
  and ``ARCHIVE::SerializeSave`` (:152), native host code (csrc/mvs_writer.cpp).

Image encoding (``cv::imwrite`` of the PNGs) is the caller's; ``toOpenMVS``
returns the undistorted images for that.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Sequence

import numpy as np

from ._lib import lib, check, SfmxError


class sfmx_undistort_image(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("width", C.c_int32), ("height", C.c_int32),
                ("channels", C.c_int32), ("_pad", C.c_int32), ("src_pitch", C.c_int64), ("dst_pitch", C.c_int64),
                ("K", C.c_double * 9), ("dist", C.c_double * 5)]


class sfmx_mvs_camera(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("K", C.c_double * 9)]


class sfmx_mvs_shot(C.Structure):
    _fields_ = [("camera", C.c_int32), ("recovered", C.c_int32), ("pose", C.c_double * 12),
                ("image_name", C.c_char_p)]


def _desc(src_ptr, dst_ptr, h, w, cn, src_pitch, dst_pitch, K, dist):
    d = sfmx_undistort_image()
    d.src, d.dst = src_ptr, dst_ptr
    d.width, d.height, d.channels = int(w), int(h), int(cn)
    d.src_pitch, d.dst_pitch = int(src_pitch), int(dst_pitch)
    d.K[:] = [float(v) for v in np.asarray(K, np.float64).reshape(9)]
    dd = np.zeros(5)
    dd[:len(np.ravel(dist))] = np.ravel(dist)[:5]
    d.dist[:] = [float(v) for v in dd]
    return d


def undistort(images: Sequence[np.ndarray], Ks, dists, device: int = 0, stream: int = 0):
    """cv::undistort(img, out, K, dist) for every H x W [x C] uint8 image (host
    arrays; copied through the device) -> list of undistorted images."""
    imgs = [np.ascontiguousarray(a, np.uint8) for a in images]
    outs = [np.empty_like(a) for a in imgs]
    descs = (sfmx_undistort_image * max(len(imgs), 1))()
    for i, (a, o) in enumerate(zip(imgs, outs)):
        cn = 1 if a.ndim == 2 else a.shape[2]
        descs[i] = _desc(a.ctypes.data, o.ctypes.data, a.shape[0], a.shape[1], cn, a.strides[0], o.strides[0],
                         Ks[i], dists[i])
    check(lib.sfmx_undistort_images(descs, len(imgs), 0, int(device), stream or None), "sfmx_undistort_images")
    return outs


def undistort_device(srcs, dsts, Ks, dists, device: int = 0, stream: int = 0):
    """Same over resident torch uint8 tensors (H x W [x C], rows may be padded)."""
    descs = (sfmx_undistort_image * max(len(srcs), 1))()
    for i, (a, o) in enumerate(zip(srcs, dsts)):
        if a.dtype.itemsize != 1 or a.stride(-1) != 1 or o.shape != a.shape:
            raise ValueError("uint8 images with unit element stride and matching shapes expected")
        cn = 1 if a.dim() == 2 else a.shape[2]
        descs[i] = _desc(a.data_ptr(), o.data_ptr(), a.shape[0], a.shape[1], cn, a.stride(0), o.stride(0),
                         Ks[i], dists[i])
    check(lib.sfmx_undistort_images(descs, len(srcs), 1, int(device), stream or None), "sfmx_undistort_images")


def last_kernel_ms() -> float:
    return float(lib.sfmx_undistort_last_kernel_ms())


def _scene_args(cameras, shots, points, origin_offsets, origin_shot):
    cams = (sfmx_mvs_camera * max(len(cameras), 1))()
    for i, (w, h, K) in enumerate(cameras):
        cams[i].width, cams[i].height = int(w), int(h)
        cams[i].K[:] = [float(v) for v in np.asarray(K, np.float64).reshape(9)]
    names = [n.encode() if isinstance(n, str) else n for (_, _, _, n) in shots]
    sh = (sfmx_mvs_shot * max(len(shots), 1))()
    for i, (cam, rec, pose, _) in enumerate(shots):
        sh[i].camera, sh[i].recovered = int(cam), int(bool(rec))
        sh[i].pose[:] = [float(v) for v in np.asarray(pose, np.float64).reshape(12)]
        sh[i].image_name = names[i]
    pts = np.ascontiguousarray(points, np.float64).reshape(-1, 3)
    oo = np.ascontiguousarray(origin_offsets, np.int64)
    osh = np.ascontiguousarray(origin_shot, np.int32)
    keep = (cams, sh, names, pts, oo, osh)
    return keep, (cams, len(cameras), sh, len(shots), pts.ctypes.data_as(C.POINTER(C.c_double)), len(pts),
                  oo.ctypes.data_as(C.POINTER(C.c_int64)), osh.ctypes.data_as(C.POINTER(C.c_int32)) if len(osh) else None)


def _serialize_bound(cameras, shots, n_points: int, n_origins: int) -> int:
    """An upper bound of the Interface size: every shot an image and a pose, every point a vertex
    with all its origins as views (the native call reports the exact size)."""
    names = sum(len(n.encode() if isinstance(n, str) else n) for (_, _, _, n) in shots)
    return (64 + len(cameras) * (8 + 8 + 8 + 8 + 72 + 72 + 24 + 8) + len(shots) * (96 + 8 + 16) + names +
            n_points * (12 + 8) + n_origins * 8 + 8 * 5 + 128)


def serialize(cameras, shots, points, origin_offsets, origin_shot, version: int = 1):
    """openMVS Interface bytes as OpenMvsUtils::toOpenMVS would write them.
    cameras: [(width, height, K 3x3)]; shots: [(camera index or -1, recovered,
    pose 3x4 [R|t], image name)]; points n x 3; origins: CSR of origin shot
    indices per point.  -> (bytes, n_images, n_vertices)
    One native call into a buffer of the bound above (a second one only if that ever fell short)."""
    keep, args = _scene_args(cameras, shots, points, origin_offsets, origin_shot)
    oo = keep[4]
    size = C.c_int64(0)
    ni, nv = C.c_int32(0), C.c_int32(0)
    cap = _serialize_bound(cameras, shots, len(keep[3]), int(oo[-1]) if len(oo) else 0)
    for _ in range(2):
        buf = bytearray(max(cap, 1))
        cbuf = (C.c_uint8 * len(buf)).from_buffer(buf)
        rc = lib.sfmx_openmvs_serialize(int(version), *args, cbuf, cap, C.byref(size), C.byref(ni), C.byref(nv))
        del cbuf
        if rc != -4:   # SFMX_ECAPACITY: size holds the exact size; go again with it
            break
        cap = size.value
    check(rc, "sfmx_openmvs_serialize")
    del keep
    return bytes(memoryview(buf)[:size.value]), ni.value, nv.value


def toOpenMVS(cameras, shots, points, origin_offsets, origin_shot, path: str, filename: str = "mvs.bin",
              relativePaths: bool = False, images=None, dists=None, version: int = 1, device: int = 0):
    """OpenMvsUtils::toOpenMVS (OpenMvsUtils.cpp:31-154).  shots: [(camera index,
    recovered, pose 3x4)]; image names are images/<shot index>.png, absolute or
    relative to `path` (the reference uses the shot's address, :38-40).  When
    `images` (one uint8 array per shot, or None) and `dists` are given, the
    recovered shots' images are undistorted on the GPU and returned as
    {file name: image} for the caller to encode (:141-150).
    -> (interface file path, n_images, n_vertices, undistorted images)"""
    os.makedirs(os.path.join(path, "images"), exist_ok=True)
    named = []
    for s, (cam, rec, pose) in enumerate(shots):
        f = os.path.join(path, "images", f"{s}.png")
        named.append((cam, rec, pose, os.path.relpath(f, path) if relativePaths else os.path.abspath(f)))
    keep, args = _scene_args(cameras, named, points, origin_offsets, origin_shot)
    ni, nv = C.c_int32(0), C.c_int32(0)
    out = os.path.join(path, filename)
    check(lib.sfmx_openmvs_write(out.encode(), int(version), *args, C.byref(ni), C.byref(nv)), "sfmx_openmvs_write")
    del keep
    undist = {}
    if images is not None:
        sel = [s for s, (cam, rec, _) in enumerate(shots) if rec and images[s] is not None]
        if sel:
            res = undistort([images[s] for s in sel], [cameras[shots[s][0]][2] for s in sel],
                            [dists[shots[s][0]] for s in sel], device=device)
            undist = {named[s][3]: r for s, r in zip(sel, res)}
    return out, ni.value, nv.value, undist


__all__ = ["undistort", "undistort_device", "last_kernel_ms", "serialize", "toOpenMVS", "SfmxError"]
