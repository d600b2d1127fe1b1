"""Synthetic grayscale images for the SIFT extraction row:
Gaussian blobs of several scales and contrasts on a smooth background, plus
mild noise, so the detector finds extrema on several octaves."""
import numpy as np


def blob_image(h, w, n_blobs=40, seed=0, noise=2.0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = 100 + 30 * np.sin(xx / 37.0) * np.cos(yy / 29.0)
    for _ in range(n_blobs):
        cy, cx = rng.uniform(0, h), rng.uniform(0, w)
        s = rng.uniform(1.5, min(h, w) / 10)
        a = rng.uniform(-90, 90)
        sx, sy = s, s * rng.uniform(0.5, 1.0)
        img += a * np.exp(-(((xx - cx) / sx) ** 2 + ((yy - cy) / sy) ** 2) / 2)
    img += rng.normal(0, noise, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def big_blob_image(h, w, seed=0, n=12, smin=8.0, smax=20.0):
    """Only large blobs on a flat background: every keypoint comes from octave >= 0, so
    SIFT::compute (called after detect, SfM.cpp:586-587) rebuilds an un-doubled pyramid
    (firstOctave = 0) for the descriptors."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    img = np.full((h, w), 110.0)
    for _ in range(n):
        cy, cx = rng.uniform(0, h), rng.uniform(0, w)
        s = rng.uniform(smin, smax)
        img += rng.uniform(-90, 90) * np.exp(-(((xx - cx) / s) ** 2 + ((yy - cy) / s) ** 2) / 2)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def big_photo_37mp():
    """6144 x 6144 u8: noisy flat background plus six 512 x 512 blob patches (fixture
    tests/golden/sift_37mp.npz, generator tests/golden/make_sift_big.py)."""
    rng = np.random.default_rng(37)
    img = np.clip(np.rint(rng.normal(120, 2.0, (6144, 6144))), 0, 255).astype(np.uint8)
    for i, (y, x) in enumerate([(300, 400), (300, 5000), (2900, 2800), (5400, 700), (5300, 5300), (4000, 3900)]):
        img[y:y + 512, x:x + 512] = blob_image(512, 512, n_blobs=120, seed=100 + i)
    return img
