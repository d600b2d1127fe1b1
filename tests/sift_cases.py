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
