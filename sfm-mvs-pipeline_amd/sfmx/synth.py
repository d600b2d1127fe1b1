"""Synthetic inputs of the BASELINE.json shapes, fixed seeds.

Not part of the hot path: generates descriptor sets and BA problems for the
bench and the tests (there is no network for real image sets, and the
reference's insel JPEGs cannot be featurised here without OpenCV SIFT).
"""
from __future__ import annotations

import numpy as np

SIFT_SEED = 0x5F3D
ORB_SEED = 0x0B256


def _sift_quantise(x: np.ndarray) -> np.ndarray:
    """OpenCV-style SIFT descriptor quantisation: L2-normalise, clamp 0.2,
    renormalise, x512, round + saturate to [0,255] -> integer-valued float32."""
    x = x / np.maximum(np.linalg.norm(x, axis=-1, keepdims=True), 1e-12)
    x = np.minimum(x, 0.2)
    x = x / np.maximum(np.linalg.norm(x, axis=-1, keepdims=True), 1e-12)
    return np.clip(np.rint(x * 512.0), 0, 255).astype(np.float32)


def sift_images(n_images: int, n_desc: int, seed: int = SIFT_SEED, shared: float = 0.25,
                noise: float = 8.0, uniform: bool = False) -> list:
    """n_images x (n_desc x 128) float32 integer-valued SIFT-like descriptors.

    Images sit on a ring; image i re-observes (perturbed, sigma=noise,
    re-quantised) ``shared`` of its rows from a landmark pool it shares with
    its neighbours, so the ratio test accepts a realistic fraction of queries.
    ``uniform=True`` draws raw uniform 0..255 values instead (exercises the
    float-sqrt collision range)."""
    rng = np.random.default_rng(seed)
    if uniform:
        return [rng.integers(0, 256, size=(n_desc, 128)).astype(np.float32) for _ in range(n_images)]
    n_sh = int(n_desc * shared)
    pool_n = max(n_sh * 4, 1)
    pool = _sift_quantise(np.abs(rng.standard_normal((pool_n, 128), dtype=np.float32)))
    out = []
    for i in range(n_images):
        fresh = _sift_quantise(np.abs(rng.standard_normal((n_desc - n_sh, 128), dtype=np.float32)))
        start = (i * n_sh) % pool_n
        sel = (start + rng.permutation(n_sh * 2)[:n_sh]) % pool_n
        obs = np.clip(np.rint(pool[sel] + rng.normal(0, noise, size=(n_sh, 128))), 0, 255).astype(np.float32)
        img = np.concatenate([obs, fresh], axis=0)
        out.append(np.ascontiguousarray(img[rng.permutation(n_desc)]))
    return out


def orb_images(n_images: int, n_desc: int, seed: int = ORB_SEED, shared: float = 0.25, max_flips: int = 24) -> list:
    """n_images x (n_desc x 32) uint8 ORB-like 256-bit descriptors: uniform bits
    plus ``shared`` planted landmark copies with 0..max_flips flipped bits."""
    rng = np.random.default_rng(seed)
    n_sh = int(n_desc * shared)
    pool_n = max(n_sh * 4, 1)
    pool = rng.integers(0, 256, size=(pool_n, 32), dtype=np.uint8)
    out = []
    for i in range(n_images):
        fresh = rng.integers(0, 256, size=(n_desc - n_sh, 32), dtype=np.uint8)
        start = (i * n_sh) % pool_n
        sel = (start + rng.permutation(n_sh * 2)[:n_sh]) % pool_n
        obs = pool[sel].copy()
        bits = np.unpackbits(obs, axis=1)
        nflip = rng.integers(0, max_flips + 1, size=n_sh)
        for r in range(n_sh):
            bits[r, rng.choice(256, size=nflip[r], replace=False)] ^= 1
        obs = np.packbits(bits, axis=1)
        img = np.concatenate([obs, fresh], axis=0)
        out.append(np.ascontiguousarray(img[rng.permutation(n_desc)]))
    return out
