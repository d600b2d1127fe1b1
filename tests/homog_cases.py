"""Shared synthetic cases for the homography step:
match graphs of planted-homography scenes plus hand-built edge cases.
Inputs only — the expected ratios come from oracle/homography_oracle.cpp."""
import numpy as np

from sfmx import synth
from sfmx.matching import DMATCH_DTYPE


def scene_case(n_img=6, n_desc=2000, seed=3):
    """Descriptor scene -> exact BF matches (oracle) -> planted-plane keypoints."""
    from oracle import oracle
    imgs, src, pn = synth.sift_images(n_img, n_desc, seed=seed, with_pool=True)
    kps = synth.scene_keypoints(src, pn, seed=seed + 1)
    pairs = oracle.pairs_unordered(n_img)
    m, off = oracle.match_pairs(imgs, pairs)
    return kps, [(720, 405)] * n_img, pairs, m, off


def _pack(lists):
    off = np.zeros(len(lists) + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in lists])
    m = np.zeros(int(off[-1]), DMATCH_DTYPE)
    k = 0
    for x in lists:
        for q, t in x:
            m[k] = (q, t, 0, 1.0)
            k += 1
    return m, off


def edge_case(seed=11):
    """Image 0/1 with crafted correspondences per pair:
      p0: 3 matches (< 4: ratio -1)       p1: exactly 4 matches
      p2: 4 collinear correspondences     p3: 5 copies of one point (every subset degenerate -> 0)
      p4: 3000 matches, 55 % on a homography (> LDS capacity, global path)
      p5: 600 matches, 90 % inliers       p6: 200 pure-noise matches
    """
    rng = np.random.default_rng(seed)
    n = 6000
    k0 = rng.uniform([0, 0], [1280, 720], (n, 2)).astype(np.float32)
    H = np.array([[0.9, 0.08, 40.0], [-0.05, 1.1, -20.0], [1e-4, -2e-4, 1.0]])
    ph = np.concatenate([k0, np.ones((n, 1), np.float32)], 1) @ H.T
    k1 = (ph[:, :2] / ph[:, 2:3] + rng.normal(0, 0.8, (n, 2))).astype(np.float32)
    k1[n // 2:] = rng.uniform([0, 0], [1280, 720], (n - n // 2, 2))      # second half: no relation
    k0[10:14] = np.array([[100, 100], [200, 200], [300, 300], [400, 400]], np.float32)
    k1[10:14] = np.array([[110, 90], [210, 190], [310, 290], [410, 390]], np.float32)
    lists = [
        [(0, 0), (1, 1), (2, 2)],
        [(20, 20), (21, 21), (22, 22), (23, 23)],
        [(10, 10), (11, 11), (12, 12), (13, 13)],
        [(5, 5)] * 5,
        [(i, i) for i in rng.choice(n // 2, 1650, replace=False)] + [(i, i) for i in rng.choice(np.arange(n // 2, n), 1350, replace=False)],
        [(i, i) for i in rng.choice(n // 2, 540, replace=False)] + [(i, i) for i in rng.choice(np.arange(n // 2, n), 60, replace=False)],
        [(i, i) for i in rng.choice(np.arange(n // 2, n), 200, replace=False)],
    ]
    m, off = _pack(lists)
    pairs = np.zeros((len(lists), 2), np.int32)
    pairs[:, 1] = 1
    return [k0, k1], [(1280, 720), (1280, 720)], pairs, m, off


def speculation_case(seed=21):
    """Pairs that stress the subset draw's speculation (homography.hip step 1): tiny lists (5 .. 12
    matches: repeated indices within an attempt are frequent), a list whose points are mostly on one line
    (most attempts fail checkSubset, so the rejections run on across speculation rounds), and a duplicated
    list (the same correspondence many times: every attempt repeats indices)."""
    rng = np.random.default_rng(seed)
    n = 400
    k0 = rng.uniform([0, 0], [1280, 720], (n, 2)).astype(np.float32)
    H = np.array([[1.05, 0.03, -12.0], [0.02, 0.97, 8.0], [5e-5, 1e-5, 1.0]])
    ph = np.concatenate([k0, np.ones((n, 1), np.float32)], 1) @ H.T
    k1 = (ph[:, :2] / ph[:, 2:3] + rng.normal(0, 0.5, (n, 2))).astype(np.float32)
    t = rng.uniform(0, 1, 120).astype(np.float32)   # points 200..319 on one line in both images
    k0[200:320] = np.stack([100 + 900 * t, 80 + 500 * t], 1)
    k1[200:320] = np.stack([130 + 880 * t, 60 + 520 * t], 1)
    lists = [[(int(i), int(i)) for i in rng.choice(200, m, replace=False)] for m in range(5, 13)]
    lists.append([(i, i) for i in range(200, 316)] + [(i, i) for i in range(4)])
    lists.append([(i % 7, i % 7) for i in range(60)])
    m, off = _pack(lists)
    pairs = np.zeros((len(lists), 2), np.int32)
    pairs[:, 1] = 1
    return [k0, k1], [(1280, 720), (1280, 720)], pairs, m, off
