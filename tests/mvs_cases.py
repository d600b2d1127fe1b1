"""Shared cases for the openMVS export row: synthetic scenes
for the Interface writer and synthetic images + cameras for the undistortion."""
import numpy as np


def rot(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    a, b, c, d = q
    return np.array([[a*a+b*b-c*c-d*d, 2*(b*c-a*d), 2*(b*d+a*c)],
                     [2*(b*c+a*d), a*a-b*b+c*c-d*d, 2*(c*d-a*b)],
                     [2*(b*d-a*c), 2*(c*d+a*b), a*a-b*b-c*c+d*d]])


def interface_scene(n_cams=2, n_shots=9, n_points=300, seed=0):
    """cameras [(w, h, K)], shots [(camera or -1, recovered, pose 3x4, name)],
    points n x 3, origins CSR (with duplicates, unrecovered and camera-less
    shots mixed in)."""
    rng = np.random.default_rng(seed)
    cameras = []
    for c in range(n_cams):
        w, h = int(rng.integers(300, 5000)), int(rng.integers(200, 4000))
        f = float(rng.uniform(0.6, 1.4) * max(w, h))
        cameras.append((w, h, np.array([[f, 0, w / 2 + rng.normal()], [0, f, h / 2 + rng.normal()], [0, 0, 1]])))
    shots = []
    for s in range(n_shots):
        cam = int(rng.integers(0, n_cams)) if s % 7 != 5 else -1
        rec = bool(s % 4 != 3)
        pose = np.hstack([rot(rng), rng.normal(0, 3, (3, 1))])
        shots.append((cam, rec, pose, f"images/{1000 + 37 * s}.png" if s % 2 else f"/tmp/omvs/images/shot_{s}.png"))
    points = rng.normal(0, 10, (n_points, 3))
    lists = []
    for p in range(n_points):
        k = int(rng.integers(0, 6))
        lists.append(list(rng.integers(0, n_shots, k)))       # duplicates allowed (getOriginShots dedups)
    oo = np.zeros(n_points + 1, np.int64)
    oo[1:] = np.cumsum([len(x) for x in lists])
    osh = np.array([s for x in lists for s in x], np.int32)
    return cameras, shots, points, oo, osh


def image(rng, h, w, cn):
    """Smooth + noisy 8-bit image (so bilinear sums cover the whole range)."""
    yy, xx = np.mgrid[0:h, 0:w]
    base = 127.5 + 127.5 * np.sin(xx[..., None] * 0.05 + yy[..., None] * 0.031 + np.arange(cn) * 1.7)
    img = np.clip(base + rng.normal(0, 20, (h, w, cn)), 0, 255).astype(np.uint8)
    return img[..., 0] if cn == 1 else img


def camera(rng, h, w, strength=1.0):
    f = float(rng.uniform(0.5, 1.5) * max(w, h))
    K = np.array([[f, 0, w / 2 + rng.normal(0, 3)], [0, f, h / 2 + rng.normal(0, 3)], [0, 0, 1]])
    dist = np.array([rng.normal(0, 0.15), rng.normal(0, 0.05), rng.normal(0, 2e-3), rng.normal(0, 2e-3), 0.0]) * strength
    return K, dist


def undistort_cases(seed=0):
    """(img, K, dist) covering: 1/2/3/4 channels, widths not divisible by 4,
    > 4096 columns (one-row stripes), a 1 x 1 and a 1-row image, strong
    distortion (maps far outside the source), zero distortion, the SimpleRadial
    (k1, k2 only) model, a non-integral principal point."""
    rng = np.random.default_rng(seed)
    out = []
    for (h, w, cn, st) in [(97, 131, 3, 1.0), (64, 64, 1, 1.0), (45, 4103, 1, 0.5), (203, 149, 4, 3.0),
                           (31, 57, 2, 1.0), (1, 1, 3, 1.0), (1, 77, 1, 1.0), (120, 161, 3, 0.0),
                           (150, 90, 3, 20.0)]:
        K, dist = camera(rng, h, w, st)
        out.append((image(rng, h, w, cn), K, dist))
    K, dist = camera(rng, 80, 100)
    dist[2:] = 0                                              # SimpleRadialCamera: k1, k2
    out.append((image(rng, 80, 100, 3), K, dist))
    return out
