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
                noise: float = 8.0, uniform: bool = False, with_pool: bool = False):
    """n_images x (n_desc x 128) float32 integer-valued SIFT-like descriptors.

    Images sit on a ring; image i re-observes (perturbed, sigma=noise,
    re-quantised) ``shared`` of its rows from a landmark pool it shares with
    its neighbours, so the ratio test accepts a realistic fraction of queries.
    ``uniform=True`` draws raw uniform 0..255 values instead (exercises the
    float-sqrt collision range).  ``with_pool=True`` also returns, per image,
    the landmark-pool index of every row (-1 for fresh rows) and the pool size."""
    rng = np.random.default_rng(seed)
    if uniform:
        return [rng.integers(0, 256, size=(n_desc, 128)).astype(np.float32) for _ in range(n_images)]
    n_sh = int(n_desc * shared)
    pool_n = max(n_sh * 4, 1)
    pool = _sift_quantise(np.abs(rng.standard_normal((pool_n, 128), dtype=np.float32)))
    out, src = [], []
    for i in range(n_images):
        fresh = _sift_quantise(np.abs(rng.standard_normal((n_desc - n_sh, 128), dtype=np.float32)))
        start = (i * n_sh) % pool_n
        sel = (start + rng.permutation(n_sh * 2)[:n_sh]) % pool_n
        obs = np.clip(np.rint(pool[sel] + rng.normal(0, noise, size=(n_sh, 128))), 0, 255).astype(np.float32)
        img = np.concatenate([obs, fresh], axis=0)
        perm = rng.permutation(n_desc)
        out.append(np.ascontiguousarray(img[perm]))
        src.append(np.concatenate([sel, np.full(n_desc - n_sh, -1)]).astype(np.int64)[perm])
    return (out, src, pool_n) if with_pool else out


def scene_keypoints(src: list, pool_n: int, width: int = 720, height: int = 405, seed: int = 0x4B50,
                    noise_px: float = 0.7, plane_frac: float = 0.85) -> list:
    """Keypoints (n x 2 float32, cv::KeyPoint::pt) for the rows of sift_images(...,
    with_pool=True): a landmark on the dominant scene plane (``plane_frac`` of the
    pool) is seen by image i through a per-image homography H_i of the plane (a
    camera sliding along the insel-like sequence), + Gaussian pixel noise; other
    landmarks and fresh rows land uniformly in the image.  Pairs therefore carry
    a strong homography (the quantity SfM::calculateHomography measures,
    SfM.cpp:599-637) plus outliers."""
    rng = np.random.default_rng(seed)
    plane = rng.uniform(0, 1, (pool_n, 2))
    on_plane = rng.uniform(0, 1, pool_n) < plane_frac
    off_xy = np.stack([rng.uniform(0, width, pool_n), rng.uniform(0, height, pool_n)], axis=1)
    out = []
    for i, sidx in enumerate(src):
        a = 0.02 * i
        H = np.array([[0.8 * width * np.cos(a), -0.15 * height * np.sin(a), 0.1 * width + 3.0 * i],
                      [0.15 * width * np.sin(a), 0.8 * height * np.cos(a), 0.1 * height + 1.0 * i],
                      [0.05 * np.sin(0.3 * i), 0.04 * np.cos(0.2 * i), 1.0]])
        n = len(sidx)
        xy = np.stack([rng.uniform(0, width, n), rng.uniform(0, height, n)], axis=1)
        m = sidx >= 0
        p = sidx[m]
        ph = np.concatenate([plane[p], np.ones((len(p), 1))], axis=1) @ H.T
        proj = ph[:, :2] / ph[:, 2:3] + rng.normal(0, noise_px, (len(p), 2))
        xy[m] = np.where(on_plane[p][:, None], proj, off_xy[p] + rng.normal(0, noise_px, (len(p), 2)))
        out.append(np.ascontiguousarray(xy.astype(np.float32)))
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
        if max_flips > 0 and n_sh > 0:   # nflip[r] distinct random bits per planted row
            pos = np.argsort(rng.random((n_sh, 256)), axis=1)[:, :max_flips]
            valid = np.arange(max_flips)[None, :] < nflip[:, None]
            bits[np.nonzero(valid)[0], pos[valid]] ^= 1
        obs = np.packbits(bits, axis=1)
        img = np.concatenate([obs, fresh], axis=0)
        out.append(np.ascontiguousarray(img[rng.permutation(n_desc)]))
    return out


BA_SEED = 0xBA200


def _aa_from_R(R):
    """angle-axis of a rotation matrix (numpy, for synthetic truth only)."""
    c = np.clip((np.trace(R) - 1) / 2, -1, 1)
    th = np.arccos(c)
    if th < 1e-12:
        return np.zeros(3)
    v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    return v / (2 * np.sin(th)) * th


def _R_from_aa(aa):
    th = np.linalg.norm(aa)
    if th < 1e-12:
        return np.eye(3)
    k = aa / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def ba_problem(n_cams: int = 200, n_points: int = 200_000, obs_per_point: int = 6, noise_px: float = 0.5,
               seed: int = BA_SEED, cam_model: int = 3, width: int = 720, height: int = 405, perturb: bool = True,
               truth: bool = False):
    """BASELINE config 5 shape: cameras on a ring looking at the centre (insel
    720x405, f = 1.2 * 720 = 864 as PhotogrammetrieCli.cpp:312-314 sets it),
    every point seen by exactly `obs_per_point` consecutive cameras, pixel noise
    `noise_px`, initial perturbation 1e-2 rad / 1% translation / 1% f / 1e-2
    point noise.  Observations point-major, as the reference
    adds residual blocks (BundleAdjustment.cpp:50-90).  -> (BAProblem kwargs dict, truth dict)."""
    rng = np.random.default_rng(seed)
    f = 1.2 * max(width, height)
    cx, cy = width / 2.0, height / 2.0
    radius = 10.0
    poses = np.zeros((n_cams, 6))
    for c in range(n_cams):
        ang = 2 * np.pi * c / n_cams
        Cw = np.array([radius * np.cos(ang), radius * np.sin(ang), 0.3 * np.sin(3 * ang)])
        z = -Cw / np.linalg.norm(Cw)
        up = np.array([0.0, 0.0, 1.0])
        x = np.cross(up, z); x /= np.linalg.norm(x)
        y = np.cross(z, x)
        R = np.stack([x, y, z])            # world -> camera rows
        poses[c, :3] = _aa_from_R(R)
        poses[c, 3:] = -R @ Cw
    pts = np.concatenate([rng.uniform(-2.5, 2.5, (n_points, 2)), rng.uniform(-1.5, 1.5, (n_points, 1))], axis=1)
    k = cam_model
    intr = np.zeros(k)
    intr[0] = f
    if k == 7:
        intr[1], intr[2] = cx, cy
    start = rng.integers(0, n_cams, n_points)
    obs_point = np.repeat(np.arange(n_points, dtype=np.int32), obs_per_point)
    obs_cam = ((start[:, None] + np.arange(obs_per_point)[None, :]) % n_cams).astype(np.int32).reshape(-1)
    Rs = np.stack([_R_from_aa(p[:3]) for p in poses])
    Xc = np.einsum("oij,oj->oi", Rs[obs_cam], pts[obs_point]) + poses[obs_cam, 3:]
    xy = f * Xc[:, :2] / Xc[:, 2:3]
    xy = xy + np.array([cx, cy]) + rng.normal(0.0, noise_px, xy.shape)
    tr = {"points": pts.copy(), "poses": poses.copy(), "intr": intr.copy()}
    if perturb:
        poses = poses.copy()
        poses[:, :3] += rng.normal(0, 1e-2, (n_cams, 3))
        poses[:, 3:] *= 1.0 + rng.normal(0, 1e-2, (n_cams, 3))
        intr = intr.copy()
        intr[0] *= 1.0 + 0.01 * rng.standard_normal()
        pts = pts + rng.normal(0, 1e-2, pts.shape)
    prob = dict(cam_model=k, points=pts, poses=poses, intr=intr, obs_point=obs_point, obs_cam=obs_cam,
                obs_xy=xy, cx=cx, cy=cy)
    return (prob, tr) if truth else prob


def ba_registered(p: dict, n_cams: int) -> dict:
    """The BA problem of a scene after its first `n_cams` cameras are registered (SfM.cpp:235 / :371
    run BundleAdjustment after every registration): their observations of the points seen by at
    least two of them (a point exists once triangulated), in the original point order."""
    obs_point, obs_cam = np.asarray(p["obs_point"]), np.asarray(p["obs_cam"])
    keep_o = obs_cam < n_cams
    cnt = np.bincount(obs_point[keep_o], minlength=len(p["points"]))
    keep_p = cnt >= 2
    keep_o &= keep_p[obs_point]
    remap = np.cumsum(keep_p) - 1
    out = dict(p, points=np.asarray(p["points"])[keep_p], poses=np.asarray(p["poses"])[:n_cams],
               obs_point=remap[obs_point[keep_o]].astype(np.int32), obs_cam=obs_cam[keep_o].astype(np.int32),
               obs_xy=np.asarray(p["obs_xy"])[keep_o])
    if p.get("pose_intr") is not None:
        out["pose_intr"] = np.asarray(p["pose_intr"])[:n_cams]
    return out


def ba_sfm_order(p: dict) -> dict:
    """The same problem with its points in the order an incremental SfM creates them (SfM.cpp:235 /
    :371, cameras registered in index order): a point is triangulated when its second camera is
    registered, and the scene appends it then (ties: the original order); each point's observations
    in registration order.  ba_registered(ba_sfm_order(p), n) is the scene after n registrations."""
    obs_point, obs_cam = np.asarray(p["obs_point"]), np.asarray(p["obs_cam"])
    P = len(p["points"])
    o = np.lexsort((obs_cam, obs_point))                  # per point, cameras ascending
    op, oc = obs_point[o], obs_cam[o]
    start = np.searchsorted(op, np.arange(P + 1))
    cnt = np.diff(start)
    second = np.where(cnt >= 2, oc[np.minimum(start[:-1] + 1, len(oc) - 1)], np.iinfo(np.int32).max)
    pord = np.lexsort((np.arange(P), second))             # new point i = old point pord[i]
    rank = np.empty(P, np.int64)
    rank[pord] = np.arange(P)
    o2 = np.lexsort((oc, rank[op]))
    out = dict(p, points=np.asarray(p["points"])[pord], obs_point=rank[op][o2].astype(np.int32),
               obs_cam=oc[o2].astype(np.int32), obs_xy=np.asarray(p["obs_xy"])[o][o2])
    return out


def ba_problem_multi(n_cams: int = 24, n_points: int = 3000, cameras=((3, 1.0), (3, 1.1)), obs_per_point: int = 6,
                     noise_px: float = 0.5, seed: int = BA_SEED + 7, width: int = 720, height: int = 405,
                     perturb: bool = True, pose_intr=None):
    """Several physical cameras (scene.getCameras(), BundleAdjustment.cpp:45-48): camera m is
    (model k_m, focal scale s_m) with its own f = 1.2 * max(W, H) * s_m and principal point;
    pose c uses camera pose_intr[c] (default c % M), each residual its shot's camera
    (:81-89).  Ring geometry of ba_problem.  -> BAProblem kwargs dict (intr = the blocks back
    to back; DISTORTION blocks carry cx, cy as parameters)."""
    base, tr = ba_problem(n_cams, n_points, obs_per_point, 0.0, seed, 3, width, height, False, True)
    rng = np.random.default_rng(seed + 1)
    M = len(cameras)
    models = np.array([k for k, _ in cameras], np.int32)
    pim = np.asarray(pose_intr if pose_intr is not None else np.arange(n_cams) % M, np.int32)
    f = np.array([1.2 * max(width, height) * sc for _, sc in cameras])
    centers = np.stack([width / 2.0 + rng.uniform(-8, 8, M), height / 2.0 + rng.uniform(-8, 8, M)], 1)
    poses, pts = tr["poses"], tr["points"]
    obs_point, obs_cam = base["obs_point"], base["obs_cam"]
    Rs = np.stack([_R_from_aa(p[:3]) for p in poses])
    Xc = np.einsum("oij,oj->oi", Rs[obs_cam], pts[obs_point]) + poses[obs_cam, 3:]
    m_o = pim[obs_cam]
    xy = f[m_o, None] * Xc[:, :2] / Xc[:, 2:3] + centers[m_o] + rng.normal(0.0, noise_px, (len(obs_cam), 2))
    blocks = []
    for m, k in enumerate(models):
        b = np.zeros(k)
        b[0] = f[m]
        if k == 7:
            b[1], b[2] = centers[m]
        blocks.append(b)
    if perturb:
        poses = poses.copy()
        poses[:, :3] += rng.normal(0, 1e-2, (n_cams, 3))
        poses[:, 3:] *= 1.0 + rng.normal(0, 1e-2, (n_cams, 3))
        for b in blocks:
            b[0] *= 1.0 + 0.01 * rng.standard_normal()
        pts = pts + rng.normal(0, 1e-2, pts.shape)
    return dict(cam_model=int(models[0]), points=pts, poses=poses, intr=np.concatenate(blocks), obs_point=obs_point,
                obs_cam=obs_cam, obs_xy=xy, cx=0.0, cy=0.0, intr_models=models, pose_intr=pim, centers=centers)


def point_cloud_origins(src: list, kps: list, min_views: int = 2):
    """Point-cloud origin records (include/sfmx_scene.h layout) for a synthetic
    scene: every landmark of the pool seen by >= min_views images is a 3-D
    point; its origins are (image, keypoint position) of the rows carrying it,
    in image order — what PointcloudElement::getOriginPoints lists after
    triangulating the landmark from its matches (Scene.cpp:162-185).
    -> (origin_offsets[int64], origin_shot[int32], origin_xy[n x 2 float64])."""
    rows = []
    for i, s in enumerate(src):
        r = np.nonzero(s >= 0)[0]
        rows.append(np.stack([s[r], np.full(len(r), i), r], axis=1))
    allr = np.concatenate(rows) if rows else np.zeros((0, 3), np.int64)
    order = np.lexsort((allr[:, 2], allr[:, 1], allr[:, 0]))   # landmark, image, row
    allr = allr[order]
    lm, start, cnt = np.unique(allr[:, 0], return_index=True, return_counts=True)
    keep = cnt >= min_views
    sel = np.concatenate([np.arange(s, s + c) for s, c in zip(start[keep], cnt[keep])]) if keep.any() else np.zeros(0, int)
    recs = allr[sel]
    off = np.zeros(int(keep.sum()) + 1, np.int64)
    off[1:] = np.cumsum(cnt[keep])
    xy = np.array([kps[int(i)][int(r)] for _, i, r in recs], np.float64).reshape(-1, 2)
    return off, recs[:, 1].astype(np.int32), xy


def gray_photo(height: int, width: int, seed: int = 0, density: float = 1 / 400) -> np.ndarray:
    """Synthetic 8-bit grayscale "photo" for the SIFT extraction row (SURVEY.md
    §8 f3): a smooth shaded background plus many small Gaussian blobs of random
    scale (1.2-6 px) and contrast, plus sensor noise -- enough structure for the
    reference's contrast threshold 0.09 to keep thousands of keypoints."""
    r = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:height, 0:width].astype(np.float32)
    img = 110 + 40 * np.sin(xx / 23.0 + r.uniform(0, 6)) * np.cos(yy / 17.0)
    n = int(height * width * density)
    cy, cx = r.uniform(0, height, n), r.uniform(0, width, n)
    s = r.uniform(1.2, 6.0, n)
    a = r.uniform(-90, 90, n)
    for i in range(n):
        y0, y1 = int(max(cy[i] - 3 * s[i], 0)), int(min(cy[i] + 3 * s[i] + 1, height))
        x0, x1 = int(max(cx[i] - 3 * s[i], 0)), int(min(cx[i] + 3 * s[i] + 1, width))
        if y1 <= y0 or x1 <= x0:
            continue
        img[y0:y1, x0:x1] += a[i] * np.exp(-((xx[y0:y1, x0:x1] - cx[i]) ** 2 + (yy[y0:y1, x0:x1] - cy[i]) ** 2)
                                           / (2 * s[i] ** 2))
    return np.clip(np.rint(img + r.normal(0, 3, img.shape)), 0, 255).astype(np.uint8)
