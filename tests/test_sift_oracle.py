"""SIFT extraction oracle on the CPU: known-answer
behaviour of the restatement of OpenCV 4.5.1 SIFT::detectAndCompute
(oracle/sift_oracle.cpp) on synthetic images.  Parity against OpenCV itself
is unpinned (OpenCV is not available here)."""
import numpy as np

from oracle import oracle
import sift_cases


def test_single_blob_found_at_its_centre():
    h, w = 96, 128
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.clip(np.rint(60 + 150 * np.exp(-((xx - 70.3) ** 2 + (yy - 41.6) ** 2) / (2 * 6.0 ** 2))), 0, 255).astype(np.uint8)
    k, d = oracle.sift(img)
    assert len(k) >= 1
    best = k[np.argmax(k["response"])]
    assert abs(best["x"] - 70.3) < 1.0 and abs(best["y"] - 41.6) < 1.0
    # blob sigma 6 -> keypoint size ~ 2 * sqrt(2) * 6 (the DoG scale of a Gaussian blob)
    assert 8 < best["size"] < 30
    assert d.shape == (len(k), 128) and np.all(d == np.rint(d)) and d.min() >= 0 and d.max() <= 255


def test_outputs_sorted_unique_and_retain_best():
    img = sift_cases.blob_image(150, 200, n_blobs=150, seed=3)
    k, d = oracle.sift(img, contrast_threshold=0.04)                   # OpenCV's default: more points
    assert len(k) > 30
    key = [(r["x"], r["y"], -r["size"], r["angle"]) for r in k]
    assert key == sorted(key) and len(set(key)) == len(key)          # removeDuplicatedSorted order
    n = len(k) // 2
    k2, d2 = oracle.sift(img, nfeatures=n, contrast_threshold=0.04)
    thr = np.sort(k["response"])[::-1][n - 1]
    assert len(k2) >= n and np.all(k2["response"] >= thr)              # retainBest keeps boundary ties
    sel = k["response"] >= thr
    # retainBest reorders in place (nth_element + partition, OpenCV 4.5.1): same kept set, rows follow the keypoints
    order = np.lexsort((k2["angle"], -k2["size"], k2["y"], k2["x"]))
    assert np.array_equal(k2[order], k[sel]) and np.array_equal(d2[order], d[sel])
    assert np.all(k2["response"][:n] >= thr) and np.all(k2["response"][n:] == thr)   # nth_element boundary
    assert not np.array_equal(k2, k[sel])            # the reorder is visible on this case
    assert np.all((k["octave"] & 255).astype(np.int8) >= -1)           # firstOctave = -1 rescale


def test_descriptor_norm_and_rotation_behaviour():
    img = sift_cases.blob_image(160, 160, n_blobs=50, seed=5)
    k, d = oracle.sift(img)
    norms = np.linalg.norm(d, axis=1)
    assert np.all((norms > 400) & (norms < 560))                       # 512 / ||v|| scaling, integer rounding
    rot = np.ascontiguousarray(np.rot90(img))                          # 90 deg: same points, angles shifted
    kr, dr = oracle.sift(rot)
    assert abs(len(kr) - len(k)) <= max(3, len(k) // 5)
