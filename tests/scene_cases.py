"""Inputs for the scene-bookkeeping tests: a synthetic
scene with its point-cloud origins, and a hand-built edge case.  Expected
outputs come from oracle/scene_oracle.cpp (the reference's literal loops)."""
import numpy as np

from sfmx import synth
from sfmx.matching import DMATCH_DTYPE


def scene_case(n_img=8, n_desc=1500, seed=3):
    from oracle import oracle
    imgs, src, pn = synth.sift_images(n_img, n_desc, seed=seed, with_pool=True)
    kps = synth.scene_keypoints(src, pn, seed=seed + 2)
    oo, osh, oxy = synth.point_cloud_origins(src, kps)
    pairs = oracle.pairs_unordered(n_img)
    m, off = oracle.match_pairs(imgs, pairs)
    return kps, pairs, m, off, oo, osh, oxy


def edge_case():
    """Shot 0 is the new shot.  Covered: the first of two pairs joining the same
    shots wins; duplicate keypoint positions (the first DMatch in list order
    wins); shot 0 on the right of a pair (the other side is queryIdx); an origin
    on shot 0 itself; a shot without a pair; a position that is not a float;
    NaN; -0.0 equal to +0.0; an empty pair list entry."""
    rng = np.random.default_rng(1)
    kps = [rng.uniform(0, 500, (12, 2)).astype(np.float32) for _ in range(4)]
    kps[1][9] = kps[1][5]                       # duplicate positions in image 1
    kps[2][4] = (0.0, 5.0)
    pairs = np.array([[0, 1], [2, 0], [0, 1], [1, 2], [3, 1]], np.int32)
    lists = [
        [(2, 9), (3, 5), (6, 7)],               # pair 0 (0,1): kp1[9] == kp1[5]; first in list is (2, 9)
        [(4, 8), (7, 1), (1, 2)],               # pair 1 (2,0): shot 0 on the right
        [(10, 7), (11, 0)],                     # pair 2 (0,1) again: never used (pair 0 comes first)
        [(0, 0)],                               # pair 3 (1,2)
        [],                                     # pair 4 (3,1): empty
    ]
    off = np.zeros(len(lists) + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in lists])
    m = np.zeros(int(off[-1]), DMATCH_DTYPE)
    k = 0
    for x in lists:
        for q, t in x:
            m[k] = (q, t, 0, 1.0)
            k += 1
    k1, k2 = kps[1].astype(np.float64), kps[2].astype(np.float64)
    origins = [
        [(1, k1[5]), (2, k2[7])],               # duplicate position -> DMatch (2, 9); image 2 kp7 -> pair 1 match (7, 1)
        [(0, kps[0][3].astype(np.float64)), (1, k1[7])],   # origin on shot 0 itself; (6, 7) in pair 0
        [(3, kps[3][2].astype(np.float64))],    # shot 3 has a pair only with 1: no match
        [(1, k1[0] + [1e-9, 0.0])],             # not a float position: no match
        [(2, np.array([np.nan, 3.0]))],         # NaN: no match
        [(2, np.array([-0.0, 5.0])), (1, k1[8])],  # -0.0 == +0.0 -> (4, 8) in pair 1; k1[8] not in pair 0
    ]
    oo = np.zeros(len(origins) + 1, np.int64)
    oo[1:] = np.cumsum([len(x) for x in origins])
    osh = np.array([s for x in origins for s, _ in x], np.int32)
    oxy = np.array([p for x in origins for _, p in x], np.float64).reshape(-1, 2)
    return kps, pairs, m, off, oo, osh, oxy
