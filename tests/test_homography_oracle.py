"""CPU checks of the homography restatement (oracle/homography_oracle.cpp, the
parity reference for the GPU kernel of SURVEY.md §8 row f1).  The reference's
arithmetic lives in OpenCV 4.5.1 (absent): parity against it is unpinned; these
tests pin the restatement's own behaviour on cases whose answer is known."""
import numpy as np

from oracle import oracle
import homog_cases


def test_edge_cases_known_answers():
    kps, sizes, pairs, m, off = homog_cases.edge_case()
    r = oracle.homography_ratios(kps, sizes, pairs, m, off, threshold=-3.0)
    assert r[0] == -1.0                       # < 4 matches: skipped (SfM.cpp:606-609)
    assert r[1] == 1.0                        # 4 points: direct kernel, mask all ones
    assert r[3] == 0.0                        # every minimal subset degenerate: RANSAC fails
    assert 0.45 < r[4] <= 0.55                # planted 55 % inliers (minimal-sample models, no refit)
    assert 0.80 < r[5] <= 0.90
    assert r[6] < 0.2                         # noise only
    # deterministic (cv::RNG((uint64)-1)) and thread-count independent
    r2 = oracle.homography_ratios(kps, sizes, pairs, m, off, threshold=-3.0, nthreads=1)
    assert np.array_equal(r, r2)


def test_relative_threshold_and_scene():
    kps, sizes, pairs, m, off = homog_cases.scene_case(5, 1500, seed=4)
    a = oracle.homography_ratios(kps, sizes, pairs, m, off, threshold=-3.0)
    b = oracle.homography_ratios(kps, sizes, pairs, m, off, threshold=3.0 / 720)   # max(w, h, h, h) * t = 3 px
    assert np.array_equal(a, b)
    counts = np.diff(off)
    assert np.all((a == -1) == (counts < 4))
    assert np.all(a[counts >= 20] > 0.5)      # the planted plane dominates the accepted matches
