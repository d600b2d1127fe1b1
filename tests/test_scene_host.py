"""Scene bookkeeping on the CPU: the oracle's literal
restatement of Scene::find3d2dMatches on a hand-built case with known answers,
and the native host builder of the BA observation arrays
(sfmx_ba_observations_from_origins, no device work) against the oracle's
find_if loop of BundleAdjustment.cpp:50-91."""
import numpy as np

from oracle import oracle
import scene_cases


def test_find_3d2d_edge_case_known_answers():
    kps, pairs, m, off, oo, osh, oxy = scene_cases.edge_case()
    k, p = oracle.find_3d2d_matches(kps, pairs, m, off, oo, osh, oxy, 0)
    #            dup pos  kp7@2   self   (6,7)   no pair  not float  NaN   -0.0   not in pair
    assert list(k) == [2, 1, -1, 6, -1, -1, -1, 8, -1]
    assert list(p) == [0, 1, -1, 0, -1, -1, -1, 1, -1]


def test_ba_observations_native_vs_oracle():
    import sfmx
    kps, pairs, m, off, oo, osh, oxy = scene_cases.scene_case(6, 800, seed=9)
    rng = np.random.default_rng(2)
    oxy = oxy + rng.normal(0, 1e-6, oxy.shape)           # exercise the cv::Point2f rounding
    got = sfmx.scene.ba_observations_from_origins(oo, osh, oxy, 6)
    op, oc, ox, sop = oracle.ba_observations(oo, osh, oxy, 6)
    assert np.array_equal(got["obs_point"], op) and np.array_equal(got["obs_cam"], oc)
    assert np.array_equal(got["obs_xy"], ox) and np.array_equal(got["shot_of_pose"], sop)
    assert np.array_equal(got["pose_of_shot"][sop], np.arange(len(sop)))
