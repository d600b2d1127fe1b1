"""GPU parity for the homography step: the HIP RANSAC
kernel (through the C ABI) against oracle/homography_oracle.cpp, bit-exact:
both restate OpenCV 4.5.1's deterministic findHomography RANSAC with the same
operation order and no FMA contraction."""
import numpy as np
import pytest
import torch

import sfmx
from sfmx import homography
import homog_cases

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [3, 8])
def test_scene_graph_bit_exact(seed):
    from oracle import oracle
    kps, sizes, pairs, m, off = homog_cases.scene_case(7, 2500, seed=seed)
    exp = oracle.homography_ratios(kps, sizes, pairs, m, off)
    got = homography.homography_ratios(kps, sizes, pairs, m, off)
    assert np.array_equal(got, exp), (got, exp)


def test_edge_cases_bit_exact():
    from oracle import oracle
    kps, sizes, pairs, m, off = homog_cases.edge_case()
    for thr, iters, conf in ((-3.0, 2000, 0.995), (-1.0, 50, 0.9), (0.004, 2000, 0.999)):
        exp = oracle.homography_ratios(kps, sizes, pairs, m, off, thr, iters, conf)
        got = homography.homography_ratios(kps, sizes, pairs, m, off, thr, iters, conf)
        assert np.array_equal(got, exp), (thr, got, exp)


def test_device_inputs_and_strategy_mirror():
    kps, sizes, pairs, m, off = homog_cases.scene_case(5, 1500, seed=6)
    host = homography.homography_ratios(kps, sizes, pairs, m, off)
    dk = [torch.from_numpy(k).cuda() for k in kps]
    dm = torch.from_numpy(m.view(np.uint8)).cuda()
    do = torch.from_numpy(off).cuda()
    dev = homography.homography_ratios_device([t.data_ptr() for t in dk], [len(k) for k in kps], sizes, pairs,
                                              dm.data_ptr(), do.data_ptr())
    assert np.array_equal(host, dev)
    scene = sfmx.Scene([sfmx.Shot(f"img{i}", None, k, s) for i, (k, s) in enumerate(zip(kps, sizes))])
    sms = [sfmx.ShotMatches(int(l), int(r), m[off[p]:off[p + 1]]) for p, (l, r) in enumerate(pairs)]
    homography.calculateHomography(scene, sms)
    assert np.array_equal([s.getHomographyInlierRatio() for s in sms], host)


def test_invalid_index_rejected():
    kps, sizes, pairs, m, off = homog_cases.edge_case()
    m = m.copy()
    m["trainIdx"][5] = 10 ** 6
    with pytest.raises(ValueError):
        homography.homography_ratios(kps, sizes, pairs, m, off)


def test_device_list_past_the_scratch_bound_is_nan():
    # device inputs are not read back: the scratch for lists over 2048 matches is sized from the
    # host-known keypoint counts (one match per query keypoint); a list past that bound is NaN, the
    # same list from the host is solved (sfmx_homography.h)
    kps, sizes, pairs, m, off = homog_cases.scene_case(5, 1500, seed=6)
    l = int(pairs[0][0])
    n = max(len(kps[l]) + 600, 2100)
    mm = np.resize(m[off[0]:off[1]], n)
    one = np.asarray(pairs[:1])
    o = np.array([0, n], np.int64)
    host = homography.homography_ratios(kps, sizes, one, mm, o)
    assert np.isfinite(host[0])
    dk = [torch.from_numpy(k).cuda() for k in kps]
    dm = torch.from_numpy(mm.view(np.uint8)).cuda()
    do = torch.from_numpy(o).cuda()
    dev = homography.homography_ratios_device([t.data_ptr() for t in dk], [len(k) for k in kps], sizes, one,
                                              dm.data_ptr(), do.data_ptr())
    assert np.isnan(dev[0])


def test_speculated_subset_draw_edge_cases_bit_exact():
    # tiny lists, a mostly collinear list (rejections across speculation rounds) and repeated matches,
    # each through several iteration budgets: the speculated draw takes the serial draw's subsets
    from oracle import oracle
    kps, sizes, pairs, m, off = homog_cases.speculation_case()
    for thr, iters, conf in ((-3.0, 2000, 0.995), (2.0, 37, 0.9), (-1.0, 2000, 0.999999)):
        exp = oracle.homography_ratios(kps, sizes, pairs, m, off, thr, iters, conf)
        got = homography.homography_ratios(kps, sizes, pairs, m, off, thr, iters, conf)
        assert np.array_equal(got, exp), (thr, iters, got, exp)
