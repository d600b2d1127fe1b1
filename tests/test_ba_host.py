"""CPU: host-side BA pieces of libsfmx (no GPU): pose conversions
(CeresUtils::toCeresPose / toOpenCvPose), problem validation, synthetic shapes."""
import numpy as np
import pytest

from sfmx import ba, synth


def rot(axis, ang):
    axis = np.asarray(axis, float) / np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K


@pytest.mark.parametrize("axis,ang", [((1, 0, 0), 0.3), ((0, 1, 1), 2.0), ((1, 2, 3), 3.1), ((0, 0, 1), 0.0),
                                       ((1, -1, 0.5), 1e-9), ((0.2, 0.1, -1), np.pi - 1e-6)])
def test_pose_round_trip(axis, ang):
    R = rot(axis, ang)
    Rt = np.hstack([R, np.array([[1.0], [-2.0], [3.0]])])
    pose = ba.pose_to_ceres(Rt)
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    if ang > 1e-6:
        np.testing.assert_allclose(pose[:3], a * ang, atol=1e-6)
    np.testing.assert_allclose(pose[3:], [1, -2, 3])
    np.testing.assert_allclose(ba.pose_from_ceres(pose), Rt, atol=1e-9)


def test_problem_validation():
    p = synth.ba_problem(3, 10, seed=1)
    with pytest.raises(ValueError):
        ba.BAProblem(**{**p, "intr": np.zeros(2)})
    with pytest.raises(ValueError):
        ba.BAProblem(**{**p, "cam_model": 2, "intr": np.zeros(2)})


def test_c5_shape():
    p = synth.ba_problem(200, 2000, seed=2)       # C5 topology, fewer points (fast)
    assert p["poses"].shape == (200, 6) and len(p["obs_point"]) == 6 * 2000
    assert np.all(np.diff(p["obs_point"]) >= 0)   # point-major observations
    cams = p["obs_cam"].reshape(-1, 6)
    assert np.all((cams[:, 1:] - cams[:, :-1]) % 200 == 1)


# ---- the point-group topology the group kernels index (ba_solver.hip check_topology) ------------

def _ragged_problem(seed, n_cams, n_points, big_every=0, dup_every=0, empty_every=0, shuffle=False):
    """Ring-like tracks of 2..9 cameras, plus (optionally) long tracks (> 64 observations: big
    groups), a repeated camera inside a track (big) and points without observations."""
    rng = np.random.default_rng(seed)
    op, oc = [], []
    for p in range(n_points):
        if empty_every and p % empty_every == 3:
            continue
        if big_every and p % big_every == 1:
            cams = rng.integers(0, n_cams, 70)
        else:
            m = int(rng.integers(2, 10))
            cams = (int(rng.integers(0, n_cams)) + np.arange(m)) % n_cams
            if dup_every and p % dup_every == 2:
                cams = np.append(cams, cams[0])
        op += [p] * len(cams)
        oc += list(cams)
    op, oc = np.array(op, np.int32), np.array(oc, np.int32)
    if shuffle:                      # not point-major: the ordering's counting path
        perm = rng.permutation(len(op))
        op, oc = op[perm], oc[perm]
    xy = rng.uniform(0, 700, (len(op), 2))
    return ba.BAProblem(3, rng.normal(size=(n_points, 3)), rng.normal(size=(n_cams, 6)), np.array([800.0, 0.0, 0.0]),
                        op, oc, xy, 360.0, 200.0)


TOPO_CASES = [dict(seed=1, n_cams=10, n_points=1000), dict(seed=2, n_cams=40, n_points=3000, big_every=97),
              dict(seed=3, n_cams=7, n_points=2500, dup_every=13, empty_every=29),
              dict(seed=4, n_cams=200, n_points=20000, big_every=501, dup_every=333, shuffle=True),
              dict(seed=5, n_cams=3, n_points=300)]


@pytest.mark.parametrize("case", range(len(TOPO_CASES)))
@pytest.mark.parametrize("gpts", [1, 2, 3, 17, 99, 0])
def test_point_group_topology_holds_every_kernel_bound(case, gpts):
    """every index the group kernels derive from the host-built topology (group /
    chunk / batch ranges, feature rows, lane-map slots, camera slots, assembly entries inside sg / hbig
    / rg) is checked against the limits the kernels assume, for group sizes down to 1 point (the
    regime of the r03 launch failure), big and duplicate-camera points, empty points, and a
    non-point-major observation order."""
    from diag import diag_lib
    from sfmx import _lib
    P = _ragged_problem(**TOPO_CASES[case])
    st = P.struct()
    n = diag_lib().sfmx_ba_debug_check_topology(st, gpts, None)
    assert n > 0, _lib.lib.sfmx_last_error() or diag_lib().sfmx_last_error()


# ---- the incremental update's host half (sfmx_ba_update: unchanged camera buckets are kept) ----

def _inc_check(a, b, gpts=0):
    import ctypes as C
    from diag import diag_lib
    from sfmx import _lib
    out = (C.c_int32 * 2)()
    ms = (C.c_double * 11)()   # sfmx_ba_debug_incremental_check writes 11
    Pa, Pb = ba.BAProblem(**a), ba.BAProblem(**b)
    rc = diag_lib().sfmx_ba_debug_incremental_check(Pa.struct(), Pb.struct(), gpts, out, ms)
    assert rc == 0, diag_lib().sfmx_last_error()
    return out[0], out[1]


def test_sfm_order_is_a_permutation_of_the_same_problem():
    p = synth.ba_problem(30, 3000, seed=5)
    q = synth.ba_sfm_order(p)
    assert np.all(np.diff(q["obs_point"]) >= 0)
    key = lambda d: sorted(zip(map(tuple, np.round(np.asarray(d["points"])[d["obs_point"]], 12)), d["obs_cam"],
                               map(tuple, d["obs_xy"])))
    assert key(p) == key(q)


@pytest.mark.parametrize("steps", [(20, 40), (40, 41), (60, 80), (199, 200), (180, 200)])
def test_incremental_layout_equals_fresh_on_a_growing_scene(steps):
    """the grown scene's layout from the kept buckets equals a fresh load's
    bit for bit (orders, permutations, every topology array), and an SfM-ordered growth by one
    camera redoes only the buckets near the new camera (plus the ring's closing bucket)."""
    base = synth.ba_sfm_order(synth.ba_problem(200, 20000, seed=7))
    n_dirty, n_all = _inc_check(synth.ba_registered(base, steps[0]), synth.ba_registered(base, steps[1]))
    if steps[1] - steps[0] == 1:
        assert n_dirty <= 3, (n_dirty, n_all)


@pytest.mark.parametrize("case", ["xy", "points_gone", "cams_shrink", "not_point_major", "K_change", "same"])
def test_incremental_layout_equals_fresh_on_edits(case):
    rng = np.random.default_rng(11)
    a = synth.ba_sfm_order(synth.ba_problem(60, 8000, seed=12))
    b = dict(a)
    if case == "xy":            # a few pixels re-measured: their buckets redone
        xy = np.array(a["obs_xy"]); xy[rng.integers(0, len(xy), 5)] += 0.25; b["obs_xy"] = xy
    elif case == "points_gone":  # the last points dropped
        keep = a["obs_point"] < 7000
        b = dict(a, points=a["points"][:7000], obs_point=a["obs_point"][keep], obs_cam=a["obs_cam"][keep],
                 obs_xy=a["obs_xy"][keep])
    elif case == "cams_shrink":
        b = synth.ba_registered(a, 30)
    elif case == "not_point_major":
        perm = rng.permutation(len(a["obs_point"]))
        b = dict(a, obs_point=a["obs_point"][perm], obs_cam=a["obs_cam"][perm], obs_xy=a["obs_xy"][perm])
    elif case == "K_change":
        b = dict(a, cam_model=1, intr=a["intr"][:1])
    n_dirty, n_all = _inc_check(a, b)
    if case == "same":
        assert n_dirty == 0
    if case == "xy":
        assert 1 <= n_dirty <= 5
