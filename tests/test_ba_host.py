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
