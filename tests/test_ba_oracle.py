"""CPU: the bundle-adjustment oracle (LM + DENSE_SCHUR restatement) pinned by
known optima, finite differences and the pose-conversion round trips."""
import numpy as np
import pytest

from oracle import oracle
from sfmx import synth


@pytest.mark.parametrize("model", [1, 3, 7])
def test_noise_free_converges_to_zero(model):
    p = synth.ba_problem(8, 300, seed=11, noise_px=0.0, cam_model=model)
    sol, sm, _ = oracle.ba_solve(p)
    assert sm["initial_cost"] > 1e3
    assert sm["final_cost"] < 1e-8 * sm["initial_cost"]
    assert sm["termination_type"] == 0          # CONVERGENCE


def test_noisy_reaches_noise_floor():
    p = synth.ba_problem(10, 800, seed=12, noise_px=0.5)
    sol, sm, tr = oracle.ba_solve(p, trace_cap=100)
    O = len(p["obs_point"])
    # E[cost] at the optimum ~ 1/2 * sigma^2 * (2 O - dof); allow a wide band
    assert 0.1 * 0.25 * O < sm["final_cost"] < 0.5 * 0.25 * 2 * O
    assert (np.diff(tr[tr[:, 2] == 1, 0]) <= 0).all()   # accepted steps never increase the cost


@pytest.mark.parametrize("model", [1, 3, 7])
def test_autodiff_matches_finite_differences(model):
    p = synth.ba_problem(4, 30, seed=13, cam_model=model)
    r, Je, Jc, Ji = oracle.ba_jacobian(p)
    h = 1e-6
    for o in (0, 7, 50):
        pt, cam = p["obs_point"][o], p["obs_cam"][o]
        for blk, J, n, key in (("points", Je, 3, pt), ("poses", Jc, 6, cam), ("intr", Ji, model, None)):
            for i in range(n):
                q1 = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in p.items()}
                q2 = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in p.items()}
                arr1, arr2 = q1[blk], q2[blk]
                if key is None:
                    step = h * max(1.0, abs(arr1[i]))
                    arr1[i] += step; arr2[i] -= step
                else:
                    step = h * max(1.0, abs(arr1[key][i]))
                    arr1[key][i] += step; arr2[key][i] -= step
                fd = (oracle.ba_jacobian(q1)[0][o] - oracle.ba_jacobian(q2)[0][o]) / (2 * step)
                np.testing.assert_allclose(J[o][:, i], fd, rtol=1e-4, atol=1e-6 * max(1.0, np.abs(fd).max()))


def test_zero_rotation_branch():
    # angle-axis exactly 0 takes AngleAxisRotatePoint's first-order branch; derivatives stay consistent
    p = synth.ba_problem(3, 20, seed=14)
    p["poses"][0, :3] = 0.0
    r, Je, Jc, Ji = oracle.ba_jacobian(p)
    o = int(np.nonzero(p["obs_cam"] == 0)[0][0])
    h = 1e-7
    for i in range(3):
        q1 = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in p.items()}
        q1["poses"][0, i] += h
        fd = (oracle.ba_jacobian(q1)[0][o] - r[o]) / h
        np.testing.assert_allclose(Jc[o][:, i], fd, rtol=1e-3, atol=1e-3)


# ---- several cameras (BundleAdjustment.cpp:45-48 registers every scene camera, :81-89 binds
# each residual to its shot's camera block) ----------------------------------------------------

MIXED = [((3, 1.0), (3, 1.1)), ((1, 1.0), (3, 0.95)), ((1, 1.0), (1, 1.05)), ((1, 1.0), (3, 1.1), (1, 0.9))]


def _split_by_camera(p, m):
    """The observations of camera m alone as a single-camera problem (same points / poses)."""
    models, pim = p["intr_models"], p["pose_intr"]
    off = np.concatenate([[0], np.cumsum(models)])
    sel = pim[p["obs_cam"]] == m
    q = dict(cam_model=int(models[m]), points=p["points"], poses=p["poses"], intr=p["intr"][off[m]:off[m + 1]],
             obs_point=p["obs_point"][sel], obs_cam=p["obs_cam"][sel], obs_xy=p["obs_xy"][sel],
             cx=float(p["centers"][m, 0]), cy=float(p["centers"][m, 1]))
    return q, sel, off


@pytest.mark.parametrize("cams", MIXED)
def test_multi_camera_jacobian_is_each_cameras_own(cams):
    """Known answer: an observation's residual and Jacobian are those of the single-camera problem
    of its camera (same functor, same block), its Ji columns sit at its camera's block of the
    caller's intr array and every other camera's columns are 0."""
    p = synth.ba_problem_multi(9, 200, cameras=cams, seed=31)
    r, Je, Jc, Ji = oracle.ba_jacobian(p)
    assert Ji.shape[2] == len(p["intr"])
    for m in range(len(cams)):
        q, sel, off = _split_by_camera(p, m)
        r1, Je1, Jc1, Ji1 = oracle.ba_jacobian(q)
        assert np.array_equal(r[sel], r1) and np.array_equal(Je[sel], Je1) and np.array_equal(Jc[sel], Jc1)
        assert np.array_equal(Ji[sel][:, :, off[m]:off[m + 1]], Ji1)
        mask = np.ones(len(p["intr"]), bool)
        mask[off[m]:off[m + 1]] = False
        assert not Ji[sel][:, :, mask].any()


@pytest.mark.parametrize("cams", MIXED + [((7, 1.0),), ((3, 1.0), (7, 1.02))])
def test_multi_camera_noise_free_converges_to_zero(cams):
    """Known optimum: noise-free observations of several cameras (mixed models) -> cost ~ 0 and
    every camera's focal length recovered to the generating value."""
    p = synth.ba_problem_multi(12, 600, cameras=cams, noise_px=0.0, seed=32)
    truth = synth.ba_problem_multi(12, 600, cameras=cams, noise_px=0.0, seed=32, perturb=False)
    sol, sm, _ = oracle.ba_solve(p)
    assert sm["initial_cost"] > 1e3 and sm["final_cost"] < 1e-8 * sm["initial_cost"]
    assert sm["termination_type"] == 0
    off = np.concatenate([[0], np.cumsum(p["intr_models"])])
    for m in range(len(cams)):
        assert abs(sol["intr"][off[m]] - truth["intr"][off[m]]) < 1e-3 * truth["intr"][off[m]]


def test_one_camera_block_form_equals_single_form():
    """n_intr = 1 describes the same Ceres problem as the single-block fields."""
    q = synth.ba_problem(10, 800, seed=5)
    q2 = dict(q, intr_models=np.array([3]), pose_intr=np.zeros(10, np.int32), centers=np.array([[q["cx"], q["cy"]]]))
    assert abs(oracle.ba_cost(q) - oracle.ba_cost(q2)) <= 1e-13 * oracle.ba_cost(q)   # OpenMP reduction order
    s1, m1, t1 = oracle.ba_solve(q, trace_cap=100)
    s2, m2, t2 = oracle.ba_solve(q2, trace_cap=100)
    assert abs(m1["final_cost"] - m2["final_cost"]) <= 1e-12 * m1["final_cost"]   # OpenMP sums: rounding only
    assert np.array_equal(t1[:, 2], t2[:, 2]) and m1["termination_type"] == m2["termination_type"]


def test_unreferenced_camera_is_not_a_parameter():
    """A camera no residual names is not in the Ceres problem: its block stays as it was and the
    solve is the one without it."""
    q = synth.ba_problem(10, 800, seed=5)
    q3 = dict(q, intr_models=np.array([7, 3]), pose_intr=np.ones(10, np.int32),
              centers=np.array([[1.0, 2.0], [q["cx"], q["cy"]]]), intr=np.concatenate([np.arange(7.0), q["intr"]]))
    s1, m1, t1 = oracle.ba_solve(q, trace_cap=100)
    s3, m3, t3 = oracle.ba_solve(q3, trace_cap=100)
    assert np.array_equal(s3["intr"][:7], np.arange(7.0))
    assert abs(m1["final_cost"] - m3["final_cost"]) <= 1e-12 * m1["final_cost"]
    assert np.array_equal(t1[:, 2], t3[:, 2])
