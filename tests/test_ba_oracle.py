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
