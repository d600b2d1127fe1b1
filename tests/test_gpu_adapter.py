"""GPU: the compiled C++ caller of the ABI (tests/cpp/adapter_main.cpp + INTEGRATION.md §2's
GpuFeatureMatchingStrategy, built by __graft_entry__.build()) run as a separate process, as
the reference's SfM.cpp:545 would call calculateShotMatches.  Its ShotMatches must equal the
oracle's lists byte for byte, for SIFT (unordered / video) and ORB (grid)."""
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

import sfmx
from sfmx import synth

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "cpp", "adapter_test")


def _write(path, imgs, mode, seq, row_len):
    with open(path, "wb") as f:
        f.write(struct.pack("<4i", len(imgs), mode, seq, row_len))
        for x in imgs:
            f.write(struct.pack("<3i", x.shape[0], x.shape[1], 5 if x.dtype == np.float32 else 0))
            f.write(np.ascontiguousarray(x).tobytes())


def _read(path):
    out = []
    with open(path, "rb") as f:
        (n,) = struct.unpack("<q", f.read(8))
        for _ in range(n):
            l, r, c = struct.unpack("<iiq", f.read(16))
            m = np.frombuffer(f.read(16 * c), dtype=sfmx.DMATCH_DTYPE) if c else np.zeros(0, sfmx.DMATCH_DTYPE)
            out.append((l, r, m))
    return out


@pytest.mark.parametrize("case", ["sift_unordered", "sift_video", "orb_grid"])
def test_compiled_adapter_equals_oracle(case):
    from oracle import oracle
    assert os.path.exists(EXE), "tests/cpp/adapter_test not built (run __graft_entry__.build())"
    if case == "sift_unordered":
        imgs, mode, seq, rl = synth.sift_images(6, 2000, seed=71), 0, 2, 0
        imgs[2] = imgs[2][:777]
        pairs = sfmx.pairs_unordered(6)
    elif case == "sift_video":
        imgs, mode, seq, rl = synth.sift_images(5, 1500, seed=72), 1, 3, 0
        pairs = sfmx.pairs_video(5, 3)
    else:
        imgs, mode, seq, rl = synth.orb_images(6, 1800, seed=73), 2, 3, 3
        pairs = sfmx.pairs_grid(6, 3, 3, 0)
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        _write(fin, imgs, mode, seq, rl)
        r = subprocess.run([EXE, fin, fout], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        got = _read(fout)
    exp, eoff = oracle.match_pairs(imgs, pairs)
    assert [(l, r) for l, r, _ in got] == [tuple(p) for p in pairs]
    for p, (_, _, m) in enumerate(got):
        assert m.tobytes() == exp[eoff[p]:eoff[p + 1]].tobytes()


# ---- BundleAdjustment::doBundleAdjustment(Scene&) compiled -----------------
BA_EXE = os.path.join(HERE, "cpp", "ba_adapter_test")


def _ba_scene(p):
    """A reference-shaped scene of a problem dict (tests/cpp/ba_adapter_main.cpp's input): cameras
    (model, f, cx, cy, distortion), shots (camera, 3x4 pose), points with their origin points.
    Returns (bytes, the problem as the adapter hands it to the solver: poses through
    CeresUtils::toCeresPose, shots in first-appearance order)."""
    from sfmx import ba
    multi = p.get("intr_models") is not None
    models = np.asarray(p["intr_models"] if multi else [p["cam_model"]], np.int32)
    centers = np.asarray(p["centers"] if multi else [[p["cx"], p["cy"]]], np.float64).reshape(-1, 2)
    pim = np.asarray(p["pose_intr"] if multi else np.zeros(len(p["poses"])), np.int32)
    off = np.concatenate([[0], np.cumsum(models)])
    cams = np.zeros((len(models), 7))
    for m, k in enumerate(models):
        b = p["intr"][off[m]:off[m + 1]]
        cams[m, :3] = [b[0], centers[m, 0], centers[m, 1]]
        if k == 3:
            cams[m, 3:5] = b[1:3]
        if k == 7:
            cams[m, 1:3] = b[1:3]
            cams[m, 3:7] = b[3:7]
    Rt = np.stack([ba.pose_from_ceres(x) for x in p["poses"]])
    out = [struct.pack("<3i", len(models), len(Rt), len(p["points"]))]
    for m in range(len(models)):
        out.append(struct.pack("<i", int(models[m])) + cams[m].tobytes())
    for s in range(len(Rt)):
        out.append(struct.pack("<i", int(pim[s])) + Rt[s].tobytes())
    obs_point, obs_cam = np.asarray(p["obs_point"]), np.asarray(p["obs_cam"])
    order = np.argsort(obs_point, kind="stable")
    cnt = np.bincount(obs_point, minlength=len(p["points"]))
    rec = np.zeros(len(order), dtype=[("s", "<i4"), ("x", "<f8"), ("y", "<f8")])
    rec["s"], rec["x"], rec["y"] = obs_cam[order], p["obs_xy"][order, 0], p["obs_xy"][order, 1]
    starts = np.concatenate([[0], np.cumsum(cnt)])
    for q in range(len(p["points"])):
        out.append(np.asarray(p["points"][q], np.float64).tobytes() + struct.pack("<i", int(cnt[q])))
        out.append(rec[starts[q]:starts[q + 1]].tobytes())
    # what the adapter's solver sees: shots in first-appearance order (BundleAdjustment.cpp:64-79),
    # poses through toCeresPose, observations point-major as Point2f
    first = []
    seen = set()
    for s in obs_cam[order]:
        if s not in seen:
            seen.add(s)
            first.append(int(s))
    remap = np.full(len(Rt), -1, np.int32)
    remap[first] = np.arange(len(first))
    solver = dict(p, poses=np.stack([ba.pose_to_ceres(Rt[s]) for s in first]), obs_point=obs_point[order],
                  obs_cam=remap[obs_cam[order]], obs_xy=p["obs_xy"][order].astype(np.float32).astype(np.float64))
    if multi:
        solver["pose_intr"] = pim[first]
    return b"".join(out), solver, first


def _run_ba_adapter(p, td):
    fin, fout = os.path.join(td, "ba_in.bin"), os.path.join(td, "ba_out.bin")
    data, solver, first = _ba_scene(p)
    with open(fin, "wb") as f:
        f.write(data)
    r = subprocess.run([BA_EXE, fin, fout], capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return r, None, solver, first
    b = open(fout, "rb").read()
    conv, term, succ, unsucc = struct.unpack_from("<4i", b, 0)
    c0, c1 = struct.unpack_from("<2d", b, 16)
    P, S, M = len(p["points"]), len(p["poses"]), len(np.atleast_1d(p.get("intr_models", [0])))
    a = np.frombuffer(b, np.float64, offset=32)
    res = dict(converged=conv, termination=term, successful=succ, unsuccessful=unsucc, initial_cost=c0, final_cost=c1,
               points=a[:3 * P].reshape(P, 3), Rt=a[3 * P:3 * P + 12 * S].reshape(S, 3, 4),
               cams=a[3 * P + 12 * S:3 * P + 12 * S + 7 * M].reshape(M, 7))
    return r, res, solver, first


@pytest.mark.parametrize("cams", [((3, 1.0), (3, 1.1)), ((1, 1.0), (3, 0.95), (1, 1.05))])
def test_compiled_ba_adapter_several_cameras_equals_oracle(cams):
    """doBundleAdjustment on a scene with several cameras (mixed models): every camera's block
    registered and written back through ceresApplyParameters, each residual on its shot's camera;
    the final cost / termination / camera parameters equal the oracle's on the same problem."""
    from oracle import oracle
    assert os.path.exists(BA_EXE), "tests/cpp/ba_adapter_test not built (run __graft_entry__.build())"
    p = synth.ba_problem_multi(16, 1500, cameras=cams, seed=51)
    with tempfile.TemporaryDirectory() as td:
        r, res, solver, _ = _run_ba_adapter(p, td)
    assert r.returncode == 0, r.stderr
    sol, osm, _ = oracle.ba_solve(solver)
    assert res["termination"] == osm["termination_type"] and res["converged"] == (osm["termination_type"] == 0)
    assert abs(res["initial_cost"] - osm["initial_cost"]) <= 1e-12 * osm["initial_cost"]
    assert abs(res["final_cost"] - osm["final_cost"]) <= 1e-5 * osm["final_cost"]
    off = np.concatenate([[0], np.cumsum(p["intr_models"])])
    for m, k in enumerate(p["intr_models"]):
        b = sol["intr"][off[m]:off[m + 1]]
        np.testing.assert_allclose(res["cams"][m, 0], b[0], rtol=1e-5)                 # f (setFocalLength)
        if k == 3:
            np.testing.assert_allclose(res["cams"][m, 3:5], b[1:3], rtol=1e-3, atol=1e-7)   # k1, k2 (distortion)
        np.testing.assert_allclose(res["cams"][m, 1:3], p["centers"][m])               # centre kept (not a parameter)


def test_compiled_ba_adapter_rejects_over_capacity_loudly():
    """Three SIMPLE_RADIAL cameras (9 intrinsics parameters > SFMX_BA_MAX_INTR): the adapter throws
    instead of solving a different problem."""
    p = synth.ba_problem_multi(9, 200, cameras=((3, 1.0), (3, 1.1), (3, 0.9)), seed=52)
    with tempfile.TemporaryDirectory() as td:
        r, res, _, _ = _run_ba_adapter(p, td)
    assert r.returncode == 1 and "SFMX_BA_MAX_INTR" in r.stderr


@pytest.mark.timeout(600)
def test_compiled_ba_adapter_c5_equals_python_path_bit_for_bit():
    """BASELINE config 5 (200 cameras, 200k points, 1.2M observations, one SimpleRadial camera)
    through the compiled doBundleAdjustment: the same bits as the Python-path solve of the problem
    the adapter builds (shots in first-appearance order, poses through toCeresPose), whose C5 parity
    with the oracle test_gpu_fullsize.py checks."""
    from sfmx import ba
    p = synth.ba_problem(200, 200_000)
    with tempfile.TemporaryDirectory() as td:
        r, res, solver, first = _run_ba_adapter(p, td)
    assert r.returncode == 0, r.stderr
    P = ba.BAProblem(**solver)
    sm, _ = ba.solve(P)
    assert res["termination"] == sm["termination_type"] and res["final_cost"] == sm["final_cost"]
    assert res["successful"] == sm["num_successful_steps"] and res["unsuccessful"] == sm["num_unsuccessful_steps"]
    assert np.array_equal(res["points"], P.points)
    Rt = np.stack([ba.pose_from_ceres(x) for x in P.poses])
    assert np.array_equal(res["Rt"][first], Rt)
    assert res["cams"][0, 0] == P.intr[0] and np.array_equal(res["cams"][0, 3:5], P.intr[1:3])
