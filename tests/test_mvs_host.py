"""openMVS export on the CPU: the native Interface
writer (sfmx_openmvs_serialize, host code) byte-for-byte against the oracle's
plain-Python restatement of OpenMvsUtils::toOpenMVS + ARCHIVE::SerializeSave,
and the C undistortion oracle against an independent numpy restatement of
cv::undistort (vectorised map, np.add.accumulate for the sequential _x sum)."""
import numpy as np
import pytest

from oracle import oracle
import mvs_cases


@pytest.mark.parametrize("version", [1, 2, 3])
@pytest.mark.parametrize("seed", [0, 1])
def test_serialize_matches_oracle(version, seed):
    import sfmx
    cams, shots, pts, oo, osh = mvs_cases.interface_scene(seed=seed)
    got, ni, nv = sfmx.mvs.serialize(cams, shots, pts, oo, osh, version=version)
    iface = oracle.openmvs_interface(cams, shots, pts, oo, osh)
    want = oracle.openmvs_serialize(iface, version)
    assert got == want
    assert ni == len(iface["images"]) and nv == len(iface["vertices"])
    back = oracle.openmvs_parse(got)
    assert back["version"] == version and len(back["platforms"]) == len(cams)
    for v in back["vertices"]:
        ids = [i for i, _ in v["views"]]
        assert len(ids) >= 2 and ids == sorted(set(ids))


def test_interface_semantics():
    """toOpenMVS rules on a hand-made scene: unrecovered / camera-less shots are
    not images; poses go to their camera's platform in shot order; C = -R^T t;
    vertices need two distinct image views."""
    import sfmx
    K = np.array([[500., 0, 320], [0, 500, 240], [0, 0, 1]])
    R = mvs_cases.rot(np.random.default_rng(3))
    t = np.array([1., -2., 3.])
    P = np.hstack([R, t[:, None]])
    cams = [(640, 480, K), (800, 600, 2 * K)]
    shots = [(0, True, P, "a"), (1, True, P, "b"), (0, False, P, "c"), (-1, True, P, "d"), (0, True, P, "e")]
    pts = np.array([[1., 2, 3], [4, 5, 6], [7, 8, 9], [0.1, 0.2, 0.3]])
    lists = [[0, 1], [0, 0, 2], [4, 3, 1, 4], [2, 3]]
    oo = np.r_[0, np.cumsum([len(x) for x in lists])]
    osh = np.array(sum(lists, []), np.int32)
    buf, ni, nv = sfmx.mvs.serialize(cams, shots, pts, oo, osh)
    d = oracle.openmvs_parse(buf)
    assert [im["name"] for im in d["images"]] == ["a", "b", "e"]
    assert [(im["platformID"], im["poseID"]) for im in d["images"]] == [(0, 0), (1, 0), (0, 1)]
    assert len(d["platforms"][0]["poses"]) == 2 and len(d["platforms"][1]["poses"]) == 1
    np.testing.assert_allclose(d["platforms"][0]["poses"][0]["C"], -R.T @ t, rtol=1e-15, atol=1e-15)
    assert d["platforms"][1]["cameras"][0]["width"] == 800
    np.testing.assert_array_equal(d["platforms"][1]["cameras"][0]["R"], np.eye(3))
    assert [[i for i, _ in v["views"]] for v in d["vertices"]] == [[0, 1], [1, 2]]
    np.testing.assert_array_equal(d["vertices"][1]["X"], np.float32([7, 8, 9]))
    assert (ni, nv) == (3, 2)


def test_capacity_and_errors(tmp_path):
    import sfmx
    import ctypes as C
    cams, shots, pts, oo, osh = mvs_cases.interface_scene(seed=4)
    keep, args = sfmx.mvs._scene_args(cams, shots, pts, oo, osh)
    size = C.c_int64(0)
    small = (C.c_uint8 * 16)()
    assert sfmx._lib.lib.sfmx_openmvs_serialize(1, *args, small, 16, C.byref(size), None, None) == -4
    full, _, _ = sfmx.mvs.serialize(cams, shots, pts, oo, osh)
    assert size.value == len(full) and bytes(small) == full[:16]
    assert sfmx._lib.lib.sfmx_openmvs_serialize(4, *args, None, 0, C.byref(size), None, None) == -1
    bad = osh.copy()
    bad[0] = len(shots)
    with pytest.raises(ValueError, match="origin shot out of range"):   # SFMX_EINVAL
        sfmx.mvs.serialize(cams, shots, pts, oo, bad)
    out, ni, nv, _ = sfmx.mvs.toOpenMVS(cams, [s[:3] for s in shots], pts, oo, osh, str(tmp_path / "omvs"),
                                        relativePaths=True)
    d = oracle.openmvs_parse(open(out, "rb").read())
    assert len(d["images"]) == ni and all(im["name"].startswith("images/") for im in d["images"])


def _np_undistort(img, K, dist):
    """Independent numpy restatement of cv::undistort (the C oracle's twin)."""
    img3 = img[..., None] if img.ndim == 2 else img
    H, W, cn = img3.shape
    K = np.asarray(K, np.float64).reshape(3, 3)
    k1, k2, p1, p2, k3 = np.r_[np.ravel(dist), np.zeros(5)][:5]
    fx, fy, u0, v0 = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    stripe0 = min(max(1, 4096 // W), H)
    det = fx * fy
    d = 1.0 / det
    t0, t2, t4, t8 = fy * d, (0.0 - u0 * fy) * d, fx * d, det * d
    xs = np.add.accumulate(np.r_[0.0 + t2, np.full(W - 1, t0)])
    Y = np.arange(H)
    ys = (Y // stripe0) * stripe0
    t5 = (0.0 - fx * (v0 - ys)) * d
    yr = (Y - ys) * t4 + t5
    w = 1.0 / t8
    x = (xs * w)[None, :]
    y = (yr * w)[:, None]
    x2, y2 = x * x, y * y
    r2 = x2 + y2
    _2xy = 2 * x * y
    kr = 1 + ((k3 * r2 + k2) * r2 + k1) * r2
    xd = x * kr + p1 * _2xy + p2 * (r2 + 2 * x2)
    yd = y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy
    u, v = fx * xd + u0, fy * yd + v0

    def rnd(a):
        r = np.rint(a * 32)
        bad = ~((r >= -2**31) & (r <= 2**31 - 1))
        return np.where(bad, -2**31, np.where(bad, 0, r)).astype(np.int64)
    iu, iv = rnd(u), rnd(v)
    sx = ((iu >> 5) & 0xFFFF).astype(np.uint16).view(np.int16).astype(np.int64)
    sy = ((iv >> 5) & 0xFFFF).astype(np.uint16).view(np.int16).astype(np.int64)
    a, b = iu & 31, iv & 31
    w0 = np.minimum((32 - b) * (32 - a) * 32, 32767)
    ws = [w0, (32 - b) * a * 32, b * (32 - a) * 32, b * a * 32]
    acc = np.zeros((H, W, cn), np.int64)
    for (dx, dy), wk in zip([(0, 0), (1, 0), (0, 1), (1, 1)], ws):
        px, py = sx + dx, sy + dy
        ok = (px >= 0) & (px < W) & (py >= 0) & (py < H)
        vals = img3[np.clip(py, 0, H - 1), np.clip(px, 0, W - 1)].astype(np.int64)
        acc += np.where(ok[..., None], vals * wk[..., None], 0)
    out = np.clip((acc + 16384) >> 15, 0, 255).astype(np.uint8)
    return out[..., 0] if img.ndim == 2 else out


def test_undistort_oracle_vs_numpy_restatement():
    for img, K, dist in mvs_cases.undistort_cases(seed=5):
        np.testing.assert_array_equal(oracle.undistort(img, K, dist), _np_undistort(img, K, dist))


def test_undistort_oracle_identity_and_shift():
    """Zero distortion, integral principal point: the output is the input."""
    rng = np.random.default_rng(0)
    img = mvs_cases.image(rng, 60, 83, 3)
    K = np.array([[70., 0, 41], [0, 70, 30], [0, 0, 1]])
    np.testing.assert_array_equal(oracle.undistort(img, K, np.zeros(4)), img)


def test_undistort_rejects_bad_input():
    import sfmx
    img = np.zeros((10, 10, 3), np.uint8)
    K = np.array([[10., 0.5, 5], [0, 10, 5], [0, 0, 1]])            # skew: not an ICamera K
    with pytest.raises(ValueError, match="camera matrix"):             # validated before any device call
        sfmx.mvs.undistort([img], [K], [np.zeros(4)])
    with pytest.raises(ValueError, match="channels"):
        sfmx.mvs.undistort([np.zeros((10, 10, 5), np.uint8)], [np.eye(3)], [np.zeros(4)])


def test_serialize_capacity_retry_and_errors(monkeypatch):
    """The wrapper's one native call into a bound-sized buffer: a bound that falls short takes the
    exact size from SFMX_ECAPACITY and calls again (same bytes); invalid origins still raise."""
    import sfmx
    cams, shots, pts, oo, osh = mvs_cases.interface_scene(seed=0)
    want, ni, nv = sfmx.mvs.serialize(cams, shots, pts, oo, osh)
    monkeypatch.setattr(sfmx.mvs, "_serialize_bound", lambda *a: 16)
    got, ni2, nv2 = sfmx.mvs.serialize(cams, shots, pts, oo, osh)
    assert got == want and (ni2, nv2) == (ni, nv)
    bad = np.array(osh, np.int32).copy()
    bad[0] = len(shots) + 5
    with pytest.raises(Exception):
        sfmx.mvs.serialize(cams, shots, pts, oo, bad)
