"""openMVS export on the GPU: sfmx_undistort_images
(csrc/mvs.hip) bit-exact against the restatement of OpenCV's cv::undistort in
oracle/mvs_oracle.cpp, through the C ABI, in host and device modes."""
import numpy as np
import pytest

from oracle import oracle
import mvs_cases

pytestmark = pytest.mark.gpu


def test_cases_one_launch_bit_exact():
    import sfmx
    cases = mvs_cases.undistort_cases(seed=11)
    got = sfmx.mvs.undistort([c[0] for c in cases], [c[1] for c in cases], [c[2] for c in cases])
    for (img, K, dist), g in zip(cases, got):
        np.testing.assert_array_equal(g, oracle.undistort(img, K, dist), err_msg=f"{img.shape}")


@pytest.mark.parametrize("seed", [1, 2])
def test_photo_size_bit_exact(seed):
    """A 12 MP RGB photo with a SimpleRadial camera (the reference's model)."""
    import sfmx
    rng = np.random.default_rng(seed)
    img = mvs_cases.image(rng, 3000, 4000, 3)
    K, dist = mvs_cases.camera(rng, 3000, 4000)
    dist[2:] = 0
    (g,) = sfmx.mvs.undistort([img], [K], [dist])
    np.testing.assert_array_equal(g, oracle.undistort(img, K, dist))


def test_device_mode_padded_and_unaligned_rows():
    import torch
    import sfmx
    rng = np.random.default_rng(3)
    dev = torch.device("cuda:0")
    shapes = [(77, 131, 3), (64, 257, 1), (33, 4099, 1)]
    srcs, dsts, Ks, ds, want, parents = [], [], [], [], [], []
    for (h, w, cn) in shapes:
        img = mvs_cases.image(rng, h, w, cn)
        K, dist = mvs_cases.camera(rng, h, w)
        big = torch.zeros((h, w + 5) + ((cn,) if cn > 1 else ()), dtype=torch.uint8, device=dev)
        big[:, :w] = torch.from_numpy(img).to(dev)
        srcs.append(big[:, :w])                                  # padded src rows
        out = torch.full((h, w + 3) + ((cn,) if cn > 1 else ()), 7, dtype=torch.uint8, device=dev)
        dsts.append(out[:, 1:w + 1])                             # odd pitch and base: byte stores
        parents.append(out)
        Ks.append(K)
        ds.append(dist)
        want.append(oracle.undistort(img, K, dist))
    sfmx.mvs.undistort_device(srcs, dsts, Ks, ds)
    torch.cuda.synchronize()
    for d, w_, out, (h, w, cn) in zip(dsts, want, parents, shapes):
        np.testing.assert_array_equal(d.cpu().numpy(), w_)
        assert bool((out[:, 0] == 7).all()) and bool((out[:, w + 1:] == 7).all())   # padding untouched
    assert sfmx.mvs.last_kernel_ms() > 0


def test_to_openmvs_end_to_end(tmp_path):
    """toOpenMVS: interface file + undistorted images of the recovered shots."""
    import sfmx
    cams, shots, pts, oo, osh = mvs_cases.interface_scene(n_cams=2, n_shots=5, n_points=200, seed=8)
    rng = np.random.default_rng(8)
    small = [(96, 128, np.array([[110., 0, 64.5], [0, 110, 47.5], [0, 0, 1]])), (80, 60, np.array([[70., 0, 30], [0, 70, 40], [0, 0, 1]]))]
    images = [mvs_cases.image(rng, small[c][1], small[c][0], 3) if c >= 0 else None for (c, _, _, _) in shots]
    dists = [np.array([-0.1, 0.02, 0, 0]), np.array([0.05, 0.0, 0, 0])]
    out, ni, nv, und = sfmx.mvs.toOpenMVS(small, [s[:3] for s in shots], pts, oo, osh, str(tmp_path),
                                          images=images, dists=dists)
    d = oracle.openmvs_parse(open(out, "rb").read())
    assert len(d["images"]) == ni
    for s, (c, rec, _, _) in enumerate(shots):
        name = str(tmp_path / "images" / f"{s}.png")
        if rec and images[s] is not None:
            np.testing.assert_array_equal(und[name], oracle.undistort(images[s], small[c][2], dists[c]))
        else:
            assert name not in und


def test_shared_map_units_bit_exact():
    """Images with identical size, K and distortion (the reference's toOpenMVS: one
    camera for every shot) form one unit that reads a shared inverse map
    (map_kernel); mixed here with singleton images, other channel counts, a
    second shared camera, a -0.0 distortion term (bitwise-different key: its own
    unit) and, in device mode, padded rows and unaligned destinations inside a unit."""
    import torch
    import sfmx
    rng = np.random.default_rng(21)
    KA, dA = mvs_cases.camera(rng, 61, 203)
    dA[2:] = 0
    KB, dB = mvs_cases.camera(rng, 40, 1030, strength=2.0)
    dAz = dA.copy()
    dAz[4] = -0.0
    spec = [(61, 203, 3, KA, dA), (40, 1030, 1, KB, dB), (61, 203, 3, KA, dA), (61, 203, 1, KA, dA),
            (61, 203, 3, KA, dAz), (40, 1030, 1, KB, dB), (61, 203, 3, KA, dA), (61, 203, 1, KA, dA),
            (40, 1030, 1, KB, dB), (33, 47, 3, KA, dA)]
    imgs = [mvs_cases.image(rng, h, w, cn) for (h, w, cn, _, _) in spec]
    want = [oracle.undistort(i, K, d) for i, (_, _, _, K, d) in zip(imgs, spec)]
    got = sfmx.mvs.undistort(imgs, [s[3] for s in spec], [s[4] for s in spec])
    for g, w_, s in zip(got, want, spec):
        np.testing.assert_array_equal(g, w_, err_msg=f"host mode {s[:3]}")
    dev = torch.device("cuda:0")
    srcs, dsts, parents = [], [], []
    for k, (img, (h, w, cn, _, _)) in enumerate(zip(imgs, spec)):
        tail = (cn,) if cn > 1 else ()
        pad = 3 if k % 2 else 0
        big = torch.zeros((h, w + pad) + tail, dtype=torch.uint8, device=dev)
        big[:, :w] = torch.from_numpy(img).to(dev)
        srcs.append(big[:, :w])
        off = k % 3
        out = torch.full((h, w + 2) + tail, 9, dtype=torch.uint8, device=dev)
        dsts.append(out[:, off:off + w])
        parents.append(out)
    sfmx.mvs.undistort_device(srcs, dsts, [s[3] for s in spec], [s[4] for s in spec])
    torch.cuda.synchronize()
    for d, w_, s in zip(dsts, want, spec):
        np.testing.assert_array_equal(d.cpu().numpy(), w_, err_msg=f"device mode {s[:3]}")
