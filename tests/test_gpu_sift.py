"""SIFT extraction on the GPU: sfmx_sift_detect_compute
(csrc/sift_features.hip) bit-identical to the restatement in
oracle/sift_oracle.cpp -- keypoints (all seven cv::KeyPoint fields) and
descriptors -- through the C ABI, host and device modes."""
import numpy as np
import pytest

from oracle import oracle
import sift_cases

pytestmark = pytest.mark.gpu


def _check(img, **kw):
    import sfmx
    k, d = sfmx.features.SIFT.create(**kw).detectAndCompute(img)
    ok = {"nfeatures": kw.get("nfeatures", 0), "contrast_threshold": kw.get("contrastThreshold", 0.09)}
    ek, ed = oracle.sift(img, **ok)
    assert len(k) == len(ek), (len(k), len(ek))
    assert k.tobytes() == ek.tobytes()
    assert np.array_equal(d, ed)
    return k


@pytest.mark.parametrize("shape,seed", [((120, 160), 1), ((97, 131), 2), ((64, 300), 3), ((240, 320), 4)])
def test_bit_exact_reference_setting(shape, seed):
    _check(sift_cases.blob_image(*shape, n_blobs=80, seed=seed))


def test_bit_exact_many_points_and_limit():
    img = sift_cases.blob_image(300, 400, n_blobs=300, seed=7)
    k = _check(img, contrastThreshold=0.04)
    assert len(k) > 50
    _check(img, contrastThreshold=0.04, nfeatures=len(k) // 3)


@pytest.mark.parametrize("seed,nf", [(0, 0), (2, 0), (3, 1), (4, 2), (5, 0)])
def test_compute_from_undoubled_pyramid(seed, nf):
    """No kept keypoint from the doubled octave -> compute() rebuilds the pyramid from
    firstOctave = 0 (OpenCV 4.5.1 SIFT_Impl::detectAndCompute with useProvidedKeypoints)."""
    img = sift_cases.big_blob_image(160, 200, seed=seed)
    k = _check(img, nfeatures=nf)
    assert len(k) > 0 and np.all((k["octave"] & 255).astype(np.int8) >= 0)


def test_nfeatures_reorders_like_retain_best():
    """retainBest's nth_element + partition reorder the kept keypoints; descriptor rows follow."""
    img = sift_cases.blob_image(260, 300, n_blobs=260, seed=17)
    ek, _ = oracle.sift(img, contrast_threshold=0.04)
    for nf in (len(ek) // 2, len(ek) // 5, 7):
        _check(img, contrastThreshold=0.04, nfeatures=nf)


def test_37mp_image_fits_the_arena():
    """A 6144 x 6144 photo (37.7 MP), host input: the scratch arena must hold both doubled-size
    float buffers, the staged image and the staged descriptors. Expected output is the oracle's,
    committed (tests/golden/sift_37mp.npz, tests/golden/make_sift_big.py: ~2 min of oracle time)."""
    import hashlib
    import os
    import sfmx
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "sift_37mp.npz"))
    img = sift_cases.big_photo_37mp()
    assert hashlib.sha256(img.tobytes()).digest() == g["sha256"].tobytes(), "fixture image changed"
    k, d = sfmx.features.SIFT.create(nfeatures=3000).detectAndCompute(img)
    assert len(k) == len(g["keypoints"]) > 100
    assert k.tobytes() == g["keypoints"].tobytes()
    assert np.array_equal(d, g["descriptors"].astype(np.float32))


def test_large_sigma_uses_the_two_pass_blur():
    """sigma 3.2: the top layers' kernels exceed the fused tile's radius (16) and
    take the row/column/DoG kernels; both paths must agree with the oracle."""
    import sfmx
    img = sift_cases.blob_image(180, 220, n_blobs=120, seed=12)
    k, d = sfmx.features.SIFT.create(contrastThreshold=0.04, sigma=3.2).detectAndCompute(img)
    ek, ed = oracle.sift(img, contrast_threshold=0.04, sigma=3.2)
    assert len(ek) > 0 and k.tobytes() == ek.tobytes() and np.array_equal(d, ed)


def test_tiny_and_flat_images():
    import sfmx
    for img in [np.full((40, 40), 128, np.uint8), np.zeros((8, 9), np.uint8), sift_cases.blob_image(23, 17, seed=1),
                np.full((1, 50), 9, np.uint8), np.full((30, 1), 9, np.uint8)]:
        k, d = sfmx.features.SIFT.create().detectAndCompute(img)
        ek, ed = oracle.sift(img)
        assert k.tobytes() == ek.tobytes() and np.array_equal(d, ed)


def test_device_mode_feeds_the_matcher():
    import torch
    import sfmx
    img = sift_cases.blob_image(200, 260, n_blobs=150, seed=9)
    dev = torch.device("cuda:0")
    ti = torch.from_numpy(img).to(dev)
    kt = torch.zeros((4096, 7), dtype=torch.int32, device=dev)
    dt = torch.zeros((4096, 128), dtype=torch.float32, device=dev)
    s = sfmx.features.SIFT.create(contrastThreshold=0.04)
    n = s.detectAndCompute_device(ti, kt, dt)
    torch.cuda.synchronize()
    ek, ed = oracle.sift(img, contrast_threshold=0.04)
    assert n == len(ek)
    assert kt[:n].cpu().numpy().tobytes() == ek.tobytes()
    assert np.array_equal(dt[:n].cpu().numpy(), ed)
    assert sfmx.features.last_kernel_ms() > 0


def test_batch_streams_equal_oracle():
    """sfmx_sift_detect_compute_batch (SfM::extractFeatures' loop over shots) with
    3 worker streams over images of different sizes: every image bit-identical to
    the oracle, twice (the workers' arenas are reused)."""
    import torch
    import sfmx
    imgs = [sift_cases.blob_image(120 + 17 * i, 160 + 29 * i, n_blobs=60 + 20 * i, seed=20 + i) for i in range(7)]
    imgs.append(np.full((40, 40), 128, np.uint8))
    dev = torch.device("cuda:0")
    ts = [torch.from_numpy(i).to(dev) for i in imgs]
    kts = [torch.zeros((4096, 7), dtype=torch.int32, device=dev) for _ in imgs]
    dts = [torch.zeros((4096, 128), dtype=torch.float32, device=dev) for _ in imgs]
    s = sfmx.features.SIFT.create(contrastThreshold=0.04)
    expect = [oracle.sift(i, contrast_threshold=0.04) for i in imgs]
    for _ in range(2):
        counts = s.detectAndCompute_batch_device(ts, kts, dts, n_streams=3)
        torch.cuda.synchronize()
        for n, kt, dt, (ek, ed) in zip(counts, kts, dts, expect):
            assert n == len(ek)
            assert kt[:n].cpu().numpy().tobytes() == ek.tobytes()
            assert np.array_equal(dt[:n].cpu().numpy(), ed)
    with pytest.raises(sfmx._lib.SfmxError):   # capacity too small for one image: its status decides the return code
        s.detectAndCompute_batch_device(ts[:2], [kts[0], kts[1][:3]], [dts[0], dts[1][:3]], n_streams=2)
