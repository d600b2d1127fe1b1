"""ORB extraction on the GPU:
sfmx_orb_detect_compute (csrc/orb_features.hip) bit-identical to the restatement in
oracle/orb_oracle.cpp -- all seven cv::KeyPoint fields, keypoint order (retainBest's
nth_element / partition order) and the 32-byte descriptors -- through the C ABI,
host, device and batch modes.  Parity with OpenCV itself: unpinned (no OpenCV here)."""
import os

import numpy as np
import pytest

from oracle import oracle
import sift_cases

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _insel(i):
    from sfmx import cli
    return cli.load_gray(os.path.join(REPO, "tests", "golden", "insel", f"{i}.jpg"))


def _check(img, **kw):
    import sfmx
    k, d = sfmx.features.ORB.create(**kw).detectAndCompute(img)
    ok = {"nfeatures": kw.get("nfeatures", 500), "scale_factor": kw.get("scaleFactor", 1.2),
          "nlevels": kw.get("nlevels", 8), "edge_threshold": kw.get("edgeThreshold", 31),
          "fast_threshold": kw.get("fastThreshold", 20)}
    ek, ed = oracle.orb(img, **ok)
    assert len(k) == len(ek), (len(k), len(ek))
    assert k.tobytes() == ek.tobytes(), [(a, b) for a, b in zip(k, ek) if a.tobytes() != b.tobytes()][:3]
    assert np.array_equal(d, ed), np.nonzero((d != ed).any(1))[0][:5]
    return k, d


@pytest.mark.parametrize("i", [1, 2, 3])
@pytest.mark.parametrize("nf", [30000, 500, 7])
def test_insel_bit_exact(i, nf):
    k, _ = _check(_insel(i), nfeatures=nf)
    assert len(k) >= min(nf, 7)


@pytest.mark.parametrize("shape,seed", [((120, 160), 1), ((97, 131), 2), ((300, 400), 3), ((481, 641), 4)])
def test_blob_images_bit_exact(shape, seed):
    _check(sift_cases.blob_image(*shape, n_blobs=120, seed=seed, noise=6.0), nfeatures=2000)


def test_ties_at_the_retain_best_boundary():
    """A flat image with a sparse checkerboard of identical corners: FAST scores and Harris
    responses tie massively, so retainBest's partition keeps > n and the order is
    nth_element's."""
    img = np.full((240, 320), 100, np.uint8)
    img[40:200:8, 40:280:8] = 200
    img[44:196:16, 44:276:16] = 10
    k, _ = _check(img, nfeatures=50)
    assert len(k) > 50


def test_large_photo_and_parameters():
    img = sift_cases.blob_image(1080, 1920, n_blobs=400, seed=11, noise=8.0)
    k, _ = _check(img, nfeatures=30000)
    assert len(k) > 1000
    _check(img, nfeatures=3000, scaleFactor=1.5, nlevels=5, fastThreshold=12, edgeThreshold=40)
    # r04 kernels' edge regimes: the resize's staged source span at its limit (scale 2) and past it
    # (2.6: the per-pixel form), edge threshold 19 (rBRIEF windows touching the level's edge)
    _check(img, nfeatures=2000, scaleFactor=2.0, nlevels=4, edgeThreshold=19)
    _check(img, nfeatures=1000, scaleFactor=2.6, nlevels=3, edgeThreshold=19, fastThreshold=8)


def test_degenerate_inputs():
    import sfmx
    assert len(_check(np.zeros((40, 40), np.uint8))[0]) == 0         # below 2 x edgeThreshold
    assert len(_check(sift_cases.blob_image(200, 200, seed=5), nfeatures=0)[0]) == 0   # retainBest(0) clears
    assert len(_check(np.full((100, 100), 7, np.uint8))[0]) == 0     # no corners
    with pytest.raises(ValueError):                                  # SFMX_EINVAL
        sfmx.features.ORB.create(100, WTA_K=3).detectAndCompute(np.zeros((64, 64), np.uint8))
    with pytest.raises(ValueError):
        sfmx.features.ORB.create(100, edgeThreshold=-1).detectAndCompute(np.zeros((64, 64), np.uint8))


@pytest.mark.parametrize("edge", [18, 16, 10, 5, 3, 0])
def test_small_edge_thresholds_read_the_bordered_pyramid(edge):
    # below 19 rBRIEF's samples (below 15 the angle patch, below 4 the Harris window) leave their level and
    # read OpenCV's bordered pyramid: the level's BORDER_REFLECT_101 copy, unblurred (compute() blurs each
    # level in place inside it); r04 refused these parameters
    img = sift_cases.blob_image(300, 420, n_blobs=160, seed=13, noise=6.0)
    k, _ = _check(img, nfeatures=1500, edgeThreshold=edge, nlevels=5)
    assert len(k) > 100
    if edge <= 10:   # some keypoints close enough to their level's edge for rBRIEF's border reads
        s = np.float32(1.2) ** k["octave"].astype(np.float64)
        x, y = k["x"] / s, k["y"] / s
        w, h = np.round(420 / s), np.round(300 / s)
        assert (np.minimum(np.minimum(x, y), np.minimum(w - 1 - x, h - 1 - y)) < 18).any()
    _check(img, nfeatures=800, edgeThreshold=edge, scaleFactor=1.6, nlevels=4, fastThreshold=10)


def test_device_and_batch_modes_match():
    import torch
    import sfmx
    imgs = [_insel(i) for i in (1, 2, 3)] + [sift_cases.blob_image(300, 500, n_blobs=150, seed=9, noise=5.0)]
    orb = sfmx.features.ORB.create(30000)
    ref = [orb.detectAndCompute(im) for im in imgs]
    got = orb.detectAndCompute_batch(imgs, n_streams=3)
    for (k0, d0), (k1, d1) in zip(ref, got):
        assert k0.tobytes() == k1.tobytes() and np.array_equal(d0, d1)
    t = torch.from_numpy(imgs[0]).cuda()
    kt = torch.zeros((1 << 15, 7), dtype=torch.int32, device="cuda")
    dt = torch.zeros((1 << 15, 32), dtype=torch.uint8, device="cuda")
    n = orb.detectAndCompute_device(t, kt, dt)
    torch.cuda.synchronize()
    assert n == len(ref[0][0])
    assert kt[:n].cpu().numpy().tobytes() == ref[0][0].tobytes()
    assert np.array_equal(dt[:n].cpu().numpy(), ref[0][1])


@pytest.mark.parametrize("n_streams", [1, 2])
def test_batched_chunks_equal_the_oracle(n_streams):
    """r04: a batch runs as chunks of up to 16 same-size images, each chunk ONE set of launches
    (image g's arrays at g x the per-image block, its counters in a stats row).  Mixed sizes split
    the chunks; every image -- corner-rich, tie-heavy, cornerless, below 2 x edgeThreshold -- must
    equal the oracle's one-image result, host and device modes."""
    import torch
    import sfmx
    ties = np.full((240, 320), 100, np.uint8)
    ties[40:200:8, 40:280:8] = 200
    ties[44:196:16, 44:276:16] = 10
    imgs = [sift_cases.blob_image(240, 320, n_blobs=120, seed=s, noise=6.0) for s in (31, 32, 33)]
    imgs += [ties, np.full((240, 320), 7, np.uint8), sift_cases.blob_image(240, 320, n_blobs=60, seed=34)]
    imgs += [np.zeros((40, 40), np.uint8), sift_cases.blob_image(97, 131, n_blobs=40, seed=35, noise=4.0)]
    imgs += [sift_cases.blob_image(240, 320, n_blobs=200, seed=36, noise=9.0)]
    orb = sfmx.features.ORB.create(2000)
    got = orb.detectAndCompute_batch(imgs, capacity=4096, n_streams=n_streams)
    for im, (k, d) in zip(imgs, got):
        ek, ed = oracle.orb(im, nfeatures=2000)
        assert k.tobytes() == ek.tobytes() and np.array_equal(d, ed)
    dev = [torch.from_numpy(im).cuda() for im in imgs]
    kt = [torch.zeros((4096, 7), dtype=torch.int32, device="cuda") for _ in imgs]
    dt = [torch.zeros((4096, 32), dtype=torch.uint8, device="cuda") for _ in imgs]
    ns = orb.detectAndCompute_batch_device(dev, kt, dt, n_streams=n_streams)
    torch.cuda.synchronize()
    for (k, d), n, a, b in zip(got, ns, kt, dt):
        assert n == len(k)
        assert a[:n].cpu().numpy().tobytes() == k.tobytes() and np.array_equal(b[:n].cpu().numpy(), d)


def test_large_images_through_several_streams():
    """every chunk reserves its per-image scratch (~15 GB for a 16384^2 photo) for
    each of its images on each stream, so 24 such images on 8 streams (chunks of 3) asked for ~375 GB.
    The batch now cuts the chunk size to the free device memory (and re-runs a failing chunk image by
    image): every image comes back OK and equal to its one-image call."""
    import torch
    import sfmx
    tile = torch.from_numpy(sift_cases.blob_image(2048, 2048, n_blobs=900, seed=41, noise=6.0)).cuda()
    base = tile.repeat(8, 8).contiguous()                     # 16384 x 16384
    imgs = [torch.roll(base, shifts=37 * i, dims=1).contiguous() for i in range(24)]
    orb = sfmx.features.ORB.create(30000)
    cap = 1 << 15
    kt = [torch.zeros((cap, 7), dtype=torch.int32, device="cuda") for _ in imgs]
    dt = [torch.zeros((cap, 32), dtype=torch.uint8, device="cuda") for _ in imgs]
    counts = orb.detectAndCompute_batch_device(imgs, kt, dt, n_streams=8)
    torch.cuda.synchronize()
    assert all(c > 0 for c in counts)
    for i in (0, 13, 23):
        k1 = torch.zeros((cap, 7), dtype=torch.int32, device="cuda")
        d1 = torch.zeros((cap, 32), dtype=torch.uint8, device="cuda")
        n = orb.detectAndCompute_device(imgs[i], k1, d1)
        torch.cuda.synchronize()
        assert n == counts[i]
        assert torch.equal(k1[:n], kt[i][:n]) and torch.equal(d1[:n], dt[i][:n])
    del imgs, kt, dt
    torch.cuda.empty_cache()
