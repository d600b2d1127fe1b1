"""GPU parity: the HIP matcher (through the C ABI) against the golden fixtures
and the oracle, bit-exact (queryIdx, trainIdx, imgIdx, distance bits, order)."""
import contextlib
import os

import numpy as np
import pytest

import sfmx
from sfmx import _lib, synth
import fixtures
from diag import diagnostic

pytestmark = pytest.mark.gpu


def run(imgs, pairs, ratio=0.7, distinct=False, min_count=0, norm=None):
    norm = norm or (sfmx.NORM_L2 if imgs[0].dtype == np.float32 else sfmx.NORM_HAMMING)
    m = sfmx.BFMatcher(norm)
    try:
        m.set_images(imgs)
        m.run(pairs, ratio, distinct, min_count)
        out = m.fetch()
        stats = m.stats()
    finally:
        m.close()
    return out + (stats,)


def assert_same(got, off, exp, exp_off):
    assert np.array_equal(off, exp_off), (off, exp_off)
    if got.tobytes() != exp.tobytes():
        bad = np.nonzero(got != exp)[0][:5] if len(got) == len(exp) else []
        raise AssertionError(f"mismatch at {bad}: got {got[bad] if len(bad) else got[:5]} exp {exp[bad] if len(bad) else exp[:5]}")


def test_device_visible():
    assert _lib.lib.sfmx_device_count() >= 1


def test_sqrt_exhaustive():
    n = 1 << 23                       # covers every SIFT squared distance (< 8,323,201)
    out = np.zeros(n, np.uint32)
    _lib.check(_lib.lib.sfmx_selftest_sqrt(0, n, out.ctypes.data_as(_lib.C.POINTER(_lib.C.c_uint32))), "sqrt")
    ref = np.sqrt(np.arange(n, dtype=np.float32)).view(np.uint32)
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("name", fixtures.desc_sets())
def test_golden(name):
    d = fixtures.load(name)
    m, off, keep, stats = run(d["imgs"], d["pairs"], d["ratio"])
    assert_same(m, off, d["matches"], d["offsets"])
    if name.startswith("sift_extreme"):
        # The two-pass path settles these far queries in the screening pass; the
        # single-pass kernel (variant 100) sends every query whose best-2 reach
        # s >= 2^22 to the exact float-sqrt slow path.  Same matches either way.
        with diagnostic(SFMX_SIFT_VARIANT="100"):
            m1, off1, _, stats1 = run(d["imgs"], d["pairs"], d["ratio"])
        assert_same(m1, off1, d["matches"], d["offsets"])
        assert stats1[0] == 250


@pytest.mark.parametrize("distinct", [0, 1])
def test_filters_golden(distinct):
    d = fixtures.load("sift_small")
    f = fixtures.load(f"sift_small_filter_d{distinct}")
    m, off, keep, _ = run(d["imgs"], d["pairs"], 0.7, distinct, 20)
    assert_same(m, off, f["matches"], f["offsets"])
    assert np.array_equal(keep, f["keep"])


def test_ragged_sizes_vs_oracle():
    from oracle import oracle
    sizes = [1, 31, 33, 64, 255, 257, 511, 513, 1000, 1300]
    base = synth.sift_images(len(sizes), 1300, seed=21)
    imgs = [b[:n] for b, n in zip(base, sizes)]
    pairs = sfmx.pairs_unordered(len(imgs))
    m, off, _, stats = run(imgs, pairs)
    em, eoff = oracle.match_pairs(imgs, pairs)
    assert_same(m, off, em, eoff)
    assert stats == (0, 0)


# Screening-pass shapes (103: 32x32x32 MFMA, 106-108: 16x16x64) and pass 2 forms
# (SFMX_SIFT_P2: 10 = the subset pass 2, the default; full-row GATHER items of
# 1/3 = 256 queries, 4 = 512, 0 = 128): every shipped or tuned kernel form must give
# the oracle's matches.  The uniform set has many queries whose best two share a
# screening subset, so pass 2 sees both accepted and undecided queries; 1100-query
# images split a pair's list over several items; images of 1 and 33 rows leave
# row subsets empty (r >= nt) or hold a single row.
@pytest.mark.parametrize("variant,p2", [("103", "0"), ("106", "4"), ("107", "1"), ("108", "3"), ("0", "0"),
                                        ("0", "10")])
def test_two_pass_variants_vs_oracle(variant, p2):
    from oracle import oracle
    sizes = [1, 33, 257, 513, 1100, 1100]
    base = synth.sift_images(len(sizes), 1100, seed=57)
    imgs = [b[:n] for b, n in zip(base, sizes)]
    rng = np.random.default_rng(58)
    imgs.append(rng.integers(0, 256, (900, 128)).astype(np.float32))
    pairs = sfmx.pairs_unordered(len(imgs))
    default = (variant, p2) == ("0", "10")   # the product library's form
    with contextlib.nullcontext() if default else diagnostic(SFMX_SIFT_VARIANT=variant, SFMX_SIFT_P2=p2):
        m, off, _, stats = run(imgs, pairs)
        m2, off2, _, _ = run(imgs, pairs, ratio=0.95)
    em, eoff = oracle.match_pairs(imgs, pairs)
    assert_same(m, off, em, eoff)
    em2, eoff2 = oracle.match_pairs(imgs, pairs, 0.95)
    assert_same(m2, off2, em2, eoff2)


def test_non_integral_fp32_fallback():
    from oracle import oracle
    rng = np.random.default_rng(9)
    imgs = [rng.random((300, 128), dtype=np.float32) * 50, rng.random((250, 128), dtype=np.float32) * 50,
            synth.sift_images(1, 200, seed=3)[0]]
    pairs = sfmx.pairs_unordered(3)
    m, off, _, stats = run(imgs, pairs)
    em, eoff = oracle.match_pairs(imgs, pairs)
    assert_same(m, off, em, eoff)
    assert stats[1] == 3                      # every pair touches a non-integral image


def test_orb_ragged_vs_oracle():
    from oracle import oracle
    base = synth.orb_images(5, 1500, seed=31)
    imgs = [b[:n] for b, n in zip(base, [1500, 1, 700, 513, 256])]
    pairs = sfmx.pairs_grid(5, 3, 2)
    m, off, _, _ = run(imgs, pairs)
    em, eoff = oracle.match_pairs(imgs, pairs)
    assert_same(m, off, em, eoff)


@pytest.mark.parametrize("variant", ["0", "12"])
@pytest.mark.parametrize("ratio", [0.0, 0.7, 0.95, 1.0, 1.5])
def test_orb_two_pass_ratios_vs_oracle(ratio, variant):
    """The ORB screening pass settles rejections from subset-maxima bounds; every
    ratio (none accepted at 0, ties accepted only above 1) must give the oracle's
    list, with the subset pass 2 (default, 0) and the r01 full-row pass 2 (12).
    Planted rows with few flipped bits plus exact duplicates (ties)."""
    from oracle import oracle
    base = synth.orb_images(4, 1200, seed=61)
    base[1][:40] = base[0][:40]
    base[2][100:140] = base[2][:40]
    imgs = [base[0], base[1][:900], base[2], base[3][:2]]
    pairs = sfmx.pairs_unordered(4)
    with contextlib.nullcontext() if variant == "0" else diagnostic(SFMX_ORB_VARIANT=variant):
        m, off, _, _ = run(imgs, pairs, ratio=ratio)
    em, eoff = oracle.match_pairs(imgs, pairs, ratio)
    assert_same(m, off, em, eoff)


def test_full_size_sift_spot_check_and_determinism():
    """C2 shape subset: 8 images x 8192 (all 28 pairs on the GPU), 3 pairs re-derived by the
    oracle; two GPU runs bit-identical; no slow-path / fp32 traffic on SIFT-like data."""
    from oracle import oracle
    imgs = synth.sift_images(8, 8192)
    pairs = sfmx.pairs_unordered(8)
    m1, off1, _, stats = run(imgs, pairs)
    m2, off2, _, _ = run(imgs, pairs)
    assert m1.tobytes() == m2.tobytes() and np.array_equal(off1, off2)
    assert stats == (0, 0)
    for p in (0, 13, 27):
        l, r = pairs[p]
        exp = oracle.match_pair(imgs[l], imgs[r])
        assert m1[off1[p]:off1[p + 1]].tobytes() == exp.tobytes()
    assert off1[-1] > 1000                    # the ratio test accepts planted neighbours


def test_full_size_orb_spot_check():
    from oracle import oracle
    imgs = synth.orb_images(3, 16384)
    pairs = np.array([[0, 1], [1, 2]], np.int32)
    m, off, _, _ = run(imgs, pairs)
    exp = oracle.match_pair(imgs[0], imgs[1])
    assert m[off[0]:off[1]].tobytes() == exp.tobytes()


def test_orb_multichunk_ties_and_narrow_rows():
    """ORB FP4-MFMA path beyond one 16384-row key chunk: train images of 40000
    rows (3 chunks folded with strict '<'), planted duplicate rows in different
    chunks (a query one bit away from both copies must report the LOWER train
    index), ratio 1.5 so ties are accepted; plus narrow rows (cols = 17 < 32)."""
    from oracle import oracle
    rng = np.random.default_rng(5)
    t = rng.integers(0, 256, size=(40000, 32), dtype=np.uint8)
    t[35000:35100] = t[100:200]                      # duplicates: chunk 0 and chunk 2
    t[20000:20050] = t[16000:16050]                  # duplicates: both in chunk 1
    dup = np.concatenate([t[100:200], t[16000:16050]]).copy()
    dup[:, 3] ^= 0x10                                # one flipped bit -> hamming 1 to both copies
    q = np.concatenate([t[rng.choice(40000, 1400, replace=False)], dup, rng.integers(0, 256, (300, 32), dtype=np.uint8)])
    imgs = [q, t, t[:16385].copy()]
    pairs = np.array([[0, 1], [0, 2], [2, 0]], np.int32)
    for ratio in (0.7, 1.5):
        m, off, _, _ = run(imgs, pairs, ratio)
        em, eoff = oracle.match_pairs(imgs, pairs, ratio)
        assert_same(m, off, em, eoff)
    got = m[off[0]:off[1]]
    sel = got[(got["queryIdx"] >= 1400) & (got["queryIdx"] < 1550)]
    assert len(sel) == 150 and np.all(sel["trainIdx"] == np.r_[100:200, 16000:16050]) and np.all(sel["distance"] == 1.0)
    narrow = [x[:, :17].copy() for x in synth.orb_images(3, 900, seed=41)]
    pairs = sfmx.pairs_unordered(3)
    m, off, _, _ = run(narrow, pairs)
    em, eoff = oracle.match_pairs(narrow, pairs)
    assert_same(m, off, em, eoff)


def test_match_pairs_oneshot_and_strategy():
    d = fixtures.load("sift_small")
    m, off, keep = sfmx.match_pairs(d["imgs"], d["pairs"], n_gpus=1)
    assert_same(m, off, d["matches"], d["offsets"])
    scene = sfmx.Scene([sfmx.Shot(f"img{i}", x) for i, x in enumerate(d["imgs"])])
    matcher = sfmx.BFMatcher(sfmx.NORM_L2)
    sm = sfmx.UnorderedFeatureMatchingStrategy().calculateShotMatches(scene, matcher)
    assert [(s.left, s.right) for s in sm] == [tuple(p) for p in d["pairs"]]
    for p, s in enumerate(sm):
        assert s.getMatches().tobytes() == d["matches"][d["offsets"][p]:d["offsets"][p + 1]].tobytes()
        assert s.homographyInlierRatio == -1.0
    f = fixtures.load("sift_small_filter_d1")
    kept = sfmx.calculate_shot_matches(scene, sfmx.UnorderedFeatureMatchingStrategy(), matcher, True, 20)
    assert len(kept) == int(f["keep"].sum())


def test_device_resident_inputs():
    torch = pytest.importorskip("torch")
    d = fixtures.load("sift_small")
    ts = [torch.from_numpy(x).cuda() for x in d["imgs"]]
    m = sfmx.BFMatcher(sfmx.NORM_L2)
    s = torch.cuda.current_stream().cuda_stream
    m.set_images_device(ts, stream=s)
    m.run(d["pairs"], stream=s)
    got, off, _ = m.fetch(stream=s)
    m.close()
    assert_same(got, off, d["matches"], d["offsets"])


def test_device_inputs_non_integral_rerun_on_read():
    """r05: set_images_device no longer waits for the integrality flags (the run assumes integral SIFT
    rows, the check happens when results are read).  A non-integral image there must still give the
    oracle's exact result: fetch, stats and device_results each re-run the last run on the fp32 path
    (every pair touching the image); a later integral batch in the same matcher runs on int8 again;
    two runs before one fetch: the last one's results."""
    import torch
    from oracle import oracle
    rng = np.random.default_rng(19)
    imgs = [synth.sift_images(1, 400, seed=5)[0], rng.random((300, 128), dtype=np.float32) * 50,
            synth.sift_images(1, 350, seed=6)[0]]
    pairs = sfmx.pairs_unordered(3)
    em, eoff = oracle.match_pairs(imgs, pairs)
    em2, eoff2 = oracle.match_pairs(imgs, pairs, 0.9)
    s = torch.cuda.current_stream().cuda_stream
    ts = [torch.from_numpy(x).cuda() for x in imgs]
    m = sfmx.BFMatcher(sfmx.NORM_L2)
    try:
        for first in ("fetch", "stats", "device"):
            m.set_images_device(ts, stream=s)
            m.run(pairs, 0.9, stream=s)          # superseded by the next run
            m.run(pairs, stream=s)
            if first == "stats":
                assert m.stats(stream=s)[1] == 2  # the two pairs with image 1 on the fp32 path
            elif first == "device":
                mp, op, _ = m.device_results()   # resolves (re-runs) before it hands out the pointers

                class _View:
                    def __init__(self, ptr, n):
                        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (ptr, False), "version": 3}
                torch.cuda.synchronize()
                dev = torch.as_tensor(_View(mp, 16 * int(eoff[-1])), device="cuda").cpu().numpy()
                assert dev.tobytes() == em.tobytes()
            got, off, _ = m.fetch(stream=s)
            assert_same(got, off, em, eoff)
            assert m.stats(stream=s)[1] == 2
        # an integral batch after it: the int8 path again, exact
        ok = [torch.from_numpy(x).cuda() for x in (imgs[0], imgs[2])]
        m.set_images_device(ok, stream=s)
        m.run(np.array([[0, 1]], np.int32), 0.9, stream=s)
        got, off, _ = m.fetch(stream=s)
        e3, eo3 = oracle.match_pairs([imgs[0], imgs[2]], np.array([[0, 1]], np.int32), 0.9)
        assert_same(got, off, e3, eo3)
        assert m.stats(stream=s)[1] == 0
    finally:
        m.close()


def test_errors():
    m = sfmx.BFMatcher(sfmx.NORM_L2)
    with pytest.raises(ValueError):
        m.set_images([np.zeros((3, 129), np.float32)])
    with pytest.raises(_lib.SfmxError):
        m.run(np.array([[0, 1]]))             # run before set_images -> SFMX_ESTATE
    m.set_images([np.zeros((3, 128), np.float32)] * 2)
    with pytest.raises(ValueError):
        m.run(np.array([[0, 5]]))
    m.close()


# Kernel builds that gave wrong results in r01, selectable again:
#   ORB pass 2 with 2 / 4 query tiles per wave (128- / 256-query items, variants 13 / 14): the r01
#   builds kept compact_work_kernel's item size at 512 queries while a block covered 128 / 256,
#   so pass 2 skipped the rest of each item (now a static_assert, and assemble_kernel counts any
#   forwarded query pass 2 left unwritten: the run fails with SFMX_EINTERNAL);
#   ORB16 single pass 4 tiles x 8 waves (7), 32x32 ORB with MINW = 1 (9, 4), SIFT single pass with
#   MINW = 1 (30, 31).
ORB_KATS = ["kat_orb_ties", "kat_orb_ties_r15", "orb_small"]
SIFT_KATS = ["kat_sift_nt1_nt0", "kat_sift_ties", "kat_sift_ties_r15", "sift_small"]


@pytest.mark.parametrize("env,variant", [("SFMX_ORB_VARIANT", "13"), ("SFMX_ORB_VARIANT", "14"),
                                         ("SFMX_ORB_VARIANT", "7"), ("SFMX_ORB_VARIANT", "9"),
                                         ("SFMX_ORB_VARIANT", "4"), ("SFMX_SIFT_VARIANT", "30"),
                                         ("SFMX_SIFT_VARIANT", "31")])
def test_previously_failing_variants(env, variant):
    from oracle import oracle
    names = ORB_KATS if env == "SFMX_ORB_VARIANT" else SIFT_KATS
    with diagnostic(**{env: variant}):
        for name in names:
            d = fixtures.load(name)
            m, off, _, _ = run(d["imgs"], d["pairs"], d["ratio"])
            assert_same(m, off, d["matches"], d["offsets"])
        if env == "SFMX_ORB_VARIANT":
            base = synth.orb_images(4, 1200, seed=61)
            base[1][:40] = base[0][:40]
            imgs = [base[0], base[1][:900], base[2], base[3][:2]]
        else:
            base = synth.sift_images(5, 1100, seed=57)
            imgs = [b[:n] for b, n in zip(base, [1, 33, 513, 1100, 1100])]
        pairs = sfmx.pairs_unordered(len(imgs))
        for ratio in (0.7, 1.5):
            m, off, _, _ = run(imgs, pairs, ratio)
            em, eoff = oracle.match_pairs(imgs, pairs, ratio)
            assert_same(m, off, em, eoff)


@pytest.mark.parametrize("persist", ["1", "0"])
@pytest.mark.parametrize("kind", ["sift", "orb"])
def test_persistent_screen_vs_oracle(kind, persist):
    """r04: the screens as a grid of resident workgroups fed by a ticket counter (PERSIST,
    SFMX_SCREEN_PERSIST=1, measured slower and kept in the diagnostic build only) and the product's
    one-workgroup-per-item grid (SFMX_SCREEN_PERSIST=0) both give the
    oracle's matches: mixed sizes, a 1-row image (the full-size C2 / C3 / C4 tests run many more
    items than resident slots, i.e. several items per workgroup)."""
    from oracle import oracle
    if kind == "sift":
        sizes = [1, 2048, 700, 1100, 1600, 513, 900, 2048]
        base = synth.sift_images(len(sizes), 2048, seed=94)
        imgs = [b[:n] for b, n in zip(base, sizes)]
    else:
        base = synth.orb_images(8, 2048, seed=95)
        imgs = [b[:n] for b, n in zip(base, [2048, 1, 700, 513, 1500, 256, 1200, 2048])]
    pairs = sfmx.pairs_unordered(len(imgs))
    with diagnostic(SFMX_SCREEN_PERSIST=persist):
        m, off, _, _ = run(imgs, pairs)
    em, eoff = oracle.match_pairs(imgs, pairs)
    assert_same(m, off, em, eoff)


@pytest.mark.parametrize("batches", ["1", "2", "3", "64"])
@pytest.mark.parametrize("kind", ["sift", "orb"])
def test_overlapped_two_pass_batches_vs_oracle(kind, batches):
    """the screen launches of consecutive batches alternate between two streams
    and each batch's pass 2 runs on a third stream behind its screen (launch_two_pass_overlap); any
    batch count, including one batch per pair (64) and the single-launch form (1), gives the oracle's
    matches, with mixed-size pairs, empty-ish images and a non-integral image (an fp32 pair inside
    a batch: no screen items, pass 2 skips it)."""
    from oracle import oracle
    if kind == "sift":
        sizes = [1, 33, 700, 1100, 1100, 513, 900]
        base = synth.sift_images(len(sizes), 1100, seed=91)
        imgs = [b[:n] for b, n in zip(base, sizes)]
        imgs.append(np.random.default_rng(92).random((300, 128), dtype=np.float32) * 40)
        pairs = sfmx.pairs_unordered(len(imgs))
    else:
        base = synth.orb_images(7, 1500, seed=93)
        imgs = [b[:n] for b, n in zip(base, [1500, 1, 700, 513, 1500, 256, 1200])]
        pairs = sfmx.pairs_grid(7, 3, 2)
    with diagnostic(SFMX_MATCH_BATCHES=batches):
        m, off, _, _ = run(imgs, pairs)
        m2, off2, _, _ = run(imgs, pairs, ratio=1.5)
    em, eoff = oracle.match_pairs(imgs, pairs)
    assert_same(m, off, em, eoff)
    em2, eoff2 = oracle.match_pairs(imgs, pairs, 1.5)
    assert_same(m2, off2, em2, eoff2)
