"""Generate the committed golden fixtures under tests/golden/ (run from repo root:
``python tests/golden/make_golden.py``).

Inputs are seeded synthetic descriptor sets and adversarial KATs; expected
outputs come from the C++ oracle (oracle/match_oracle.cpp) and are asserted
equal to the independent numpy restatement (tests/refnp.py) before saving.
The reference itself cannot run here (no OpenCV/Ceres), so
these fixtures pin our restatement, not the reference binary ("parity
unpinned" vs the reference).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "sfm-mvs-pipeline_amd")]

from oracle import oracle  # noqa: E402
import refnp  # noqa: E402
import kat  # noqa: E402
from sfmx import synth  # noqa: E402


def packed_oracle(imgs, pairs, ratio=0.7):
    m, off = oracle.match_pairs(imgs, pairs, ratio)
    # cross-check every pair against the numpy restatement
    for p, (l, r) in enumerate(pairs):
        ref = refnp.match_pair(imgs[l], imgs[r], ratio)
        got = m[off[p]:off[p + 1]]
        assert len(ref) == len(got) and (ref.tobytes() == got.tobytes()), f"oracle != numpy on pair {p}"
    return m, off


def save(name, **arrs):
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
    print("wrote", name, {k: v.shape for k, v in arrs.items()})


def desc_set(name, imgs, pairs, ratio=0.7):
    m, off = packed_oracle(imgs, pairs, ratio)
    d = {f"img{i}": (x.astype(np.uint8) if x.dtype == np.float32 else x) for i, x in enumerate(imgs)}
    kind = np.array(0 if imgs[0].dtype == np.float32 else 1)
    save(name, kind=kind, n_imgs=np.array(len(imgs)), ratio=np.array(ratio), pairs=pairs, matches=m, offsets=off, **d)
    return m, off


def main():
    # 1. SIFT-like, ragged sizes (none a multiple of the 512-row work item)
    base = synth.sift_images(4, 600, seed=11)
    imgs = [base[0], base[1][:517], base[2][:64], base[3][:1]]
    pairs = oracle.pairs_unordered(4)
    m, off = desc_set("sift_small", imgs, pairs)
    # filters on the same result (SfM.cpp:547-570)
    for distinct in (0, 1):
        fm, foff, keep = oracle.filter_matches(m, off, distinct, 20)
        save(f"sift_small_filter_d{distinct}", matches=fm, offsets=foff, keep=keep)
    # 2. uniform 0..255 values
    desc_set("sift_uniform", synth.sift_images(3, 300, seed=12, uniform=True), oracle.pairs_unordered(3))
    # 3. collision-range stress (every query on the exact slow path)
    q, t = kat.sift_extreme()
    desc_set("sift_extreme", [q, t], np.array([[0, 1], [1, 0]], np.int32))
    # ratio > 1 accepts equal-distance neighbours, so the reported trainIdx
    # exposes the tie-break / float-sqrt ranking (ratio < 1 output is invariant to it)
    desc_set("sift_extreme_r15", [q, t], np.array([[0, 1], [1, 0]], np.int32), ratio=1.5)
    # 4. ORB
    ob = synth.orb_images(4, 700, seed=13)
    desc_set("orb_small", [ob[0], ob[1][:333], ob[2][:32], ob[3][:2]], oracle.pairs_unordered(4))
    # 5. KATs
    q, t = kat.sift_ties()
    desc_set("kat_sift_ties", [q, t], np.array([[0, 1]], np.int32))
    desc_set("kat_sift_ties_r15", [q, t], np.array([[0, 1]], np.int32), ratio=1.5)
    q, t = kat.sift_sqrt_collision()
    desc_set("kat_sift_sqrt_collision", [q, t], np.array([[0, 1]], np.int32))
    desc_set("kat_sift_sqrt_collision_r15", [q, t], np.array([[0, 1]], np.int32), ratio=1.5)
    for i, (q, t) in enumerate(kat.sift_ratio_boundary()):
        desc_set(f"kat_sift_ratio_{i}", [q, t], np.array([[0, 1]], np.int32))
    q, t = kat.orb_ties()
    desc_set("kat_orb_ties", [q, t], np.array([[0, 1]], np.int32))
    desc_set("kat_orb_ties_r15", [q, t], np.array([[0, 1]], np.int32), ratio=1.5)
    # Nt = 1 and Nt = 0 / Nq = 0
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, (70, 128)).astype(np.float32)
    desc_set("kat_sift_nt1_nt0", [a, a[:1], a[:0]], np.array([[0, 1], [0, 2], [2, 0], [1, 0]], np.int32))
    # 6. pair lists
    save("pairs", unordered7=oracle.pairs_unordered(7), video10_3=oracle.pairs_video(10, 3),
         video5_2=oracle.pairs_video(5, 2), grid20_3_5=oracle.pairs_grid(20, 3, 5, 1),
         grid23_3_5_ref=oracle.pairs_grid(23, 3, 5, 0), grid23_3_5_int=oracle.pairs_grid(23, 3, 5, 1),
         grid200_3_20=oracle.pairs_grid(200, 3, 20, 1))


if __name__ == "__main__":
    main()
