"""Full-size GPU parity on the BASELINE configs:
the whole-loop semantics of UnorderedFeatureMatchingStrategy.cpp:40-88 (every pair of
the job) and BundleAdjustment.cpp:50-95 (the whole Ceres problem), at the sizes the
bench measures.  The oracle runs with OpenMP on the box's host cores (tens of seconds).

  C2  50 x 8192 SIFT, all 1225 unordered pairs: DMatch lists byte-equal to the oracle.
  C4  200 x 16384 ORB-256, grid seq 3 / rowLen 20 (881 pairs): byte-equal to the oracle.
  C3  pair-sharded matching: 2 ranks (gloo, both on this GPU) merged == 1 rank, byte-equal;
      at its full size (200 x 8192 SIFT, all 19 900 unordered pairs) plus a stride sample of
      1 048 pairs spread over the whole list byte-equal to the oracle.
  C5  200 cams / 200k points / 1.2M obs BA: final cost within 1e-5 relative of the oracle,
      same termination, same accept/reject sequence.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import sfmx
from sfmx import ba, synth

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
THREADS = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 16)


def _match(imgs, pairs, norm):
    m = sfmx.BFMatcher(norm, device=0)
    try:
        m.set_images(imgs)
        m.run(pairs, sfmx.LOWE_RATIO)
        got, off, _ = m.fetch()
        stats = m.stats()
    finally:
        m.close()
    return got, off, stats


def test_c2_all_pairs_byte_equal_to_oracle():
    from oracle import oracle
    imgs = synth.sift_images(50, 8192)
    pairs = sfmx.pairs_unordered(50)
    got, off, stats = _match(imgs, pairs, sfmx.NORM_L2)
    exp, eoff = oracle.match_pairs(imgs, pairs, 0.7, THREADS)
    assert len(pairs) == 1225 and stats == (0, 0)
    assert np.array_equal(off, eoff)
    assert got.tobytes() == exp.tobytes()
    assert off[-1] > 500_000


def test_c4_all_pairs_byte_equal_to_oracle():
    from oracle import oracle
    imgs = synth.orb_images(200, 16384)
    pairs = sfmx.pairs_grid(200, 3, 20)
    got, off, _ = _match(imgs, pairs, sfmx.NORM_HAMMING)
    exp, eoff = oracle.match_pairs(imgs, pairs, 0.7, THREADS)
    assert len(pairs) == 881
    assert np.array_equal(off, eoff)
    assert got.tobytes() == exp.tobytes()


@pytest.mark.parametrize("kind,n_img", [("sift", 100), ("orb", 60)])
def test_pair_sharded_two_ranks_equal_one_rank(kind, n_img):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr=127.0.0.1", "--master-port=29533", os.path.join(HERE, "mp_match_worker.py"),
                          kind, str(n_img)], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert r["covered"] and r["equal"], r
    assert min(r["per_rank_pairs"]) > 0 and r["matches"] > 0


@pytest.mark.timeout(900)
def test_c3_full_size_sharded_equal_one_rank_and_oracle_sample():
    """BASELINE config 3 at its size (UnorderedFeatureMatchingStrategy.cpp:32-40): 200 x 8192
    SIFT, 19 900 pairs, pair-sharded over 2 ranks; merged == 1 rank, and every 19th pair
    (1 048 pairs, up to pair 19 893 = images (197, 199)) byte-equal to oracle.match_pairs."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr=127.0.0.1", "--master-port=29534", os.path.join(HERE, "mp_match_worker.py"),
                          "sift", "200", "19"], capture_output=True, text=True, timeout=900, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert r["pairs"] == 19_900 and r["covered"] and r["equal"], r
    assert r["oracle_pairs"] == 1048 and r["max_pair_index"] > 19_800, r
    assert r["oracle_bad"] == [] and r["oracle_matches"] > 400_000, r


def test_c5_full_ba_matches_oracle():
    from oracle import oracle
    p = synth.ba_problem(200, 200_000)
    assert len(p["obs_point"]) == 1_200_000
    _, osm, otr = oracle.ba_solve(p, trace_cap=1024, nthreads=THREADS)
    P = ba.BAProblem(**p)
    sm, tr = ba.solve(P, ba.default_options(), trace_cap=1024)
    assert sm["termination_type"] == osm["termination_type"]
    assert abs(sm["initial_cost"] - osm["initial_cost"]) <= 1e-12 * osm["initial_cost"]
    assert abs(sm["final_cost"] - osm["final_cost"]) <= 1e-5 * osm["final_cost"]
    assert len(tr) == len(otr) and np.array_equal(tr[:, 2], otr[:, 2])      # accept/reject sequence
    np.testing.assert_allclose(tr[:, 0], otr[:, 0], rtol=1e-6)
