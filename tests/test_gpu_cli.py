"""GPU: the run-scripts' flag sets replayed end to end through the Photogrammetrie
driver (sfmx/cli.py -> csrc/cli.cpp flags -> SIFT / matching / filters / homography
kernels) on the reference's insel images (BASELINE config C1, tests/golden/insel/),
and every artefact compared with the oracle chain on the same decoded pixels:

    oracle.sift(limit, 3, 0.09) | oracle.orb(limit)  ->  strategy pairs  ->  oracle.match_pairs (exact 2-NN,
    ratio 0.7)  ->  oracle.filter_matches(--distinct-matches, -Pmatch-threshold)  ->
    oracle.homography_ratios(-Pransac-matching-threshold) over the kept pairs.

Keypoints, descriptors and match lists bit-exact; homography inlier ratios equal.
(The JPEG decode itself is PIL's libjpeg grayscale output on both sides: 'parity
unpinned' against an OpenCV build's decoder, see sfmx/cli.py:load_gray.)"""
import csv
import json
import os
import sys

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INSEL = os.path.join(REPO, "tests", "golden", "insel")
RUN_SCRIPTS = json.load(open(os.path.join(REPO, "tests", "golden", "run_scripts.json")))

CASES = [  # (script, $1, $2, extra flags)
    ("run-sequence-flann.sh", "2", "", []),                  # C1: SIFT -> Video(seq=2) -> filters -> homography
    ("run-sequence.sh", "3", "", ["--distinct-matches"]),
    ("run-grid-featurelimit.sh", "2", "1", []),
    ("run-unordered-flann.sh", "", "", ["-Pmatch-threshold=4", "-Pransac-matching-threshold=0.01"]),
    ("run-grid-flann-distortion.sh", "3", "3", ["-Pfeature-limit=150"]),
    ("run-orb-sequence-flann.sh", "2", "", []),              # ORB(30000) -> Hamming
    ("run-orb-grid.sh", "2", "1", ["--distinct-matches"]),
    ("run-orb-unordered.sh", "", "", ["-Pfeature-limit=400"]),
]


def _argv(script, a1, a2, extra, out):
    words = [w.replace("$1", a1).replace("$2", a2) for w in RUN_SCRIPTS[script]]
    words = [("-Pimage=" + INSEL if w == "-Pimage=./images" else w) for w in words if w not in ("-Pfeature-sequence=",
                                                                                                  "-Pfeature-gridlength=")]
    for e in extra:                    # getArg takes the first value: an override replaces the script's word
        key = e.split("=", 1)[0] + "="
        words = [w for w in words if not w.startswith(key)]
    return words + extra + ["-Pout=" + str(out)]


@pytest.mark.parametrize("script,a1,a2,extra", CASES, ids=[c[0] + "_" + c[1] + c[2] for c in CASES])
def test_run_script_replay_matches_oracle(script, a1, a2, extra, tmp_path):
    from sfmx import cli
    out = tmp_path / "reconstruction"
    argv = _argv(script, a1, a2, extra, out)
    assert cli.main(argv) == 0
    summary = json.load(open(out / "sfmx_pipeline.json"))
    cfg = summary["config"]
    paths = summary["images"]
    assert [os.path.basename(p) for p in paths] == ["1.jpg", "2.jpg", "3.jpg"]

    # oracle chain on the same pixels
    imgs = [cli.load_gray(p, summary["camera"]["resolution"]) for p in paths]
    if cfg["feature_detector"] == 1:
        feats = [oracle.orb(im, nfeatures=cfg["feature_limit"]) for im in imgs]
    else:
        feats = [oracle.sift(im, nfeatures=cfg["feature_limit"], contrast_threshold=cfg["sift_contrast_threshold"])
                 for im in imgs]
    for i, (k, d) in enumerate(feats):
        z = np.load(out / "features" / f"{i}{os.path.basename(paths[i])}.npz")
        assert z["keypoints"].tobytes() == k.tobytes(), i
        assert np.array_equal(z["descriptors"], d), i
    pairs = np.asarray(summary["pairs"], np.int32).reshape(-1, 2)
    m, off = oracle.match_pairs([d for _, d in feats], pairs)
    m, off, keep = oracle.filter_matches(m, off, bool(cfg["distinct_matches"]), cfg["match_threshold"])
    kept = [p for p in range(len(pairs)) if keep[p]]
    assert summary["kept_pairs"] == pairs[kept].tolist()
    assert len(kept) >= 1
    km = [m[off[p]:off[p + 1]] for p in kept]
    for j, p in enumerate(kept):
        l, r = pairs[p]
        got = np.load(out / "matches" / f"{j}{os.path.basename(paths[l])}-{os.path.basename(paths[r])}.npy")
        assert got.tobytes() == km[j].tobytes(), (l, r)
    koff = np.concatenate([[0], np.cumsum([len(x) for x in km])]).astype(np.int64)
    ratios = oracle.homography_ratios([np.stack([k["x"], k["y"]], 1) for k, _ in feats],
                                      [summary["camera"]["resolution"]] * 3, pairs[kept], np.concatenate(km), koff,
                                      cfg["ransac_matching_threshold"])
    assert summary["homography_inlier_ratios"] == [float(x) for x in ratios]
    rows = list(csv.DictReader(open(out / "shot_matches.csv")))
    assert [int(r["matches"]) for r in rows] == [len(x) for x in km]
    assert os.path.exists(out / "app.stat.csv")                                # --stats
