"""CPU: the reference's command line (VERDICT r01 ★ row) through the native parser
(include/sfmx_cli.h, csrc/cli.cpp) and the Photogrammetrie driver (sfmx/cli.py).

- grammar: AppArgs::parseArgs / getArg / getArgs / isFlag (cli/util/AppArgs.cpp:29-88),
  checked against a plain-Python restatement of those lines;
- one test per flag PhotogrammetrieCli / App read: its default, a set value, the
  warning or the SfM setter rejection (PhotogrammetrieCli.cpp:94-112, 288-392;
  SfM.cpp:66-129; App.cpp:34-50);
- every run-scripts/run-*.sh flag set (tests/golden/run_scripts.json) replayed through
  `Photogrammetrie ... --sfmx-plan`, which resolves images, camera, strategy and pairs
  and stops before device work.  The GPU replay is tests/test_gpu_cli.py.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "sfm-mvs-pipeline_amd"))

from sfmx import cli  # noqa: E402

INSEL = os.path.join(REPO, "tests", "golden", "insel")
EXE = os.path.join(REPO, "sfm-mvs-pipeline_amd", "bin", "Photogrammetrie")
HW = os.cpu_count()


# ---- grammar --------------------------------------------------------------------

def spec_parse(argv):
    """AppArgs.cpp:29-53 restated: list of (key, value) in multimap order
    (key-sorted, equal keys in insertion order)."""
    kv = []
    for arg in argv:
        if len(arg.encode()) < 3 or not arg.startswith("-"):
            kv.append(("", arg))
            continue
        eq = arg.find("=")
        typ = arg[:2]
        key = arg[2:] if eq < 0 else arg[2:eq]
        val = "" if eq < 0 else arg[eq + 1:]
        if typ == "-P":
            kv.append((key, val))
        elif typ == "--":
            kv.append((key, "1"))
    return sorted(kv, key=lambda p: p[0].encode())   # stable: equal keys keep order


GRAMMAR_CASES = [
    ["-Pa=b"], ["-Pa"], ["--flag"], ["--flag=x"], ["-X=5", "-Xfoo"], ["ab", "x", "-", "--", "-P"],
    ["-Pk=v=w"], ["-P=v"], ["-Pimage=1", "-Pimage=2", "-Pimage=3"], ["--dense", "-Pdense=0"],
    ["-Pdense=0", "--dense"], ["-Pdense=1"], ["-Pdense=true"], ["--a=", "-Pb="], ["image.jpg", "-Pout=/tmp/x y"],
    ["-p=lower", "-Pz=1", "-PA=2", "-Pa=3"], ["-Pü=ä"],
]


@pytest.mark.parametrize("argv", GRAMMAR_CASES, ids=[" ".join(c) for c in GRAMMAR_CASES])
def test_grammar_matches_appargs(argv):
    a = cli.AppArgs(argv)
    kv = spec_parse(argv)
    assert a.toString() == "\n".join(f"{k} -> {v}" for k, v in kv)
    for key in {k for k, _ in kv} | {"missing"}:
        vals = [v for k, v in kv if k == key]
        assert a.getArgs(key) == vals
        assert a.getArgCount(key) == len(vals)
        assert a.getArg(key, "dflt") == (vals[0] if vals else "dflt")
        assert a.isFlag(key) == ((vals[0] if vals else "0") == "1")


def test_getarg_first_value_and_reparse():
    a = cli.AppArgs(["-Pimage=1", "-Pimage=2"])
    assert a.getArg("image") == "1" and a.getArgs("image") == ["1", "2"]
    a.parseArgs(["-Pout=x"])                          # parseArgs replaces (AppArgs.cpp:30)
    assert a.getArgCount("image") == 0 and a.getArg("out") == "x"


def test_abi_errors():
    a = cli.AppArgs(["-Pimage=1"])
    with pytest.raises(Exception):
        cli._string(cli.lib.sfmx_args_get_at, a._h, b"image", 1)
    assert cli.lib.sfmx_args_count(None, b"x") == -1
    assert cli.lib.sfmx_cli_usage(b"x", 7, None, 0) == -1


# ---- per-flag configuration ---------------------------------------------------------

BASE = ["-Prun=photogrammetrie", "-Pimage=x.jpg"]


def conf(*flags):
    return cli.configure(cli.AppArgs(BASE + list(flags)))


def warnings(log):
    return [m for lvl, m in log if lvl == cli.LOG_WARN]


def rejected(*flags):
    with pytest.raises(cli.ConfigError) as e:
        conf(*flags)
    return str(e.value)


def test_defaults():
    c, log = conf()
    assert log == []
    assert (c.run, c.loglevel, c.omp_cpu_threads, c.help, c.n_images) == (1, 2, HW, 0, 1)
    assert (c.camera_model, c.feature_detector, c.feature_limit, c.sift_n_octave_layers) == (3, 0, 10000, 3)
    assert c.sift_contrast_threshold == 0.09
    assert (c.feature_matcher, c.norm, c.strategy, c.feature_sequence, c.feature_gridlength) == (0, 4, 0, 0, 0)
    assert (c.omp_feature_threads, c.match_threshold, c.baseline_homography_threshold, c.distinct_matches) == \
        (HW, 20, 100, 0)
    assert (c.ransac_matching_threshold, c.ransac_baseline_threshold, c.ransac_pose_threshold) == (0.006, -1.0, -8.0)
    assert (c.homography_inlier_ratio_threshold, c.pose_inlier_ratio_threshold) == (0.4, 0.4)
    assert (c.reprojection_error_threshold, c.pointcloud_feature_merge_distance,
            c.pointcloud_point_merge_distance) == (10.0, 20.0, 0.01)
    assert [getattr(c, f) for f in ("colored", "dense", "sgm", "mesh", "no_decimate", "refine_mesh", "stats",
                                    "artifacts")] == [0] * 8
    assert c.out == b"./reconstruction"


def test_flag_run():
    for v, want in (("photogrammetrie", 1), ("pcl-stats", 2), ("help", 0), ("bogus", 0)):
        c, _ = cli.configure(cli.AppArgs([f"-Prun={v}", "-Pimage=x"]))
        assert c.run == want
    c, _ = cli.configure(cli.AppArgs(["-Pimage=x"]))
    assert c.run == 0


def test_flag_loglevel():
    assert conf("-Ploglevel=0")[0].loglevel == 0
    assert conf("-Ploglevel= 4x")[0].loglevel == 4          # std::stoi: leading blanks, trailing text
    assert "loglevel" in rejected("-Ploglevel=high")


def test_flag_omp_cpu_threads():
    assert conf("-Pomp-cpu-threads=3")[0].omp_cpu_threads == 3
    assert "omp-cpu-threads" in rejected("-Pomp-cpu-threads=")


def test_flag_force_colored_output():
    assert conf("--forceColoredOutput")[0].force_colored_output == 1


def test_flag_help_and_image_count_stop_reading():
    c, log = cli.configure(cli.AppArgs(BASE + ["--help", "-Pcamera-model=Nope"]))
    assert c.help == 1 and log == [] and c.camera_model == 3     # usage + exit before prepareScene
    c, log = cli.configure(cli.AppArgs(["-Prun=photogrammetrie", "-Pcamera-model=Nope"]))
    assert c.n_images == 0 and log == []
    c, _ = conf("-Pimage=y.jpg", "-Pimage=dir")
    assert c.n_images == 3


def test_flag_out():
    assert conf("-Pout=/tmp/w")[0].out == b"/tmp/w"
    assert conf("-Pout=")[0].out == b""
    assert "out" in rejected("-Pout=" + "x" * 1024)


@pytest.mark.parametrize("v,model,warn", [("SimpleRadial", 3, False), ("Distortion", 7, False), ("Simple", 1, False),
                                          ("simple", 3, True), ("", 3, True), ("Pinhole", 3, True)])
def test_flag_camera_model(v, model, warn):
    c, log = conf(f"-Pcamera-model={v}")
    assert c.camera_model == model
    assert bool(warnings(log)) == warn and c.n_warnings == int(warn)


@pytest.mark.parametrize("v,det,norm,warn", [("SIFT", 0, 4, False), ("ORB", 1, 6, False), ("", 0, 4, False),
                                              ("orb", 0, 4, True), ("SURF", 0, 4, True)])
def test_flag_feature_detector(v, det, norm, warn):
    c, log = conf(f"-Pfeature-detector={v}")
    assert (c.feature_detector, c.norm) == (det, norm)
    assert bool(warnings(log)) == warn


def test_flag_feature_limit():
    assert conf("-Pfeature-limit=0")[0].feature_limit == 0
    assert conf("-Pfeature-limit=30000")[0].feature_limit == 30000
    assert "feature-limit" in rejected("-Pfeature-limit=many")
    assert "feature-limit" in rejected("-Pfeature-limit=99999999999")     # std::out_of_range


@pytest.mark.parametrize("det,v,m,warn", [("SIFT", "FLANN", 1, False), ("SIFT", "BF", 0, False), ("SIFT", "", 0, False),
                                          ("ORB", "FLANN", 1, False), ("ORB", "flann", 0, True),
                                          ("SIFT", "KNN", 0, True)])
def test_flag_feature_matcher(det, v, m, warn):
    c, log = conf(f"-Pfeature-detector={det}", f"-Pfeature-matcher={v}")
    assert c.feature_matcher == m
    assert c.norm == (6 if det == "ORB" else 4)
    assert bool(warnings(log)) == warn


@pytest.mark.parametrize("seq,grid,strategy,warn", [(None, None, 0, False), ("0", None, 0, False), ("1", None, 0, True),
                                                    ("-3", None, 0, True), ("2", None, 1, False), ("5", "0", 1, False),
                                                    ("3", "20", 2, False), ("2", "1", 2, False),
                                                    (None, "4", 0, False), ("1", "4", 0, True)])
def test_flag_feature_sequence_and_gridlength(seq, grid, strategy, warn):
    flags = ([f"-Pfeature-sequence={seq}"] if seq is not None else []) + \
            ([f"-Pfeature-gridlength={grid}"] if grid is not None else [])
    c, log = conf(*flags)
    assert c.strategy == strategy
    assert bool(warnings(log)) == warn
    assert "feature-sequence" in rejected("-Pfeature-sequence=x")
    assert "feature-gridlength" in rejected("-Pfeature-gridlength=x")


def test_flag_omp_feature_threads():
    assert conf("-Pomp-feature-threads=8")[0].omp_feature_threads == 8
    assert conf("-Pomp-feature-threads=0")[0].omp_feature_threads == HW       # SfM.cpp:66-71
    assert conf("-Pomp-feature-threads=-2")[0].omp_feature_threads == 1


def test_flag_match_threshold():
    assert conf("-Pmatch-threshold=4")[0].match_threshold == 4
    assert "match-threshold" in rejected("-Pmatch-threshold=3")               # SfM.cpp:73-78


def test_flag_baseline_homography_threshold():
    assert conf("-Pbaseline-homography-threshold=50")[0].baseline_homography_threshold == 50
    assert "baseline-homography-threshold" in rejected("-Pbaseline-homography-threshold=0")


@pytest.mark.parametrize("flag,field,ok,bad", [
    ("ransac-matching-threshold", "ransac_matching_threshold", ["0", "1", "0.01"], ["-0.5", "1.5"]),
    ("ransac-baseline-threshold", "ransac_baseline_threshold", ["-3", "1", "0.2"], ["0", "2"]),
    ("ransac-pose-threshold", "ransac_pose_threshold", ["-8", "0.5"], ["0", "1.01"]),
    ("homography-inlier-ratio-threshold", "homography_inlier_ratio_threshold", ["0", "1", "0.25"], ["-0.1", "1.1"]),
    ("pose-inlier-ratio-threshold", "pose_inlier_ratio_threshold", ["0", "0.9"], ["2"]),
    ("reprojection-error-threshold", "reprojection_error_threshold", ["0", "3.5", "1e3"], ["-1"]),
    ("pointcloud-feature-merge-distance", "pointcloud_feature_merge_distance", ["-5", "7.5"], []),
    ("pointcloud-point-merge-distance", "pointcloud_point_merge_distance", ["0.5", "inf"], []),
])
def test_flag_thresholds(flag, field, ok, bad):
    for v in ok:
        assert getattr(conf(f"-P{flag}={v}")[0], field) == float(v)
    for v in bad + ["abc"]:
        assert flag in rejected(f"-P{flag}={v}")


def test_flag_distinct_matches():
    assert conf("--distinct-matches")[0].distinct_matches == 1
    assert conf("-Pdistinct-matches=1")[0].distinct_matches == 1             # isFlag compares with "1"
    assert conf("-Pdistinct-matches=yes")[0].distinct_matches == 0


@pytest.mark.parametrize("flag", ["colored", "dense", "sgm", "mesh", "no-decimate", "refine-mesh", "stats", "artifacts"])
def test_stage_flags(flag):
    c, _ = conf(f"--{flag}")
    assert getattr(c, flag.replace("-", "_")) == 1


def test_warning_order_and_first_error_wins():
    c, log = conf("-Pcamera-model=X", "-Pfeature-detector=Y", "-Pfeature-matcher=Z", "-Pfeature-sequence=1")
    assert [m.split(":")[0] for m in warnings(log)] == ["unknown camera model", "unknown feature detector",
                                                        "unknown feature matcher", "invalid sequence length"]
    msg = rejected("-Pmatch-threshold=2", "-Pransac-pose-threshold=0")
    assert "match-threshold" in msg                                           # setters run in :94-112 order


def test_usage_texts():
    for which in (0, 1):
        u = cli.usage("Photogrammetrie", which)
        assert u.startswith("usage: Photogrammetrie")
    u = cli.usage("P", 1)
    for flag in ("image", "out", "camera-model", "feature-detector", "feature-limit", "feature-matcher",
                 "feature-sequence", "feature-gridlength", "match-threshold", "ransac-matching-threshold",
                 "distinct-matches", "artifacts"):
        assert flag in u


# ---- the driver ---------------------------------------------------------------------

def run_exe(args, cwd=None):
    env = dict(os.environ, SFMX_NO_TORCH="1")
    return subprocess.run([sys.executable, EXE] + list(args), capture_output=True, text=True, cwd=cwd, env=env,
                          timeout=120)


def test_driver_usage_exits():
    assert run_exe([]).returncode == 255                                     # -Prun missing -> App usage
    r = run_exe(["-Prun=photogrammetrie", "-Pimage=x", "--help"])
    assert r.returncode == 255 and "usage:" in r.stdout
    r = run_exe(["-Prun=photogrammetrie"])
    assert r.returncode == 255 and "no images" in r.stdout
    r = run_exe(["-Prun=photogrammetrie", "-Pimage=" + os.path.join(INSEL, "1.jpg"), "-Pimage=/nonexistent"])
    assert r.returncode == 255 and "not found" in r.stdout and "at least two" in r.stdout
    r = run_exe(["-Prun=photogrammetrie", "-Pimage=" + INSEL, "-Pmatch-threshold=2", "--sfmx-plan"])
    assert r.returncode == 255 and "match-threshold" in r.stdout
    assert run_exe(["-Prun=pcl-stats"]).returncode == 255
    assert run_exe(["-Prun=photogrammetrie", "-Ploglevel=x"]).returncode == 255


def test_driver_loglevel_filters():
    base = ["-Prun=photogrammetrie", "-Pimage=" + INSEL, "-Pcamera-model=Foo", "--sfmx-plan"]
    assert "[WARN]" in run_exe(base).stdout
    out = run_exe(base + ["-Ploglevel=4"]).stdout
    assert "[WARN]" not in out and "[INFO]" not in out


def _expected_pairs(n, seq, grid):
    from oracle import oracle
    if seq >= 2 and grid >= 1:
        return oracle.pairs_grid(n, seq, grid, 1)
    if seq >= 2:
        return oracle.pairs_video(n, seq)
    return oracle.pairs_unordered(n)


RUN_SCRIPTS = json.load(open(os.path.join(REPO, "tests", "golden", "run_scripts.json")))


@pytest.mark.parametrize("script", sorted(RUN_SCRIPTS), ids=sorted(RUN_SCRIPTS))
def test_run_script_replay_plan(script, tmp_path):
    """run-scripts/<script> with $1 = 2, $2 = 1, -Pimage=./images -> the insel images."""
    argv = [w.replace("$1", "2").replace("$2", "1") for w in RUN_SCRIPTS[script][1:]] + ["--sfmx-plan"]
    os.symlink(INSEL, tmp_path / "images")
    r = run_exe(argv, cwd=tmp_path)
    if "-Prun=pcl-stats" in argv:
        assert r.returncode == 255 and "outside the sfmx hot path" in r.stdout
        return
    assert r.returncode == 0, r.stdout + r.stderr
    plan = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    flags = dict(w[2:].split("=", 1) for w in argv if w.startswith("-P"))
    c = plan["config"]
    assert [os.path.basename(p) for p in plan["images"]] == ["1.jpg", "2.jpg", "3.jpg"]
    assert plan["camera"] == {"model": flags["camera-model"], "focal_length": 864.0, "cx": 360.0, "cy": 202.5,
                              "resolution": [720, 405]}
    assert c["feature_detector"] == (1 if flags["feature-detector"] == "ORB" else 0)
    assert c["norm"] == (6 if flags["feature-detector"] == "ORB" else 4)
    assert c["feature_limit"] == int(flags["feature-limit"])
    assert c["feature_matcher"] == (1 if flags.get("feature-matcher") == "FLANN" else 0)
    assert c["omp_feature_threads"] == (int(flags.get("omp-feature-threads", "0")) or HW)
    seq, grid = int(flags.get("feature-sequence", "0")), int(flags.get("feature-gridlength", "0"))
    assert plan["strategy"] == ("Grid" if seq >= 2 and grid >= 1 else "Video" if seq >= 2 else "Unordered")
    assert plan["pairs"] == _expected_pairs(3, seq, grid).tolist()
    for f in ("colored", "dense", "mesh", "stats", "artifacts", "sgm"):
        assert c[f] == int(f"--{f}" in argv)
    assert c["loglevel"] == 2 and c["force_colored_output"] == 1 and c["n_warnings"] == 0


def test_prepare_working_dir_refuses_dangerous_targets(tmp_path, monkeypatch):
    """prepareWorkingDir (PhotogrammetrieCli.cpp:399-402) clears -Pout; the restatement keeps that
    but refuses the filesystem root, the home directory and the current directory or its ancestors."""
    import logging
    from sfmx import cli
    log = logging.getLogger("t")
    monkeypatch.chdir(tmp_path)
    (tmp_path / "keep.txt").write_text("x")
    for bad in (os.sep, os.path.expanduser("~"), ".", str(tmp_path), str(tmp_path.parent)):
        with pytest.raises(ValueError):
            cli.prepare_working_dir(bad, log)
    assert (tmp_path / "keep.txt").exists()
    out = tmp_path / "out"
    out.mkdir()
    (out / "stale.txt").write_text("x")
    cli.prepare_working_dir(str(out), log)
    assert out.is_dir() and not (out / "stale.txt").exists()
