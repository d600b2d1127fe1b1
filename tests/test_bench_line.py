"""The printed bench line stays parseable by the driver (r04's 21.1 KB line
was recorded with parsed: null).  Built here from a recorded full result (profiles/r04z_bench_line.json,
the r04 line as the bench then printed it), no GPU."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

HEAD = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]


def _full():
    with open(os.path.join(REPO, "profiles", "r04z_bench_line.json")) as f:
        return json.load(f)


def test_compact_line_small_with_headline_first():
    full = _full()
    assert len(json.dumps(full)) > 20000          # the line r04's driver could not parse
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    assert len(s) <= bench.LINE_MAX_BYTES <= 12 * 1024
    assert list(line)[:len(HEAD)] == HEAD
    json.loads(s)                                  # strict round trip
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in line["roofline"]
    assert line["roofline"]["frac"] == pytest.approx(full["roofline"]["frac"], rel=1e-5)
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in line["cpu_baseline"]
    assert line["value"] == pytest.approx(full["value"], rel=1e-5)
    assert line["config"]["workload"].startswith("50 images")
    assert line["parity"] is True
    assert line["detail"] == "gpurun_out/bench_detail.json"


def test_every_leg_summary_under_600_bytes():
    full = _full()
    line = bench.compact_line(full)
    assert set(line["legs"]) >= {"orb", "c3", "ba", "ba_calls", "homography", "find_3d2d", "mvs", "features",
                                 "features_orb"}
    for name, leg in line["legs"].items():
        assert len(json.dumps(leg)) <= bench.LEG_MAX_BYTES, name
    for name in ("orb", "c3", "mvs", "features", "features_orb"):
        assert line["legs"][name]["frac"] is not None, name
        assert line["legs"][name]["cpu_baseline"] is not None, name
        assert line["legs"][name]["parity"] is True, name
    ba = line["legs"]["ba"]
    assert ba["unit"] == "ms" and ba["vs_cpu"] == pytest.approx(full["ba"]["cpu_baseline"]["value"] / full["ba"]["value"],
                                                                 rel=1e-3)
    assert len(line["legs"]["ba_calls"]["single_camera_steps_setup_frac"]) == 4


def test_oversized_legs_are_cut_not_the_headline():
    full = _full()
    # a pathological leg (long strings everywhere) must not push the line past the limit
    for name in ("orb", "c3", "mvs"):
        full[name]["unit"] = "x" * 3000
    line = bench.compact_line(full)
    s = json.dumps(line)
    assert len(s) <= bench.LINE_MAX_BYTES
    assert list(line)[:len(HEAD)] == HEAD and line["roofline"]["frac"] is not None


def test_write_detail_side_file(tmp_path, monkeypatch):
    p = tmp_path / "d.json"
    monkeypatch.setenv("SFMX_BENCH_DETAIL", str(p))
    full = _full()
    rel = bench.write_detail(full)
    assert rel is not None and json.loads(p.read_text())["ba"]["calls"]["calls"] == full["ba"]["calls"]["calls"]


def test_failed_legs_leave_an_error_not_a_missing_line():
    full = _full()
    full["ba"] = {"error": "SfmxError: ncclCommInitRank: unhandled system error"}
    full["mvs"] = {"error": "RuntimeError: x" * 100}
    line = bench.compact_line(full)
    assert line["legs"]["ba"]["error"].startswith("SfmxError")
    assert len(line["legs"]["mvs"]["error"]) <= 300
    assert "ba_calls" not in line["legs"]
    assert len(json.dumps(line)) <= bench.LINE_MAX_BYTES and line["roofline"]["frac"] is not None


def test_recorded_r06_line_kernel_time_within_the_step():
    """the line's kernel time comes from the timed steps' own events (the
    matcher's per-run event ring), so it cannot exceed the step it is part of."""
    with open(os.path.join(REPO, "profiles", "r06n_bench_line.json")) as f:
        line = json.loads(f.read())
    assert list(line)[:len(HEAD)] == HEAD
    rf = line["roofline"]
    assert 0 < rf["kernel_ms_per_launch"] <= line["ms_per_step"]
    assert rf["frac"] == pytest.approx(rf["achieved"] / rf["peak"], rel=1e-4)
    assert line["n_gpus"] == 1 and line["config"]["workload"].startswith("50 images")
