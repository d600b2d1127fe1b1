"""CPU: the C-ABI library loads, exports every symbol include/*.h declares,
and its host-only entry points (pair enumeration, argument validation) behave
like the reference strategies.  No compute calls: there is no GPU here."""
import glob
import os
import re

import numpy as np
import pytest

import sfmx
from sfmx import _lib
import fixtures

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*[A-Za-z_][\w\s\*]*?\b(sfmx_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_entry_points():
    names = declared_functions()
    assert "sfmx_matcher_run" in names and "sfmx_pairs_grid" in names
    assert len(names) >= 15


@pytest.mark.parametrize("name", declared_functions())
def test_library_exports(name):
    assert hasattr(_lib.lib, name), f"libsfmx.so does not export {name}"
    assert name in _lib.PROTOTYPES, f"no ctypes prototype for {name}"


def test_pairs_match_golden():
    p = fixtures.load("pairs")
    assert np.array_equal(sfmx.pairs_unordered(7), p["unordered7"])
    assert np.array_equal(sfmx.pairs_video(10, 3), p["video10_3"])
    assert np.array_equal(sfmx.pairs_video(5, 2), p["video5_2"])
    assert np.array_equal(sfmx.pairs_grid(20, 3, 5), p["grid20_3_5"])
    assert np.array_equal(sfmx.pairs_grid(23, 3, 5, 0), p["grid23_3_5_ref"])
    assert np.array_equal(sfmx.pairs_grid(23, 3, 5, 1), p["grid23_3_5_int"])
    assert np.array_equal(sfmx.pairs_grid(200, 3, 20), p["grid200_3_20"])


def test_pair_counts_of_configs():
    assert len(sfmx.pairs_unordered(50)) == 1225        # C2
    assert len(sfmx.pairs_unordered(200)) == 19900      # C3
    assert len(sfmx.pairs_grid(200, 3, 20)) == 881      # C4 (assumed seq=3, rowLen=20)
    assert len(sfmx.pairs_video(3, 2)) == 2             # C1 insel, seq=2
    assert sfmx.pairs_video(3, 3).tolist() == [[0, 1], [0, 2], [1, 2]]
    assert len(sfmx.pairs_unordered(0)) == 0 and len(sfmx.pairs_unordered(1)) == 0


def test_strategy_argument_errors():
    with pytest.raises(ValueError):
        sfmx.VideoFeatureMatchingStrategy(1)
    with pytest.raises(ValueError):
        sfmx.GridFeatureMatchingStrategy(1, 5)
    with pytest.raises(ValueError):
        sfmx.GridFeatureMatchingStrategy(3, 0)
    with pytest.raises(ValueError):
        sfmx.pairs_video(5, 1)
    with pytest.raises(ValueError):
        sfmx.pairs_grid(5, 3, 0)


def test_no_gpu_fails_loudly():
    if _lib.lib.sfmx_device_count() > 0:
        pytest.skip("a gfx950 device is visible")
    with pytest.raises(_lib.SfmxError):
        sfmx.BFMatcher(sfmx.NORM_L2)
