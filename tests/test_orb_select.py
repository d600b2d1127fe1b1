"""CPU: the parallel formulation of KeyPointsFilter::retainBest for a device selection (the r03
orb_retain_kernel, tools/archive/r03_unvalidated_orb_device_retain.patch; DESIGN.md, "retainBest on
the device") against libstdc++'s own std::nth_element / std::partition / std::__introselect (small
depth limits: the __heap_select fallback), on random arrays with many ties.  The reference calls
retainBest through OpenCV's ORB (PhotogrammetrieCli.cpp:347-348 -> cv::ORB::detectAndCompute ->
KeyPointsFilter::retainBest); the permutation it leaves decides the keypoint order, hence the
descriptor rows the matcher sees."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "cpp", "orb_select_sim.cpp")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_parallel_retain_best_matches_libstdcxx(tmp_path):
    exe = str(tmp_path / "orb_select_sim")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, SRC], check=True, capture_output=True, text=True, timeout=300)
    r = subprocess.run([exe, "3000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
