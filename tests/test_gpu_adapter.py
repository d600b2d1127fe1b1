"""GPU: the compiled C++ caller of the ABI (tests/cpp/adapter_main.cpp + INTEGRATION.md §2's
GpuFeatureMatchingStrategy, built by __graft_entry__.build()) run as a separate process, as
the reference's SfM.cpp:545 would call calculateShotMatches.  Its ShotMatches must equal the
oracle's lists byte for byte, for SIFT (unordered / video) and ORB (grid)."""
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

import sfmx
from sfmx import synth

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "cpp", "adapter_test")


def _write(path, imgs, mode, seq, row_len):
    with open(path, "wb") as f:
        f.write(struct.pack("<4i", len(imgs), mode, seq, row_len))
        for x in imgs:
            f.write(struct.pack("<3i", x.shape[0], x.shape[1], 5 if x.dtype == np.float32 else 0))
            f.write(np.ascontiguousarray(x).tobytes())


def _read(path):
    out = []
    with open(path, "rb") as f:
        (n,) = struct.unpack("<q", f.read(8))
        for _ in range(n):
            l, r, c = struct.unpack("<iiq", f.read(16))
            m = np.frombuffer(f.read(16 * c), dtype=sfmx.DMATCH_DTYPE) if c else np.zeros(0, sfmx.DMATCH_DTYPE)
            out.append((l, r, m))
    return out


@pytest.mark.parametrize("case", ["sift_unordered", "sift_video", "orb_grid"])
def test_compiled_adapter_equals_oracle(case):
    from oracle import oracle
    assert os.path.exists(EXE), "tests/cpp/adapter_test not built (run __graft_entry__.build())"
    if case == "sift_unordered":
        imgs, mode, seq, rl = synth.sift_images(6, 2000, seed=71), 0, 2, 0
        imgs[2] = imgs[2][:777]
        pairs = sfmx.pairs_unordered(6)
    elif case == "sift_video":
        imgs, mode, seq, rl = synth.sift_images(5, 1500, seed=72), 1, 3, 0
        pairs = sfmx.pairs_video(5, 3)
    else:
        imgs, mode, seq, rl = synth.orb_images(6, 1800, seed=73), 2, 3, 3
        pairs = sfmx.pairs_grid(6, 3, 3, 0)
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        _write(fin, imgs, mode, seq, rl)
        r = subprocess.run([EXE, fin, fout], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        got = _read(fout)
    exp, eoff = oracle.match_pairs(imgs, pairs)
    assert [(l, r) for l, r, _ in got] == [tuple(p) for p in pairs]
    for p, (_, _, m) in enumerate(got):
        assert m.tobytes() == exp[eoff[p]:eoff[p + 1]].tobytes()
