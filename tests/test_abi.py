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


# ---- header <-> binding agreement --------------------------------

_SCALARS = {"int32_t": "c_int32", "int64_t": "c_int64", "uint32_t": "c_uint32", "double": "c_double",
            "float": "c_float", "int": "c_int", "char": "c_char"}


def _declarations():
    """(name, return type, [param types]) of every function the headers declare."""
    out = []
    for h in sorted(glob.glob(os.path.join(REPO, "include", "*.h"))):
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        src = re.sub(r"typedef[^;]*;", "", src)
        src = re.sub(r"^\s*#[^\n]*", "", src, flags=re.M)
        src = src.replace('extern "C" {', "")
        for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(sfmx_\w+)\s*\(([^()]*)\)\s*;", src):
            ret, name, params = " ".join(m.group(1).split()), m.group(2), " ".join(m.group(3).split())
            ps = [] if params in ("", "void") else [re.sub(r"\s*\b\w+$", "", p.strip()) for p in params.split(",")]
            out.append((name, ret, ps))
    return out


def _ctype_ok(ctype_decl, ct):
    import ctypes as C
    t = ctype_decl.replace("const", "").strip()
    if t == "void":
        return ct is None
    if t == "sfmx_allreduce_fn":
        return ct is _lib.ALLREDUCE_FN
    if "*" in t:
        base = t.replace("*", "").strip()
        if base == "char" and t.count("*") == 1:
            return ct in (C.c_char_p, C.c_void_p)
        return ct is C.c_void_p or (isinstance(ct, type) and issubclass(ct, C._Pointer))
    return ct is getattr(C, _SCALARS[t])


@pytest.mark.parametrize("name,ret,params", _declarations(), ids=[d[0] for d in _declarations()])
def test_ctypes_prototype_matches_header(name, ret, params):
    assert name in _lib.PROTOTYPES, name
    res, args = _lib.PROTOTYPES[name]
    assert len(args) == len(params), f"{name}: header has {len(params)} params, binding {len(args)}"
    assert _ctype_ok(ret, res), f"{name}: return {ret} vs {res}"
    for i, (p, a) in enumerate(zip(params, args)):
        assert _ctype_ok(p, a), f"{name}: param {i} {p} vs {a}"


def test_struct_layouts_match_header(tmp_path):
    """sizeof/offsetof of the ABI structs from a C compile of the headers == the ctypes mirrors."""
    import ctypes as C
    import subprocess
    structs = {"sfmx_dmatch": _lib.sfmx_dmatch, "sfmx_desc": _lib.sfmx_desc, "sfmx_ba_problem": _lib.sfmx_ba_problem,
               "sfmx_ba_options": _lib.sfmx_ba_options, "sfmx_ba_summary": _lib.sfmx_ba_summary,
               "sfmx_cli_config": _lib.sfmx_cli_config}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "sfmx.h"', '#include "sfmx_ba.h"', '#include "sfmx_cli.h"',
             'int main(void){']
    for s, cls in structs.items():
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n") if l)
    for s, cls in structs.items():
        assert int(got[s]) == C.sizeof(cls), s
        for f, _ in cls._fields_:
            assert int(got[f"{s}.{f}"]) == getattr(cls, f).offset, f"{s}.{f}"


def test_integration_adapter_is_the_compiled_one():
    """INTEGRATION.md §2 shows exactly the adapter body tests/cpp compiles and the GPU suite runs."""
    body = open(os.path.join(REPO, "tests", "cpp", "GpuFeatureMatchingStrategy.h")).read()
    adapter = body[body.index("// --- adapter begin ---\n") + 24: body.index("// --- adapter end ---")]
    assert adapter in open(os.path.join(REPO, "INTEGRATION.md")).read()
    assert os.path.exists(os.path.join(REPO, "tests", "cpp", "adapter_test")), "build() compiles tests/cpp/adapter_test"


def test_product_library_reads_no_tuning_variables():
    """a drop-in library whose output changes with a stray environment
    variable is a hazard.  The kernel variants, timing probes and alternative factorization
    forms live only in lib/libsfmx_diag.so (csrc/diag.hpp); the product library carries no
    SFMX_* variable name and no getenv of its own."""
    blob = open(_lib.LIB_PATH, "rb").read()
    for var in (b"SFMX_PROBE_XOR80", b"SFMX_SIFT_VARIANT", b"SFMX_SIFT_P2", b"SFMX_ORB_VARIANT", b"SFMX_BA_ORDER",
                b"SFMX_BA_BACK", b"SFMX_BA_SPLIT", b"SFMX_BA_DAG", b"SFMX_BA_SPEC", b"SFMX_SIFT_SMALL"):
        assert var not in blob, var
    names = set(re.findall(rb"SFMX_[A-Z0-9_]+", blob))
    assert names <= {b"SFMX_CAM_SIMPLE", b"SFMX_NORM_L2", b"SFMX_NORM_HAMMING", b"SFMX_BA_MAX_INTR"}, names   # messages


def test_diagnostic_library_exports_the_same_entry_points():
    import diag
    dl = diag.diag_lib()
    for name in declared_functions():
        assert hasattr(dl, name), name
    assert b"SFMX_SIFT_VARIANT" in open(diag.DIAG_PATH, "rb").read()


def test_integration_ba_adapter_is_the_compiled_one():
    """INTEGRATION.md §4 shows exactly the doBundleAdjustment adapter tests/cpp compiles and the GPU
    suite runs (several cameras: one intrinsics block per ICamera, getCenter, dynamic_cast)."""
    body = open(os.path.join(REPO, "tests", "cpp", "GpuBundleAdjustment.h")).read()
    adapter = body[body.index("// --- adapter begin ---\n") + 24: body.index("// --- adapter end ---")]
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    assert adapter in text
    assert "getCenter(cx, cy)" in adapter and "ceresParameterCount" not in text and "getCx" not in text
    assert os.path.exists(os.path.join(REPO, "tests", "cpp", "ba_adapter_test")), "build() compiles tests/cpp/ba_adapter_test"


def test_ba_problem_struct_layout():
    """The ctypes mirror of sfmx_ba_problem has the header's field offsets (several-camera fields)."""
    import ctypes as C
    S = _lib.sfmx_ba_problem
    assert S.n_intr.offset == 4 * 4 + 6 * 8 + 2 * 8 and S.intr_model.offset == S.n_intr.offset + 8
    assert C.sizeof(S) == S.intr_center.offset + 8
