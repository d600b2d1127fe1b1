"""Phase cycle totals of the BA group kernels from the diagnostic stamp build
(make -C sfm-mvs-pipeline_amd stamps -> lib/libsfmx_stamps.so; SFMX_BA_STAMPS, ba_group.hpp).
Runs the C5 bench problem once and prints, per stamp slot, the s_memtime cycles of thread 0
summed over workgroups and divided by the number of LM steps.  GPU box only (tooling)."""
import ctypes as C
import os
import sys

os.environ.setdefault("SFMX_LIB_NAME", "libsfmx_stamps.so")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sfm-mvs-pipeline_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from sfmx import ba, synth  # noqa: E402
from sfmx._lib import lib  # noqa: E402

NAMES = {0: "gschur round MFMA", 1: "gschur wave combine", 2: "gschur store", 3: "gschur obs phase",
         4: "gschur point phase", 5: "gschur round H fill", 8: "glin zero G + sync",
         9: "glin dual numbers + stores", 10: "glin barrier wait", 11: "glin point sums + gram + sync",
         12: "glin epilogue",
         16: "gupdate obs", 17: "gupdate point", 18: "gupdate model", 19: "gupdate epilogue",
         24: "camred cam loads", 25: "camred cam combine", 26: "camred intr loads", 27: "camred intr sum",
         28: "camred cam WGs (count)", 29: "camred cam WG max", 30: "camred intr WGs (count)",
         31: "camred intr WG max", 32: "assemble pose WGs", 33: "assemble pose WG max",
         34: "assemble cam-intr WGs", 35: "assemble cam-intr WG max", 36: "assemble intr WGs",
         37: "assemble intr WG max",
         40: "fin fold", 41: "fin group sums", 42: "fin (cand loop)", 43: "fin barrier", 44: "fin rows",
         45: "fin copy + reduce", 46: "fin publish", 47: "fin calls",
         48: "finC fold", 49: "finC group sums", 50: "finC cand loop", 51: "finC barrier", 52: "finC rows",
         53: "finC copy + reduce", 54: "finC publish", 55: "finC calls"}
prob = synth.ba_problem(200, 200_000)
ctx = ba.BAContext(ba.BAProblem(**prob), ba.default_options())
ctx.run(max_iterations=1)
ctx.reset()
f = lib.sfmx_ba_debug_stamps
f.argtypes, f.restype = [C.POINTER(C.c_ulonglong), C.c_int32], C.c_int
buf = (C.c_ulonglong * 64)()
f(buf, 64)   # clear
sm, _ = ctx.run()
f(buf, 64)
steps = sm["num_successful_steps"] + sm["num_unsuccessful_steps"] - 1
print(f"LM steps {steps}; cycles per step (thread 0 of each workgroup, summed over workgroups):")
for i, v in enumerate(buf):
    if v:
        if 40 <= i < 56 and i % 8 != 7:   # ba_finalize phases: cycles per call (one workgroup)
            n = buf[47 if i < 48 else 55]
            print(f"  [{i:2d}] {NAMES.get(i, '?'):22s} {v / max(n, 1):10.0f} cyc/call")
        elif i in (47, 55):
            print(f"  [{i:2d}] {NAMES.get(i, '?'):22s} {v:10d}")
        elif i in (29, 31, 33, 35, 37):   # the longest single workgroup (s_memtime cycles), not a total
            print(f"  [{i:2d}] {NAMES.get(i, '?'):22s} {v:10d} cyc")
        elif i in (28, 30, 32, 34, 36):
            print(f"  [{i:2d}] {NAMES.get(i, '?'):22s} {v / max(steps, 1):10.1f} per step")
        else:
            print(f"  [{i:2d}] {NAMES.get(i, '?'):22s} {v / max(steps, 1) / 1e6:10.2f} Mcyc")
