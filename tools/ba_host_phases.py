"""BA host setup phase times of an SfM update (C5 ring grown 199 -> 200 cameras, SfM point order):
sfmx_ba_debug_incremental_check (diagnostic library) -> the update's and a fresh load's host time and
the update's phases (HostScratch::tm).  CPU only; run on the GPU box for its CPU.  (tooling)
python tools/ba_host_phases.py [REPEATS]"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sfm-mvs-pipeline_amd"), os.path.join(REPO, "tests")]
from diag import diag_lib  # noqa: E402
from sfmx import ba, synth  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
base = synth.ba_sfm_order(synth.ba_problem(200, 200000))
a, b = ba.BAProblem(**synth.ba_registered(base, 199)), ba.BAProblem(**synth.ba_registered(base, 200))
names = ["view", "compare", "bucket_lists", "order_groups", "layout", "merge", "tasks", "shadows", "(ordering part)"]
best = None
for _ in range(reps):
    out, ms = (C.c_int32 * 2)(), (C.c_double * 11)()
    rc = diag_lib().sfmx_ba_debug_incremental_check(a.struct(), b.struct(), 0, out, ms)
    assert rc == 0, diag_lib().sfmx_last_error()
    best = list(ms) if best is None else [min(x, y) for x, y in zip(best, ms)]
print(f"cpus {os.cpu_count()}  buckets redone {out[0]} of {out[1]}  (minimum over {reps} runs, ms)")
print(f"update {best[0]:.3f}  fresh load {best[1]:.3f}")
print("  " + "  ".join(f"{n} {v:.3f}" for n, v in zip(names, best[2:])))
