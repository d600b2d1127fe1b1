"""r06 debug (tooling): final costs of one small BA problem through the one-rank path (fused ba_assemble
+ camera terms), the one-rank path with ba_add_cam (SFMX_BA_NOFUSE=1, diagnostic library) and the
all-reduce-hook path (ba_add_cam after the all-reduce)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sfm-mvs-pipeline_amd")]
os.environ.setdefault("SFMX_LIB_NAME", "libsfmx_diag.so")
import torch  # noqa
from sfmx import ba, synth
p = synth.ba_problem(10, 1500, seed=25)
def run(hook, mask):
    os.environ["SFMX_BA_FUSE"] = str(mask)
    ctx = ba.BAContext(ba.BAProblem(**p), allreduce=(lambda ptr, n, op, st: None) if hook else None)
    s, tr = ctx.run()
    ctx.close()
    return s["final_cost"], tr
for hook, mask in ((True, 0),) + tuple((False, m) for m in range(8)):
    c, tr = run(hook, mask)
    print(f"hook={hook} fuse_mask={mask} final={c!r}")
