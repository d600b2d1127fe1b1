"""Timeline of one chol_factor launch at C5 (diagnostic library, ba_chol.hpp CHOL_TRACE; tooling, not
product): per ticket the item (leaf k, or task (a, b) from source k), its row masks, and the times (us
from the first start) at which it started, had its operands, had W_k, finished its products, knew
whether it finishes the task, started the inverse, and ended.  GPU box only:
  SFMX_LIB_NAME=libsfmx_diag.so python tools/chol_trace.py [cams] [points]"""
import ctypes as C
import os
import sys

os.environ.setdefault("SFMX_LIB_NAME", "libsfmx_diag.so")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sfm-mvs-pipeline_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from sfmx import ba, synth  # noqa: E402
from sfmx._lib import lib  # noqa: E402

cams = int(sys.argv[1]) if len(sys.argv) > 1 else 200
pts = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
prob = synth.ba_problem(cams, pts)
ctx = ba.BAContext(ba.BAProblem(**prob), ba.default_options())
ctx.run(max_iterations=2)
f = lib.sfmx_ba_debug_chol_items
f.argtypes, f.restype = [C.c_void_p, C.c_void_p, C.c_int32], C.c_int
n = f(ctx._h, None, 0)
it = np.zeros(8 * n, np.int32)
f(ctx._h, it.ctypes.data, len(it))
items, masks = it[:4 * n].reshape(n, 4), it[4 * n:].reshape(n, 4)
g = lib.sfmx_ba_debug_chol_trace
g.argtypes, g.restype = [C.c_void_p, C.c_int32], C.c_int
tr = np.zeros((n, 16), np.int64)
g(tr.ctypes.data, n)
# the plan's tasks (same graph as the solver's)
op, oc = np.asarray(prob["obs_point"]), np.asarray(prob["obs_cam"])
adj = np.zeros((cams, cams), np.uint8)
st = np.searchsorted(op, np.arange(len(prob["points"]) + 1))
for p in range(len(prob["points"])):
    cs = oc[st[p]:st[p + 1]]
    adj[np.ix_(cs, cs)] = 1
np.fill_diagonal(adj, 0)
pl = ba.factor_plan(adj, {'natural': 0, 'nd': 1, 'nd1': 2, 'nd2': 3, 'nd4': 4}.get(os.environ.get('SFMX_BA_ORDER', ''), -1))
tasks, src = pl["tasks"], pl["src"]
t0 = tr[:, 0][tr[:, 0] > 0].min()
us = lambda v: (v - t0) / 100.0 if v > 0 else float("nan")   # 100 MHz ticks
print(f"items {n}; launch span {(tr[:, 13].max() - t0) / 100.0:.1f} us")
print("tk  item                 masks(ra rb gc pad ka kb)      start  opnds  W_k   Wld    G    upd   fin   inv   sw0   sw1   sw2   sw3  Wpub   end  xcc/cu")
for tk in range(n):
    x, y, z, w = items[tk]
    if y < 0:
        desc = f"leaf {x}"
    else:
        l, a, b, inv, s0, s1 = tasks[x]
        desc = f"L{l} ({a},{b})<-{src[y]} n{w & 0xffff}{' I' if w >> 16 else ''}"
    mx = masks[tk, 0]
    m = f"{mx & 15:x} {(mx >> 4) & 15:x} {(mx >> 8) & 15:x} {(mx >> 12) & 15:x} {masks[tk, 1] & 0xffff:04x} {masks[tk, 2] & 0xffff:04x}"
    hw = int(tr[tk, 15])
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    print(f"{tk:3d} {desc:20s} {m:30s} " + " ".join(f"{us(v):5.1f}" for v in tr[tk, :14]) + f"  x{hw >> 32} se{se} cu{cu}")
