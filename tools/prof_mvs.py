"""Undistortion kernel alone on the bench workload (50 x 12 MP RGB), for rocprofv3."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sfm-mvs-pipeline_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from sfmx import mvs  # noqa: E402

H, W, C, N = 3000, 4000, 3, int(os.environ.get("MVS_N", "50"))
g = torch.Generator(device="cuda:0").manual_seed(1)
srcs = [torch.randint(0, 256, (H, W, C), dtype=torch.uint8, device="cuda:0", generator=g) for _ in range(N)]
dsts = [torch.empty_like(t) for t in srcs]
rng = np.random.default_rng(1)
Ks = [np.array([[4000.0, 0, 2000.3], [0, 4000.0, 1500.2], [0, 0, 1]]) for _ in range(N)]
ds = [np.array([rng.normal(0, 0.1), rng.normal(0, 0.03), 0, 0, 0]) for _ in range(N)]
if os.environ.get("MVS_DISTINCT", "0") != "1":   # the reference's export: one camera for every shot
    ds = [ds[0]] * N
for _ in range(int(os.environ.get("MVS_REPS", "5"))):
    mvs.undistort_device(srcs, dsts, Ks, ds)
    print(f"kernel_ms {mvs.last_kernel_ms():.3f}", flush=True)
