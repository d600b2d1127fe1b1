"""SIFT extraction alone (sfmx_sift_detect_compute) on synthetic photos, for rocprofv3."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sfm-mvs-pipeline_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import sfmx  # noqa: E402
import sift_cases  # noqa: E402

H, W, N = int(os.environ.get("SIFT_H", "1080")), int(os.environ.get("SIFT_W", "1920")), int(os.environ.get("SIFT_N", "4"))
from sfmx import synth  # noqa: E402
imgs = [synth.gray_photo(H, W, seed=s) for s in range(N)]
dev = torch.device("cuda:0")
s = sfmx.features.SIFT.create(nfeatures=8192)
kt = torch.zeros((1 << 16, 7), dtype=torch.int32, device=dev)
dt = torch.zeros((1 << 16, 128), dtype=torch.float32, device=dev)
tis = [torch.from_numpy(i).to(dev) for i in imgs]
for r in range(2):
    for i, ti in enumerate(tis):
        t = time.perf_counter()
        n = s.detectAndCompute_device(ti, kt, dt)
        torch.cuda.synchronize()
        print(f"img {i} n={n} kernel_ms={sfmx.features.last_kernel_ms():.2f} wall_ms={(time.perf_counter() - t) * 1e3:.2f}", flush=True)
