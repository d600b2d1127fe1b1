"""ORB extraction on one stream (serialized kernels, for a per-kernel time breakdown under
rocprofv3 --kernel-trace): 32 synthetic 1920x1080 photos resident in HBM, chunks of 16, twice.
GPU box only (tooling)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sfm-mvs-pipeline_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from sfmx import features, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
base = [synth.gray_photo(1080, 1920, seed=2000 + i) for i in range(2)]
imgs = [torch.from_numpy(np.ascontiguousarray(np.roll(base[j % 2], 41 * j, axis=1))).cuda() for j in range(n)]
orb = features.ORB.create(30000)
kts = [torch.zeros((1 << 15, 7), dtype=torch.int32, device="cuda") for _ in imgs]
dts = [torch.zeros((1 << 15, 32), dtype=torch.uint8, device="cuda") for _ in imgs]
for _ in range(2):
    counts = orb.detectAndCompute_batch_device(imgs, kts, dts, n_streams=1)
torch.cuda.synchronize()
print("keypoints per image", float(np.mean(counts)), "kernel ms per image", features.orb_last_kernel_ms())
