"""Golden fixture loader (test helper)."""
import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def desc_sets():
    """Names of the descriptor-set fixtures (those holding images + expected matches)."""
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))):
        with np.load(f) as d:
            if "img0" in d.files:
                out.append(os.path.basename(f)[:-4])
    return out


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz")) as d:
        data = {k: d[k] for k in d.files}
    if "img0" in data:
        n = int(data["n_imgs"])
        l2 = int(data["kind"]) == 0
        data["imgs"] = [data[f"img{i}"].astype(np.float32) if l2 else data[f"img{i}"] for i in range(n)]
        data["ratio"] = float(data.get("ratio", 0.7))
    return data
