"""Generate tests/golden/sift_37mp.npz (run from repo root: ``python tests/golden/make_sift_big.py``).

A 6144 x 6144 (37.7 MP) synthetic photo: flat noisy background with blob patches at
six places. The SIFT oracle (oracle/sift_oracle.cpp, OpenCV 4.5.1 SIFT restated) takes
about two minutes on it, too long for the GPU suite, so its keypoints and descriptors
are committed here and tests/test_gpu_sift.py::test_37mp_image_fits_the_arena compares
the GPU output with them. The image is regenerated from the seed in the test and
checked against the stored SHA-256 first.
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

import sift_cases  # noqa: E402


def main():
    from oracle import oracle
    img = sift_cases.big_photo_37mp()
    k, d = oracle.sift(img, nfeatures=3000)
    np.savez_compressed(os.path.join(HERE, "sift_37mp.npz"), keypoints=k, descriptors=d.astype(np.uint8),
                        sha256=np.frombuffer(hashlib.sha256(img.tobytes()).digest(), np.uint8))
    print("wrote sift_37mp.npz", len(k), "keypoints")


if __name__ == "__main__":
    main()
