"""Adversarial known-answer inputs for the matcher (test helper).

Each builder returns (query, train) descriptor matrices that force one of the
semantics the reference inherits from cv::BFMatcher [ext]: ties broken by the
lower train index, ranking on float-sqrt bits (collisions), the double-precision
ratio boundary, and the <2-neighbour / empty-train rules."""
import numpy as np


def _four_squares(r: int):
    """r (< 4*255^2) as a sum of <= 4 squares with parts <= 255 (Lagrange)."""
    import math
    for a in range(min(255, math.isqrt(r)), -1, -1):
        ra = r - a * a
        for b in range(min(a, math.isqrt(ra)), -1, -1):
            rb = ra - b * b
            for c in range(min(b, math.isqrt(rb)), -1, -1):
                rc = rb - c * c
                d = math.isqrt(rc)
                if d * d == rc and d <= c:
                    return [a, b, c, d]
    raise ValueError(r)


def _row_with_sq(target: int, dim: int = 128) -> np.ndarray:
    """Non-negative integer row (values <= 255) whose sum of squares == target."""
    r = np.zeros(dim, np.float32)
    n255 = max(0, target // 65025 - 1)
    rem = target - n255 * 65025
    parts = [255] * n255 + _four_squares(rem)
    if len(parts) > dim:
        raise ValueError("target not representable")
    r[: len(parts)] = parts
    assert int((r.astype(np.int64) ** 2).sum()) == target
    return r


def sift_ties(seed=1):
    rng = np.random.default_rng(seed)
    t = rng.integers(0, 256, (40, 128)).astype(np.float32)
    t[7] = t[3]            # duplicate train rows
    t[20] = t[3]
    q = np.stack([t[3], t[3] + 1, t[10], np.clip(t[3] + 2, 0, 255)]).astype(np.float32)
    q = np.clip(q, 0, 255)
    return q, t


def sift_sqrt_collision():
    """Query = 0; train rows at squared distances that collide under float sqrt
    (s >= 4,197,201), placed so integer ranking and float-bit ranking differ."""
    q = np.zeros((3, 128), np.float32)
    rows = []
    # s values: find a colliding adjacent pair (s-1, s) with sqrtf equal
    s_pairs = []
    s = 4197201
    while len(s_pairs) < 3:
        if np.sqrt(np.float32(s)) == np.sqrt(np.float32(s - 1)):
            s_pairs.append((s - 1, s))
        s += 1
    (a0, a1), (b0, b1), (c0, c1) = s_pairs
    # j=0: far filler; j=1: larger s of the first colliding pair; j=2: its smaller s;
    # so integer ranking says (2,1) but float-bit ranking says (1,2).
    rows = [_row_with_sq(8000000), _row_with_sq(a1), _row_with_sq(a0), _row_with_sq(b1), _row_with_sq(b0),
            _row_with_sq(c0), _row_with_sq(c1)]
    t = np.stack(rows).astype(np.float32)
    q[1, 0] = 0
    q[2] = 0
    return q, t


def sift_ratio_boundary():
    """List of (q, t): q = one zero row, t = rows at s0 and s1 with s0/s1
    around 0.49 (d0/d1 around 0.7 in reals), so the float-then-double ratio
    test decides on rounding."""
    cases = [(49 * 4, 100 * 4), (49 * 9, 100 * 9), (49 * 100 - 1, 100 * 100), (49 * 100 + 1, 100 * 100),
             (49 * 2500, 100 * 2500), (49 * 10000, 100 * 10000), (49 * 40000, 100 * 40000)]
    out = []
    for s0, s1 in cases:
        q = np.zeros((1, 128), np.float32)
        t = np.stack([_row_with_sq(s1), _row_with_sq(s0), _row_with_sq(s1 + 12345)])
        out.append((q, t))
    return out


def orb_ties(seed=2):
    rng = np.random.default_rng(seed)
    t = rng.integers(0, 256, (50, 32), dtype=np.uint8)
    t[9] = t[4]
    t[30] = t[4]
    q = np.stack([t[4], t[4] ^ np.uint8(1), t[11]]).astype(np.uint8)
    return q, t


def sift_extreme(nq=200, nt=300, seed=3):
    """Queries near 0, train near 255: every best-2 lies in the float-sqrt
    collision range (s >= 2^22), so every query takes the exact slow path.
    Train rows 0..49 are near-copies of queries 0..49 (accepted at ratio 0.7)."""
    rng = np.random.default_rng(seed)
    q = rng.integers(0, 21, (nq, 128)).astype(np.float32)
    t = rng.integers(235, 256, (nt, 128)).astype(np.float32)
    t[:50] = np.clip(q[:50] + rng.integers(-3, 4, (50, 128)), 0, 255)
    return q, t
