"""The FAST score formulation of the device kernel (orb_features.hip fast_score_lds, r04) against the
bit-mask test + cornerScore<16> loops it replaced, which restate OpenCV 4.5.1's FAST_t<16> and
cornerScore<16> (oracle/orb_oracle.cpp): on random, near-threshold and arc-shaped rings the corner
decision and the score agree for every threshold, and the kernel's quick pre-test passes every corner.  CPU only (test infrastructure)."""
import numpy as np


def _mask_form(v, p, t):
    d = [v - x for x in p]
    dark = sum(1 << k for k in range(16) if p[k] < v - t)
    bright = sum(1 << k for k in range(16) if p[k] > v + t)
    dd, bb = dark | (dark << 16), bright | (bright << 16)
    rd, rb = dd, bb
    for s in range(1, 9):
        rd &= dd >> s
        rb &= bb >> s
    if not ((rd | rb) & 0xFFFF):
        return 0
    a0 = t
    for k in range(0, 16, 2):
        a = min(d[(k + j) & 15] for j in range(1, 9))
        a0 = max(a0, min(a, d[k]), min(a, d[(k + 9) & 15]))
    b0 = -a0
    for k in range(0, 16, 2):
        b = max(d[(k + j) & 15] for j in range(1, 9))
        b0 = min(b0, max(b, d[k]), max(b, d[(k + 9) & 15]))
    return (-b0 - 1) & 255


def _arc_form(v, p, t):   # the kernel's: sliding minima / maxima of width 3, arcs of three runs
    d = [v - x for x in p]
    m3 = [min(d[k], d[(k + 1) & 15], d[(k + 2) & 15]) for k in range(16)]
    x3 = [max(d[k], d[(k + 1) & 15], d[(k + 2) & 15]) for k in range(16)]
    M = max(min(m3[k], m3[(k + 3) & 15], m3[(k + 6) & 15]) for k in range(16))
    N = min(max(x3[k], x3[(k + 3) & 15], x3[(k + 6) & 15]) for k in range(16))
    e = max(M, -N)
    return e - 1 if e > t else 0


def _quick_pass(v, p, t):   # the kernel's pre-test: ring pixels 0, 4, 8, 12 pairwise 4 apart
    d = [v - p[k] for k in (0, 4, 8, 12)]
    M = max(min(d[k], d[(k + 1) % 4]) for k in range(4))
    N = min(max(d[k], d[(k + 1) % 4]) for k in range(4))
    return M > t or N < -t


def test_arc_form_equals_mask_test_and_corner_score():
    rng = np.random.default_rng(7)
    corners = 0
    for it in range(24000):
        v = int(rng.integers(0, 256))
        mode = it % 4
        if mode == 0:
            p = rng.integers(0, 256, 16)
        elif mode == 1:
            p = np.clip(v + rng.integers(-40, 41, 16), 0, 255)
        elif mode == 2:   # an arc of 7..11 pixels clearly darker or brighter
            p = np.clip(v + rng.integers(-5, 6, 16), 0, 255)
            s, n, sg = rng.integers(0, 16), rng.integers(7, 12), rng.choice([-1, 1])
            for j in range(n):
                p[(s + j) % 16] = np.clip(v + sg * rng.integers(15, 60), 0, 255)
        else:
            p = np.clip(v + rng.integers(-25, 26, 16), 0, 255)
        t = int(rng.choice([0, 1, 5, 20, 40, 254, 255]))
        p = [int(x) for x in p]
        a = _mask_form(v, p, t)
        assert a == _arc_form(v, p, t), (v, p, t)
        assert a == 0 or _quick_pass(v, p, t), (v, p, t)   # the pre-test never rejects a corner
        corners += a > 0
    assert corners > 3000
