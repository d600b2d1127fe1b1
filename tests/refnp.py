"""Independent numpy restatement of the matcher semantics (test helper).

Deliberately a different computation from oracle/match_oracle.cpp: exact
int64 squared distances by matrix product, numpy's correctly-rounded float32
sqrt, and a stable sort on the 64-bit key (float bits << 32 | train index).
Used to cross-check the C++ oracle (which in turn checks the GPU path)."""
import numpy as np


def knn2_l2_int(q: np.ndarray, t: np.ndarray):
    """q, t integer-valued float32 -> (idx[nq,2], dist[nq,2]) with idx=-1 for absent."""
    qi = q.astype(np.int64)
    ti = t.astype(np.int64)
    s = (qi * qi).sum(1)[:, None] + (ti * ti).sum(1)[None, :] - 2 * (qi @ ti.T)
    d = np.sqrt(s.astype(np.float32))            # s < 2^24: exact in f32; sqrt correctly rounded
    return _top2(d.view(np.uint32).astype(np.int64), d, t.shape[0])


def knn2_hamming(q: np.ndarray, t: np.ndarray):
    x = np.bitwise_xor(q[:, None, :], t[None, :, :])
    d = np.unpackbits(x, axis=2).sum(2).astype(np.int64)
    return _top2(d, d.astype(np.float32), t.shape[0])


def _top2(keyhi: np.ndarray, d: np.ndarray, nt: int):
    nq = keyhi.shape[0]
    idx = np.full((nq, 2), -1, np.int32)
    dist = np.zeros((nq, 2), np.float32)
    if nt == 0:
        return idx, dist
    key = (keyhi << 32) | np.arange(nt, dtype=np.int64)[None, :]
    k = min(2, nt)
    part = np.argsort(key, axis=1, kind="stable")[:, :k]
    idx[:, :k] = part
    dist[:, :k] = np.take_along_axis(d, part, axis=1)
    return idx, dist


def ratio_filter(idx, dist, nt, ratio=0.7):
    out = []
    for i in range(idx.shape[0]):
        if nt == 0:
            continue
        if nt >= 2:
            if float(dist[i, 0]) < float(dist[i, 1]) * ratio:
                out.append((i, int(idx[i, 0]), 0, dist[i, 0]))
        else:
            out.append((i, int(idx[i, 0]), 0, dist[i, 0]))
    return np.array(out, dtype=[("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"), ("distance", "<f4")])


def match_pair(q, t, ratio=0.7):
    if q.dtype == np.uint8:
        idx, dist = knn2_hamming(q, t)
    else:
        idx, dist = knn2_l2_int(q, t)
    return ratio_filter(idx, dist, t.shape[0], ratio)
