"""Pair sharding across ranks (§8e): image pairs are independent units, so each
rank (one process per GPU) takes a contiguous slice of the pair list balanced
by sum Nq*Nt, with no collective on the data path.  Mirrors the reference's
pair-parallel OpenMP loop (UnorderedFeatureMatchingStrategy.cpp:40) one level up."""
from __future__ import annotations

import numpy as np


def shard_bounds(cost: np.ndarray, world: int) -> np.ndarray:
    """Cut points [world+1] of a contiguous split of `cost` into `world` slices
    of near-equal sum (slice r = [b[r], b[r+1]))."""
    cost = np.asarray(cost, dtype=np.float64)
    n = len(cost)
    b = np.zeros(world + 1, np.int64)
    b[-1] = n
    if n == 0 or world == 1:
        return b
    cum = np.cumsum(cost)
    tot = cum[-1]
    for r in range(1, world):
        b[r] = int(np.searchsorted(cum, tot * r / world, side="left")) + 1
    b = np.maximum.accumulate(np.minimum(b, n))
    return b


def shard_pairs(pairs: np.ndarray, rows: np.ndarray, rank: int, world: int):
    """-> (this rank's pair slice, (lo, hi) indices into `pairs`)."""
    pairs = np.asarray(pairs, np.int32).reshape(-1, 2)
    rows = np.asarray(rows, np.int64)
    cost = rows[pairs[:, 0]] * rows[pairs[:, 1]] if len(pairs) else np.zeros(0)
    b = shard_bounds(cost, world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    return pairs[lo:hi], (lo, hi)


def images_for_weak_scaling(world: int, pairs_per_gpu: int = 1225) -> int:
    """Image count n whose unordered pair set has about world * pairs_per_gpu
    pairs (n = 50 at one GPU: BASELINE config 2)."""
    target = world * pairs_per_gpu
    return int(round((1 + np.sqrt(1 + 8 * target)) / 2))
