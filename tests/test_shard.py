"""CPU: the multi-rank paths' host logic — pair sharding (matching, weak
scaling) and point sharding (BA) — exercised with a world_size-2 gloo group."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import sfmx
from sfmx import shard, synth
from sfmx.dist import shard_ba_problem


def test_shard_bounds_balanced_and_covering():
    rows = np.array([8192] * 50)
    pairs = sfmx.pairs_unordered(50)
    for world in (1, 2, 4, 8):
        parts = [shard.shard_pairs(pairs, rows, r, world)[1] for r in range(world)]
        assert parts[0][0] == 0 and parts[-1][1] == len(pairs)
        assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
        sizes = np.array([hi - lo for lo, hi in parts])
        assert sizes.max() - sizes.min() <= 1


def test_weak_scaling_image_counts():
    assert [shard.images_for_weak_scaling(w) for w in (1, 2, 4, 8)] == [50, 71, 99, 141]


def test_ba_point_shards_partition_observations():
    p = synth.ba_problem(10, 503, seed=4)
    shards = [shard_ba_problem(p, r, 3) for r in range(3)]
    assert sum(len(s["points"]) for s in shards) == 503
    assert sum(len(s["obs_point"]) for s in shards) == len(p["obs_point"])
    for s in shards:
        lo, hi = s["point_range"]
        assert s["obs_point"].min() == 0 and s["obs_point"].max() == hi - lo - 1
        np.testing.assert_array_equal(s["poses"], p["poses"])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows = np.array([1000 + 37 * i for i in range(20)])
    pairs = sfmx.pairs_unordered(20)
    mine, (lo, hi) = shard.shard_pairs(pairs, rows, rank, world)
    t = torch.tensor([lo, hi, len(mine)], dtype=torch.int64)
    allt = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allt, t)
    # the bench's max-over-ranks timing reduction
    el = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put(([x.tolist() for x in allt], float(el.item()), len(pairs)))
    dist.destroy_process_group()


def test_gloo_world2_pair_shards():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29000 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    shards, el, npairs = got
    assert shards[0][0] == 0 and shards[0][1] == shards[1][0] and shards[1][1] == npairs
    assert shards[0][2] + shards[1][2] == npairs
    assert el == 2.0


class _FakeCtx:
    def __init__(self):
        self.args = None

    def set_comm(self, uid, nranks, rank):
        self.args = (bytes(uid), nranks, rank)


def _rccl_worker(rank, world, port, q):
    """sfmx.dist.rccl_comm's id hand-off over gloo (no RCCL here: the id source is injected)."""
    from sfmx.dist import rccl_comm
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    made = []

    def uid():
        made.append(rank)
        return bytes([rank + 1]) * 128
    c = _FakeCtx()
    rccl_comm(c, unique_id=uid)
    # a subgroup whose rank 0 is global rank 1 (the broadcast source is a global rank)
    sub = dist.new_group([1, 2])
    c2 = _FakeCtx()
    if rank in (1, 2):
        rccl_comm(c2, group=sub, unique_id=uid)
    q.put((rank, c.args, c2.args, made))
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_comm_unique_id_hand_off_gloo_world3():
    """VERDICT r03 item 6 (CPU half): every rank gets the id its group's rank 0 made, with the group
    size and its group rank; in a subgroup the id comes from the subgroup's first member."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29100 + os.getpid() % 800
    procs = [ctx.Process(target=_rccl_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
    for rank, a, b, made in got:
        assert a == (bytes([1]) * 128, 3, rank)
        if rank in (1, 2):
            assert b == (bytes([2]) * 128, 2, rank - 1)
        else:
            assert b is None
    assert [m for _, _, _, m in got] == [[0], [1], []]
