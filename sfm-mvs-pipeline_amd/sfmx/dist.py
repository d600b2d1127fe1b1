"""Multi-GPU plumbing: one process per GPU, torch.distributed (RCCL over xGMI on
MI355X, gloo on CPU for tests).

* Matching shards image pairs (sfmx.shard): no collective on the data path.
* Bundle adjustment shards POINTS (with their observations); cameras and the
  shared intrinsics are replicated.  libsfmx calls the all-reduce hook on the
  reduced camera system S + rhs once per LM step, on the camera/intrinsics
  column norms once per linearisation, and on a few scalars (include/sfmx_ba.h).
  The reference has no distributed path at all (OpenMP only).
"""
from __future__ import annotations

import numpy as np

REDUCE_SUM, REDUCE_MAX = 0, 1


def shard_ba_problem(prob: dict, rank: int, world: int) -> dict:
    """A contiguous point range with its observations, cut so that every rank holds about
    the same number of OBSERVATIONS (the per-step work of ba_glin / ba_gschur / ba_gupdate
    is per observation; real tracks have 2 to hundreds of them); cameras and intrinsics
    replicated.  Observation order (point-major) is preserved."""
    from .shard import shard_bounds
    P = len(prob["points"])
    op = np.asarray(prob["obs_point"])
    b = shard_bounds(np.bincount(op, minlength=P), world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    sel = (op >= lo) & (op < hi)
    out = dict(prob)
    out["points"] = np.asarray(prob["points"])[lo:hi]
    out["obs_point"] = (op[sel] - lo).astype(np.int32)
    out["obs_cam"] = np.asarray(prob["obs_cam"])[sel]
    out["obs_xy"] = np.asarray(prob["obs_xy"])[sel]
    out["point_range"] = (lo, hi)
    return out


def rccl_comm(ctx, group=None, unique_id=None) -> None:
    """Give a BAContext native RCCL collectives (sfmx_ba_set_comm): the group's rank 0 creates the
    id, torch.distributed broadcasts it (any backend), every rank initialises its communicator.
    `unique_id` replaces sfmx.ba.comm_unique_id (tests of the hand-off without RCCL)."""
    import torch.distributed as dist
    from .ba import comm_unique_id as _uid
    comm_unique_id = unique_id or _uid
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    obj = [comm_unique_id() if rank == 0 else None]
    # broadcast_object_list takes a GLOBAL source rank: the group's rank 0
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast_object_list(obj, src=src, group=group)
    ctx.set_comm(obj[0], world, rank)


class _DevView:
    """Zero-copy view of a raw device buffer (doubles) for torch.as_tensor."""

    def __init__(self, ptr: int, count: int):
        self.__cuda_array_interface__ = {"shape": (count,), "typestr": "<f8", "data": (ptr, False), "version": 3}


def torch_allreduce(group=None, cpu_staging: bool = False):
    """-> callable(ptr, count, op, stream) for sfmx.ba.BAContext(allreduce=...).
    The collective is ordered on the solver's HIP stream (ExternalStream); with
    cpu_staging the buffer goes through host memory (gloo)."""
    import torch
    import torch.distributed as dist

    def fn(ptr: int, count: int, op: int, stream: int):
        rop = dist.ReduceOp.SUM if op == REDUCE_SUM else dist.ReduceOp.MAX
        t = torch.as_tensor(_DevView(ptr, count), device="cuda")
        if cpu_staging:
            torch.cuda.synchronize()
            h = t.cpu()
            dist.all_reduce(h, op=rop, group=group)
            t.copy_(h)
            torch.cuda.synchronize()
            return
        s = torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()
        with torch.cuda.stream(s):
            dist.all_reduce(t, op=rop, group=group)

    return fn
