"""VERDICT r04 item 8 (CPU half of the BA sharding): every rank of a point-sharded solve must build
the SAME factorization plan, from the co-visibility all-reduced over the ranks (ensure_plan in
ba_solver.hip: the upper triangle as doubles, SUM, > 0), or the ranks would lay S out differently
and the all-reduce of the reduced camera system would add unrelated tiles.  World 4 over gloo on the
40-camera ring in SfM point order, whose shards see different camera pairs; no GPU (the adjacency
comes from the diagnostic library's host setup, the plan from sfmx_ba_plan)."""
import ctypes as C
import os
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sfm-mvs-pipeline_amd"), os.path.join(REPO, "tests")]


def _adjacency(p):
    from diag import diag_lib
    from sfmx import ba
    P = ba.BAProblem(**p)
    n = len(P.poses)
    adj = np.zeros((n, n), np.uint8)
    rc = diag_lib().sfmx_ba_debug_adjacency(P.struct(), 0, adj.ctypes.data_as(C.POINTER(C.c_uint8)))
    assert rc >= 0, diag_lib().sfmx_last_error()
    return adj


def _plan_key(adj):
    from sfmx import ba
    pl = ba.factor_plan(adj)
    return {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in pl.items() if k != "predicted_us"}


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sfmx import synth
    from sfmx.dist import shard_ba_problem
    p = synth.ba_sfm_order(synth.ba_problem(40, 4000, seed=7))
    local = shard_ba_problem(p, rank, world)
    local.pop("point_range")
    adj = _adjacency(local)
    n = adj.shape[0]
    iu = np.triu_indices(n, 1)
    h = torch.from_numpy(adj[iu].astype(np.float64))     # the ensure_plan payload
    dist.all_reduce(h, op=dist.ReduceOp.SUM)
    g = np.zeros((n, n), np.uint8)
    g[iu] = (h.numpy() > 0).astype(np.uint8)
    g = g | g.T
    plans = [None] * world
    dist.all_gather_object(plans, _plan_key(g))
    locals_ = [None] * world
    dist.all_gather_object(locals_, adj.tolist())
    if rank == 0:
        full = _adjacency(p)
        q.put((plans, locals_, g.tolist(), full.tolist(), _plan_key(full)))
    dist.barrier()
    dist.destroy_process_group()


def test_every_rank_plans_the_same_from_the_all_reduced_covisibility_world4():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29300 + os.getpid() % 700
    procs = [ctx.Process(target=_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    plans, locals_, g, full, full_plan = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    # the shards really see different camera pairs (else the all-reduce would be moot)
    assert any(locals_[r] != locals_[0] for r in range(1, 4))
    assert any(np.asarray(l).sum() < np.asarray(full).sum() for l in locals_)
    # the all-reduced graph is the whole problem's co-visibility, and every rank's plan is the one
    # a single rank builds for the whole problem
    assert g == full
    assert all(pl == plans[0] for pl in plans)
    assert plans[0] == full_plan
    assert plans[0]["height"] >= 1 and len(plans[0]["camrow"]) == 40
