"""Worker for test_gpu_ba_multirank: point-sharded BA across ranks (torchrun),
all ranks on one GPU, gloo all-reduce with host staging.  Prints one JSON line
(rank 0) with the final cost."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "sfm-mvs-pipeline_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from sfmx import ba, synth
    from sfmx.dist import shard_ba_problem, torch_allreduce
    if len(sys.argv) > 4 and sys.argv[4] == "multi":   # several cameras: every rank must derive the same border
        p = synth.ba_problem_multi(int(sys.argv[1]), int(sys.argv[2]), cameras=((1, 1.0), (3, 1.1)), seed=int(sys.argv[3]))
    elif len(sys.argv) > 4 and sys.argv[4] == "ring":   # SfM point order: the shards see different camera pairs
        p = synth.ba_sfm_order(synth.ba_problem(int(sys.argv[1]), int(sys.argv[2]), seed=int(sys.argv[3])))
    else:
        p = synth.ba_problem(int(sys.argv[1]), int(sys.argv[2]), seed=int(sys.argv[3]))
    local = shard_ba_problem(p, rank, world)
    local.pop("point_range")
    ctx = ba.BAContext(ba.BAProblem(**local), allreduce=torch_allreduce(cpu_staging=True))
    sm, tr = ctx.run(trace_cap=256)
    sol = ctx.get()
    cams = torch.from_numpy(sol.poses.copy())
    all_cams = [torch.zeros_like(cams) for _ in range(world)]
    dist.all_gather(all_cams, cams)
    same = all(torch.equal(all_cams[0], c) for c in all_cams)
    if rank == 0:
        print(json.dumps({"final_cost": sm["final_cost"], "initial_cost": sm["initial_cost"],
                          "termination": sm["termination_type"], "iters": sm["num_successful_steps"] +
                          sm["num_unsuccessful_steps"], "cameras_identical": bool(same)}), flush=True)
    ctx.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
