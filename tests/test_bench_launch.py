"""bench.py --gpus N starts N ranks itself when no launcher did (the flag was
parsed and never read, so a driver call `python bench.py --gpus 8` would have measured one GPU).
CPU only: the ranks run the --launch-probe body (gloo rendezvous + all-reduce, no torch.cuda)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402

DIST_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in DIST_ENV}
    env.update({k: str(v) for k, v in kw.items()})
    return env


def _run(args, env, timeout=120):
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_resolve_world_rules():
    a = bench.parse(["--gpus", "4"])
    assert bench.resolve_world(a, {}) == (4, True)                    # no launcher: start 4 ranks here
    assert bench.resolve_world(a, {"WORLD_SIZE": "4"}) == (4, False)  # launched: this process is one rank
    with pytest.raises(SystemExit):
        bench.resolve_world(a, {"WORLD_SIZE": "2"})                   # mismatch: refuse
    assert bench.resolve_world(bench.parse([]), {}) == (1, False)       # default: one GPU, in process
    assert bench.resolve_world(bench.parse([]), {"WORLD_SIZE": "3"}) == (3, False)
    assert bench.resolve_world(bench.parse(["--gpus", "1"]), {}) == (1, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(bench.parse(["--gpus", "0"]), {})


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    r = _run(["--gpus", str(n), "--launch-probe"], _env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout                     # exactly rank 0's line is forwarded
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["rank_sum"] == n * (n - 1) / 2 and d["local_rank"] == 0


def test_mismatch_with_launcher_env_is_refused():
    r = _run(["--gpus", "4", "--launch-probe"], _env(WORLD_SIZE=2, RANK=0, LOCAL_RANK=0), timeout=60)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_failed_rank_fails_the_launch():
    # rank 1 exits before the rendezvous; rank 0 would block in it forever: the launcher ends it
    r = _run(["--gpus", "2", "--launch-probe"], _env(SFMX_BENCH_PROBE_FAIL_RANK=1), timeout=120)
    assert r.returncode != 0 and "rank(s) failed" in r.stderr
